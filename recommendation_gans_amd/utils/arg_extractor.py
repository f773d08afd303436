"""Command-line flags shared by the CLIs (utils/arg_extractor.py:15-77 of the
reference): every reference flag with its default, plus additive flags only
(SURVEY §5): --mf_loss, --synthetic, --zipf, --seed_random."""
import argparse


def str2bool(v):
    if isinstance(v, bool):
        return v
    if v.lower() in ("yes", "true", "t", "y", "1"):
        return True
    if v.lower() in ("no", "false", "f", "n", "0"):
        return False
    raise argparse.ArgumentTypeError("Boolean value expected.")


def build_parser():
    p = argparse.ArgumentParser(description="MI355X MF / NCF / cGAN training (recommendation_Gans drop-in)")
    # reference flags (same names, types and defaults)
    p.add_argument("--use_gpu", nargs="?", type=str2bool, default=False)
    p.add_argument("--l2_regularizer", type=float, default=1e-5)
    p.add_argument("--on_cluster", type=str2bool, default=False)
    p.add_argument("--model", type=str, default="mf")
    p.add_argument("--dataset", type=str, default="100K")
    p.add_argument("--experiment_name", type=str, default="matrix_model")
    p.add_argument("--precision_recall", type=str2bool, default=True)
    p.add_argument("--map_recall", type=str2bool, default=True)
    p.add_argument("--rmse", type=str2bool, default=True)
    p.add_argument("--mf_embedding_dim", type=int, default=50)
    p.add_argument("--mlp_embedding_dim", type=int, default=16)
    p.add_argument("--training_epochs", type=int, default=50)
    p.add_argument("--batch_size", type=int, default=256)
    p.add_argument("--learning_rate", type=float, default=1e-3)
    p.add_argument("--optim", type=str, default="adam")
    p.add_argument("--k", type=int, default=3)
    p.add_argument("--neg_examples", type=int, default=5)
    p.add_argument("--optim_gan", type=str, default="rms")
    p.add_argument("--gan_embedding_dim", type=int, default=5)
    p.add_argument("--gan_hidden_layer", type=int, default=10)
    p.add_argument("--loss", type=str, default="bce")
    p.add_argument("--slate_size", type=int, default=3)
    # additive flags
    p.add_argument("--mf_loss", type=str, default="pointwise",
                   help="pointwise (the reference CLI's effective loss) / bpr (= adaptive hinge, as the "
                        "reference maps it) / hinge / adaptive_hinge / pairwise_bpr (1 - sigmoid(pos - neg))")
    p.add_argument("--synthetic", type=str2bool, default=None,
                   help="synthetic MovieLens-shaped data when the dataset cache files are absent (default: auto)")
    p.add_argument("--zipf", type=float, default=1.0, help="item popularity skew of the synthetic data")
    # additive: data-parallel MF training, one process per GPU under torchrun (the reference's
    # single process at batch world_size * batch_size)
    p.add_argument("--world_size", type=int, default=1)
    return p


def get_args(argv=None):
    return build_parser().parse_args(argv)
