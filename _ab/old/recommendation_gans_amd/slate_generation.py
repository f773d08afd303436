"""CLI: cGAN slate generation (drop-in for the reference's slate_generation.py:1-104).

    python -m recommendation_gans_amd.slate_generation --use_gpu True --dataset 20M \
        --slate_size 5 --gan_hidden_layer 256 --training_epochs 5

Same flags, seeding (RandomState(0), torch.manual_seed(0)), data provider call,
network shapes (G hidden [H/2, H], D hidden [2H, H, H/2], noise 100), optimizer
(``--optim_gan``, default rms) and fit / test calls as the reference; training runs
through the fused discriminator / generator iterations (rg_gan.hip)."""
import logging

import numpy as np
import torch

from .CGANs import CGAN
from .spotlight import optimizers
from .spotlight.dnn_models.cGAN_models import discriminator, generator
from .utils.arg_extractor import get_args
from .utils.slate_data_provider import slate_data_provider


def main(argv=None):
    logging.basicConfig(format="%(message)s", level=logging.INFO)
    args = get_args(argv)
    logging.info("DataSet MovieLens_%s will be used" % args.dataset)
    path = "/disk/scratch/s1877727/datasets/movielens/" if args.on_cluster else "datasets/movielens/"
    seed = 0
    random_state = np.random.RandomState(seed)
    torch.manual_seed(seed)
    loader = slate_data_provider(path, args.dataset, min_viewers=5, slate_size=args.slate_size, min_movies=0,
                                 movies_to_keep=-1, synthetic=args.synthetic, zipf=args.zipf)
    (train_vec, train_slates, test_vec, test_set, num_users, num_movies, valid_vec, valid_cold_users,
     valid_set) = loader.get_data()
    cold_start_users = loader.get_cold_start_users()
    noise_dim = 100
    H = args.gan_hidden_layer
    Gen = generator(num_items=num_movies, noise_dim=noise_dim, embedding_dim=args.gan_embedding_dim,
                    hidden_layer=[H // 2, H], output_dim=args.slate_size)
    Disc = discriminator(num_items=num_movies, embedding_dim=args.gan_embedding_dim,
                         hidden_layers=[2 * H, H, H // 2], input_dim=args.slate_size)
    optim = getattr(optimizers, args.optim_gan + "_optimizer")
    model = CGAN(n_iter=args.training_epochs, z_dim=noise_dim, embedding_dim=args.gan_embedding_dim,
                 hidden_layer=H, batch_size=args.batch_size, loss_fun=args.loss, slate_size=args.slate_size,
                 learning_rate=args.learning_rate, use_cuda=args.use_gpu, experiment_name=args.experiment_name,
                 G_optimizer_func=optim, D_optimizer_func=optim, G=Gen, D=Disc, random_state=random_state)
    logging.info(" Training session: {}  epochs, {} batch size {} learning rate.  {} users x  {} items".format(
        args.training_epochs, args.batch_size, args.learning_rate, num_users, num_movies))
    logging.info("Model set, training begins")
    model.fit(train_vec, train_slates, num_users, num_movies, valid_vec, valid_cold_users, valid_set)
    logging.info("Model is ready, testing performance")
    results = model.test(test_vec, test_set.tocsr(), cold_start_users)
    logging.info("precision {} and recall {}".format(results["precision"], results["recall"]))
    logging.info("Training complete")
    return model, results


if __name__ == "__main__":
    main()
