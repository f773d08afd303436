"""CLI: matrix factorisation training (drop-in for the reference's mf_spotlight.py:1-75).

    python -m recommendation_gans_amd.mf_spotlight --use_gpu True --dataset 20M \
        --mf_embedding_dim 64 --batch_size 8192 --training_epochs 5 [--mf_loss pairwise_bpr]

Same flags, seeding (RandomState(0) for the model, torch.manual_seed(0) before the
representation), data provider, model construction, fit / test calls and log
lines as the reference; ``--mf_loss`` is additive (the reference CLI never passes
a loss, so its runs are pointwise, the default here too)."""
import logging
import os
import sys

import numpy as np
import torch

from .implicit import ImplicitFactorizationModel
from .spotlight import optimizers
from .spotlight.factorization.representations import BilinearNet
from .utils.arg_extractor import get_args
from .utils.data_provider import data_provider


def init_data_parallel(world_size):
    """--world_size N (additive): one process per GPU under torchrun; rank, local rank and the
    rendezvous come from the environment.  Called before any GPU work.  The process group
    carries the RCCL id and the final table gather; the step's exchanges run over RCCL inside
    the native step (mf_engine.MFEngine dp="owner")."""
    import torch.distributed as dist
    if world_size <= 1:
        return 0
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    torch.cuda.set_device(local)
    dist.init_process_group(os.environ.get("RG_DP_BACKEND", "nccl"), world_size=world_size,
                            device_id=torch.device("cuda", local))
    return dist.get_rank()


def main(argv=None):
    logging.basicConfig(format="%(message)s", level=logging.INFO)
    args = get_args(argv)
    rank = init_data_parallel(args.world_size)
    logging.info("DataSet MovieLens_%s will be used" % args.dataset)
    path = "/disk/scratch/s1877727/datasets/movielens/" if args.on_cluster else "datasets/movielens/"
    seed = 0
    random_state = np.random.RandomState(seed)
    torch.manual_seed(seed)
    loader = data_provider(path, args.dataset, args.neg_examples, movies_to_keep=-1, synthetic=args.synthetic,
                           zipf=args.zipf)
    train, valid, test, neg_examples, item_popularity = loader.get_timebased_data()
    users, movies = train.num_users, train.num_items
    embedding_dim = args.mf_embedding_dim
    technique = BilinearNet(users, movies, embedding_dim, sparse=False)
    optim = getattr(optimizers, args.optim + "_optimizer")
    model = ImplicitFactorizationModel(n_iter=args.training_epochs, neg_examples=neg_examples,
                                       num_negative_samples=args.neg_examples, model_name="mf",
                                       embedding_dim=embedding_dim, l2=args.l2_regularizer,
                                       representation=technique, random_state=random_state,
                                       batch_size=args.batch_size, use_cuda=bool(args.use_gpu),
                                       learning_rate=args.learning_rate, optimizer_func=optim,
                                       experiment_name=args.experiment_name, loss=args.mf_loss,
                                       world_size=args.world_size)
    logging.info("Model set, training begins")
    model.fit(train, valid, verbose=rank == 0)
    if rank != 0:                       # every rank holds the gathered model; rank 0 evaluates and logs
        return model
    logging.info("Model is ready, testing performance")
    model.test(test, item_popularity, args.k, rmse_flag=args.rmse, precision_recall=args.precision_recall,
               map_recall=args.map_recall)
    logging.info("Training session: {} latent dimensions, {} epochs, {} batch size {} learning rate {} "
                 "l2_regularizer.  {} users x  {} items".format(embedding_dim, args.training_epochs,
                                                               args.batch_size, args.learning_rate,
                                                               args.l2_regularizer, users, movies))
    return model


if __name__ == "__main__":
    main()
