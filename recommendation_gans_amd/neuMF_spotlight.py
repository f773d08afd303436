"""CLI: NeuMF training (drop-in for the reference's neuMF_spotlight.py:1-78).

    python -m recommendation_gans_amd.neuMF_spotlight --use_gpu True --dataset 20M \
        --mlp_embedding_dim 16 --mf_embedding_dim 50 --batch_size 8192 --training_epochs 5

Same flags, seeding, tower sizes ([2**x for x in reversed(range(3, log2(2E) + 1))],
neuMF_spotlight.py:53-55), data provider, model construction (model_name 'neuMf', the
model's default loss) and fit / test calls as the reference; training runs through
the fused NCF step with the GMF branch (rg_ncf.hip, rg_neumf_apply)."""
import logging

import numpy as np
import torch

from .implicit import ImplicitFactorizationModel
from .ncf_spotlight import mlp_layers
from .spotlight import optimizers
from .spotlight.dnn_models.neuMF import NeuMF
from .mf_spotlight import init_data_parallel
from .utils.arg_extractor import get_args
from .utils.data_provider import data_provider


def main(argv=None):
    logging.basicConfig(format="%(message)s", level=logging.INFO)
    args = get_args(argv)
    rank = init_data_parallel(args.world_size)     # additive --world_size (torchrun, one process per GPU)
    logging.info("DataSet MovieLens_%s will be used" % args.dataset)
    path = "/disk/scratch/s1877727/datasets/movielens/" if args.on_cluster else "datasets/movielens/"
    seed = 0
    random_state = np.random.RandomState(seed)
    torch.manual_seed(seed)
    loader = data_provider(path, args.dataset, args.neg_examples, movies_to_keep=-1, synthetic=args.synthetic,
                           zipf=args.zipf)
    train, valid, test, neg_examples, item_popularity = loader.get_timebased_data()
    users, movies = train.num_users, train.num_items
    E, M = args.mlp_embedding_dim, args.mf_embedding_dim
    layers = mlp_layers(E)
    logging.info(layers)
    technique = NeuMF(layers, users, movies, mf_embedding_dim=M, mlp_embedding_dim=E)
    logging.info(technique)
    optim = getattr(optimizers, args.optim + "_optimizer")
    model = ImplicitFactorizationModel(n_iter=args.training_epochs, neg_examples=neg_examples,
                                       num_negative_samples=args.neg_examples, model_name="neuMf", embedding_dim=E,
                                       l2=args.l2_regularizer, representation=technique, random_state=random_state,
                                       batch_size=args.batch_size, use_cuda=bool(args.use_gpu),
                                       learning_rate=args.learning_rate, optimizer_func=optim,
                                       experiment_name=args.experiment_name, world_size=args.world_size)
    logging.info("Model set, training begins")
    model.fit(train, valid, verbose=rank == 0)
    if rank != 0:                       # replicated model: rank 0 evaluates and logs
        return model
    logging.info("Model is ready, testing performance")
    model.test(test, item_popularity, args.k, rmse_flag=args.rmse, precision_recall=args.precision_recall,
               map_recall=args.map_recall)
    logging.info("Training session: {} latent dimensions, {} epochs, {} batch size {} learning rate {} "
                 "l2_regularizer.  {} users x  {} items".format(E, args.training_epochs, args.batch_size,
                                                               args.learning_rate, args.l2_regularizer, users,
                                                               movies))
    return model


if __name__ == "__main__":
    main()
