"""ImplicitFactorizationModel -- drop-in for the reference's implicit.py:31-471.

Same constructor arguments, attributes, ``fit(train_set, valid_set, verbose)``,
``run_train_iteration`` / ``run_val_iteration``, ``predict``, ``test`` and output
files (``experiments_results/<name>/result_outputs/{configuration.json,
summary.csv, test_summary.json}``, ``saved_models/best_model`` =
``torch.save({'network': state_dict})``).  Training of a BilinearNet runs
through the fused MI355X step (``mf_engine.MFEngine`` over librg_hip.so); there
is no CPU training path.

Semantics kept from the reference:
* ``loss``: 'pointwise' -> pointwise, 'hinge' -> hinge, anything else of the
  allowed names ('bpr', 'adaptive_hinge') -> adaptive hinge (implicit.py:194-199);
  the build's pairwise BPR is the additive name 'pairwise_bpr';
* negatives: ``random.choices(neg_examples, k=num_negative_samples * batch_size)``
  from the module-level ``random`` stream (implicit.py:352), shared by training and
  validation; the device stream starts at ``random.getstate()`` and is written
  back with ``random.setstate`` after ``fit``;
* one shuffle with the model's RandomState before the epochs (implicit.py:262),
  ``set_seed(random_state.randint(-1e8, 1e8))`` at construction (:146);
* the optimizer is what ``optimizer_func(params, weight_decay=l2, lr=lr)`` builds
  (Adam when None), applied densely to every row every step;
* best-by-validation-loss model, degenerate-loss ValueError, id-range ValueErrors.
"""
import copy
import json
import logging
import os
import random

import numpy as np
import torch

from . import _mtstate
from .mf_engine import MFEngine
from .ncf_engine import NCFEngine
from .spotlight.factorization.representations import BilinearNet
from .spotlight.optimizers import describe
from .spotlight.sampling import NegativePool
from .spotlight.torch_utils import set_seed, shuffle
from .spotlight import evaluation
from .spotlight import losses
from .utils.storage_utils import save_statistics

logging.basicConfig(format="%(message)s", level=logging.INFO)

_LOSS_MAP = {"pointwise": "pointwise", "hinge": "hinge", "bpr": "adaptive_hinge",
             "adaptive_hinge": "adaptive_hinge", "pairwise_bpr": "bpr"}


class ImplicitFactorizationModel:
    def __init__(self, loss="pointwise", embedding_dim=32, n_iter=10, batch_size=256, l2=0.0,
                 experiment_name="Implicit_Feedback", learning_rate=1e-2, optimizer_func=None, use_cuda=False,
                 representation=None, sparse=False, model_name="mf", random_state=None, neg_examples=None,
                 num_negative_samples=3, world_size=1):
        self.exeriment_name = experiment_name
        self.experiment_folder = os.path.abspath("experiments_results/" + experiment_name)
        self.experiment_logs = os.path.join(self.experiment_folder, "result_outputs")
        self.experiment_saved_models = os.path.join(self.experiment_folder, "saved_models")
        self.starting_epoch = 0
        for d in (self.experiment_logs, self.experiment_saved_models):
            os.makedirs(d, exist_ok=True)
        assert loss in _LOSS_MAP, loss
        self._loss = loss
        self._embedding_dim = embedding_dim
        self._n_iter = n_iter
        self._learning_rate = learning_rate
        self._batch_size = batch_size
        self._l2 = l2
        self._use_cuda = use_cuda
        self._representation = representation
        self._sparse = sparse
        self._optimizer_func = optimizer_func
        self._random_state = random_state or np.random.RandomState()
        self._num_negative_samples = num_negative_samples
        self.neg_examples = neg_examples
        self._num_users = None
        self._num_items = None
        self._net = None
        self._engine = None
        self.best_model = None
        self.best_validation = None
        self.model_name = model_name
        self.best_epoch = -1
        # additive: data-parallel training over world_size processes (one per GPU, under
        # torchrun, torch.distributed initialised by the caller before any GPU work); the
        # reference's single process at batch world_size * batch_size, reproduced by the
        # owner-sharded layout (mf_engine.MFEngine dp="owner")
        self._world = int(world_size)
        self._rank = 0
        self._full_tables = None
        if self._world > 1:
            import torch.distributed as dist
            if not dist.is_initialized() or dist.get_world_size() != self._world:
                raise RuntimeError("world_size > 1 needs torch.distributed initialised with that many ranks "
                                   "(torchrun; mf_spotlight.py --world_size)")
            self._rank = dist.get_rank()
        set_seed(self._random_state.randint(-10 ** 8, 10 ** 8), cuda=self._use_cuda)

    def __repr__(self):
        return "<ImplicitFactorizationModel: {}>".format(
            "uninitialised" if self._net is None else f"{self._num_users} users x {self._num_items} items, "
                                                      f"d={self._embedding_dim}, loss={self._loss}")

    @property
    def _initialized(self):
        return self._net is not None

    # ------------------------------------------------------------------ setup
    def _device(self):
        if not self._use_cuda:
            raise RuntimeError("this implementation trains on the GPU only (librg_hip.so): pass use_cuda=True")
        return torch.device("cuda", torch.cuda.current_device())

    def _initialize(self, interactions):
        self._num_users, self._num_items = interactions.num_users, interactions.num_items
        dev = self._device()
        net = self._representation
        if net is None:
            net = BilinearNet(self._num_users, self._num_items, self._embedding_dim, sparse=self._sparse)
        self._net = net.to(dev)
        self._opt = describe(self._optimizer_func, self._learning_rate, self._l2)
        # the reference's loss selection (implicit.py:194-199); the fused step computes the same
        # loss in its kernel, this is the function for callers that score pairs themselves
        self._loss_func = losses.bpr_loss if self._loss == "pairwise_bpr" else losses.loss_for(self._loss)
        # implicit.py:351-360: without a negative pool the loss sees the positives only --
        # self._loss_func(positive_prediction) -- and no draw is taken from `random`
        self._no_negatives = not self.neg_examples
        if self._no_negatives:
            if self._loss != "pointwise":   # the reference's pairwise losses need the negatives argument
                raise TypeError(f"{self._loss_func.__name__}() missing 1 required positional argument: "
                                f"'negative_predictions'")
            if self._world > 1:
                raise NotImplementedError("data-parallel training needs a negative pool")
        self._pool = NegativePool.from_pairs([(0, 0)] if self._no_negatives else self.neg_examples)
        engine_loss = "pointwise_pos" if self._no_negatives else _LOSS_MAP[self._loss]
        o = self._opt
        common = dict(loss=engine_loss, optimizer=o["kind"], lr=o["lr"], weight_decay=o["weight_decay"],
                      betas=o.get("betas", (0.9, 0.999)), eps=o.get("eps", 1e-8), alpha=o.get("alpha", 0.99),
                      n_neg=self._num_negative_samples, batch_size=self._batch_size, device=dev)
        ncf_dp = {}
        if self._world > 1:
            import torch.distributed as dist
            comm = None
            if dist.get_backend() == "nccl":           # RCCL: the exchanges run inside the native step
                from .comm import RcclComm
                comm = RcclComm(dev)
            ncf_dp = dict(rank=self._rank, world_size=self._world, comm=comm)
        is_mf = hasattr(net, "user_embeddings") and hasattr(net, "item_biases")
        if self._no_negatives and not is_mf:   # before any engine (and its device state) is built
            raise NotImplementedError("training without a negative pool is implemented for BilinearNet")
        if hasattr(net, "embedding_user_mlp") and hasattr(net, "affine_output"):   # NeuMF (neuMF.py:7-55)
            self._kind = "ncf"
            self._params = [net.embedding_user_mlp.weight, net.embedding_item_mlp.weight,
                            net.embedding_user_mf.weight, net.embedding_item_mf.weight]
            for lin in [m_ for m_ in net.layers if isinstance(m_, torch.nn.Linear)] + [net.affine_output]:
                self._params += [lin.weight, lin.bias]
            self._embedding_dim = net.embedding_user_mlp.weight.shape[1]
            w = [p.detach() for p in self._params]
            self._engine = NCFEngine(w[0], w[1], w[4:], self._pool.user_ids, self._pool.item_ids, _mtstate.current(),
                                     seed=int(torch.randint(0, 2 ** 31 - 1, (1,)).item()), mf_user_w=w[2],
                                     mf_item_w=w[3], **common, **ncf_dp)
        elif hasattr(net, "embedding_user") and hasattr(net, "layers"):          # NCF MLP (mlp.py:5-46)
            self._kind = "ncf"
            self._params = [net.embedding_user.weight, net.embedding_item.weight]
            for lin in [m_ for m_ in net.layers if isinstance(m_, torch.nn.Linear)]:
                self._params += [lin.weight, lin.bias]
            self._embedding_dim = net.embedding_user.weight.shape[1]
            self._engine = NCFEngine(self._params[0].detach(), self._params[1].detach(),
                                     [p.detach() for p in self._params[2:]], self._pool.user_ids,
                                     self._pool.item_ids, _mtstate.current(),
                                     seed=int(torch.randint(0, 2 ** 31 - 1, (1,)).item()), **common, **ncf_dp)
        elif hasattr(net, "user_embeddings") and hasattr(net, "item_biases"):   # BilinearNet
            self._kind = "mf"
            self._params = [net.user_embeddings.weight, net.item_embeddings.weight, net.user_biases.weight,
                            net.item_biases.weight]
            self._embedding_dim = net.user_embeddings.weight.shape[1]
            w = [p.detach() for p in self._params]
            dp = {}
            if self._world > 1:
                dp = dict(rank=self._rank, world_size=self._world, dp="owner", comm=ncf_dp["comm"])
            self._engine = MFEngine(w[0], w[1], w[2].reshape(-1), w[3].reshape(-1), self._pool.user_ids,
                                    self._pool.item_ids, _mtstate.current(), **common, **dp)
        else:
            raise NotImplementedError("the fused steps train BilinearNet, the NCF MLP and NeuMF representations")
        self.configuration = {"num_users": self._num_users, "num_items": self._num_items,
                              "weight_decay": self._l2, "lr": self._learning_rate,
                              "embedding_dim": self._embedding_dim, "batch_size": self._batch_size,
                              "epochs": self._n_iter}
        if self._rank == 0:            # one writer per experiment folder in a data-parallel fit
            with open(os.path.join(self.experiment_logs, "configuration.json"), "w") as fp:
                json.dump(self.configuration, fp)

    def _check_input(self, user_ids, item_ids, allow_items_none=False):
        user_id_max = user_ids if isinstance(user_ids, int) else user_ids.max()
        if user_id_max >= self._num_users:
            raise ValueError("Maximum user id greater than number of users in model.")
        if allow_items_none and item_ids is None:
            return
        item_id_max = item_ids if isinstance(item_ids, int) else item_ids.max()
        if item_id_max >= self._num_items:
            raise ValueError("Maximum item id greater than number of items in model.")

    # ------------------------------------------------------------------ training
    def fit(self, train_set, valid_set, verbose=False):
        self.train_set = train_set
        users, items = shuffle(train_set.user_ids, train_set.item_ids, random_state=self._random_state)
        if not self._initialized:
            self._initialize(train_set)
        self._check_input(train_set.user_ids, train_set.item_ids)
        e, dev = self._engine, self._engine.device
        b = self._batch_size
        B = b * self._world                        # the global batch (one process at world * batch_size)
        R, r = self._world, self._rank
        owner = R > 1 and self._kind == "mf"       # MF: owner-sharded; NCF / NeuMF: replicated columns
        allreduce = None
        if R > 1 and e.comm is None:               # gloo process group: exchanges through torch.distributed
            import torch.distributed as dist
            allreduce = dist.all_reduce
        e.set_mt_state(_mtstate.current())
        tu = torch.from_numpy(np.ascontiguousarray(users, dtype=np.int64)).to(dev)
        ti = torch.from_numpy(np.ascontiguousarray(items, dtype=np.int64)).to(dev)
        vu = torch.from_numpy(np.ascontiguousarray(valid_set.user_ids, dtype=np.int64)).to(dev)
        vi = torch.from_numpy(np.ascontiguousarray(valid_set.item_ids, dtype=np.int64)).to(dev)
        nb = (len(tu) + B - 1) // B
        losses = torch.zeros(nb, dtype=torch.float32, device=dev)
        total = {"train_loss": [], "validation_loss": [], "curr_epoch": []}
        # the batches repeat every epoch (one shuffle): plans (and MF step inputs) are built once
        # (one launch builds every batch's plan, rg_mf_plans_build)
        if owner:
            plans = e.make_plans(ti, users=tu)
        elif R > 1:                                # this rank's columns [r*b, (r+1)*b) of each global batch
            plans = e.make_plans(ti, offset=r * b, stride=B, n_batches=nb)
        else:
            plans = e.make_plans(ti)
        vplans = e.make_plans(vi, users=vu) if owner else None

        def cols(x, s):                            # this rank's columns of global batch s (NCF / NeuMF)
            lo = min(s * B + r * b, len(x))
            return x[lo:min(lo + b, (s + 1) * B, len(x))]
        if self._kind == "mf":
            inputs = [e.step_input(tu[s * B:(s + 1) * B], ti[s * B:(s + 1) * B], None, plans[s]) for s in range(nb)]
        for epoch in range(self._n_iter):
            for s in range(nb):
                nxt = inputs[s + 1] if self._kind == "mf" and s + 1 < nb else None
                if self._kind == "mf" and allreduce is not None:
                    e.train_step_owner_exchange(inputs[s], nxt, allreduce, loss_out=losses[s:s + 1])
                elif self._kind == "mf":
                    e.train_step_in(inputs[s], nxt, loss_out=losses[s:s + 1])
                else:
                    nxt = (cols(tu, s + 1), cols(ti, s + 1), plans[s + 1]) if s + 1 < nb else None
                    e.train_step(cols(tu, s), cols(ti, s), global_pos=min(B, len(tu) - s * B), plan=plans[s],
                                 loss_out=losses[s:s + 1], next_step=nxt, allreduce=allreduce)
            tl = [float(x) for x in losses.cpu().numpy()]          # loss.item() per batch
            train_epoch_loss = sum(tl) / nb
            if np.isnan(train_epoch_loss) or train_epoch_loss == 0.0:
                raise ValueError("Degenerate epoch loss: {}".format(train_epoch_loss))
            if owner:
                vl = [float(e.val_loss(vu[s:s + B], vi[s:s + B], plan=vplans[s // B], allreduce=allreduce)[0])
                      for s in range(0, len(vu), B)]
            elif R > 1:
                vl = [float(e.val_loss(cols(vu, s), cols(vi, s), global_pos=min(B, len(vu) - s * B),
                                       allreduce=allreduce)[0]) for s in range(-(-len(vu) // B))]
            else:
                vl = [float(e.val_loss(vu[s:s + B], vi[s:s + B])[0]) for s in range(0, len(vu), B)]
            valid_epoch_loss = sum(vl) / len(vl)
            if self.best_validation is None or valid_epoch_loss < self.best_validation:
                self.best_model = [t.detach().clone() for t in e.params()]
                self.best_validation = valid_epoch_loss
                self.best_epoch = epoch
            if verbose:
                logging.info("Epoch {}: training_loss {:10.5f}".format(epoch, train_epoch_loss))
                logging.info("Epoch {}: validation_loss {:10.5f}".format(epoch, valid_epoch_loss))
            total["train_loss"].append(np.mean(tl))
            total["validation_loss"].append(np.mean(vl))
            total["curr_epoch"].append(epoch)
            if self._rank == 0:
                save_statistics(experiment_log_dir=self.experiment_logs, filename="summary.csv", stats_dict=total,
                                current_epoch=epoch, continue_from_mode=(self.starting_epoch != 0 or epoch > 0))
        if not self._no_negatives:                     # the Python stream continues after fit
            _mtstate.restore(e.mt_state())
        if self._kind == "mf":
            e.set_params(*self.best_model)
        else:
            e.set_params(self.best_model)
        if owner:                                      # every rank gets the full best tables
            self.best_model = self._gather_tables(self.best_model)
            self._full_tables = [t.to(dev) for t in self.best_model]
        self._load_into_net(self.best_model)
        if self._rank == 0:
            self.save_readable_model(self.experiment_saved_models, self._net.state_dict())
        logging.info("Model chosen from epoch %d", self.best_epoch)

    def _gather_tables(self, local):
        """Full (user_w, item_w, user_b, item_b) from every rank's user rows (u % R == rank,
        local row u // R) and the replicated items."""
        import torch.distributed as dist
        from . import sharding
        mine = [t.detach().cpu().numpy() for t in local]
        shards = [None] * self._world
        dist.all_gather_object(shards, mine[0::2])     # user rows and user biases
        uw = sharding.unshard_rows([x[0] for x in shards], self._num_users)
        ub = sharding.unshard_rows([x[1] for x in shards], self._num_users)
        return [torch.from_numpy(uw), torch.from_numpy(mine[1]).clone(), torch.from_numpy(ub),
                torch.from_numpy(mine[3]).clone()]

    def _tables(self):
        """The MF tables the evaluation reads: the engine's, or after a data-parallel fit
        (the engine then holds this rank's users only) the gathered full tables."""
        return self._full_tables if self._full_tables is not None else self._engine.params()

    def _load_into_net(self, tables):
        with torch.no_grad():
            for p, t in zip(self._params, tables):
                p.copy_(t.reshape(p.shape))

    def run_train_iteration(self, batch_user, batch_item):
        """One fused step on this batch (implicit.py:347-364); returns the loss (device, shape (1,))."""
        e = self._engine
        return e.train_step(batch_user.to(e.device, torch.int64).contiguous(),
                            batch_item.to(e.device, torch.int64).contiguous())

    def run_val_iteration(self, batch_user, batch_item):
        e = self._engine
        return e.val_loss(batch_user.to(e.device, torch.int64).contiguous(),
                          batch_item.to(e.device, torch.int64).contiguous())

    # ------------------------------------------------------------------ inference
    def predict(self, user_ids, item_ids=None):
        self._check_input(user_ids, item_ids, allow_items_none=True)
        if item_ids is None:
            item_ids = np.arange(self._num_items, dtype=np.int64)
        if np.isscalar(user_ids):
            user_ids = np.array(user_ids, dtype=np.int64)
        u = torch.from_numpy(np.asarray(user_ids, dtype=np.int64).reshape(-1))
        i = torch.from_numpy(np.asarray(item_ids, dtype=np.int64).reshape(-1))
        if u.numel() != i.numel():
            u = u.expand(i.numel())
        if self._kind == "mf" and self._full_tables is not None:
            from . import _lib
            dev = self._engine.device
            U, I, ub, ib = self._full_tables
            u, i = u.to(dev).contiguous(), i.to(dev).contiguous()
            out = torch.empty(u.numel(), dtype=torch.float32, device=dev)
            lib = _lib.load()
            _lib.check(lib.rg_mf_scores(_lib.stream_handle(), _lib.ptr(U), _lib.ptr(I), _lib.ptr(ub), _lib.ptr(ib),
                                        U.shape[1], _lib.ptr(u), _lib.ptr(i), u.numel(), _lib.ptr(out)),
                       "rg_mf_scores")
            return out.cpu().numpy().flatten()
        return self._engine.scores(u, i).detach().cpu().numpy().flatten()

    def _device_scores(self, u):
        """(len(u), num_items) fp32 scores on the device: one GEMM of the tables (MF), or
        the eval-mode MLP / NeuMF over the block x items pairs."""
        if self._kind == "mf":
            U, I, ub, ib = self._tables()
            return torch.sigmoid(U[u] @ I.T + ub[u][:, None] + ib[None, :])
        items = torch.arange(self._num_items, device=u.device)
        s = self._engine.scores(u.repeat_interleave(self._num_items), items.repeat(len(u)))
        return s.reshape(len(u), self._num_items).detach()

    def score_users(self, users):
        """Scores of every item for a block of users, (len(users), num_items) float32 on
        the host (evaluation helper)."""
        u = torch.as_tensor(np.asarray(users, dtype=np.int64), device=self._engine.device)
        return self._device_scores(u).cpu().numpy()

    def topk_users(self, users, k, exclude_csr=None):
        """The first k entries of argsort(-scores) for a block of users (evaluation.py:
        precision/recall@k, hit ratio, MAP@k), ranked on the device by rg_topk_rows;
        items of ``exclude_csr``'s rows rank last (the reference's FLOAT_MAX).  Returns
        (len(users), k) int64 on the host."""
        from . import _lib
        dev = self._engine.device
        ub = np.asarray(users, dtype=np.int64)
        u = torch.as_tensor(ub, device=dev)
        s = self._device_scores(u).to(torch.float32).contiguous()
        if exclude_csr is not None:
            sub = exclude_csr[ub]
            if sub.nnz:
                rows = np.repeat(np.arange(len(ub)), np.diff(sub.indptr))
                s[torch.as_tensor(rows, device=dev), torch.as_tensor(sub.indices.astype(np.int64), device=dev)] = \
                    float("-inf")
        out = torch.empty(len(ub), k, dtype=torch.int32, device=dev)
        lib = _lib.load()
        _lib.check(lib.rg_topk_rows(_lib.stream_handle(), _lib.ptr(s), len(ub), self._num_items, self._num_items,
                                    int(k), _lib.ptr(out)), "rg_topk_rows")
        return out.cpu().numpy().astype(np.int64)

    def test(self, test_set, item_popularity, k=5, rmse_flag=False, precision_recall=False, map_recall=True):
        test_results = {"k": k}
        if rmse_flag:
            dev = self._engine.device
            tu = torch.from_numpy(np.asarray(test_set.user_ids, dtype=np.int64))
            ti = torch.from_numpy(np.asarray(test_set.item_ids, dtype=np.int64))
            total = 0.0
            for s in range(0, len(tu), self._batch_size):
                total += evaluation.rmse_score(self._net, tu[s:s + self._batch_size].to(dev),
                                               ti[s:s + self._batch_size].to(dev))
            total /= len(test_set)
            logging.info("BCE: {}".format(np.sqrt(total)))
            test_results["bce"] = float(np.sqrt(total))
        if precision_recall:
            pop_p, pop_r = evaluation.evaluate_popItems(item_popularity, test_set, k=k)
            rand_p, rand_r = evaluation.evaluate_random(item_popularity, test_set, k=k)
            p, r = evaluation.precision_recall_score(self, test=test_set, k=k)
            logging.info(self.model_name + " precision@{} {} recall@{} {}".format(k, p, k, r))
            logging.info("Random: precision@{} {} recall@{} {}".format(k, rand_p, k, rand_r))
            logging.info("PopItem Algorithm: precision@{} {} recall@{} {}".format(k, pop_p, k, pop_r))
            test_results.update(precision=float(p), recall=float(r), rand_prec=float(rand_p),
                                rand_rec=float(rand_r), pop_prec=float(pop_p), pop_rec=float(pop_r), at_k=k)
        if map_recall:
            map_k = evaluation.map_at_k(self, test=test_set, k=k)
            _, r = evaluation.precision_recall_score(self, test=test_set, k=k)
            logging.info(self.model_name + " map@{} {} recall@{} {}".format(k, map_k, k, r))
            test_results["map"] = float(map_k)
        with open(os.path.join(self.experiment_logs, "test_summary.json"), "w") as fp:
            json.dump(test_results, fp)
        return test_results

    def save_readable_model(self, model_save_dir, state_dict):
        fname = os.path.join(model_save_dir, "best_model")
        logging.info("Saving state in {}".format(fname))
        torch.save({"network": {k: v.detach().cpu() for k, v in state_dict.items()}}, f=fname)
