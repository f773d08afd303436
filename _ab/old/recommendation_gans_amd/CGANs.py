"""Conditional GAN for slate generation (CGANs.py of the reference), on the fused
HIP iterations of rg_gan.hip (recommendation_gans_amd.gan_engine).

``CGAN(G, D, z_dim, n_iter, batch_size, loss_fun, learning_rate, slate_size,
G_optimizer_func, embedding_dim, hidden_layer, D_optimizer_func,
experiment_name, use_cuda, random_state)`` with the reference's methods:
``fit`` (CGANs.py:230-336), ``train_discriminator_iteration`` (:410-457),
``train_generator_iteration`` (:370-408), ``test`` (:507-561),
``one_hot_encoding``, ``preprocess_train``, ``save_readable_model``.  The G / D
modules (spotlight.dnn_models.cGAN_models) supply the architecture and the
initial parameters; training runs on the device and the modules receive the
trained parameters back (``G`` is the best-validation generator after ``fit``).

Behaviour kept from the reference: z ~ U[0, 1) (``torch.rand``), the +-0.01 clamp of
every D parameter at each D iteration, one G iteration every ``n_critic`` = 5 D
iterations on the same batch, weight_decay 0, the per-epoch validation precision
and best-generator snapshot, summary.csv columns, and the training precision /
recall of ``precision_recall_slates_atk`` (0 for every row: the reference's set
intersection of identity-hashed 0-d tensors).  Differences: the reference's
``fit`` raises NameError after its first epoch (``real_score`` is undefined at
CGANs.py:326); here that log line reports the last D iteration's mean D(real)
and training continues.  ``run_val_iteration`` references undefined targets in
the reference (:497-503) and is not provided.
"""
import copy
import json
import logging
import math
import os

import numpy as np
import torch
import torch.nn as nn

from .gan_engine import GANBatch, GANEngine
from .spotlight import optimizers as sp_optimizers
from .spotlight.evaluation import precision_recall_score_slates, precision_recall_slates_atk
from .spotlight.torch_utils import minibatch
from .utils.storage_utils import save_statistics

logging.basicConfig(format="%(message)s", level=logging.INFO)


class CGAN:
    def __init__(self, G=None, D=None, z_dim=100, n_iter=15, batch_size=128, loss_fun="bce", learning_rate=1e-4,
                 slate_size=3, G_optimizer_func=None, embedding_dim=5, hidden_layer=16, D_optimizer_func=None,
                 experiment_name="CGANs", use_cuda=False, random_state=None):
        self.exeriment_name = experiment_name
        self.experiment_folder = os.path.abspath("experiments_results/" + experiment_name)
        self.experiment_logs = os.path.abspath(os.path.join(self.experiment_folder, "result_outputs"))
        self.experiment_saved_models = os.path.abspath(os.path.join(self.experiment_folder, "saved_models"))
        for d in ("experiments_results", self.experiment_folder, self.experiment_logs, self.experiment_saved_models):
            os.makedirs(d, exist_ok=True)
        self.starting_epoch = 0
        self.training = True
        self._n_iter = n_iter
        self.G, self.D = G, D
        self.slate_size = slate_size
        self._learning_rate = learning_rate
        self._use_cuda = self.use_cuda = use_cuda
        self.G_optimizer_func, self.D_optimizer_func = G_optimizer_func, D_optimizer_func
        self._random_state = random_state or np.random.RandomState()
        self.hidden_layer, self.embedding_dim, self.z_dim = hidden_layer, embedding_dim, z_dim
        self.loss_fun = loss_fun
        self.weight_cliping_limit = 0.01
        self.n_critic = 5
        self._batch_size = batch_size
        self.logistic = nn.Sigmoid()
        self.chosen_epoch = -1
        self.best_model = None
        self.best_precision = -1
        self.gamma = 10
        # the fused path runs on the GPU whatever use_cuda says (there is no CPU path)
        self.device = torch.device("cuda")
        self.dtype = torch.cuda.FloatTensor
        self.engine = None
        self._batches = {}
        assert loss_fun in ("mse", "bce")

    # ------------------------------------------------------------------ setup
    def _opt_kind(self, func):
        d = sp_optimizers.describe(func if func is not None else sp_optimizers.adam_optimizer, self._learning_rate,
                                   0.0)
        return d

    def _initialize(self):
        """CGANs.py:140-179: optimizers (weight_decay 0, lr), configuration.json."""
        gd, dd = self._opt_kind(self.G_optimizer_func), self._opt_kind(self.D_optimizer_func)
        if (gd["kind"], gd.get("alpha"), gd.get("betas")) != (dd["kind"], dd.get("alpha"), dd.get("betas")):
            raise NotImplementedError("G and D optimizers of different kinds are not supported")
        self.criterion = nn.BCEWithLogitsLoss() if self.loss_fun == "mse" else nn.MSELoss()
        S, N, E = self.slate_size, self.num_items, self.embedding_dim
        H = self.G.mult_heads["head_0"].in_features
        self.engine = GANEngine(self.G.state_dict(), self.D.state_dict(), N, S, H, self.G.y, self.G.z,
                                batch_max=self._batch_size, optimizer=gd["kind"], lr=gd["lr"],
                                alpha=gd.get("alpha", 0.99), betas=gd.get("betas", (0.5, 0.999)),
                                eps=gd.get("eps", 1e-8), seed=int(self._random_state.randint(0, 2 ** 31 - 1)))
        configuration = {"batch_size": self._batch_size, "z_dim": self.z_dim, "slate_size": self.slate_size,
                         "n_iter": self._n_iter, "learning_rate": self._learning_rate, "users": self.num_users,
                         "movies": self.num_items, "hidden_layer": self.hidden_layer,
                         "embedding_dim": self.embedding_dim}
        with open(os.path.join(self.experiment_logs, "configuration.json"), "w") as fp:
            json.dump(configuration, fp)

    def _sync_modules(self):
        self.G.load_state_dict(self.engine.g_state_dict())
        self.D.load_state_dict(self.engine.d_state_dict())

    def _batch(self, hist, slates=None, key=None):
        if key is not None and key in self._batches:
            return self._batches[key]
        h = hist.detach().cpu().numpy() if torch.is_tensor(hist) else np.asarray(hist)
        s = None
        if slates is not None:
            s = slates.detach().cpu().numpy() if torch.is_tensor(slates) else np.asarray(slates)
        b = GANBatch(h.astype(np.int64), None if s is None else s.astype(np.int64), self.num_items,
                     self.slate_size, self.device)
        if key is not None:
            self._batches[key] = b
        return b

    # ------------------------------------------------------------------ reference API
    def one_hot_encoding(self, slates, num_items):
        """CGANs.py:181-198: (B, S * num_items) one-hot rows (the fused D step never
        builds them; kept for callers)."""
        oh = nn.functional.one_hot(torch.as_tensor(slates).to(torch.int64), num_classes=num_items)
        return oh.reshape(oh.shape[0], -1).float()

    def preprocess_train(self, interactions):
        """CGANs.py:200-224."""
        from .utils.slate_data_provider import preprocess_train
        rows, vec, _ = preprocess_train(interactions, interactions.shape[0], self.num_items)
        return rows, vec

    def sigmoid(self, x):
        return 1 / (1 + math.exp(-x))

    def train_discriminator_iteration(self, batch_user, batch_slate, _key=None):
        """CGANs.py:410-457.  Returns d_loss (float)."""
        out = self.engine.d_step(self._batch(batch_user, batch_slate, _key))
        self._last_d = out
        return float(out[0])

    def train_generator_iteration(self, batch_user, batch_slate, _key=None):
        """CGANs.py:370-408.  Returns (g_loss, precision list, recall list)."""
        g, slates = self.engine.g_step(self._batch(batch_user, batch_slate, _key), slates=True)
        precision, recall = precision_recall_slates_atk(slates.type(torch.int64), batch_slate, k=self.slate_size)
        return float(g[0]), precision, recall

    def fit(self, train_vec, train_slates, users, movies, valid_vec, valid_cold_users, valid_set):
        self.num_users, self.num_items = users, movies
        self._initialize()
        steps_performed = 0
        user_slate_tensor = torch.from_numpy(np.asarray(train_slates)).float()
        logging.info("training start!!")
        total_losses = {"G_loss": [], "D_loss": [], "G_pre": [], "G_rec": [], "curr_epoch": [], "Val_prec": []}
        real_score = float("nan")
        for epoch_num in range(self._n_iter):
            g_losses, d_losses = [], []
            cur = {"G_loss": [], "D_loss": [], "G_pre": [], "G_rec": [], "Val_prec": []}
            for bi, (batch_user, batch_slate) in enumerate(minibatch(train_vec, user_slate_tensor,
                                                                     batch_size=self._batch_size)):
                steps_performed += 1
                b = self._batch(batch_user, batch_slate, key=("train", bi))
                d_out = self.engine.d_step(b)
                d_losses.append(d_out)
                if steps_performed % self.n_critic == 0:
                    g, slates = self.engine.g_step(b, slates=True)
                    pre, rec = precision_recall_slates_atk(slates.type(torch.int64), batch_slate,
                                                           k=self.slate_size)
                    g_losses.append(g)
                    cur["G_loss"].append(g)
                    cur["D_loss"].append(d_out)
                    cur["G_pre"] += pre
                    cur["G_rec"] += rec
            # one host sync per epoch for the loss logs
            cur["G_loss"] = [float(t[0]) for t in cur["G_loss"]]
            cur["D_loss"] = [float(t[0]) for t in cur["D_loss"]]
            if d_losses:
                real_score = float(d_losses[-1][1])
            results = self.test(valid_vec, valid_set, valid_cold_users)
            logging.info(str(results["precision"]))
            if results["precision"] > self.best_precision:
                self.best_model = self.engine.g_state_dict()
                self.best_precision = results["precision"]
                self.chosen_epoch = epoch_num
            cur["Val_prec"].append(results["precision"])
            total_losses["curr_epoch"].append(epoch_num)
            for key, value in cur.items():
                total_losses[key].append(np.mean(value))
            save_statistics(experiment_log_dir=self.experiment_logs, filename="summary.csv", stats_dict=total_losses,
                            current_epoch=epoch_num,
                            continue_from_mode=True if (self.starting_epoch != 0 or epoch_num > 0) else False)
            logging.info("--------------- Epoch %d ---------------" % epoch_num)
            logging.info("G_Loss: {}".format(np.mean([float(t[0]) for t in g_losses]) if g_losses else float("nan")))
            logging.info("D_Loss: {} D(x): {}".format(np.mean([float(t[0]) for t in d_losses]), self.sigmoid(real_score)))
        self._sync_modules()
        if self.best_model is not None:
            self.engine.load_g_state(self.best_model)
            self.G.load_state_dict(self.best_model)
        logging.info("Model chosen from: {}".format(self.chosen_epoch))
        self.save_readable_model(self.experiment_saved_models, self.G.state_dict())
        self.training = False

    def test(self, train_vec, test, cold_start_users=None):
        """CGANs.py:507-561: precision / recall@slate_size of the eval-mode generator's
        slates against each user's held-out items; cold-start users condition on the
        padding item only.  Writes test_results.json."""
        if self.engine is None:
            raise RuntimeError("call fit() first")
        total = {"precision": [], "recall": []}
        test = test.tocsr()
        for n, user_batch in enumerate(minibatch(train_vec, batch_size=self._batch_size)):
            z = torch.rand(user_batch.shape[0], self.z_dim, device=self.device)
            slates = self.engine.generate(self._batch(user_batch), z=z).cpu().type(torch.int64)
            r0 = n * self._batch_size
            p, r = precision_recall_score_slates(slates, test[r0:r0 + user_batch.shape[0], :], k=self.slate_size)
            total["precision"] += p
            total["recall"] += r
        if cold_start_users is not None and cold_start_users.shape[0] > 0:
            cold = torch.empty((cold_start_users.shape[0], self.embedding_dim)).fill_(self.num_items)
            cold_csr = cold_start_users.tocsr()
            for n, user_batch in enumerate(minibatch(cold, batch_size=self._batch_size)):
                z = torch.rand(user_batch.shape[0], self.z_dim, device=self.device)
                slates = self.engine.generate(self._batch(user_batch), z=z).cpu().type(torch.int64)
                r0 = n * self._batch_size
                p, r = precision_recall_score_slates(slates, cold_csr[r0:r0 + user_batch.shape[0], :],
                                                     k=self.slate_size)
                total["precision"] += p
                total["recall"] += r
        res = {"precision": float(np.mean(total["precision"])) if total["precision"] else float("nan"),
               "recall": float(np.mean(total["recall"])) if total["recall"] else float("nan"),
               "at": self.slate_size}
        with open(os.path.join(self.experiment_logs, "test_results.json"), "w") as fp:
            json.dump(res, fp)
        return res

    def save_readable_model(self, model_save_dir, state_dict):
        fname = os.path.join(model_save_dir, "generator")
        logging.info("Saving state in {}".format(fname))
        torch.save({"network": state_dict}, f=fname)
