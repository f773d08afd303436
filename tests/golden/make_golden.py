"""Generate golden vectors by importing the REFERENCE itself (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [/root/reference]

The reference (Stamatios-Korres/recommendation_Gans, pure Python/PyTorch) is
imported read-only from its checkout; each fixture records inputs and the
reference's outputs at small sizes.  The fixtures (.npz, data only) are what
travels; this script and /root/reference never run on the GPU box.

Fixtures:
  rng_golden.npz    CPython random.choices indices + states; NumPy legacy
                    RandomState randint / shuffle / choice.
  pool_golden.npz   spotlight.sampling.get_negative_samples on tiny Interactions,
                    both the normal (has_key False) and the has_key-True branch.
  mf_<loss>_<opt>_d<d>.npz
                    3 training steps (one of them a partial batch) through the
                    reference's BilinearNet + loss + optimizer + autograd.
                    pointwise / adaptive_hinge run the reference's own
                    ImplicitFactorizationModel.run_train_iteration (implicit.py:347);
                    bpr / hinge run the reference loss functions on the
                    neg.view(n, B) pairing the build defines.
  mf_fit_golden.npz ImplicitFactorizationModel.fit over 2 epochs with
                    validation interleaving (shared random stream) + test-time
                    predict scores.
  mlp_<loss>_e<E>.npz
                    3 training steps of the reference's NCF MLP
                    (spotlight/dnn_models/mlp.py, layers as ncf_spotlight.py:53-56)
                    through ImplicitFactorizationModel.run_train_iteration, with
                    every dropout mask recorded by forward hooks (the masks come
                    from torch's CPU generator; the GPU path is fed them).
"""
import os
import random
import sys
import tempfile

import numpy as np
import torch

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)

import implicit as ref_implicit  # noqa: E402
from spotlight import losses as ref_losses  # noqa: E402
from spotlight import optimizers as ref_optim  # noqa: E402
from spotlight import sampling as ref_sampling  # noqa: E402
from spotlight.factorization.representations import BilinearNet  # noqa: E402
from spotlight.interactions import Interactions  # noqa: E402
from spotlight.dnn_models.mlp import MLP as RefMLP  # noqa: E402

torch.set_num_threads(1)


def save(name, **arrays):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print("wrote", path, os.path.getsize(path), "bytes")


# ------------------------------------------------------------------ RNG
def make_rng():
    out = {}
    seeds = [0, 1, 12345, 2 ** 40 + 7]
    ns = [1, 7, 1682, 8_100_000, 2 ** 31 + 11]
    for si, s in enumerate(seeds):
        random.seed(s)
        out[f"py_state_seed{si}"] = np.array(random.getstate()[1], dtype=np.uint32)
        for ni, n in enumerate(ns):
            out[f"py_choices_s{si}_n{ni}"] = np.array(random.choices(range(n), k=700), dtype=np.int64)
        out[f"py_state_end{si}"] = np.array(random.getstate()[1], dtype=np.uint32)
    out["py_seeds"] = np.array([0, 1, 12345, 0], dtype=np.int64)  # last one is 2**40+7 (stored separately)
    out["py_ns"] = np.array(ns, dtype=np.int64)
    # mid-block start: three random() calls first
    random.seed(99)
    for _ in range(3):
        random.random()
    out["py_mid_state"] = np.array(random.getstate()[1], dtype=np.uint32)
    out["py_mid_choices"] = np.array(random.choices(range(40960), k=5000), dtype=np.int64)
    # NumPy legacy
    rs = np.random.RandomState(0)
    out["np_seed0_randint"] = np.array([rs.randint(-10 ** 8, 10 ** 8)], dtype=np.int64)
    for n in [1, 2, 10, 1000, 100003]:
        rs = np.random.RandomState(0)
        a = np.arange(n)
        rs.shuffle(a)
        out[f"np_shuffle_{n}"] = a.astype(np.int64)
    np.random.seed(7)
    out["np_choice_u"] = np.random.choice(136677, 3000).astype(np.int64)
    out["np_choice_i"] = np.random.choice(20108, 3000).astype(np.int64)
    # the model's set_seed draw after RandomState(0) (implicit.py:146) then shuffle (implicit.py:262)
    rs = np.random.RandomState(0)
    out["np_model_seed"] = np.array([rs.randint(-10 ** 8, 10 ** 8)], dtype=np.int64)
    a = np.arange(5000)
    rs.shuffle(a)
    out["np_model_shuffle_5000"] = a.astype(np.int64)
    save("rng_golden.npz", **out)


# ------------------------------------------------------------------ pool
def make_pool():
    out = {}
    rs = np.random.RandomState(3)
    nu, ni, nnz = 30, 25, 200
    u = rs.randint(0, nu, nnz).astype(np.int32)
    i = rs.randint(0, ni, nnz).astype(np.int32)
    key = np.unique(u.astype(np.int64) * ni + i)
    u = (key // ni).astype(np.int32)
    i = (key % ni).astype(np.int32)
    for tag, rating in (("raw4", 4.0), ("ones", 1.0)):
        inter = Interactions(u, i, ratings=np.full(len(u), rating, dtype=np.float32),
                             num_users=nu, num_items=ni)
        np.random.seed(11)
        pool = ref_sampling.get_negative_samples(inter, 400)
        out[f"{tag}_pool"] = np.array(pool, dtype=np.int64)
    out["pos_u"] = u.astype(np.int64)
    out["pos_i"] = i.astype(np.int64)
    out["shape"] = np.array([nu, ni, 400], dtype=np.int64)
    save("pool_golden.npz", **out)


# ------------------------------------------------------------------ MF steps
def mf_case(loss, opt, dim, wd, seed=0, U=50, I=40, B=16, n=5):
    torch.manual_seed(seed)
    net = BilinearNet(U, I, dim, sparse=False)
    init = {k: v.detach().clone().numpy() for k, v in net.state_dict().items()}
    prs = np.random.RandomState(seed + 1)
    pool_u = prs.randint(0, U, 300)
    pool_i = prs.randint(0, I, 300)
    pool = list(zip(pool_u.tolist(), pool_i.tolist()))
    # positives: 3 steps, the second a partial batch (B_actual = 11); include duplicates
    steps_pos = []
    for s, bp in enumerate([B, 11, B]):
        pu = prs.randint(0, U, bp)
        pi = prs.randint(0, I, bp)
        pu[0] = pu[1]  # duplicate user rows inside one batch
        pi[2] = pi[3] = pi[4]
        steps_pos.append((pu, pi))
    optimizer_func = getattr(ref_optim, opt + "_optimizer")
    with tempfile.TemporaryDirectory() as td:
        cwd = os.getcwd()
        os.chdir(td)
        try:
            model = ref_implicit.ImplicitFactorizationModel(
                loss={"pointwise": "pointwise", "adaptive_hinge": "adaptive_hinge",
                      "bpr": "pointwise", "hinge": "pointwise"}[loss],
                embedding_dim=dim, n_iter=1, batch_size=B, l2=wd, learning_rate=1e-2,
                optimizer_func=optimizer_func, representation=net,
                random_state=np.random.RandomState(seed), neg_examples=pool,
                num_negative_samples=n)
            inter = Interactions(np.zeros(1, np.int32), np.zeros(1, np.int32), num_users=U, num_items=I)
            model._initialize(inter)
        finally:
            os.chdir(cwd)
    random.seed(1234 + seed)
    rec = {"init_" + k.replace(".", "_"): v for k, v in init.items()}
    rec["pool_u"], rec["pool_i"] = pool_u.astype(np.int64), pool_i.astype(np.int64)
    rec["meta"] = np.array([U, I, dim, B, n], dtype=np.int64)
    rec["wd"] = np.array([wd])
    rec["lr"] = np.array([1e-2])
    for s, (pu, pi) in enumerate(steps_pos):
        st = random.getstate()
        rec[f"s{s}_mt_state"] = np.array(st[1], dtype=np.uint32)
        rep = random.Random()
        rep.setstate(st)
        rec[f"s{s}_neg_idx"] = np.array(rep.choices(range(len(pool)), k=n * B), dtype=np.int64)
        rec[f"s{s}_pos_u"], rec[f"s{s}_pos_i"] = pu.astype(np.int64), pi.astype(np.int64)
        bu = torch.from_numpy(pu).long()
        bi = torch.from_numpy(pi).long()
        if loss in ("pointwise", "adaptive_hinge"):
            # the reference's own step (implicit.py:347-364)
            captured = {}
            orig = model._loss_func

            def spy(pos, neg, _orig=orig):
                captured["pos"], captured["neg"] = pos.detach().clone(), neg.detach().clone()
                out = _orig(pos, neg)
                captured["loss"] = float(out)
                return out

            model._loss_func = spy
            orig_step = model._optimizer.step

            def step_spy(*a, **k):
                captured["grads"] = [p.grad.detach().clone() for p in model._net.parameters()]
                return orig_step(*a, **k)

            model._optimizer.step = step_spy
            model.run_train_iteration(bu, bi)
            model._loss_func = orig
            model._optimizer.step = orig_step
        else:
            # same sequence as run_train_iteration, with the build's neg.view(n, B) pairing
            captured = {}
            pos = model._net(bu, bi)
            model._optimizer.zero_grad()
            nu, ni = zip(*random.choices(pool, k=n * B))
            neg = model._net(torch.from_numpy(np.array(nu)).long(), torch.from_numpy(np.array(ni)).long())
            negm = neg.view(n, B)[:, :len(pu)]
            fn = ref_losses.bpr_loss if loss == "bpr" else ref_losses.hinge_loss
            lv = fn(pos, negm)
            lv.backward()
            captured["pos"], captured["neg"], captured["loss"] = pos.detach(), neg.detach(), float(lv)
            captured["grads"] = [p.grad.detach().clone() for p in model._net.parameters()]
            model._optimizer.step()
        rec[f"s{s}_p_pos"] = captured["pos"].numpy()
        rec[f"s{s}_p_neg"] = captured["neg"].numpy()
        rec[f"s{s}_loss"] = np.array([captured["loss"]])
        names = [k for k, _ in model._net.named_parameters()]
        for nm, g in zip(names, captured["grads"]):
            rec[f"s{s}_grad_" + nm.replace(".", "_")] = g.numpy()
        for nm, p in model._net.named_parameters():
            rec[f"s{s}_after_" + nm.replace(".", "_")] = p.detach().clone().numpy()
    return rec


def make_mf():
    cases = [("pointwise", "adam", 8, 1e-5), ("pointwise", "adam", 64, 1e-5),
             ("bpr", "adam", 64, 1e-5), ("bpr", "adam", 8, 0.0),
             ("hinge", "adam", 8, 1e-5), ("adaptive_hinge", "adam", 8, 1e-5),
             ("pointwise", "sgd", 8, 1e-5), ("bpr", "rms", 8, 1e-5),
             ("bpr", "sgd", 32, 0.0)]
    for loss, opt, d, wd in cases:
        rec = mf_case(loss, opt, d, wd)
        save(f"mf_{loss}_{opt}_d{d}{'_wd0' if wd == 0 else ''}.npz", **rec)


# ------------------------------------------------------------------ MF fit (2 epochs)
def make_fit():
    U, I, d, B, n = 30, 20, 8, 32, 5
    rs = np.random.RandomState(5)
    tu, ti = rs.randint(0, U, 150).astype(np.int32), rs.randint(0, I, 150).astype(np.int32)
    vu, vi = rs.randint(0, U, 40).astype(np.int32), rs.randint(0, I, 40).astype(np.int32)
    train = Interactions(tu, ti, ratings=np.ones(150, np.float32), num_users=U, num_items=I)
    valid = Interactions(vu, vi, ratings=np.ones(40, np.float32), num_users=U, num_items=I)
    pool_u, pool_i = rs.randint(0, U, 150), rs.randint(0, I, 150)
    pool = list(zip(pool_u.tolist(), pool_i.tolist()))
    rec = {}
    for loss in ("pointwise", "adaptive_hinge"):
        torch.manual_seed(0)
        net = BilinearNet(U, I, d, sparse=False)
        rec[f"{loss}_init_U"] = net.user_embeddings.weight.detach().clone().numpy()
        rec[f"{loss}_init_I"] = net.item_embeddings.weight.detach().clone().numpy()
        random.seed(0)
        rec[f"{loss}_mt_state"] = np.array(random.getstate()[1], dtype=np.uint32)
        with tempfile.TemporaryDirectory() as td:
            cwd = os.getcwd()
            os.chdir(td)
            try:
                model = ref_implicit.ImplicitFactorizationModel(
                    loss=loss, embedding_dim=d, n_iter=2, batch_size=B, l2=1e-5,
                    learning_rate=1e-2, optimizer_func=ref_optim.adam_optimizer,
                    representation=net, random_state=np.random.RandomState(0),
                    neg_examples=pool, num_negative_samples=n)
                model.fit(train, valid)
                with open(os.path.join(model.experiment_logs, "summary.csv")) as f:
                    rec[f"{loss}_summary_csv"] = np.array(f.read())
                best = model._net
                rec[f"{loss}_best_epoch"] = np.array([model.best_epoch])
                for nm, p in best.named_parameters():
                    rec[f"{loss}_best_" + nm.replace(".", "_")] = p.detach().clone().numpy()
                rec[f"{loss}_predict_u3"] = model.predict(3)
            finally:
                os.chdir(cwd)
        rec[f"{loss}_mt_state_end"] = np.array(random.getstate()[1], dtype=np.uint32)
    rec["train_u"], rec["train_i"] = tu.astype(np.int64), ti.astype(np.int64)
    rec["valid_u"], rec["valid_i"] = vu.astype(np.int64), vi.astype(np.int64)
    rec["pool_u"], rec["pool_i"] = pool_u.astype(np.int64), pool_i.astype(np.int64)
    rec["meta"] = np.array([U, I, d, B, n], dtype=np.int64)
    save("mf_fit_golden.npz", **rec)


# ------------------------------------------------------------------ NCF MLP steps
def mlp_case(loss, E, seed=0, U=50, I=40, B=16, n=5):
    import math
    top = math.log2(E * 2)
    layers = [2 ** x for x in reversed(range(3, int(top) + 1))]       # ncf_spotlight.py:53-55
    torch.manual_seed(seed)
    net = RefMLP(layers=layers, num_users=U, num_items=I, embedding_dim=E)
    init = {k: v.detach().clone().numpy() for k, v in net.state_dict().items()}
    prs = np.random.RandomState(seed + 1)
    pool_u, pool_i = prs.randint(0, U, 300), prs.randint(0, I, 300)
    pool = list(zip(pool_u.tolist(), pool_i.tolist()))
    steps_pos = []
    for s_, bp in enumerate([B, 11, B]):
        pu, pi = prs.randint(0, U, bp), prs.randint(0, I, bp)
        pu[0] = pu[1]
        pi[2] = pi[3] = pi[4]
        steps_pos.append((pu, pi))
    masks = []

    def hook(mod, inp, out):
        if mod.training:
            masks.append((out != 0).to(torch.uint8).clone())

    for m in net.layers:
        if isinstance(m, torch.nn.Dropout):
            m.register_forward_hook(hook)
    with tempfile.TemporaryDirectory() as td:
        cwd = os.getcwd()
        os.chdir(td)
        try:
            model = ref_implicit.ImplicitFactorizationModel(
                loss={"pointwise": "pointwise", "adaptive_hinge": "adaptive_hinge", "bpr": "pointwise"}[loss],
                embedding_dim=E, n_iter=1, batch_size=B, l2=1e-5, learning_rate=1e-2,
                optimizer_func=ref_optim.adam_optimizer, representation=net,
                random_state=np.random.RandomState(seed), neg_examples=pool, num_negative_samples=n)
            model._initialize(Interactions(np.zeros(1, np.int32), np.zeros(1, np.int32), num_users=U, num_items=I))
        finally:
            os.chdir(cwd)
    random.seed(4321 + seed)
    rec = {"init_" + k.replace(".", "_"): v for k, v in init.items()}
    rec["layers"] = np.array(layers, dtype=np.int64)
    rec["pool_u"], rec["pool_i"] = pool_u.astype(np.int64), pool_i.astype(np.int64)
    rec["meta"] = np.array([U, I, E, B, n], dtype=np.int64)
    names = [k for k, _ in net.named_parameters()]
    rec["param_names"] = np.array(names)
    for s_, (pu, pi) in enumerate(steps_pos):
        rec[f"s{s_}_mt_state"] = np.array(random.getstate()[1], dtype=np.uint32)
        rec[f"s{s_}_pos_u"], rec[f"s{s_}_pos_i"] = pu.astype(np.int64), pi.astype(np.int64)
        bu, bi = torch.from_numpy(pu).long(), torch.from_numpy(pi).long()
        masks.clear()
        captured = {}
        if loss in ("pointwise", "adaptive_hinge"):
            orig = model._loss_func

            def spy(pos, neg, _orig=orig):
                captured["pos"], captured["neg"] = pos.detach().clone(), neg.detach().clone()
                out = _orig(pos, neg)
                captured["loss"] = float(out)
                return out

            model._loss_func = spy
            orig_step = model._optimizer.step

            def step_spy(*a, **k):
                captured["grads"] = [p.grad.detach().clone() for p in model._net.parameters()]
                return orig_step(*a, **k)

            model._optimizer.step = step_spy
            model.run_train_iteration(bu, bi)
            model._loss_func, model._optimizer.step = orig, orig_step
        else:
            # the build's BPR on the NCF scores: pos squeezed to (B,), neg.view(n, B)
            pos = model._net(bu, bi)
            model._optimizer.zero_grad()
            nu, ni = zip(*random.choices(pool, k=n * B))
            neg = model._net(torch.from_numpy(np.array(nu)).long(), torch.from_numpy(np.array(ni)).long())
            lv = ref_losses.bpr_loss(pos.view(-1), neg.view(n, B)[:, :len(pu)])
            lv.backward()
            captured.update(pos=pos.detach(), neg=neg.detach(), loss=float(lv),
                            grads=[p.grad.detach().clone() for p in model._net.parameters()])
            model._optimizer.step()
        nd = len(masks) // 2
        for k, m in enumerate(masks):
            rec[f"s{s_}_mask_{'pos' if k < nd else 'neg'}{k % nd}"] = m.numpy()
        rec[f"s{s_}_p_pos"], rec[f"s{s_}_p_neg"] = captured["pos"].numpy(), captured["neg"].numpy()
        rec[f"s{s_}_loss"] = np.array([captured["loss"]])
        for nm, g in zip(names, captured["grads"]):
            rec[f"s{s_}_grad_" + nm.replace(".", "_")] = g.numpy()
        for nm, p in model._net.named_parameters():
            rec[f"s{s_}_after_" + nm.replace(".", "_")] = p.detach().clone().numpy()
    rec["end_mt_state"] = np.array(random.getstate()[1], dtype=np.uint32)
    return rec


def make_mlp():
    for loss, E in (("pointwise", 16), ("pointwise", 64), ("adaptive_hinge", 16), ("bpr", 16)):
        save(f"mlp_{loss}_e{E}.npz", **mlp_case(loss, E))


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "mlp":
    make_mlp()
    sys.exit(0)

if __name__ == "__main__":
    make_rng()
    make_pool()
    make_mf()
    make_fit()
