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
  mf_init_golden.npz
                    torch.manual_seed(0) -> BilinearNet(U, I, d) tables (mf_spotlight.py:36-37,
                    spotlight/layers.py:30-56, representations.py:40-60) at two sizes.
  mf_fit_golden.npz ImplicitFactorizationModel.fit over 2 epochs with
                    validation interleaving (shared random stream) + test-time
                    predict scores.
  mlp_<loss>_e<E>.npz
                    3 training steps of the reference's NCF MLP
                    (spotlight/dnn_models/mlp.py, layers as ncf_spotlight.py:53-56)
                    through ImplicitFactorizationModel.run_train_iteration, with
                    every dropout mask recorded by forward hooks (the masks come
                    from torch's CPU generator; the GPU path is fed them).
  neumf_<loss>_e<E>_m<M>.npz
                    3 training steps of the reference's NeuMF (spotlight/dnn_models/neuMF.py,
                    neuMF_spotlight.py's tower sizes), as the MLP fixtures: dropout masks
                    of the tower recorded by forward hooks.
  gan_<opt>_n<N>.npz
                    6 discriminator steps and the generator step after the 5th
                    (n_critic = 5, CGANs.py:290-301) of the reference's own CGAN
                    (CGANs.py:370-457) on its generator / discriminator
                    (cGAN_models.py), slate_generation.py's layer shapes at a small
                    size: every z, every dropout mask (forward hooks), BatchNorm
                    running stats, d_loss / g_loss, D outputs, the generator's
                    inference slates and training precision/recall, and all G / D
                    parameters after every step.
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
from spotlight.dnn_models.neuMF import NeuMF as RefNeuMF  # noqa: E402
from spotlight.dnn_models import cGAN_models as ref_gan_models  # noqa: E402
import CGANs as ref_cgans  # noqa: E402

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
    return _tower_case(net, layers, loss, E, seed, U, I, B, n)


def _tower_case(net, layers, loss, E, seed, U, I, B, n, extra_meta=()):
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
    rec["meta"] = np.array([U, I, E, B, n] + list(extra_meta), dtype=np.int64)
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


def neumf_case(loss, E, M, seed=0, U=50, I=40, B=16, n=5):
    import math
    top = math.log2(E * 2)
    layers = [2 ** x for x in reversed(range(3, int(top) + 1))]       # neuMF_spotlight.py:54-55
    torch.manual_seed(seed)
    net = RefNeuMF(layers, U, I, mf_embedding_dim=M, mlp_embedding_dim=E)
    return _tower_case(net, layers, loss, E, seed, U, I, B, n, extra_meta=[M])


def make_neumf():
    for loss, E, M in (("pointwise", 16, 10), ("bpr", 8, 5), ("adaptive_hinge", 16, 12)):
        save(f"neumf_{loss}_e{E}_m{M}.npz", **neumf_case(loss, E, M))


def make_mlp():
    for loss, E in (("pointwise", 16), ("pointwise", 64), ("adaptive_hinge", 16), ("bpr", 16)):
        save(f"mlp_{loss}_e{E}.npz", **mlp_case(loss, E))


def gan_case(opt="rms", seed=0, N=50, S=5, H=16, E=5, B=8, L=7, z_dim=100, nb=3, d_steps=6, lr=1e-3,
             d_max=None):
    """slate_generation.py:46-54 shapes: G hidden [H//2, H], D hidden [2H, H, H//2].

    ``d_max``: scale each initial D tensor to max |x| = d_max.  At these sizes the
    reference's Xavier bound (~0.09) is far outside the +-0.01 clamp, so nearly every
    clamped D weight is exactly +-0.01 and pre-activations cancel to within rounding
    of the LeakyReLU kink, where the slope (1 or 0.2) is decided by summation order
    and no two implementations agree.  At the C4 size W1's Xavier bound is 0.0077,
    inside the clamp; scaled tensors plus a small lr keep the goldens in that regime."""
    torch.manual_seed(seed)
    G = ref_gan_models.generator(num_items=N, noise_dim=z_dim, embedding_dim=E, hidden_layer=[H // 2, H],
                                 output_dim=S)
    D = ref_gan_models.discriminator(num_items=N, embedding_dim=E, hidden_layers=[2 * H, H, H // 2], input_dim=S)
    if d_max is not None:
        with torch.no_grad():
            for p_ in D.parameters():
                p_.mul_(d_max / float(p_.abs().max()))
    rs = np.random.RandomState(seed + 7)
    # user histories: ragged, padded with N (slate_data_provider.py:226-234); one all-padding row
    hist = np.full((nb * B, L), N, np.float32)
    for r in range(nb * B):
        ln = 0 if r == 5 else rs.randint(1, L + 1)
        hist[r, :ln] = rs.choice(N, ln, replace=False)
    slates = np.stack([rs.choice(N, S, replace=False) for _ in range(nb * B)]).astype(np.float32)
    slates[3, 1] = slates[4, 1]             # two rows share an item in the same slot
    g_init = {k: v.detach().clone().numpy() for k, v in G.state_dict().items()}
    d_init = {k: v.detach().clone().numpy() for k, v in D.state_dict().items()}
    zs, masks, bn = [], [], []

    def z_hook(mod, args):
        zs.append(args[0].detach().clone())

    # torch's CPU dropout is the composite bernoulli_(1 - p) -> div_(1 - p) -> input * noise
    # (ATen _dropout_impl); the same ops here (bit-identical output, gradient and generator
    # position — checked below) so the noise itself is recorded: the discriminator's
    # ±0.01 clamp makes exact-zero inputs common, whose mask the output would hide
    orig_dropout = torch.nn.functional.dropout

    def rec_dropout(input, p=0.5, training=True, inplace=False):
        if not training or p == 0.0:
            return orig_dropout(input, p, training, inplace)
        noise = torch.empty_like(input).bernoulli_(1 - p)
        noise.div_(1 - p)
        masks.append((noise != 0).to(torch.uint8).clone())
        return input * noise

    x = torch.randn(16, 9)
    gs = torch.get_rng_state()
    ref_out = orig_dropout(x, 0.3, True)
    r1 = torch.rand(2)
    torch.set_rng_state(gs)
    assert torch.equal(rec_dropout(x, 0.3, True), ref_out) and torch.equal(torch.rand(2), r1)
    torch.set_rng_state(gs)
    masks.clear()
    torch.nn.functional.dropout = rec_dropout

    G.register_forward_pre_hook(z_hook)
    with tempfile.TemporaryDirectory() as td:
        cwd = os.getcwd()
        os.chdir(td)
        try:
            model = ref_cgans.CGAN(G=G, D=D, z_dim=z_dim, n_iter=1, batch_size=B, loss_fun="bce", learning_rate=lr,
                                   slate_size=S, G_optimizer_func=getattr(ref_optim, opt + "_optimizer"),
                                   D_optimizer_func=getattr(ref_optim, opt + "_optimizer"), embedding_dim=E,
                                   hidden_layer=H, experiment_name="g")
            model.num_users, model.num_items = nb * B, N
            model._initialize()
        finally:
            os.chdir(cwd)
    rec = {"g_init_" + k.replace(".", "_"): v for k, v in g_init.items()}
    rec.update({"d_init_" + k.replace(".", "_"): v for k, v in d_init.items()})
    rec["g_param_names"] = np.array([k for k, _ in G.named_parameters()])
    rec["d_param_names"] = np.array([k for k, _ in D.named_parameters()])
    rec["g_buffer_names"] = np.array([k for k, _ in G.named_buffers()])
    rec["meta"] = np.array([N, S, H, E, B, L, z_dim, nb, d_steps], np.int64)
    rec["lr"] = np.array([lr])
    rec["hist"], rec["slates"] = hist, slates
    rec["drop_scale"] = np.array([float(torch.ones(1).div_(1 - p)) for p in (0.1, 0.3)], np.float32)
    hist_t, slates_t = torch.from_numpy(hist), torch.from_numpy(slates)
    steps_performed = 0
    for k in range(d_steps):
        b = k % nb
        bu, bs = hist_t[b * B:(b + 1) * B], slates_t[b * B:(b + 1) * B]
        zs.clear()
        masks.clear()
        steps_performed += 1
        rec[f"d{k}_batch"] = np.array([b])
        dcap = []
        orig_d = D.forward

        def d_spy(x, c, _o=orig_d):
            out = _o(x, c)
            dcap.append((out.detach().clone(), x.detach().clone()))
            return out

        D.forward = d_spy
        d_loss = model.train_discriminator_iteration(bu, bs)
        D.forward = orig_d
        rec[f"d{k}_d_real"], rec[f"d{k}_d_fake"] = dcap[0][0].numpy(), dcap[1][0].numpy()
        rec[f"d{k}_fake"] = dcap[1][1].numpy()
        rec[f"d{k}_z"] = zs[0].numpy()
        for j, m in enumerate(masks):        # D(real) x3, G x2, D(fake) x3
            rec[f"d{k}_mask{j}"] = m.numpy()
        rec[f"d{k}_loss"] = np.array([d_loss])
        for nm, p in D.named_parameters():
            rec[f"d{k}_after_D_" + nm.replace(".", "_")] = p.detach().clone().numpy()
        for nm, t in G.named_buffers():
            rec[f"d{k}_after_G_" + nm.replace(".", "_")] = t.detach().clone().numpy()
        if steps_performed % model.n_critic == 0:
            zs.clear()
            masks.clear()
            cap = {}
            orig_d = D.forward

            def d_spy(x, c, _o=orig_d):
                out = _o(x, c)
                cap["d_fake"] = out.detach().clone()
                cap["fake"] = x.detach().clone()
                return out

            D.forward = d_spy
            g_loss, prec, recl = model.train_generator_iteration(bu, bs)
            D.forward = orig_d
            rec[f"g{k}_z"] = zs[0].numpy()
            assert torch.equal(zs[0], zs[1]), "inference runs on the training z"
            for j, m in enumerate(masks):    # G x2, D(fake) x3
                rec[f"g{k}_mask{j}"] = m.numpy()
            rec[f"g{k}_loss"] = np.array([g_loss])
            rec[f"g{k}_d_fake"] = cap["d_fake"].numpy()
            rec[f"g{k}_fake"] = cap["fake"].numpy()
            rec[f"g{k}_precision"], rec[f"g{k}_recall"] = np.array(prec), np.array(recl)
            G.eval()
            with torch.no_grad():
                rec[f"g{k}_slates_after"] = G(zs[0], bu, inference=True).numpy()
            G.train()
            for nm, p in G.named_parameters():
                rec[f"g{k}_after_G_" + nm.replace(".", "_")] = p.detach().clone().numpy()
            for nm, t in G.named_buffers():
                rec[f"g{k}_after_G_" + nm.replace(".", "_")] = t.detach().clone().numpy()
            rec["g_step_at"] = np.array([k])
    if "g_step_at" not in rec:
        rec["g_step_at"] = np.array([-1])
    torch.nn.functional.dropout = orig_dropout
    return rec


def make_gan():
    save("gan_rms_n50.npz", **gan_case("rms", lr=1e-4, d_max=0.004))
    save("gan_adam_n50.npz", **gan_case("adam", seed=1, nb=2, lr=1e-4, d_max=0.004))
    save("gan_sgd_n64.npz", **gan_case("sgd", seed=2, N=64, H=32, E=8, B=16, L=9, nb=2, d_steps=5, lr=1e-2,
                                       d_max=0.004))
    save("gan_rms_refinit.npz", **gan_case("rms", seed=3, d_steps=1))


def make_init():
    """the MF tables exactly as mf_spotlight.py:36-37 builds them."""
    out = {}
    for k, (U, I, d) in enumerate([(300, 200, 64), (943, 40, 32)]):
        torch.manual_seed(0)
        net = BilinearNet(U, I, d, sparse=False)
        out[f"shape{k}"] = np.array([U, I, d], dtype=np.int64)
        for name, t in net.state_dict().items():
            out[f"{name}_{k}"] = t.numpy().copy()
    save("mf_init_golden.npz", **out)


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "init":
    make_init()
    sys.exit(0)


def make_fit_noneg():
    """implicit.py:351-360's neg_examples=None branch: the loss on the positives only (pointwise,
    the only loss that accepts one argument), no draw from `random`; same data as make_fit."""
    g = np.load(os.path.join(OUT, "mf_fit_golden.npz"))
    U, I, d, B, n = (int(x) for x in g["meta"])
    tu, ti = g["train_u"].astype(np.int32), g["train_i"].astype(np.int32)
    vu, vi = g["valid_u"].astype(np.int32), g["valid_i"].astype(np.int32)
    train = Interactions(tu, ti, ratings=np.ones(len(tu), np.float32), num_users=U, num_items=I)
    valid = Interactions(vu, vi, ratings=np.ones(len(vu), np.float32), num_users=U, num_items=I)
    rec = {}
    torch.manual_seed(0)
    net = BilinearNet(U, I, d, sparse=False)
    rec["init_U"] = net.user_embeddings.weight.detach().clone().numpy()
    rec["init_I"] = net.item_embeddings.weight.detach().clone().numpy()
    random.seed(0)
    rec["mt_state"] = np.array(random.getstate()[1], dtype=np.uint32)
    with tempfile.TemporaryDirectory() as td:
        cwd = os.getcwd()
        os.chdir(td)
        try:
            model = ref_implicit.ImplicitFactorizationModel(
                loss="pointwise", embedding_dim=d, n_iter=2, batch_size=B, l2=1e-5, learning_rate=1e-2,
                optimizer_func=ref_optim.adam_optimizer, representation=net,
                random_state=np.random.RandomState(0), neg_examples=None, num_negative_samples=n)
            model.fit(train, valid)
            with open(os.path.join(model.experiment_logs, "summary.csv")) as f:
                rec["summary_csv"] = np.array(f.read())
            rec["best_epoch"] = np.array([model.best_epoch])
            for nm, p in model._net.named_parameters():
                rec["best_" + nm.replace(".", "_")] = p.detach().clone().numpy()
            rec["predict_u3"] = model.predict(3)
        finally:
            os.chdir(cwd)
    rec["mt_state_end"] = np.array(random.getstate()[1], dtype=np.uint32)
    rec["meta"] = g["meta"]
    save("mf_fit_noneg_golden.npz", **rec)


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "noneg":
    make_fit_noneg()
    sys.exit(0)

if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "refinit5":
    # the reference's own D init (clamp-bound) and lr 1e-3 over a whole
    # n_critic cycle: five D iterations, the G iteration after the fifth, one more D iteration
    save("gan_rms_refinit5.npz", **gan_case("rms", seed=3, d_steps=6, lr=1e-3))
    sys.exit(0)

if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "gan":
    make_gan()
    sys.exit(0)

if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "mlp":
    make_mlp()
    sys.exit(0)

if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "neumf":
    make_neumf()
    sys.exit(0)

if __name__ == "__main__":
    make_rng()
    make_pool()
    make_mf()
    make_fit()
