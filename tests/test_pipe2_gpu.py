"""The two-launch pipelined single-GPU MF step (rg_mf_pipe2_hot / rg_mf_pipe2_cold; A/B build,
RG_PIPE2=1, measured slower than the split step: step t's dense update of the rows step t+1's pair pass reads, then that pair pass beside the
update of every other row and step t+2's prepare) against the split step (RG_PIPE2=0): the same
per-row and per-column arithmetic, so losses, tables, optimizer state and the MT stream are
bit-identical -- after EVERY step, over several steps, with item plans and Zipf-hot rows overflowing
their lists, for every loss the pipeline takes, at d = 32 / 64 / 128 (the dense pass on its own row
layouts); with the lookahead given or not (``next2``); and when the lookahead turns out wrong
(another batch, a validation pass in between), what ran ahead is dropped."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _ab_only():
    from recommendation_gans_amd import _lib
    _lib.load()
    if not _lib.ab_build():
        # measured slower than the split step: the A/B build carries it,
        # scripts/gpu_ab_tests.sh runs this file with RG_LIB pointing at that build
        pytest.skip("A/B build only (RG_LIB=recommendation_gans_amd/_variants/librg_hip_ab.so)")


def _engine(pipe2, loss, d, U, I, B, n, seed=0):
    from oracle import rng as orng
    from recommendation_gans_amd.mf_engine import MFEngine
    old = os.environ.get("RG_PIPE2")
    os.environ["RG_PIPE2"] = "1" if pipe2 else "0"
    try:
        torch.manual_seed(seed)
        Uw, Iw = torch.empty(U, d).normal_(0, 1.0 / d), torch.empty(I, d).normal_(0, 1.0 / d)
        rs = np.random.RandomState(seed)
        pool_u, pool_i = rs.randint(0, U, 40000), rs.randint(0, I, 40000)
        e = MFEngine(Uw, Iw, torch.zeros(U), torch.zeros(I), pool_u, pool_i, orng.py_seed_state(seed), loss=loss,
                     optimizer="adam", lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B,
                     device=torch.device("cuda:0"))
    finally:
        if old is None:
            os.environ.pop("RG_PIPE2", None)
        else:
            os.environ["RG_PIPE2"] = old
    assert e.pipeline_kind == (2 if pipe2 else 0), e.pipeline_kind
    return e


def _inputs(e, U, I, B, steps, seed=1):
    rs = np.random.RandomState(seed)
    dev = torch.device("cuda:0")
    out = []
    for s in range(steps):
        pu = torch.from_numpy(rs.randint(0, U, B).astype(np.int64)).to(dev)
        pi = torch.from_numpy(np.minimum(rs.zipf(1.2, B) - 1, I - 1).astype(np.int64)).to(dev)
        out.append(e.step_input(pu, pi, B, e.make_plan(pi)))
    return out


def _state(e):
    torch.cuda.synchronize()
    t = [p.detach().cpu().clone() for p in e.params()]
    st = [x.detach().cpu().clone() for x in (e.m + e.v) if x is not None]
    return t, st, e.mt_state().copy()


def _same(a, b, what=""):
    names = ["user_w", "item_w", "user_b", "item_b"]
    for k, (x, y) in enumerate(zip(a[0] + a[1], b[0] + b[1])):
        if not torch.equal(x, y):
            bad = (x != y).reshape(x.shape[0], -1).any(1).nonzero().flatten()
            name = names[k] if k < 4 else f"optimizer state {k - 4}"
            raise AssertionError(f"{what}{name}: {len(bad)} rows differ (first {bad[:8].tolist()}), "
                                 f"max |diff| {float((x - y).abs().max()):.3e}")
    assert (a[2] == b[2]).all(), f"{what}MT state"


@pytest.mark.parametrize("loss,d,ahead", [("bpr", 64, True), ("pointwise", 64, True), ("hinge", 64, True),
                                          ("bpr", 32, True), ("bpr", 128, True), ("bpr", 64, False),
                                          ("pointwise", 50, True)])
def test_pipe2_step_is_bit_identical(loss, d, ahead):
    U, I, B, n, steps = 3000, 400, 1024, 5, 7
    ref, pipe = _engine(False, loss, d, U, I, B, n), _engine(True, loss, d, U, I, B, n)
    ins_r, ins_p = _inputs(ref, U, I, B, steps), _inputs(pipe, U, I, B, steps)
    lr, lp = [], []
    for s in range(steps):
        nx = ins_r[s + 1] if s + 1 < steps else None
        lr.append(float(ref.train_step_in(ins_r[s], nx)[0]))
        nxp = ins_p[s + 1] if s + 1 < steps else None
        nx2 = ins_p[s + 2] if ahead and s + 2 < steps else None
        lp.append(float(pipe.train_step_in(ins_p[s], nxp, next2=nx2)[0]))
        # every row is up to date after the step's two launches (the pair pass run ahead writes
        # only the next step's scratch)
        _same(_state(ref), _state(pipe), f"after step {s}: ")
        assert lr == lp, (s, lr, lp)


def test_pipe2_lookahead_dropped():
    """The lookahead given to step s names batch X for step s+1, but step s+1 trains batch Y; and a
    validation pass (rg_mf_stepper_acquire) comes between two pipelined steps: the engine ends
    bit-identical to the split step over the same sequence."""
    U, I, B, n, d = 3000, 400, 1024, 5, 64
    ref, pipe = _engine(False, "bpr", d, U, I, B, n), _engine(True, "bpr", d, U, I, B, n)
    ins_r, ins_p = _inputs(ref, U, I, B, 6), _inputs(pipe, U, I, B, 6)
    vr, vp = _inputs(ref, U, I, B, 1, seed=9)[0], _inputs(pipe, U, I, B, 1, seed=9)[0]
    # s0 announces (1, 2), but s1 trains batch 3 (announcing 4, 5); then validation; then 4, 5
    seq = [(0, 1, 2), (3, 4, 5), "val", (4, 5, None), (5, None, None)]
    lr, lp = [], []
    for item in seq:
        if item == "val":
            lr.append(float(ref.val_loss(*vr._keep[:2], plan=vr._keep[2])[0]))
            lp.append(float(pipe.val_loss(*vp._keep[:2], plan=vp._keep[2])[0]))
            continue
        a, b, c = item
        lr.append(float(ref.train_step_in(ins_r[a], ins_r[b] if b is not None else None)[0]))
        lp.append(float(pipe.train_step_in(ins_p[a], ins_p[b] if b is not None else None,
                                           next2=ins_p[c] if c is not None else None)[0]))
    assert lr == lp, (lr, lp)
    _same(_state(ref), _state(pipe))


def test_pipe2_full_size_matches_split():
    """C2's shape (U = 136,677, I = 20,108, d = 64, B = 8192, BPR, Zipf items, the full pool): five
    pipelined steps against the split step, bit for bit."""
    from recommendation_gans_amd.synthetic import ML20M, movielens_like
    from recommendation_gans_amd.mf_engine import MFEngine
    from oracle import rng as orng
    data = movielens_like(ML20M, seed=0)
    U, I, d, B, n, steps = data.num_users, data.num_items, 64, 8192, 5, 5
    engines = []
    for flag in ("0", "1"):
        os.environ["RG_PIPE2"] = flag
        try:
            torch.manual_seed(0)
            Uw, Iw = torch.empty(U, d).normal_(0, 1.0 / d), torch.empty(I, d).normal_(0, 1.0 / d)
            engines.append(MFEngine(Uw, Iw, torch.zeros(U), torch.zeros(I), data.pool_u, data.pool_i,
                                    orng.py_seed_state(0), loss="bpr", optimizer="adam", lr=1e-3, weight_decay=1e-5,
                                    n_neg=n, batch_size=B, device=torch.device("cuda:0")))
        finally:
            os.environ.pop("RG_PIPE2", None)
    ref, pipe = engines
    assert pipe.pipeline_kind == 2 and ref.pipeline_kind == 0
    dev = torch.device("cuda:0")
    tu = torch.from_numpy(data.train_u[:(steps + 2) * B].astype(np.int64)).to(dev)
    ti = torch.from_numpy(data.train_i[:(steps + 2) * B].astype(np.int64)).to(dev)
    ins = [[e.step_input(tu[s * B:(s + 1) * B], ti[s * B:(s + 1) * B], B, e.make_plan(ti[s * B:(s + 1) * B]))
            for s in range(steps + 2)] for e in engines]
    for s in range(steps):
        lr = float(ref.train_step_in(ins[0][s], ins[0][s + 1])[0])
        lp = float(pipe.train_step_in(ins[1][s], ins[1][s + 1], next2=ins[1][s + 2])[0])
        assert lr == lp, (s, lr, lp)
    _same(_state(ref), _state(pipe))
