"""Benchmark: train interactions/s, MF-BPR dim=64, MovieLens-20M-shaped, 1 -> 8 MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one pass of the hot path over one batch of B = 8192 positives per
GPU (weak scaling), each with n = 5 negatives drawn bit-exactly from the CPython
MT19937 stream, the BPR loss on the neg.view(n, B) pairing, backward, and a dense
coupled-L2 Adam update of every row of the four BilinearNet tables (the
reference's semantics: implicit.py:347-364, spotlight/optimizers.py:10-16).
The native stepper runs it as rg_mf_pairs -> rg_mf_apply_prepare (the dense
update and the next step's prepare in one launch); under an A/B build
RG_FUSED=1 selects the overlapped two-launch step (measured slower).
Inputs (positive ids, pool, tables) are resident in HBM before timing starts.

With N > 1 ranks (one process per GPU) the default is the reference-exact
owner-sharded step: rank r keeps the users u % N == r and every
item, every rank walks ONE global negative draw of n*N*B indices over the full pool and
keeps the pairs whose user it owns; the pair scores (not for pointwise) and the item
gradient are all-reduced with RCCL -- N ranks compute exactly the reference's step at
batch N*B.  --dp global_stream selects the replicated reference-exact step (rank-major
gradient reduce-scatter + table all-gather); --dp user_shard the user-sharded opt-in
(sharding.py: own sub-pool and MT stream per rank, item-gradient all-reduce), which is
NOT the reference's sampling at N > 1.

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment launches the
N rank processes itself (a torch.distributed.run child started before this process
touches the GPU) and exits with its status; it never falls back to one rank.
`--launch-check` runs only that plumbing (gloo, no GPU): rendezvous, barrier, max-over-
ranks timing, one JSON line from rank 0.  `--emulate-rank R/W` times rank R's owner step
at W-rank geometry on ONE GPU (global batch W*B, the global draw, U/W users, every item)
with the collectives replaced by same-size local copies (comm.LocalComm).

Rank 0 prints ONE JSON line.  `value` = positives processed by all ranks / the
max over ranks of the timed wall time.  `roofline` is for the dominant kernel
(rg_mf_apply_prepare: the dense optimizer pass + the next step's prepare), timed
with HIP events on the stream it is launched on; `cpu_baseline` times the CPU restatement (oracle/, the
reference's algorithm incl. its random.choices sampler) on a bounded sample.
"""
import argparse
import contextlib
import json
import os
import random
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "train interactions/sec, MF-BPR dim=64 MovieLens-20M, 1→8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak (spec)


@contextlib.contextmanager
def stdout_to_stderr():
    """Route file descriptor 1 to 2 (RCCL / gloo print init banners on stdout)."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def algorithmic_bytes(U, I, d, B, n):
    """gathers + ids + dense Adam (read+write p, m, v) per step."""
    gather = B * (1 + n) * 2 * (4 * d + 4)
    ids = B * (16 + 24 * n)
    adam = 6 * (U + I) * (4 * d + 4)
    return gather, ids, adam


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--batch", type=int, default=8192, help="positives per GPU per step")
    ap.add_argument("--neg", type=int, default=5)
    ap.add_argument("--loss", default="bpr")
    ap.add_argument("--optim", default="adam")
    ap.add_argument("--zipf", type=float, default=1.0)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-prefetch", action="store_true")
    ap.add_argument("--model", default="mf", choices=["mf", "ncf", "neumf", "gan", "eval"],
                    help="mf: the BASELINE metric (MF-BPR); ncf: config 3 (NCF MLP, MFMA roofline); "
                         "neumf: neuMF_spotlight.py defaults (mlp dim 16, mf dim 50); "
                         "gan: config 4 (cGAN slate generation, MFMA roofline); "
                         "eval: precision/recall@5 + MAP@5 of an ML-20M-shaped MF model (device top-k)")
    ap.add_argument("--mf-dim", type=int, default=50, help="NeuMF GMF dim (arg_extractor --mf_embedding_dim)")
    ap.add_argument("--mlp-dim", type=int, default=16, help="NeuMF tower dim (arg_extractor --mlp_embedding_dim)")
    ap.add_argument("--gan-batch", type=int, default=256, help="cGAN batch (arg_extractor.py --batch_size)")
    ap.add_argument("--gan-hidden", type=int, default=256)
    ap.add_argument("--gan-slate", type=int, default=5)
    ap.add_argument("--gan-emb", type=int, default=5)
    ap.add_argument("--dp", default="owner", choices=["owner", "global_stream", "user_shard"],
                    help="multi-GPU layout (N > 1): owner = reference-exact, users sharded by owner, items "
                         "replicated (score + item-gradient all-reduces); global_stream = reference-exact "
                         "replicated step (reduce-scatter + all-gather of every row); user_shard = user-sharded "
                         "opt-in (not the reference's sampling at N > 1)")
    ap.add_argument("--dp-at-1", action="store_true",
                    help="run the DP code path at N = 1 too (identity exchange; bench-path check)")
    ap.add_argument("--comm-at-1", action="store_true",
                    help="with --dp-at-1 --dp owner: the native step with a one-rank RCCL communicator")
    ap.add_argument("--launch-check", action="store_true",
                    help="only the multi-rank launch plumbing (gloo on the CPU, no GPU): every rank joins, "
                         "times a barrier, rank 0 prints the JSON line with n_gpus = WORLD_SIZE")
    ap.add_argument("--emulate-rank", default=None, metavar="R/W",
                    help="one GPU runs rank R's owner step at W-rank geometry (global batch W*B, the global draw, "
                         "U/W users, every item), collectives replaced by same-size local copies")
    ap.add_argument("--events-every", type=int, default=10,
                    help="record the dominant kernel's timing events on every k-th timed step (each event "
                         "pair leaves a ~6 us bubble on the stream: 2 pairs in the driver's 20 steps)")
    ap.add_argument("--host-ahead", type=float, default=0.0, metavar="MS",
                    help="diagnostic: a MS-long spin kernel before the timed steps lets the host enqueue them "
                         "all ahead; the step time is then taken by events after the spin (GPU-side time only, "
                         "reported as gpu_ahead_us_per_step; not the driver's line)")
    return ap.parse_args()


def cpu_baseline(data, d, B, n, loss, budget_s):
    """Time the oracle's CPU restatement (torch-CPU math + CPython random.choices over
    a list of tuples, as implicit.py:352) on a bounded number of full-size steps."""
    from oracle import mf as omf
    from oracle import rng as orng
    torch.manual_seed(0)
    U, I = data.num_users, data.num_items
    tabs = omf.init_tables(U, I, d)
    random.seed(0)
    t0 = time.time()
    o = omf.MFOracle(*tabs, data.pool_u, data.pool_i, orng.state_from_python(random.getstate()), loss=loss,
                     optimizer="adam", lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B, python_sampler=True)
    setup = time.time() - t0
    pu = torch.from_numpy(data.train_u)
    pi = torch.from_numpy(data.train_i)
    o.step(pu[:B], pi[:B])          # warm-up
    steps, t0 = 0, time.time()
    while True:
        s = (steps + 1) * B
        o.step(pu[s:s + B], pi[s:s + B])
        steps += 1
        el = time.time() - t0
        if el >= budget_s or steps >= 200:
            break
    return {"value": steps * B / el, "unit": "interactions/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"{steps} full steps (B={B}, n={n}, d={d}, {loss}, Adam over U={U} I={I}, "
                      f"pool {len(data.pool_u)}) after 1 warm-up step, {el:.1f} s timed "
                      f"(+{setup:.1f} s pool/tuple setup untimed)"}


HIDDEN_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: peak FP32 (matrix), dense


def ncf_flops_per_example(E):
    """Forward MACs of the MLP (layers 2E -> ... -> 8 -> 1) x 2 FLOP, x 3 (forward, dW, dA)."""
    sizes, h = [], 2 * E
    while h >= 8:
        sizes.append(h)
        h //= 2
    macs = sum(a * b for a, b in zip(sizes[:-1], sizes[1:])) + 8
    return 3 * 2 * macs


def ncf_cpu_baseline(params, names, data, B, n, neumf, budget_s):
    """The oracle's NCF / NeuMF step (torch-CPU fp32, dropout masks drawn on the CPU as
    torch's Dropout does) on full-size batches for ~budget_s seconds (kind "port")."""
    from oracle import ncf as oncf
    from oracle import rng as orng
    random.seed(0)
    cls = oncf.NeuMFOracle if neumf else oncf.NCFOracle
    o = cls([p.clone() for p in params], names, data.pool_u, data.pool_i,
            orng.state_from_python(random.getstate()), loss="pointwise", lr=1e-3, weight_decay=1e-5, n_neg=n,
            batch_size=B)
    units = oncf.layer_sizes(int(params[0].shape[1]))[1:]
    pu, pi = torch.from_numpy(data.train_u), torch.from_numpy(data.train_i)

    def one(s):
        mp = [torch.randint(0, 2, (B, h), dtype=torch.uint8) for h in units]
        mn = [torch.randint(0, 2, (n * B, h), dtype=torch.uint8) for h in units]
        o.step(pu[s * B:(s + 1) * B], pi[s * B:(s + 1) * B], mp, mn)
    one(0)                                           # warm-up
    steps, t0 = 0, time.time()
    while True:
        one(steps + 1)
        steps += 1
        el = time.time() - t0
        if el >= budget_s or steps >= 200:
            break
    return {"value": steps * B / el, "unit": "interactions/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{steps} full steps (B={B}, n={n}, pointwise, Adam over every parameter) after 1 warm-up "
                      f"step, {el:.1f} s timed"}


def bench_ncf(args):
    """Config 3: ncf_spotlight.py MovieLens-20M, mlp_embedding_dim=64, 1 GPU (pointwise, the CLI's
    loss; dropout from the device hash RNG).  --model neumf: neuMF_spotlight.py with the
    CLI's defaults (mlp_embedding_dim 16, mf_embedding_dim 50), same data and loop."""
    from recommendation_gans_amd import _lib
    from recommendation_gans_amd.ncf_engine import NCFEngine
    from recommendation_gans_amd.synthetic import ML20M, movielens_like
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    comm = None
    if world > 1:     # replicated, reference-exact NCF data parallelism (ncf_engine.py): RCCL all-reduce
        from recommendation_gans_amd.comm import RcclComm
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        with stdout_to_stderr():
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
            comm = RcclComm(torch.device(f"cuda:{local_rank}"))
    dev = torch.device(f"cuda:{local_rank}")
    neumf = args.model == "neumf"
    E, B, n = (args.mlp_dim if neumf else args.dim), args.batch, args.neg
    M = args.mf_dim if neumf else 0
    data = movielens_like(ML20M, seed=0, zipf_s=args.zipf)
    U, I = data.num_users, data.num_items
    torch.manual_seed(0)
    from recommendation_gans_amd.spotlight.dnn_models.mlp import MLP
    from recommendation_gans_amd.spotlight.dnn_models.neuMF import NeuMF
    from recommendation_gans_amd.ncf_spotlight import mlp_layers
    if neumf:
        net = NeuMF(mlp_layers(E), U, I, mf_embedding_dim=M, mlp_embedding_dim=E)
    else:
        net = MLP(layers=mlp_layers(E), num_users=U, num_items=I, embedding_dim=E)
    names = [k for k, _ in net.named_parameters()]
    params = [p.detach() for p in net.parameters()]
    random.seed(0)
    mt = np.asarray(random.getstate()[1], dtype=np.uint32)
    extra = dict(mf_user_w=params[2], mf_item_w=params[3]) if neumf else {}
    mlp_params = params[4:] if neumf else params[2:]
    eng = NCFEngine(params[0], params[1], mlp_params, data.pool_u, data.pool_i, mt, loss="pointwise",
                    optimizer="adam", lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B, device=dev, seed=0,
                    rank=rank, world_size=world, comm=comm, **extra)
    tu = torch.from_numpy(data.train_u).to(dev)
    ti = torch.from_numpy(data.train_i).to(dev)
    GC = B * world                      # rank r: columns [g*GC + r*B, +B) of global batch g
    nb = len(data.train_u) // GC
    nplan = min(nb, args.warmup + args.steps + 1)
    plans = eng.make_plans(ti[:nplan * GC], offset=rank * B, stride=GC)

    def cols(g):
        lo = g * GC + rank * B
        return tu[lo:lo + B], ti[lo:lo + B]
    for s in range(args.warmup):
        g = s % nplan
        eng.train_step(*cols(g), plan=plans[g])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    every = max(1, args.events_every)
    evs = []
    ahead = None
    if args.host_ahead > 0:      # diagnostic (see --host-ahead): GPU-side step time alone
        torch.cuda._sleep(int(args.host_ahead * 2.1e6))
        ahead = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ahead[0].record()
    t0 = time.perf_counter()
    for s in range(args.steps):
        g = (args.warmup + s) % nplan
        u, i = cols(g)
        if s % every == 0:
            a, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            eng.kernel_events = (a, b_)
            evs.append((a, b_))
        else:
            eng.kernel_events = None
        g2 = (args.warmup + s + 1) % nplan
        eng.train_step(u, i, plan=plans[g], next_step=(*cols(g2), plans[g2]))
    if ahead is not None:
        ahead[1].record()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ms = float(np.mean([a.elapsed_time(b_) for a, b_ in evs]))
    # NeuMF adds per example: GMF product (M) + output dot (2M) forward; dW_out (2M), the GMF
    # unit gradients (M) and both table gradients (2M) backward
    flops = (ncf_flops_per_example(E) + 8 * M) * B * (1 + n)
    ach = flops / (ms * 1e-3) / 1e12
    metric = (f"train interactions/sec, NeuMF mlp dim={E} mf dim={M} MovieLens-20M" if neumf else
              "train interactions/sec, NCF MLP dim=64 MovieLens-20M (config 3)")
    workload = (f"NeuMF tower {mlp_layers(E)} + GMF {M} -> affine_output({8 + M}), " if neumf else
                f"NCF MLP {mlp_layers(E)}->1, ")
    out = {"metric": metric, "value": args.steps * B * world / el,
           "unit": "interactions/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "f32", "data": f"synthetic ML-20M-shaped (U={U}, I={I}); MLP init as the reference",
           "config": {"workload": workload + f"batch {B}, {n} negatives, pointwise, adam, "
                                             f"dropout 0.5 (device hash RNG)", "global_batch": GC, "embedding_dim": E,
                      "mf_embedding_dim": M,
                      "parallelism": f"dp{world}" + (" replicated (embedding + MLP gradient all-reduce, "
                                                     "reference-exact)" if world > 1 else "")},
           "roofline": {"bound": "mfma", "kernel": "rg_ncf_pairs (" + ("ncf_wave_kernel" if E == 64 and not neumf
                                                                    and not (_lib.ab_build() and
                                                                             os.environ.get("RG_NCF_TILE") == "1")
                                                                    else "ncf_pairs_kernel") + ")", "achieved": ach,
                        "peak": HIDDEN_FP32_MFMA_TFLOPS, "unit": "TFLOP/s", "frac": ach / HIDDEN_FP32_MFMA_TFLOPS,
                        "traffic": None, "algorithmic_flops_per_launch": flops, "avg_launch_us": ms * 1e3},
           "final_loss": float(eng.loss_out[0]), "host_enqueue_us_per_step": t_enq / args.steps * 1e6}
    if ahead is not None:
        out["gpu_ahead_us_per_step"] = ahead[0].elapsed_time(ahead[1]) * 1e3 / args.steps
        out["ms_per_step"] = out["gpu_ahead_us_per_step"] * 1e-3
        out["value"] = B * world / (out["gpu_ahead_us_per_step"] * 1e-6)
        out["timing"] = "GPU events after a host-ahead spin (diagnostic)"
    if not args.no_cpu_baseline and world == 1:
        out["cpu_baseline"] = ncf_cpu_baseline([p.clone() for p in params], names, data, B, n, neumf,
                                               args.cpu_baseline_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        del eng
        comm.close()
        dist.destroy_process_group()


def stream_copy_gbs(dev, mib=1024, reps=10):
    """Achievable HBM bandwidth of this box: a grid-stride float4 copy of `mib` MiB
    (rg_stream_copy, read + write bytes counted) timed with events, best of `reps`."""
    from recommendation_gans_amd import _lib
    lib = _lib.load()
    n4 = mib * (1 << 20) // 16
    src = torch.ones(n4 * 4, device=dev)
    dst = torch.empty_like(src)
    st = _lib.stream_handle()
    _lib.check(lib.rg_stream_copy(st, _lib.ptr(dst), _lib.ptr(src), n4), "rg_stream_copy")
    best = float("inf")
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        lib.rg_stream_copy(st, _lib.ptr(dst), _lib.ptr(src), n4)
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e-3)
    del src, dst
    return 2 * n4 * 16 / best / 1e9


def gan_flops(N, S, H, E, Z, B):
    """Algorithmic FLOPs of one discriminator and one generator iteration:
    2 * multiply-adds of every dense contraction, the real slates' one-hot layer counted
    by its S nonzeros per row (structural zeros are not work)."""
    SN, H1, H2 = S * N, H // 2, 2 * H
    g_fwd = 2 * B * ((Z + E) * H1 + H1 * H + H * SN)
    d_l1 = 2 * B * (SN + E) * H2
    d_up = 2 * B * (H2 * H + H * H1 + H1)                 # layers 2..4, per pass
    d_real_l1 = 2 * B * (S + E) * H2
    d_step = (d_real_l1 + d_l1 + 2 * d_up + g_fwd          # forward: D(real), G(z), D(fake)
              + 2 * (2 * d_up)                             # upper layers: dW + dX, both passes
              + 2 * B * H2 * SN + 2 * 2 * B * H2 * E)      # layer-1 dW (fake dense; real sparse ~0) + history cols
    g_step = (g_fwd + d_l1 + d_up                          # G(z), D(fake)
              + 2 * d_up + 2 * B * H2 * SN                  # D backward to the slate input
              + 2 * 2 * B * SN * H                          # heads: dWH and dA2
              + 2 * 2 * B * (H * H1 + H1 * (Z + E))         # G small layers dW + dX
              + g_fwd)                                      # eval inference on the same z
    return d_step, g_step


def gan_bytes(N, S, H, E, Z, B):
    """Algorithmic HBM bytes of one discriminator and one generator iteration: the streams of size
    S*N (the slate axis: the 2H x S*N layer-1 weight W1S of D, the S*N x H heads WH of G, the B x S*N
    fake slates and their gradient), each read or written once per use; everything else (the small
    layers, histories, the real slates' sparse columns) is < 1 % and not counted.
      D iteration (CGANs.py:410-457): G(z) reads WH and writes the fake slates; D(fake) reads them
      and W1S; layer 1's dW (fused with RMSprop) reads them again and moves W1S and its square
      average v in and out (4 x W1S).
      G iteration (CGANs.py:370-408): G(z) reads WH, writes the fake slates; D(fake) reads them and
      W1S; D's backward to the slates reads W1S and writes dfake; the heads' dW (fused with RMSprop)
      reads dfake and moves WH and v in and out (4 x WH); the eval inference reads WH again."""
    f = 4
    w1s, wh, fake = 2 * H * S * N * f, S * N * H * f, B * S * N * f
    d_it = wh + fake + (fake + w1s) + (fake + 4 * w1s)
    g_it = (wh + fake) + (fake + w1s) + (w1s + fake) + (fake + 4 * wh) + wh
    return d_it, g_it


def gan_cpu_baseline(g_sd, d_sd, np_batches, N, S, H, E, Z, budget_s):
    """The oracle's cGAN iterations (oracle/gan.py, float64 NumPy, the reference's
    CGANs.py:370-457 restated) at the bench's full size: D iterations with a G iteration
    every 5th, random z and dropout masks, for ~budget_s seconds (kind "port")."""
    from oracle import gan as og
    o = og.GANOracle({k: v.numpy() for k, v in g_sd.items()}, {k: v.numpy() for k, v in d_sd.items()}, N, S, H, E,
                     Z, opt="rms", lr=1e-3)
    rs = np.random.RandomState(0)
    scales = (1.0 / 0.9, 1.0 / 0.7)
    gd, dd = og.g_hidden(H), og.d_hidden(H)

    def masks(B, widths, p):
        return [(rs.rand(B, w) >= p).astype(np.float64) for w in widths]
    steps, t0 = 0, time.time()
    while True:
        hist, sl = np_batches[steps % len(np_batches)]
        B = hist.shape[0]
        m = masks(B, dd, 0.3) + masks(B, gd, 0.1) + masks(B, dd, 0.3)
        o.d_step(hist, sl, rs.rand(B, Z), m, scales)
        if (steps + 1) % 5 == 0:
            o.g_step(hist, rs.rand(B, Z), masks(B, gd, 0.1) + masks(B, dd, 0.3), scales)
        steps += 1
        el = time.time() - t0
        if el >= budget_s or steps >= 50:
            break
    B = np_batches[0][0].shape[0]
    return {"value": steps * B / el, "unit": "slates/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{steps} steps (D iteration each, G iteration every 5th) of the float64 NumPy oracle at the "
                      f"bench size (N={N}, B={B}), {el:.1f} s"}


def bench_gan(args):
    """Config 4: slate_generation.py cGAN, MovieLens-20M, slate_size 5, gan_hidden_layer 256,
    batch 256, RMSprop (optim_gan default), n_critic 5: one step = one discriminator
    iteration plus, every 5th step, one generator iteration (CGANs.py:288-301)."""
    from recommendation_gans_amd.gan_engine import GANBatch, GANEngine
    from recommendation_gans_amd.spotlight.dnn_models.cGAN_models import discriminator, generator
    from recommendation_gans_amd.synthetic import ML20M, movielens_like
    dev = torch.device("cuda:0")
    B, H, S, E, Z = args.gan_batch, args.gan_hidden, args.gan_slate, args.gan_emb, 100
    data = movielens_like(ML20M, seed=0, zipf_s=args.zipf)
    N = data.num_items
    # per-user training lists; the last S items are the user's target slate (create_slates,
    # dataset_manilupation.py:270-316), the rest the padded history (slate_data_provider.py:226-234)
    order = np.argsort(data.train_u, kind="stable")
    uu, ii = data.train_u[order], data.train_i[order]
    starts = np.searchsorted(uu, np.arange(data.num_users + 1))
    counts = np.diff(starts)
    users = np.nonzero(counts > S)[0]
    L = int((counts[users] - S).max())
    nb = min(len(users) // B, 40)
    batches, np_batches = [], []
    for g in range(nb):
        hist = np.full((B, L), N, np.int64)
        sl = np.zeros((B, S), np.int64)
        for r, u in enumerate(users[g * B:(g + 1) * B]):
            items = ii[starts[u]:starts[u + 1]]
            hist[r, :len(items) - S] = items[:-S]
            sl[r] = items[-S:]
        batches.append(GANBatch(hist, sl, N, S, dev))
        if g < 2:
            np_batches.append((hist, sl))
    torch.manual_seed(0)
    G = generator(num_items=N, noise_dim=Z, embedding_dim=E, hidden_layer=[H // 2, H], output_dim=S)
    D = discriminator(num_items=N, embedding_dim=E, hidden_layers=[2 * H, H, H // 2], input_dim=S)
    g_sd = {k: v.detach().clone() for k, v in G.state_dict().items()}
    d_sd = {k: v.detach().clone() for k, v in D.state_dict().items()}
    eng = GANEngine(G.state_dict(), D.state_dict(), N, S, H, E, Z, batch_max=B, optimizer="rms", lr=1e-3, device=dev)
    del G, D
    steps = max(5, args.steps // 5 * 5)

    def step(k):
        bt = batches[k % nb]
        eng.d_step(bt)
        if (k + 1) % 5 == 0:
            eng.g_step(bt, slates=True)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize()
    a, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record()
    for k in range(steps):
        step(args.warmup + k)
    b_.record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ms_ev = a.elapsed_time(b_)
    fd, fg = gan_flops(N, S, H, E, Z, B)
    flops = steps * fd + steps // 5 * fg
    ach = flops / (ms_ev * 1e-3) / 1e12
    # both legs of the roofline: the iteration moves ~1.4 GB of weight / optimizer-state / slate
    # streams besides its FLOPs; frac = max(flop time at peak, byte time at peak) / measured
    bd, bg = gan_bytes(N, S, H, E, Z, B)
    nbytes = steps * bd + steps // 5 * bg
    t_meas = ms_ev * 1e-3
    t_flop, t_byte = flops / (HIDDEN_FP32_MFMA_TFLOPS * 1e12), nbytes / (HBM_PEAK_GBS * 1e9)
    out = {"metric": "train slates/sec, cGAN slate_size=5 gan_hidden_layer=256 MovieLens-20M (config 4)",
           "value": steps * B / el, "unit": "slates/s", "n_gpus": 1, "steps": steps, "warmup": args.warmup,
           "ms_per_step": el / steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "f32", "data": f"synthetic ML-20M-shaped histories (N={N}, L_max={L}); reference init",
           "config": {"workload": f"cGAN G hidden [{H // 2}, {H}], D hidden [{2 * H}, {H}, {H // 2}], S={S}, E={E}, "
                                  f"z=100, batch {B}, RMSprop lr 1e-3, n_critic 5 (1 D iteration per step, 1 G "
                                  f"iteration per 5 steps)", "global_batch": B, "parallelism": "dp1"},
           "roofline": {"bound": "mfma" if t_flop >= t_byte else "hbm",
                        "kernel": "whole D/G iterations (gemm_kernel + small kernels)",
                        "achieved": ach, "peak": HIDDEN_FP32_MFMA_TFLOPS, "unit": "TFLOP/s",
                        "frac": max(t_flop, t_byte) / t_meas, "traffic": None,
                        "algorithmic_flops_per_step": flops / steps, "d_iter_gflop": fd / 1e9,
                        "g_iter_gflop": fg / 1e9,
                        "legs": {"mfma": {"time_at_peak_us_per_step": t_flop / steps * 1e6,
                                          "frac": ach / HIDDEN_FP32_MFMA_TFLOPS},
                                 "hbm": {"algorithmic_bytes_per_step": nbytes / steps, "d_iter_MB": bd / 1e6,
                                         "g_iter_MB": bg / 1e6, "achieved_GBs": nbytes / t_meas / 1e9,
                                         "peak_GBs": HBM_PEAK_GBS, "time_at_peak_us_per_step": t_byte / steps * 1e6,
                                         "frac": nbytes / t_meas / 1e9 / HBM_PEAK_GBS}},
                        "frac_rule": "max(flop time at the fp32 MFMA peak, byte time at the HBM peak) / measured"},
           "cpu_baseline": None,
           "final": [float(x) for x in eng.d_step(batches[0]).cpu()]}
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = gan_cpu_baseline(g_sd, d_sd, np_batches, N, S, H, E, Z, args.cpu_baseline_seconds)
    print(json.dumps(out), flush=True)


def eval_model(tabs, num_items, dev):
    """A stand-in for a fitted MF ImplicitFactorizationModel holding `tabs` (user_w, item_w,
    user_b, item_b): the model's own evaluation methods (implicit.py _tables / _device_scores /
    score_users / topk_users) bound to it, so the bench times the drop-in's evaluation path
    without a fit."""
    import types
    from recommendation_gans_amd.implicit import ImplicitFactorizationModel
    m = types.SimpleNamespace(_kind="mf", _num_items=num_items, _full_tables=None,
                              _engine=types.SimpleNamespace(device=dev, params=lambda: tabs))
    for name in ("_tables", "_device_scores", "score_users", "topk_users"):
        setattr(m, name, types.MethodType(getattr(ImplicitFactorizationModel, name), m))
    return m


def bench_eval(args):
    """ImplicitFactorizationModel.test's ranking metrics
    (precision_recall_score + map_at_k, k = 5, evaluation.py:115-185, 334-353) over the
    synthetic ML-20M test split, for a d = 64 MF model of that shape.  A "step" is one
    block of 4096 test users: one GEMM of the tables + sigmoid (library GEMM) and
    rg_topk_rows; `value` = test users ranked per second over the whole split.  The CPU
    leg is the reference's ranking (numpy argsort of each user's scores) on a bounded
    sample of users."""
    import types
    from recommendation_gans_amd.spotlight import evaluation
    from recommendation_gans_amd.spotlight.interactions import Interactions
    from recommendation_gans_amd.synthetic import ML20M, movielens_like
    dev = torch.device("cuda:0")
    d, k = args.dim, 5
    data = movielens_like(ML20M, seed=0, zipf_s=args.zipf)
    U, I = data.num_users, data.num_items
    test = Interactions(data.test_u, data.test_i, num_users=U, num_items=I)
    torch.manual_seed(0)
    tabs = [torch.randn(U, d, device=dev) / d, torch.randn(I, d, device=dev) / d, torch.zeros(U, device=dev),
            torch.zeros(I, device=dev)]
    m = eval_model(tabs, I, dev)
    csr = test.tocsr()
    n_users = int((np.diff(csr.indptr) > 0).sum())
    with stdout_to_stderr():          # the metrics print the reference's cold-start count
        evaluation.precision_recall_score(m, Interactions(data.test_u[:2000], data.test_i[:2000], num_users=U,
                                                          num_items=I), k=k)       # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p, r = evaluation.precision_recall_score(m, test, k=k)
        mp = evaluation.map_at_k(m, test, k=k)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    out = {"metric": "evaluation test users/sec (precision/recall@5 + MAP@5), MF dim=64 MovieLens-20M",
           "value": 2 * n_users / el, "unit": "users/s", "n_gpus": 1, "steps": 2, "warmup": 1,
           "ms_per_step": el / 2 * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "f32", "data": f"synthetic ML-20M-shaped test split ({n_users} users, {len(data.test_u)} "
                                   f"interactions), N(0,1/d) tables",
           "config": {"workload": f"rank {I} items per test user, top {k}, two metric passes", "embedding_dim": d,
                      "parallelism": "dp1"},
           "precision": float(p), "recall": float(r), "map": float(mp), "roofline": None, "cpu_baseline": None}
    if not args.no_cpu_baseline:
        host = types.SimpleNamespace(score_users=m.score_users)
        users = np.flatnonzero(np.diff(csr.indptr) > 0)
        sel = np.isin(data.test_u, users[:1000])
        sub = Interactions(data.test_u[sel], data.test_i[sel], num_users=U, num_items=I)
        with stdout_to_stderr():
            t0 = time.perf_counter()
            evaluation.precision_recall_score(host, sub, k=k)
            evaluation.map_at_k(host, sub, k=k)
            elc = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": 2 * 1000 / elc, "unit": "users/s", "cores": 1, "kind": "port",
                               "sample": "1000 test users x 2 passes: scores from the device block, then the "
                                         "reference's per-user numpy argsort over all items on the host"}
    print(json.dumps(out), flush=True)


def launch_ranks(args):
    """`--gpus N` (N > 1) without WORLD_SIZE: start the N rank processes as ONE child,
    `torch.distributed.run` on this node over 127.0.0.1, before this process makes any
    GPU call (so no exec and no GPU state in the parent), and exit with its status --
    a failed launch is a failed bench, never a 1-rank run."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    rc = subprocess.call(cmd, env=env)
    if rc != 0:
        print(f"bench.py: the {args.gpus}-rank launch failed with status {rc}", file=sys.stderr)
    sys.exit(rc if rc != 0 else 0)


def launch_check(args):
    """The multi-rank plumbing alone (gloo, CPU): rendezvous, barrier-bracketed timing of
    a trivial all-reduce per step, max over ranks, one JSON line from rank 0."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    x = torch.ones(1024)
    for _ in range(args.warmup):
        if world > 1:
            dist.all_reduce(x)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if world > 1:
            dist.all_reduce(x)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": "launch check (gloo all-reduce of 1024 floats)", "value": args.steps / el,
                          "unit": "steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
                          "vs_baseline": None, "dtype": "f32", "data": "synthetic",
                          "config": {"workload": "launch plumbing only", "parallelism": f"dp{world}"}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args)
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}")
    if args.launch_check:
        return launch_check(args)
    if args.gpus > 1 and args.model in ("gan", "eval"):
        raise SystemExit(f"--model {args.model} runs on one GPU (cGAN: replicas only, SURVEY §8e); "
                         f"--gpus {args.gpus} refused")
    if args.model == "eval":
        return bench_eval(args)
    if args.model in ("ncf", "neumf"):
        return bench_ncf(args)
    if args.model == "gan":
        return bench_gan(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    emu = None
    if args.emulate_rank:
        if world > 1:
            raise SystemExit("--emulate-rank runs one process on one GPU")
        r_, w_ = (int(x) for x in args.emulate_rank.split("/"))
        if not (w_ > 1 and 0 <= r_ < w_):
            raise SystemExit("--emulate-rank R/W needs W > 1 and 0 <= R < W")
        emu = (r_, w_)
        args.dp = "owner"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        with stdout_to_stderr():          # stdout carries only the JSON line
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
    dev = torch.device(f"cuda:{local_rank}")
    torch.cuda.set_device(dev)

    from recommendation_gans_amd import build as rg_build
    from recommendation_gans_amd import sharding
    from recommendation_gans_amd.mf_engine import MFEngine
    from recommendation_gans_amd.synthetic import ML20M, movielens_like

    if not os.path.exists(rg_build.LIB):
        rg_build.build()
    d, B, n = args.dim, args.batch, args.neg
    # the stepper's overlapped step (rg_stepper.cpp train_fused) unless disabled
    from recommendation_gans_amd import _lib as _rglib
    fused = _rglib.ab_build() and os.environ.get("RG_FUSED", "0") == "1" and args.loss != "adaptive_hinge"
    data = movielens_like(ML20M, seed=0, zipf_s=args.zipf)
    U, I = data.num_users, data.num_items
    torch.manual_seed(0)                               # mf_spotlight.py:37
    Uw = torch.empty(U, d).normal_(0, 1.0 / d)         # ScaledEmbedding (layers.py:35)
    Iw = torch.empty(I, d).normal_(0, 1.0 / d)
    random.seed(0)
    mt = np.asarray(random.getstate()[1], dtype=np.uint32)
    comm = None
    if world > 1:
        from recommendation_gans_amd.comm import RcclComm
        with stdout_to_stderr():          # RCCL's init banner
            comm = RcclComm(dev)
    if emu is not None:
        # one GPU, rank emu[0] of emu[1]: the owner step at that geometry with local-copy exchanges
        from recommendation_gans_amd.comm import LocalComm
        comm = LocalComm(dev, emu[1], emu[0])
        rank, world = emu
    gs = args.dp == "global_stream" and (world > 1 or args.dp_at_1)
    own = args.dp == "owner" and (world > 1 or args.dp_at_1)
    solo_pg = False
    if own and comm is None and args.comm_at_1:
        # N = 1 on the DP code path: a one-rank gloo group carries the RCCL id, so the native
        # owner step runs with its two RCCL all-reduces (and the item gradient on the
        # communicator stream) exactly as at N > 1
        import socket
        from recommendation_gans_amd.comm import RcclComm
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            os.environ.setdefault("MASTER_PORT", str(sk.getsockname()[1]))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        with stdout_to_stderr():
            dist.init_process_group("gloo", rank=0, world_size=1)
            comm = RcclComm(dev)
        solo_pg = True
    if own:
        # owner-sharded, reference-exact: this rank's users (u % world == rank) + every item,
        # the full pool; every global batch of B * world positives, this rank's plan of it
        eng = MFEngine(Uw, Iw, torch.zeros(U), torch.zeros(I), data.pool_u, data.pool_i, mt, loss=args.loss,
                       optimizer=args.optim, lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B, device=dev,
                       rank=rank, world_size=world, dp="owner", prefetch=not args.no_prefetch, comm=comm)
        train_u, train_i = data.train_u, data.train_i
        U_local = eng.U
        gb = B * world
        nbatches = len(train_u) // gb
        batch_lo = [g * gb for g in range(nbatches)]
    elif gs:
        # replicated, reference-exact: full tables / pool on every rank, global batches of
        # B * world positives, this rank's columns [rank*B, (rank+1)*B) of each
        eng = MFEngine(Uw, Iw, torch.zeros(U), torch.zeros(I), data.pool_u, data.pool_i, mt, loss=args.loss,
                       optimizer=args.optim, lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B, device=dev,
                       rank=rank, world_size=world, dp="global_stream", prefetch=not args.no_prefetch, comm=comm)
        train_u, train_i = data.train_u, data.train_i
        U_local = U
        gb = B * world
        nbatches = len(train_u) // gb
        batch_lo = [g * gb + rank * B for g in range(nbatches)]
    else:
        pool_u, pool_i = sharding.shard_pool(data.pool_u, data.pool_i, rank, world)
        train_u, train_i = sharding.shard_interactions(data.train_u, data.train_i, rank, world)
        U_local = sharding.num_local_users(U, rank, world)
        eng = MFEngine(sharding.shard_rows(Uw, rank, world), Iw, torch.zeros(U_local), torch.zeros(I), pool_u,
                       pool_i, sharding.rank_mt_state(mt, rank), loss=args.loss, optimizer=args.optim, lr=1e-3,
                       weight_decay=1e-5, n_neg=n, batch_size=B, device=dev, rank=rank, world_size=world,
                       dp="user_shard" if world > 1 else None, prefetch=not args.no_prefetch, comm=comm)
        gb = B * world
        nbatches = len(train_u) // B
        batch_lo = [g * B for g in range(nbatches)]
    tu = torch.from_numpy(train_u).to(dev)
    ti = torch.from_numpy(train_i).to(dev)
    # per-batch plans: the epoch order is fixed for the whole fit (implicit.py:262), so
    # they are built once per fit, before timing (like the reference's own data
    # preparation), for EVERY batch of the epoch in one launch (rg_mf_plans_build); the
    # cost is measured (second build, warm) and reported beside the step
    pstride = batch_lo[1] - batch_lo[0] if nbatches > 1 else B
    pkw = dict(users=tu) if own else {}
    eng.make_plans(ti[:gb * 4], offset=batch_lo[0], stride=pstride, **({"users": tu[:gb * 4]} if own else {}))
    torch.cuda.synchronize()
    tp0 = time.perf_counter()
    plans = eng.make_plans(ti, offset=batch_lo[0], stride=pstride, **pkw)[:nbatches]
    torch.cuda.synchronize()
    plan_epoch_s = time.perf_counter() - tp0
    plan_us = plan_epoch_s / nbatches * 1e6
    nplan = len(plans)

    span = gb if own else B

    def batch(s):
        g = s % nbatches
        lo = batch_lo[g]
        return tu[lo:lo + span], ti[lo:lo + span], plans[g % nplan]

    # step inputs (ids + plan pointers) built before timing; each call also hands the
    # NEXT step's input to the native stepper, which generates its words ahead
    n_extra = 6          # untimed steps after the timed region (lazy-pass row counts)
    inputs = [eng.step_input(*batch(s)[:2], gb, batch(s)[2]) for s in range(args.warmup + args.steps + n_extra + 2)]

    def step(s, ev=None):
        # two steps of lookahead: the pipelined single-GPU step runs step s+1's pair pass and
        # step s+2's prepare inside step s's launch (rg_mf_stepper_train_ahead)
        return eng.train_step_in(inputs[s], inputs[s + 1], apply_events=ev, next2=inputs[s + 2])

    for s in range(args.warmup):
        step(s)
    torch.cuda.synchronize()
    every = max(1, args.events_every)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           if s % every == 0 else None for s in range(args.steps)]
    for ev in evs:   # torch creates the HIP event lazily on its first record
        if ev is not None:
            ev[0].record()
            ev[1].record()
    multi = world > 1 and emu is None     # real ranks (an emulated rank is one process)
    if multi:
        dist.barrier()
    torch.cuda.synchronize()
    ahead = None
    if args.host_ahead > 0:
        # ~2.1 GHz shader clock: the spin outlasts the host's enqueue of every timed step
        torch.cuda._sleep(int(args.host_ahead * 2.1e6))
        ahead = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ahead[0].record()
    t0 = time.perf_counter()
    for s in range(args.steps):
        step(args.warmup + s, evs[s])
    if ahead is not None:
        ahead[1].record()
    # the lazy pass leaves cold user rows behind: catching them all up is part of the timed
    # work (after this every row equals the eager pass's; no-op when eager)
    eng.flush()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    if multi:
        dist.barrier()
    el = time.perf_counter() - t0
    rccl = None
    if multi:
        # every rank's own time and what its native communicator reports (ncclCommCount /
        # ncclCommUserRank): the line shows the ranks RCCL itself saw, not only WORLD_SIZE
        cnt, urank, is_rccl = comm.info() if comm is not None else (world, rank, False)
        mine = torch.tensor([el, float(cnt), float(urank), float(is_rccl)], dtype=torch.float64, device=dev)
        allv = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
        allv = [v.tolist() for v in allv]
        el = max(v[0] for v in allv)
        rccl = {"comm_count": sorted({int(v[1]) for v in allv}), "user_ranks": [int(v[2]) for v in allv],
                "native_rccl": all(v[3] > 0 for v in allv),
                "per_rank_ms_per_step": [v[0] / args.steps * 1e3 for v in allv]}
    loss_last = float(eng.loss_out[0])
    if getattr(eng, "pipelined", False) and eng.pipe_error():
        raise RuntimeError("pipelined MF step: a pair workgroup's bounded wait ran out (results invalid)")
    lazy_rows = None
    if eng.lazy_rows(enable=True) is not None:
        # untimed: user rows the lazy pass processes per step (the counter is contended, so it
        # runs only here), over steps that continue the timed sequence
        base = args.warmup + args.steps
        for s in range(n_extra - 1):
            eng.train_step_in(inputs[base + s], inputs[base + s + 1])
        lazy_rows = eng.lazy_rows(enable=False) / (n_extra - 1)
        eng.flush()

    if ahead is not None:
        torch.cuda.synchronize()
        ahead = ahead[0].elapsed_time(ahead[1]) * 1e3 / args.steps
        if t_enq * 1e3 > args.host_ahead:
            print(f"warning: the host took {t_enq * 1e3:.2f} ms to enqueue, longer than the {args.host_ahead} ms spin",
                  file=sys.stderr)
    if emu is not None:
        return report_emulated(args, emu, eng, evs, el, U, I, d, B, n, t_enq, ahead)
    if rank == 0:
        value = args.steps * B * world / el
        # per rank: its user shard + every item go through the dense optimizer pass
        gather, ids, adam = algorithmic_bytes(U_local, I, d, B, n)
        user_adam = 6 * U_local * (4 * d + 4) if (world > 1 or own) else adam
        out = {"metric": METRIC, "value": value, "unit": "interactions/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "f32",
               "data": f"synthetic ML-20M-shaped: U={U} I={I}, {len(data.train_u)} train positives "
                       f"(lognormal users, Zipf({args.zipf}) items, 81/9/10 time split), "
                       f"pool {len(data.pool_u)} uniform pairs; tables N(0,1/d) init",
               "config": {"workload": f"MF-{args.loss.upper()} ML-20M-shaped, embedding_dim={d}, "
                                      f"batch {B}/GPU, {n} negatives, {args.optim} (coupled L2 1e-5) over all rows",
                          "global_batch": gb, "embedding_dim": d,
                          "parallelism": f"dp{world}" + (" owner-sharded users, replicated items (score + item-"
                                                         "gradient all-reduces, reference-exact)" if own else
                                                         " replicated (reduce-scatter + all-gather, reference-exact)"
                                                         if gs else "" if world == 1 else
                                                         " user-sharded (opt-in, not reference sampling)")},
               "plan_build_us_per_batch": plan_us, "plan_build_ms_per_epoch": plan_epoch_s * 1e3,
               "plan_build_note": f"item-sorted plans of all {nbatches} batches of an epoch in one HIP launch "
                                  "(rg_mf_plans_build), built once per fit (the reference shuffles once, "
                                  "implicit.py:262); not in the timed region"}
        if rccl is not None:
            out["rccl"] = rccl
        step_bytes = gather + ids + adam
        out["step_roofline"] = {"bytes_per_step": step_bytes,
                                "achieved_GBs": step_bytes / (el / args.steps) / 1e9,
                                "frac": step_bytes / (el / args.steps) / 1e9 / HBM_PEAK_GBS}
        out["host_enqueue_us_per_step"] = t_enq / args.steps * 1e6
        if ahead is not None:   # --host-ahead diagnostic (the wall time includes the spin)
            out["gpu_ahead_us_per_step"] = ahead
            out["ms_per_step"] = ahead * 1e-3
            out["value"] = B * world / (ahead * 1e-6)
            out["timing"] = "GPU events after a host-ahead spin (diagnostic)"
        if lazy_rows is not None:
            out["lazy_dense_pass"] = {
                "user_rows_per_step": lazy_rows, "user_rows": U_local,
                "note": "deferred cold user-row updates (DESIGN §4.1): a user row is processed when it has a "
                        "gradient or the next step reads it, its skipped cold updates applied in order on the "
                        "way; bit-identical to the eager dense pass (tests/test_lazy_gpu.py); the timed region "
                        "ends with the flush that brings every row up to date"}
        if any(ev is not None for ev in evs):
            from recommendation_gans_amd import _lib
            ms = [_lib.elapsed_ms(a, b) for a, b in (ev for ev in evs if ev is not None)]
            avg = float(np.mean(ms)) * 1e-3
            if own:
                # the events bracket the user rows' update with the next step's owner prepare
                alg = user_adam
                kname = "rg_mf_apply (owner: this rank's user rows; next step's owner prepare in the same launch)"
            elif gs:
                # rg_mf_grads_sharded: every row's pulled gradient written rank-major (the exchange's input)
                alg = gather + world * eng.chunk * 4
                kname = "rg_mf_grads_sharded (mf_apply_kernel<kGradOnly>, rank-major gradient for the reduce-scatter)"
            elif fused:
                # the events bracket rg_mf_step_front (pairs | next prepare | cold-row update)
                # and rg_mf_step_hot (touched-row update): the whole step's algorithmic bytes
                # (DP: up to the user-shard update; the item update follows the exchange)
                alg = gather + ids + user_adam
                kname = "rg_mf_step_front + rg_mf_step_hot (mf_front_kernel, mf_hot_kernel)"
            elif lazy_rows is not None:
                # rg_mf_apply_lazy: p, m, v of every item row and of the user rows it processes
                # (a gradient this step or a next-step mark), read + written once
                alg = 6 * (I + lazy_rows) * (4 * d + 4)
                kname = ("rg_mf_apply_lazy (mf_back_kernel<LAZY>: every item row + the user rows with a "
                         "gradient or a next-step mark; deferred cold updates applied on the way)")
            elif eng.pipelined:
                # rg_mf_pipe_step: step s's dense pass, step s+1's pair pass (row gathers) and
                # step s+2's prepare (ids) in one launch
                alg = user_adam + ids + gather
                kname = ("rg_mf_pipe_step (mf_pipe_kernel: dense update of step s + pair pass of s+1 + prepare "
                         "of s+2)")
            else:
                # rg_mf_apply_prepare: the dense optimizer pass and the next step's prepare
                # (ids in, prepared pairs out) in one launch
                alg = user_adam + ids
                kname = "rg_mf_apply_prepare (mf_back_kernel: dense update + next-step prepare)"
            ach = alg / avg / 1e9
            out["roofline"] = {"bound": "hbm", "kernel": kname, "achieved": ach,
                               "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                               "traffic": None, "algorithmic_bytes_per_launch": alg,
                               "avg_launch_us": avg * 1e6}
            # PMC traffic (scripts/pmc_apply.sh: FETCH_SIZE / WRITE_SIZE passes) of THIS build only:
            # the profile is stamped with the library's hash, a profile of another build is refused
            pmc = os.path.join(ROOT, "profiles", "pmc_step.json" if fused else "pmc_back.json")
            if world == 1 and not own and not gs and lazy_rows is None and os.path.exists(pmc):
                import hashlib
                p = json.load(open(pmc))
                sha = hashlib.sha256(open(os.environ.get("RG_LIB") or rg_build.LIB, "rb").read()).hexdigest()[:16]
                if p.get("dim") == d and p.get("batch") == B and p.get("lib_sha16") == sha:
                    out["roofline"]["traffic"] = p.get("hbm_bytes_per_step" if fused else "hbm_bytes_per_launch")
                    out["roofline"]["traffic_source"] = f"profiles/{os.path.basename(pmc)} (lib {sha})"
                else:
                    out["roofline"]["traffic_source"] = (f"profiles/{os.path.basename(pmc)} is of another build "
                                                         f"(lib {p.get('lib_sha16')} vs {sha}): not used")
        if out.get("roofline"):
            # the box's achievable HBM rate (STREAM-style copy, after the timed region), reported
            # beside the 8 TB/s nominal peak
            bw = stream_copy_gbs(dev)
            out["roofline"]["stream_copy_GBs"] = bw
            out["roofline"]["frac_of_stream_copy"] = out["roofline"]["achieved"] / bw
        out["final_loss"] = loss_last
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(data, d, B, n, args.loss, args.cpu_baseline_seconds)
        print(json.dumps(out), flush=True)
    if world > 1 or solo_pg:
        del eng
        comm.close()
        dist.destroy_process_group()


def report_emulated(args, emu, eng, evs, el, U, I, d, B, n, t_enq, ahead=None):
    """--emulate-rank: one JSON line for rank R's step at W-rank geometry (NOT the driver's
    metric line): its time per step, the user-update kernel's events, and what W ranks each
    taking this step time would process (exchange time over xGMI NOT included: the
    collectives were local copies)."""
    from recommendation_gans_amd import _lib
    r_, w_ = emu
    ms_step = el / args.steps * 1e3
    ev = [_lib.elapsed_ms(a, b) for a, b in (e for e in evs if e is not None)]
    rows_user = eng.U
    out = {"metric": f"emulated rank {r_} of {w_}: owner-sharded MF step time (local-copy exchanges)",
           "value": args.steps * B * w_ / el, "unit": "interactions/s (projected: W ranks at this step time)",
           "n_gpus": 1, "emulated_world": w_, "emulated_rank": r_, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
           "data": f"synthetic ML-20M-shaped: U={U} I={I}",
           "config": {"workload": f"MF-{args.loss.upper()} d={d}, batch {B}/rank, global batch {B * w_}, {n} "
                                  f"negatives, {args.optim}; this rank: {rows_user} user rows + {I} item rows",
                      "global_batch": B * w_, "embedding_dim": d, "parallelism": f"emulated dp{w_} owner"},
           "exchange_floats_per_step": {"scores": (1 + n) * B * w_ if args.loss != "pointwise" else 0,
                                        "item_grad": I * (d + 1) + 1},
           "user_update_us": float(np.mean(ev)) * 1e3 if ev else None,
           # host time to enqueue a step (Python + the stepper's HIP calls): close to the step
           # time means the GPU waits for the host
           "host_enqueue_us_per_step": t_enq / args.steps * 1e6,
           "mt_mode": eng.mt_mode,
           "final_loss": float(eng.loss_out[0])}
    if ahead is not None:
        # --host-ahead: every step enqueued before the GPU reached it (the wall time above
        # includes the spin): the GPU-side step time alone
        out["gpu_ahead_us_per_step"] = ahead
        out["ms_per_step"] = ahead * 1e-3
        out["value"] = B * w_ / (ahead * 1e-6)
        out["timing"] = "GPU events after a host-ahead spin (diagnostic)"
    print(json.dumps(out), flush=True)
    eng.comm.close()


if __name__ == "__main__":
    main()
