"""Diagnostic for DESIGN §0.4 row 3's NeuMF finding (test infrastructure: runs the oracle on the
CPU, no GPU): the layer-0 pre-activations of the example (user 20562, item 17554) before steps
14-16 of neuMF_spotlight.py's defaults at ML-20M shape.  Unit 2 reaches 8.4e-08 before step 16 --
inside fp32 rounding of its 32-term dot product -- which is where the GPU's rows part from the
reference (tests/parity_long_ncf.py --neumf --track ...).

Before step 16 it also names the forward orders that flip the decision: the same 32 products
plus the bias summed left to right in fp32 (on the fp32 restatement's state, the state the GPU's
run tracks bit for bit up to there) in 20,000 seeded orders, the fraction landing on each side of
the kink and the first order that lands on the side the GPU took (<= 0), and the reference's own
order (x @ W.T + b in torch fp32).  Then the oracle's kink-flip sample (oracle/ncf.py kink_flip)
of the whole run: its user row 20562 against float64 at every step (the GPU's, in
profiles/r5/parity/parity_neumf_20steps_track_r6.jsonl: 4.5e-4 at step 16, 7.4e-4 at step 19).

    python tests/neumf_relu_probe.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ncf as oncf  # noqa: E402
from oracle import rng as orng  # noqa: E402
from recommendation_gans_amd.ncf_spotlight import mlp_layers  # noqa: E402
from recommendation_gans_amd.spotlight.dnn_models.neuMF import NeuMF  # noqa: E402
from recommendation_gans_amd.synthetic import ML20M, movielens_like  # noqa: E402
data = movielens_like(ML20M, seed=0)
U, I, E, B, n = data.num_users, data.num_items, 16, 8192, 5
torch.manual_seed(0)
net = NeuMF(mlp_layers(E), U, I, mf_embedding_dim=50, mlp_embedding_dim=E)
names = [k for k, _ in net.named_parameters()]
params = [p.detach().clone() for p in net.parameters()]
kw = dict(loss="pointwise", lr=1e-3, weight_decay=1e-5, n_neg=n, batch_size=B)


def oracle(dtype, **k):
    return oncf.NeuMFOracle([t.to(dtype).clone() for t in params], names, data.pool_u, data.pool_i, orng.py_seed_state(0),
                            **kw, **k)


o, o32, ofl = oracle(torch.float64), oracle(torch.float32), oracle(torch.float32, kink_flip=4.0)
widths = oncf.layer_sizes(E)[1:]
rs = np.random.RandomState(6)
iu, ii, iw, ib = (names.index(k) for k in ('embedding_user_mlp.weight', 'embedding_item_mlp.weight',
                                           'layers.0.weight', 'layers.0.bias'))
for s in range(20):
    pu = data.train_u[s * B:(s + 1) * B].astype(np.int64)
    pi = data.train_i[s * B:(s + 1) * B].astype(np.int64)
    mp = [torch.from_numpy((rs.rand(B, w) >= 0.5).astype(np.uint8)) for w in widths]
    mn = [torch.from_numpy((rs.rand(n * B, w) >= 0.5).astype(np.uint8)) for w in widths]
    if 14 <= s <= 16:
        P = o.P.t
        x = torch.cat([P[iu][20562], P[ii][17554]])
        pre = P[iw] @ x + P[ib]
        print('before step', s, 'float64 pre-activations of (20562, 17554):', ['%.3e' % v for v in pre.tolist()[:6]])
    if s == 16:
        P = o32.P.t
        x32 = torch.cat([P[iu][20562], P[ii][17554]])
        terms = np.append((P[iw][2] * x32).numpy(), P[ib][2].numpy()).astype(np.float32)   # 32 products + bias
        ref = float((x32[None] @ P[iw].t() + P[ib])[0, 2])
        g = np.random.RandomState(0)
        vals, first = [], None
        for t in range(20000):
            perm = g.permutation(len(terms))
            acc = np.float32(0)
            for v in terms[perm]:
                acc = np.float32(acc + v)
            vals.append(float(acc))
            if first is None and acc <= 0:
                first = (t, perm.tolist(), float(acc))
        vals = np.array(vals)
        print(f'before step 16, fp32 state: unit 2 in the reference order (torch mm) {ref:.3e}; in 20,000 seeded '
              f'left-to-right fp32 orders <= 0 in {np.mean(vals <= 0):.3f} of them, > 0 in {np.mean(vals > 0):.3f} '
              f'(range {vals.min():.3e} .. {vals.max():.3e}, exact {float(pre[2]):.3e})')
        if first is not None:
            print(f'first order landing <= 0 (order #{first[0]}, value {first[2]:.3e}; index 32 = the bias): {first[1]}')
    o.step(pu, pi, mp, mn)
    o32.step(pu, pi, mp, mn)
    ofl.step(pu, pi, mp, mn)
    d = float((ofl.P.t[iu][20562].double() - o.P.t[iu][20562]).abs().max())
    print(f'step {s}: kink-flip sample flipped {ofl.flips[-1]} decisions; its user row 20562 vs float64 {d:.2e}')
