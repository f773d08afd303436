"""Diagnostic for DESIGN §0.4 row 3's open NeuMF finding (test infrastructure: runs the oracle on
the CPU, no GPU): the layer-0 pre-activations of the example (user 20562, item 17554) before
steps 14-16 of neuMF_spotlight.py's defaults at ML-20M shape, in float64.  Unit 2 reaches
8.4e-08 before step 16 -- inside fp32 rounding of its 32-term dot product -- which is where the
GPU's rows part from the reference (tests/parity_long_ncf.py --neumf --track ...).

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
o = oncf.NeuMFOracle([t.double() for t in params], names, data.pool_u, data.pool_i, orng.py_seed_state(0), **kw)
widths = oncf.layer_sizes(E)[1:]
rs = np.random.RandomState(6)
iu, ii, iw, ib = names.index('embedding_user_mlp.weight'), names.index('embedding_item_mlp.weight'), names.index('layers.0.weight'), names.index('layers.0.bias')
for s in range(17):
    pu = data.train_u[s * B:(s + 1) * B].astype(np.int64)
    pi = data.train_i[s * B:(s + 1) * B].astype(np.int64)
    mp = [torch.from_numpy((rs.rand(B, w) >= 0.5).astype(np.uint8)) for w in widths]
    mn = [torch.from_numpy((rs.rand(n * B, w) >= 0.5).astype(np.uint8)) for w in widths]
    if s >= 14:
        P = o.P.t
        x = torch.cat([P[iu][20562], P[ii][17554]])
        pre = P[iw] @ x + P[ib]
        print('before step', s, 'pre-activations of (20562, 17554):', ['%.3e' % v for v in pre.tolist()[:6]])
    o.step(pu, pi, mp, mn)
