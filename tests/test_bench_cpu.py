"""bench.py's multi-rank launch contract, on the CPU (gloo; no GPU).

`python bench.py --gpus N` without WORLD_SIZE must start N rank processes itself
(torch.distributed.run child, before any GPU call) and report n_gpus = N from rank 0;
a mismatch between --gpus and an existing WORLD_SIZE, or a failed launch, must exit
non-zero -- never a silent 1-rank run (VERDICT r2, next #1a)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(kw)
    return env


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_launches_n_ranks(n):
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launch-check", "--steps", "5", "--warmup", "1"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = _json_line(p.stdout)
    assert line["n_gpus"] == n
    assert line["steps"] == 5 and line["ms_per_step"] > 0


def test_world_size_mismatch_refused():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), cwd=ROOT)
    assert p.returncode != 0
    assert "WORLD_SIZE" in p.stderr


def test_failed_rank_fails_the_launch():
    # every rank refuses a multi-rank cGAN bench (replicas only): the launch must fail, no JSON line
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--model", "gan"], capture_output=True, text=True,
                       timeout=240, env=_env(), cwd=ROOT)
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_eval_model_stand_in_scores_like_the_tables():
    """bench.py --model eval ranks through the drop-in's own evaluation methods bound to a
    stand-in model (bench.eval_model): every attribute they read must exist (a missing one
    broke the eval line once); scores = sigmoid(U I^T + ub + ib), checked on the CPU."""
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    import bench
    g = torch.Generator().manual_seed(0)
    tabs = [torch.randn(7, 4, generator=g), torch.randn(5, 4, generator=g), torch.randn(7, generator=g),
            torch.randn(5, generator=g)]
    m = bench.eval_model(tabs, 5, torch.device("cpu"))
    got = m.score_users([0, 3, 6])
    U, I, ub, ib = tabs
    want = torch.sigmoid(U[[0, 3, 6]] @ I.T + ub[[0, 3, 6]][:, None] + ib[None, :]).numpy()
    np.testing.assert_array_equal(got, want)
