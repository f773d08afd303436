"""Bounded failure of the RCCL communicator (rg_comm.cpp watchdog, DESIGN §6 "Bounded failure"):
a rank whose collective can never complete -- its peer skips that all-reduce -- must end with
exit status 3 and a message naming it within RG_COMM_TIMEOUT_S, even though it then blocks in a
stream synchronize and enqueues nothing more (the case ADVICE r4 found untracked when only every
16th collective armed the deadline).  Needs two GPUs (RCCL refuses two ranks on one device), so
it is skipped on the one-GPU boxes; it runs on a multi-GPU node."""
import os
import subprocess
import sys
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RANK_SCRIPT = r"""
import os, sys, time
import torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from recommendation_gans_amd.comm import RcclComm
rank = int(os.environ["RANK"])
torch.cuda.set_device(rank)
dist.init_process_group("gloo", rank=rank, world_size=2)
comm = RcclComm(torch.device("cuda", rank))
buf = torch.ones(1 << 16, device=f"cuda:{rank}")
dist.barrier()
if rank == 0:
    comm.allreduce_(buf)          # the peer never joins this one
    torch.cuda.synchronize()      # blocks: only the watchdog can end this process
    print("rank 0 returned", flush=True)
    sys.exit(0)
time.sleep(60)                    # rank 1 skips the all-reduce
sys.exit(0)
"""


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                    reason="needs two GPUs (RCCL refuses two ranks on one device)")
def test_stalled_collective_exits_with_status_3(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29731", WORLD_SIZE="2",
               RG_COMM_TIMEOUT_S="5", HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, str(script), ROOT], env=dict(env, RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    t0 = time.time()
    try:
        out, err = procs[0].communicate(timeout=90)
    finally:
        procs[1].kill()
        procs[1].communicate()
    assert procs[0].returncode == 3, (procs[0].returncode, out, err[-2000:])
    assert "rank 0 of 2" in err, err[-2000:]
    assert "rank 0 returned" not in out
    assert time.time() - t0 < 85


AHEAD_SCRIPT = r"""
import os, sys, time
import torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from recommendation_gans_amd.comm import RcclComm
torch.cuda.set_device(0)
dist.init_process_group("gloo", rank=0, world_size=1)
comm = RcclComm(torch.device("cuda", 0))
x = torch.ones(4 << 20, device="cuda")
buf = torch.ones(1 << 10, device="cuda")
evs, t0, n = [], time.time(), 0
while time.time() - t0 < 4 * float(os.environ["RG_COMM_TIMEOUT_S"]):
    for _ in range(4):
        x.mul_(1.0000001)
    comm.allreduce_(buf)
    e = torch.cuda.Event()
    e.record()
    evs.append(e)
    if len(evs) > 50:          # the host stays 50 iterations ahead of the GPU, never syncing it
        evs.pop(0).synchronize()
    n += 1
torch.cuda.synchronize()
print("host-ahead run finished", n, flush=True)
"""


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_host_ahead_run_is_not_killed(tmp_path):
    """a healthy run whose host stays ahead of the GPU (enqueueing collectives, never
    waiting for the newest one) must not reach the deadline -- the watchdog times the OLDEST
    collective not yet complete (a FIFO of events), not the newest one's re-recorded event.  One
    rank (an RCCL communicator of one: rg_comm_allreduce_sum_f32 still launches ncclAllReduce)
    for four deadlines' time with RG_COMM_TIMEOUT_S = 2."""
    script = tmp_path / "ahead.py"
    script.write_text(AHEAD_SCRIPT)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29733", RG_COMM_TIMEOUT_S="2",
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, str(script), ROOT], env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, (p.returncode, p.stdout, p.stderr[-2000:])
    assert "host-ahead run finished" in p.stdout
