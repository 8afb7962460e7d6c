"""RCCL on the hardware: the bench's rank body with a real "nccl" process group.

Two ranks cannot share one GPU under RCCL (it rejects duplicate devices in a
communicator), and the leased box has one GPU, so the multi-rank RCCL path is
exercised here at world size 1 with the process group forced on
(QAMR_DIST_FORCE_PG=1): every collective of the bench -- the timed-region max and
the BER/FER counter sum -- then runs through RCCL on the MI355X,
the same calls the 8-GPU run makes.  The bench runs as a child process (fresh
process, no exec of this GPU-initialised one)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_bench_rank_body_over_rccl(gpu):
    env = dict(os.environ, QAMR_DIST_FORCE_PG="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    env.pop("QAMR_BENCH_STUB", None)
    env.pop("QAMR_BENCH_BACKEND", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--workload", "reg1008_4pam",
           "--batch", "256", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0",
           "--no-secondary", "--no-roofline"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["config"]["backend"] == "nccl" and out["n_gpus"] == 1
    assert out["ber_fer"]["frames_counted"] == 256  # the counter sum went through RCCL
    assert out["value"] > 0


@pytest.mark.gpu
def test_host_tensor_staged_through_rccl(gpu):
    """A host tensor handed to qamr.dist under RCCL is staged through the GPU (RCCL
    itself rejects host tensors: checked too)."""
    code = r"""
import os, sys, torch, torch.distributed as td
sys.path.insert(0, os.path.join(sys.argv[1], "qam-reconciliation_amd"))
from qamr import dist
w, r, _ = dist.init("nccl")
assert td.get_backend() == "nccl" and w == 1
t = torch.tensor([3, 4, 5], dtype=torch.int64)
dist.all_reduce_sum(t)
m = torch.tensor([2.5], dtype=torch.float64)
dist.all_reduce_max(m)
try:
    td.all_reduce(torch.zeros(1))
    raw = "accepted"
except Exception as e:
    raw = "rejected"
dist.barrier()
dist.finalize()
print("RESULT", t.tolist(), float(m.item()), t.device.type, raw)
"""
    env = dict(os.environ, QAMR_DIST_FORCE_PG="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, "-c", code, ROOT], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT")][-1]
    assert line.startswith("RESULT [3, 4, 5] 2.5 cpu"), line
    print(line)
