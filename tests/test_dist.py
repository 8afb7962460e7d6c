"""Multi-process CPU tests (gloo, world_size 2) of the sharding / reduction
logic used by bench.py and qamr.sim on RCCL: frame shards tile the batch
exactly, the five BER/FER counters all-reduce to the global sums, every rank
takes the same early-stop decision, and the timed region is max-reduced."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "qam-reconciliation_amd"))
    from qamr import dist

    w, r, _ = dist.init("gloo")
    assert (w, r) == (world, rank)
    out = {}
    # shards of 4096 and of a ragged 1001-frame batch
    out["shards"] = [dist.shard(n, world, rank) for n in (4096, 1001, 1)]
    # per-rank counters: bit_errors, frame_errors, successes, iter_sum, frames
    c = torch.tensor([10 * (rank + 1), rank + 1, 5 - rank, 7 * (rank + 2), 100 + rank], dtype=torch.int64)
    dist.all_reduce_sum(c)
    out["counters"] = c.tolist()
    out["stop"] = dist.early_stop(c.numpy(), ferr_count_min=3, simulation_loops=1000)
    t = torch.tensor([0.5 + rank], dtype=torch.float64)
    dist.all_reduce_max(t)
    out["tmax"] = float(t.item())
    out["seed"] = dist.rank_seed(3, rank, 7)
    dist.barrier()
    dist.finalize()
    q.put((rank, out))


def test_gloo_world2_sharding_and_reduction():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    # shards tile [0, n) without overlap
    for i, n in enumerate((4096, 1001, 1)):
        ranges = sorted(res[r]["shards"][i] for r in range(world))
        pos = 0
        for start, cnt in ranges:
            assert start == pos
            pos += cnt
        assert pos == n
    exp = [10 + 20, 1 + 2, 5 + 4, 14 + 21, 100 + 101]
    assert res[0]["counters"] == exp and res[1]["counters"] == exp
    assert res[0]["stop"] == res[1]["stop"] is True
    assert res[0]["tmax"] == res[1]["tmax"] == 1.5
    assert res[0]["seed"] != res[1]["seed"]


def test_early_stop_rule():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "qam-reconciliation_amd"))
    from qamr import dist

    # reconciliation.pyx:159-161: frame_errors >= min and wordcount > loops/20
    assert not dist.early_stop([0, 99, 0, 0, 1000], 100, 5000)
    assert not dist.early_stop([0, 100, 0, 0, 251], 100, 5000)   # wordcount 250 is not > 250
    assert dist.early_stop([0, 100, 0, 0, 252], 100, 5000)


# ---------------------------------------------------------------- bench.py rank body
BENCH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")


def _bench_line(cmd, extra_env=None):
    import json
    import subprocess
    import sys

    env = dict(os.environ, QAMR_BENCH_STUB="1")
    env.pop("WORLD_SIZE", None)
    if extra_env:
        env.update(extra_env)
    r = subprocess.run([sys.executable] + cmd, env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    return json.loads(lines[0])


def _check_world2(out):
    assert out["n_gpus"] == 2
    assert out["config"]["global_batch"] == 2 * out["config"]["batch_per_gpu"]
    assert out["config"]["parallelism"] == "dp2" and out["config"]["backend"] == "gloo"
    B = out["config"]["batch_per_gpu"]
    # StubWork rank r contributes [10(r+1), r+1, B-r-1, 7(B-r-1), B]: the line carries the sums
    assert out["counters"] == [10 + 20, 1 + 2, (B - 1) + (B - 2), 7 * ((B - 1) + (B - 2)), 2 * B]
    assert len(out["per_rank"]["ms_per_step"]) == 2
    # value = frames of all ranks / max-over-ranks timed region
    assert abs(out["value"] - 2 * B * out["steps"] / (out["ms_per_step"] * out["steps"] / 1e3)) / out["value"] < 1e-2


def test_bench_gpus2_self_launch():
    """`bench.py --gpus 2` with no WORLD_SIZE starts 2 ranks itself (the configs[4]
    path at N=2), reports the process group's world size and the summed counters."""
    _check_world2(_bench_line([BENCH, "--gpus", "2", "--steps", "3", "--warmup", "1"]))


def test_bench_gpus2_torchrun():
    """The driver's launch: torch.distributed.run --nproc-per-node 2 bench.py --gpus 2."""
    out = _bench_line(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                       "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                       BENCH, "--gpus", "2", "--steps", "2", "--warmup", "1"])
    _check_world2(out)


def test_bench_world_size_must_match_gpus():
    import subprocess
    import sys

    env = dict(os.environ, QAMR_BENCH_STUB="1", WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "must agree" in r.stderr


# ------------------------------------------------------- RCCL device capability
def _qamr_dist():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "qam-reconciliation_amd"))
    from qamr import dist
    return dist


def test_staging_follows_backend_capability():
    """RCCL reduces GPU tensors only (torch's Backend.backend_capability['nccl']);
    qamr.dist stages a host tensor through the rank's GPU, and gloo gets host tensors."""
    d = _qamr_dist()
    assert d.staging_device_type("nccl", "cpu") == "cuda"
    assert d.staging_device_type("nccl", "cuda") is None
    assert d.staging_device_type("gloo", "cpu") is None
    assert d.staging_device_type("gloo", "cuda") == "cpu"
    assert d.staging_device_type("cpu:gloo,cuda:nccl", "cpu") is None
    assert d.staging_device_type("cpu:gloo,cuda:nccl", "cuda") is None


def test_bench_rank_body_under_rccl_capability(monkeypatch, capsys):
    """The bench's whole rank body (stub GPU work) with torch.distributed faked as a
    2-rank "nccl" group whose all_reduce rejects, as RCCL does, any tensor whose device
    the backend cannot reduce on.  A host tensor is accepted only after qamr.dist has
    staged it to the GPU (recorded by the stand-in for the host->GPU copy, since this
    box has no GPU).  Round 2's timed region handed RCCL a host tensor: that fails here."""
    import json
    import sys

    import torch
    import torch.distributed as tdist

    d = _qamr_dist()
    sys.path.insert(0, os.path.dirname(BENCH))
    import bench

    cap = set(tdist.Backend.backend_capability["nccl"])
    staged, seen = set(), []

    def fake_stage(t, device_type):
        assert device_type == "cuda"
        s = t.clone()
        staged.add(id(s))
        return s

    def fake_all_reduce(t, op=None, **kw):
        ok = t.device.type in cap or id(t) in staged
        seen.append((t.device.type, ok))
        if not ok:
            raise ValueError(f"No backend type associated with device type {t.device.type}")
        if op == tdist.ReduceOp.SUM:
            t.mul_(2)  # a second rank contributing the same values

    monkeypatch.setattr(d, "_stage", fake_stage)
    monkeypatch.setattr(tdist, "is_initialized", lambda: True)
    monkeypatch.setattr(tdist, "init_process_group", lambda *a, **k: None)
    monkeypatch.setattr(tdist, "destroy_process_group", lambda *a, **k: None)
    monkeypatch.setattr(tdist, "get_world_size", lambda *a, **k: 2)
    monkeypatch.setattr(tdist, "get_rank", lambda *a, **k: 0)
    monkeypatch.setattr(tdist, "get_backend", lambda *a, **k: "nccl")
    monkeypatch.setattr(tdist, "barrier", lambda *a, **k: None)
    monkeypatch.setattr(tdist, "all_reduce", fake_all_reduce)
    monkeypatch.setattr(torch.cuda, "set_device", lambda *a, **k: None)
    for k, v in dict(QAMR_BENCH_STUB="1", QAMR_BENCH_BACKEND="nccl", WORLD_SIZE="2", RANK="0",
                     LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29500").items():
        monkeypatch.setenv(k, v)
    assert bench.main(["--gpus", "2", "--steps", "2", "--warmup", "1"]) == 0
    out = json.loads([l for l in capsys.readouterr().out.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["config"]["backend"] == "nccl"
    assert len(seen) >= 2 and all(ok for _, ok in seen)  # timed-region max + counter sum
    B = out["config"]["batch_per_gpu"]
    assert out["counters"] == [2 * 10, 2 * 1, 2 * (B - 1), 2 * 7 * (B - 1), 2 * B]


# ------------------------------------------------ configs[4]'s rank count (8 ranks, CPU)
def _check_world8(out):
    assert out["n_gpus"] == 8
    B = out["config"]["batch_per_gpu"]
    assert out["config"]["global_batch"] == 8 * B == 32768      # configs[4]: 8 x 4096 frames
    assert out["config"]["parallelism"] == "dp8" and out["config"]["backend"] == "gloo"
    # StubWork rank r contributes [10(r+1), r+1, B-r-1, 7(B-r-1), B]
    assert out["counters"] == [10 * 36, 36, 8 * B - 36, 7 * (8 * B - 36), 8 * B]
    assert out["config"]["rank_devices"] == list(range(8))     # rank r bound LOCAL_RANK r
    # the per-rank record of the first scaling run: every rank's own timed region, the line's
    # ms_per_step their max (the stub has no priced kernel: no event averages)
    pr = out["per_rank"]
    assert len(pr["ms_per_step"]) == 8 and all(v > 0 for v in pr["ms_per_step"])
    assert abs(max(pr["ms_per_step"]) - out["ms_per_step"]) <= 1e-3 * out["ms_per_step"] + 1e-3
    assert pr["avg_launch_us"] == [None] * 8 and pr["priced_kernel"] is None


def test_bench_gpus8_self_launch():
    """`bench.py --gpus 8` (configs[4]'s launch at its real rank count) starting its 8 ranks
    itself: world size, global batch 32768, summed counters, rank r bound to GPU r."""
    _check_world8(_bench_line([BENCH, "--gpus", "8", "--steps", "2", "--warmup", "1", "--batch", "4096"]))


def test_bench_gpus8_torchrun():
    """The driver's N=8 launch: torch.distributed.run --nproc-per-node 8 bench.py --gpus 8."""
    _check_world8(_bench_line(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                               BENCH, "--gpus", "8", "--steps", "2", "--warmup", "1", "--batch", "4096"]))


# synthetic per-frame results of global frame g (bit errors, success, iterations)
def _frame_synth(g):
    ferr = (g * 2654435761 % 97 + 1) if (g * 7919) % 5 == 0 else 0
    return ferr, int(g % 3 != 0), 1 + g % 29


FRAME_CASES = [  # (batch per rank, simulation_loops, ferr_count_min)
    (16, 1000, 30),      # stops inside a later batch
    (5, 37, 2),          # one ragged batch (37 < 8 x 5)
    (3, 100, 10 ** 6),   # never stops: ragged last batch
    (1, 20, 0),          # ferr_count_min 0: stops at the first wordcount > loops / 20
    (4, 6, 1),           # fewer frames than ranks: ranks 6, 7 hold none
    (7, 500, 12),
]


def _frames_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "qam-reconciliation_amd"))
    from qamr import dist
    from qamr.sim import run_frames, shard_counters

    dist.init("gloo")
    res = []
    for batch, loops, fmin in FRAME_CASES:
        def fn(bidx, start, B, batch=batch):
            g0 = bidx * batch * world + start          # every batch before the last is full
            rows = [_frame_synth(g) for g in range(g0, g0 + B)]
            ferr = torch.tensor([r[0] for r in rows], dtype=torch.int32)
            succ = torch.tensor([r[1] for r in rows], dtype=torch.uint8)
            its = torch.tensor([r[2] for r in rows], dtype=torch.int32)
            return ferr, succ, its, shard_counters(ferr, succ, its, B)
        res.append(run_frames(fn, batch, loops, fmin))
    dist.barrier()
    dist.finalize()
    q.put((rank, res))


def _sequential(loops, fmin):
    """sims/reconciliation.pyx:127-168 over the same frames, one at a time."""
    be = fe = su = it = 0
    w = -1
    for w in range(loops):
        e, s, i = _frame_synth(w)
        if s:
            it += i
            su += 1
        if e:
            fe += 1
            be += e
        if fe >= fmin and w > loops / 20:
            break
    return [be, fe, su, it, w + 1]


def test_run_frames_world8_exact_early_stop():
    """qamr.sim.run_frames (Simulator.run_snr's shard / reduce / early-stop loop) at world size 8
    over gloo with stub frames: every rank returns the counters of the reference's sequential
    loop, cut at the same frame (per-frame rule, not batch granularity)."""
    world, port = 8, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_frames_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for c, (batch, loops, fmin) in enumerate(FRAME_CASES):
        exp = _sequential(loops, fmin)
        for r in range(world):
            assert res[r][c] == exp, (c, r, res[r][c], exp)
