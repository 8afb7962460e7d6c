"""Multi-GPU plumbing: one process per GPU, frames sharded, one tiny collective.

Frames are independent: rank r decodes its own frames with no
data-path communication.  The only collectives are
  * the all-reduce (SUM) of the five int64 BER/FER counters
    {bit_errors, frame_errors, successes, iteration_sum_of_successes, frames}
    (the bookkeeping of sims/reconciliation.pyx:149-157), once per batch so
    every rank takes the same ferr_count_min early-stop decision
    (reconciliation.pyx:159-161); 40 bytes, latency-bound over xGMI;
  * the max over ranks of a timed region (benchmarking).
Works with backend "nccl" (= RCCL on ROCm, GPU tensors) and "gloo" (CPU
tensors; used by the CPU tests).
"""
from __future__ import annotations

import os


def env_world():
    """(world, rank, local_rank) from the torchrun environment (1, 0, 0 if absent)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str | None = None, device: int | None = None):
    """Initialise torch.distributed when WORLD_SIZE > 1; returns (world, rank, local).

    ``backend``: "nccl" (= RCCL on ROCm; one GPU per rank), "gloo" (CPU tensors;
    the CPU tests and the several-ranks-on-one-GPU rehearsal) or None (RCCL when a
    GPU is visible).  ``device``: the GPU this rank binds (default: LOCAL_RANK).
    The world size returned is the one the process group reports.
    ``QAMR_DIST_FORCE_PG=1`` creates the process group at world size 1 too, so a
    single-GPU run pushes every collective through RCCL (tests/test_gpu_dist.py)."""
    world, rank, local = env_world()
    if world > 1 or os.environ.get("QAMR_DIST_FORCE_PG") == "1":
        import torch
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dev = local if device is None else int(device)
        if not dist.is_initialized():
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            if backend == "nccl":
                torch.cuda.set_device(dev)
                dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
            else:
                dist.init_process_group(backend)
        world, rank = dist.get_world_size(), dist.get_rank()
    return world, rank, local


def backend():
    """The initialised backend name, or None for a single process."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        return dist.get_backend()
    return None


def _capability(backend_name: str):
    """Device types the backend's collectives accept.  A multi-device backend string
    ("cpu:gloo,cuda:nccl") accepts the union of its parts."""
    import torch.distributed as dist

    caps = set()
    for part in str(backend_name).split(","):
        name = part.split(":")[-1].strip().lower()
        caps.update(dist.Backend.backend_capability.get(name, []))
    return caps


def staging_device_type(backend_name: str, device_type: str):
    """Device type a tensor living on ``device_type`` must be staged to before a
    collective of ``backend_name``, or None when it can be reduced where it lives.
    RCCL ("nccl") reduces GPU tensors only: a host tensor goes through the rank's GPU.
    gloo is always given host tensors (its GPU path is not built for ROCm)."""
    name = str(backend_name).lower()
    if name == "gloo":
        return None if device_type == "cpu" else "cpu"
    caps = _capability(name)
    if device_type in caps:
        return None
    return "cuda" if "cuda" in caps else "cpu"


def _stage(t, device_type: str):
    """Copy ``t`` to ``device_type`` (the rank's current GPU for "cuda")."""
    import torch

    if device_type == "cuda":
        return t.to(torch.device("cuda", torch.cuda.current_device()))
    return t.to(device_type)


def _all_reduce(t, op):
    """All-reduce in place.  The tensor is staged to a device the backend reduces on
    (RCCL: the rank's GPU; gloo: the host) and copied back, so callers may hand in
    host or GPU tensors under either backend."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return t
    to = staging_device_type(dist.get_backend(), t.device.type)
    if to is None:
        dist.all_reduce(t, op=op)
    else:
        s = _stage(t, to)
        dist.all_reduce(s, op=op)
        t.copy_(s)
    return t


def shard(total: int, world: int, rank: int):
    """Contiguous frame range [start, start + count) of `total` frames for `rank`
    (frame-range sharding: GPU g takes frames [g*T/G, (g+1)*T/G))."""
    start = (total * rank) // world
    end = (total * (rank + 1)) // world
    return start, end - start


def rank_seed(seed: int, rank: int, batch_index: int) -> int:
    """Independent, reproducible RNG stream per (seed, rank, batch)."""
    return (seed * 1_000_003 + rank * 10_007 + batch_index) & 0x7FFFFFFFFFFFFFFF


def all_reduce_sum(t):
    import torch.distributed as dist

    return _all_reduce(t, dist.ReduceOp.SUM)


def all_reduce_max(t):
    import torch.distributed as dist

    return _all_reduce(t, dist.ReduceOp.MAX)


def all_reduce_min(t):
    import torch.distributed as dist

    return _all_reduce(t, dist.ReduceOp.MIN)


def barrier():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def finalize():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def early_stop(counters, ferr_count_min: int, simulation_loops: int) -> bool:
    """reconciliation.pyx:159-161 after the last frame counted: frame_errors >= ferr_count_min
    and wordcount = (frames processed - 1) > simulation_loops / 20 (qamr.sim then locates the
    first frame at which it held)."""
    frames = int(counters[4])
    return int(counters[1]) >= ferr_count_min and (frames - 1) > simulation_loops / 20


def launch_local(nprocs: int, argv, env_extra=None, poll_s: float = 0.2) -> int:
    """Start ``nprocs`` ranks of ``python argv...`` on this node (torchrun's env contract:
    RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT)
    and wait for them.  The caller must not have touched the GPU: the children are
    fresh processes (no fork/exec of a GPU-initialised process).  If a rank fails the
    others are terminated (they would otherwise wait in a collective forever).
    Returns the first non-zero exit code, else 0."""
    import socket
    import subprocess
    import sys
    import time

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(nprocs):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if env_extra:
            env.update(env_extra)
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=env))
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc
