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


def init(backend: str | None = None):
    """Initialise torch.distributed when WORLD_SIZE > 1; returns (world, rank, local)."""
    world, rank, local = env_world()
    if world > 1:
        import torch
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if not dist.is_initialized():
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            if backend == "nccl":
                torch.cuda.set_device(local)
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            else:
                dist.init_process_group(backend)
    return world, rank, local


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

    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def all_reduce_max(t):
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t


def barrier():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def finalize():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def early_stop(counters, ferr_count_min: int, simulation_loops: int) -> bool:
    """reconciliation.pyx:159-161 at batch granularity: frame_errors >= ferr_count_min
    and (frames processed - 1) > simulation_loops / 20."""
    frames = int(counters[4])
    return int(counters[1]) >= ferr_count_min and (frames - 1) > simulation_loops / 20
