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
