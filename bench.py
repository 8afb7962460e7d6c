#!/usr/bin/env python3
"""Benchmark: decoded frames/s at N=64800, 50 BP iterations (BASELINE.json metric).

One process per GPU (torch.distributed over RCCL for N > 1).  Frames are
independent, so every rank decodes its own batch (weak scaling; no collective
on the data path); the only collective is the final all-reduce of the BER/FER
counters plus the max-over-ranks of the timed region.

A "step" = one pass of the hot path over one batch of B frames resident in HBM:
  --workload dvbs2_4pam   (default, configs[2]): batched Decoder._decode of B
                           frames, max_iterations=50, EsN0 3.0 dB (every frame runs
                           all 50 iterations: the worst case / headline).
  --workload dvbs2_16pam  (configs[3]): fused NoiseMapper soft demap (16-PAM) ->
                           decode of B frames.
Inputs (symbols, AWGN, Bob's x_hat/n_hat/word/syndrome, and for dvbs2_4pam the
LAPPRs) are generated on the GPU before the timed region.

Arithmetic (--math): "strict" (default) reproduces the reference's glibc exp/log bit
for bit, so every output of the measured step equals the reference's; "fast" / "eps"
are the opt-in approximations (1e-6 on LAPPRs at configs[2], not at configs[3]).  At
N=1 the line also carries their throughput on the same batch ("alt_math").

The JSON line carries the roofline of the dominant kernel (k_fused<7>: the degree-7
check sweep of one frame half fused with the variable sweep of the other, timed with
hipEvents on its launch stream inside the timed region) -- HBM bytes and, because
the strict check sweep is fp64-VALU bound, its VALU issue rate from the committed
PMC counts -- and a CPU baseline (the oracle restatement, OpenMP over frames, on a
bounded sample, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "qam-reconciliation_amd"))

METRIC = "decoded frames/sec @ N=64800, 50 BP iters; achieved HBM GB/s vs roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# fp64 VALU: 78.6 TFLOP/s spec = 1024 SIMDs x 2.4 GHz x 16 fp64 FMA lanes: a wave64 fp64
# instruction occupies its SIMD 4 cycles, 32-bit VALU 2 cycles (MI355X_MICROARCH.md).
SIMDS, CLOCK_HZ = 1024, 2.4e9
MATH = {"strict": 0, "fast": 1, "eps": 2}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--workload", default="dvbs2_4pam", choices=["dvbs2_4pam", "dvbs2_16pam", "reg1008_4pam"])
    p.add_argument("--batch", type=int, default=4096, help="frames per GPU")
    p.add_argument("--snr", type=float, default=None, help="EsN0 [dB] (default per workload)")
    p.add_argument("--max-iter", type=int, default=50)
    p.add_argument("--alpha", type=float, default=1.0)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline time budget (0 = skip)")
    p.add_argument("--no-roofline", action="store_true", help="skip per-kernel event timing")
    p.add_argument("--math", default="strict", choices=list(MATH), help="decoder arithmetic (strict = bit-exact)")
    p.add_argument("--no-alt", action="store_true", help="skip the alt_math throughput of the other arithmetics")
    return p.parse_args()


def setup_dist(args):
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal knobs (several ranks on a 1-GPU box): QAMR_BENCH_DEVICE pins every
    # rank to one device, QAMR_BENCH_BACKEND=gloo replaces RCCL (which refuses two
    # ranks on one GPU).  The driver's N-GPU runs use neither.
    local = int(os.environ.get("QAMR_BENCH_DEVICE", local))
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if os.environ.get("QAMR_BENCH_BACKEND", "nccl") == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def reduce_(t, op):
    """All-reduce a small GPU tensor (via the host under gloo)."""
    import torch.distributed as dist

    if dist.get_backend() == "gloo":
        h = t.cpu()
        dist.all_reduce(h, op=op)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op)


def var_sweep_bytes(V, E, B):
    """Algorithmic bytes of one variable sweep over B frames: c2v read (8 B per
    edge), lappr read and post write (8 B per variable each) -- SURVEY.md 8(d)."""
    return (8 * E + 16 * V) * B


def check_class_bytes(vid, cid, degree, B):
    """Algorithmic bytes of one launch of the degree-`degree` check kernel over B
    frames: c2v read + write (16 B per edge), the unique posteriors it gathers
    (8 B per adjacent variable), the syndrome byte per check and the active flag
    per frame (SURVEY.md 8(d) B_it, restricted to that launch)."""
    deg = np.bincount(cid)
    cls = np.flatnonzero(deg == degree)
    mask = np.isin(cid, cls)
    E_d = int(mask.sum())
    V_d = int(np.unique(vid[mask]).size)
    C_d = int(cls.size)
    return (16 * E_d + 8 * V_d + C_d) * B + B, dict(E=E_d, V=V_d, C=C_d)


def cpu_baseline(args, vid, cid, pipe, batch, lappr_host_fn, budget_s):
    """Oracle restatement on the host cores for ~budget_s seconds of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count() or 1
    cores = max(1, min(aff, int(os.environ.get("OMP_NUM_THREADS", aff))))
    code = O.OracleCode(vid, cid)
    nfr = min(batch.B, cores)
    synd = batch.synd[:, :nfr].cpu().numpy().T.copy()
    if args.workload == "dvbs2_16pam":
        nm = O.OracleNoiseMapper(4, 2.0, pipe.noise_var, np.array([0, 1] * 8, np.uint8))
        nh = batch.nhat[:, :nfr].cpu().numpy().T.copy()
        xs = batch.x[:, :nfr].cpu().numpy().T.copy()
    else:
        L = lappr_host_fn(nfr)
    frames, t0 = 0, time.perf_counter()
    rounds = 0
    while True:
        if args.workload == "dvbs2_16pam":
            L = np.stack([nm.demap_lappr_array(nh[f], xs[f], nthreads=cores) * args.alpha for f in range(nfr)])
        code.decode_batch(L, synd, args.max_iter, nthreads=cores)
        frames += nfr
        rounds += 1
        el = time.perf_counter() - t0
        if el >= budget_s or rounds >= 50:
            break
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return {"value": frames / el, "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": f"{frames} frames ({rounds} rounds x {nfr}) of the same workload in {el:.1f} s, "
                      f"oracle/qamr_oracle.c (gcc -O2 -ffp-contract=off, OpenMP over frames) on {cpu_model}"}


def copy_bandwidth(dev, nbytes=2 << 30, reps=5):
    """Measured device-to-device streaming copy bandwidth (read + write bytes / time,
    libqamr's 16-B-per-lane copy kernel): the practical HBM ceiling SURVEY.md 8(d)
    asks the roofline to be related to."""
    import ctypes
    import torch
    from qamr import _lib

    a = torch.ones(nbytes // 8, dtype=torch.float64, device=dev)
    b = torch.empty_like(a)
    st = torch.cuda.current_stream(dev)
    L = _lib.load()

    def cp():
        _lib.check(L.qr_stream_copy(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()), nbytes,
                                    ctypes.c_void_p(st.cuda_stream)))
    cp()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        cp()
    e1.record(st)
    torch.cuda.synchronize(dev)
    gbps = 2 * nbytes * reps / (e0.elapsed_time(e1) / 1e3) / 1e9
    del a, b
    torch.cuda.empty_cache()
    return gbps


def main():
    args = parse()
    import torch

    world, rank, local = setup_dist(args)
    import qamr
    from qamr import codes
    from qamr.pipeline import SofteningPipeline

    if qamr.device_count() <= 0:
        raise SystemExit("bench: no HIP device")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    if args.workload == "reg1008_4pam":
        vid, cid = codes.regular_code(1008)
        bps, snr = 2, (3.0 if args.snr is None else args.snr)
        code_name = "reg-(3,6) N=1008"
    else:
        vid, cid = codes.dvbs2_like_half()
        bps = 4 if args.workload == "dvbs2_16pam" else 2
        snr = args.snr if args.snr is not None else (13.0 if bps == 4 else 3.0)
        code_name = "DVB-S2-rate-1/2-profile IRA N=64800"
    qamr._lib.tune_set("math", MATH[args.math])
    dec = qamr.Decoder(vid, cid, device=local)
    pipe = SofteningPipeline(dec, bps=bps, snr_db=snr, batch=args.batch, alpha=args.alpha,
                             max_iterations=args.max_iter, device=local)
    gen = torch.Generator(device=dev).manual_seed(args.seed * 1000 + rank)
    batch = pipe.generate(gen)
    fused = args.workload == "dvbs2_16pam"
    lappr = pipe.demap(batch)  # input LAPPRs (re-computed inside each step when fused)
    final = torch.empty_like(lappr)
    succ = torch.empty(batch.B, dtype=torch.uint8, device=dev)
    its = torch.empty(batch.B, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)

    def step():
        if fused:
            pipe.demap(batch, out=lappr)
        pipe.decode(lappr, batch, final, succ, its)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    if not args.no_roofline:
        qamr.profile_reset()
        qamr.profile_enable(True)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    qamr.profile_enable(False)

    # BER/FER bookkeeping of the last step (and the only data-path-free collective)
    pipe.count(final, batch, succ, its)
    counters = pipe.counters.clone()
    t_max = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        import torch.distributed as dist

        reduce_(t_max, dist.ReduceOp.MAX)
        reduce_(counters, dist.ReduceOp.SUM)
    elapsed = float(t_max.item())
    total_frames = world * batch.B * args.steps
    value = total_frames / elapsed

    roof = None
    kstats = {}
    if not args.no_roofline:
        for k in ("check", "check_d7", "check_d6", "check1", "fused_d7", "var", "var_init", "parity", "status",
                  "demap"):
            ms, n = qamr.profile_query(k)
            if n:
                kstats[k] = {"avg_us": 1e3 * ms / n, "launches": n, "total_ms": ms}
        V_, E_ = dec.vnum, dec.ednum
        math_mode = int(qamr._lib.tune_get("math"))
        if "fused_d7" in kstats:
            # split schedule: one launch = check sweep of one frame half + variable sweep of the other
            half = batch.ld // 2
            fr_c = min(batch.B, half)           # real frames in the checked half (first half)
            fr_v = batch.B - fr_c if batch.B > half else 0
            # both orientations alternate; price the average launch over both halves
            bc0, _ = check_class_bytes(vid, cid, 7, fr_c)
            bc1, _ = check_class_bytes(vid, cid, 7, max(batch.B - fr_c, 0))
            bytes_launch = (bc0 + bc1) / 2 + (var_sweep_bytes(V_, E_, fr_c) + var_sweep_bytes(V_, E_, fr_v)) / 2
            ar = {0: "kStrict", 1: "kFast", 2: "kEps"}.get(math_mode, "?")
            kname = f"k_fused<7,Normal,{ar}> (check sweep of one frame half + variable sweep of the other)"
            kkey = "fused_d7"
        elif "check_d7" in kstats:
            ar = {0: "kStrict", 1: "kFast", 2: "kEps"}.get(math_mode, "?")
            if int(qamr._lib.tune_get("split")) >= 3 and batch.ld % 512 == 0:
                # two-stream schedule: each launch = the check sweep of one frame half; the
                # variable sweep of the other half runs concurrently on a second stream
                half = batch.ld // 2
                fr_c = min(batch.B, half)
                bc0, _ = check_class_bytes(vid, cid, 7, fr_c)
                bc1, _ = check_class_bytes(vid, cid, 7, max(batch.B - fr_c, 0))
                bytes_launch = (bc0 + bc1) / 2
                kname = (f"k_check<7,Normal,{ar}> (check sweep of one frame half; the variable sweep of the "
                         f"other half runs concurrently on a second stream)")
            else:
                bytes_launch, _ = check_class_bytes(vid, cid, 7, batch.B)
                kname = f"k_check<7,Normal,{ar}> (degree-7 check-node sweep)"
            kkey = "check_d7"
        else:
            kkey = None
        if kkey:
            avg_s = kstats[kkey]["avg_us"] / 1e6
            ach = bytes_launch / avg_s / 1e9
            traffic, valu = None, None
            pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
            if os.path.exists(pmc):
                try:
                    t = json.load(open(pmc))
                    if t.get("workload") == args.workload and int(t.get("batch", -1)) == batch.B \
                            and t.get("kernel_key") == kkey and t.get("math") == math_mode:
                        traffic = t.get("hbm_bytes_per_launch")
                        if t.get("valu_insts_per_launch"):
                            n_all, n64 = t["valu_insts_per_launch"], t.get("valu_f64_insts_per_launch", 0)
                            busy = (4 * n64 + 2 * (n_all - n64)) / SIMDS / CLOCK_HZ  # s of SIMD issue time
                            valu = {"wave_insts_per_launch": int(n_all), "f64_wave_insts_per_launch": int(n64),
                                    "issue_ms_at_2.4GHz": round(busy * 1e3, 3),
                                    "frac": round(busy / avg_s, 4),
                                    "note": "SIMD issue time of the launch's VALU instructions (f64 4 cyc, "
                                            "other 2 cyc per wave64) / launch time; counts from "
                                            "profiles/pmc_traffic.json (rocprofv3 --pmc)"}
                except Exception:
                    traffic = None
            copy_gbps = copy_bandwidth(dev) if rank == 0 else None
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": kname,
                    "bytes_per_launch": int(bytes_launch), "avg_launch_us": round(avg_s * 1e6, 1),
                    "launches": kstats[kkey]["launches"],
                    "measured_copy_GBps": round(copy_gbps, 1) if copy_gbps else None,
                    "frac_of_copy": round(ach / copy_gbps, 4) if copy_gbps else None, "valu": valu}
    # whole-decode algorithmic bandwidth (SURVEY.md 8(d) B_frame at the iterations actually run)
    it_mean = float(its.float().mean().item())
    V, C, E = dec.vnum, dec.cnum, dec.ednum
    B_it = 24 * E + 24 * V + C
    B_frame = 16 * V + C + it_mean * B_it

    # the other arithmetics on the same resident batch (N=1 only; not the measured value)
    alt = None
    if world == 1 and not args.no_alt:
        alt = {}
        for name, code in MATH.items():
            if name == args.math:
                continue
            qamr._lib.tune_set("math", code)
            step()
            torch.cuda.synchronize(dev)
            n_alt = 2
            ta = time.perf_counter()
            for _ in range(n_alt):
                step()
            torch.cuda.synchronize(dev)
            alt[name] = round(batch.B * n_alt / (time.perf_counter() - ta), 1)
        qamr._lib.tune_set("math", MATH[args.math])
        step()  # leave `final` as the measured arithmetic produced it
        torch.cuda.synchronize(dev)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        def lappr_host(n):
            return lappr[:, :n].cpu().numpy().T.copy()
        cpu = cpu_baseline(args, vid, cid, pipe, batch, lappr_host, args.cpu_seconds)

    if rank == 0:
        snr_, ber, fer, avg_it = SofteningPipeline.summarize(counters.cpu().numpy(), pipe.K, snr)
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (GPU-generated AWGN softening frames, torch Philox RNG)",
            "config": {"workload": args.workload, "code": code_name, "V": V, "C": C, "E": E,
                       "batch_per_gpu": batch.B, "global_batch": world * batch.B, "max_iterations": args.max_iter,
                       "snr_db": snr, "bps": bps, "fused_demap": fused, "parallelism": f"dp{world}",
                       "arithmetic": args.math + (" (glibc exp/log restated: outputs bit-identical to the reference)"
                                                  if args.math == "strict" else " (approximate, opt-in)")},
            "roofline": roof,
            "cpu_baseline": cpu,
            "alt_math": {"frames_per_s": alt, "note": "opt-in approximate arithmetics, same batch, 2 steps each; "
                                                      "not bit-exact (1e-6 LAPPR bar met at configs[2] only)"}
            if alt else None,
            "decode_alg_GBps": round(B_frame * total_frames / elapsed / 1e9, 1),
            "mean_iterations": it_mean,
            "ber_fer": {"ber": ber, "fer": fer, "avg_iters_success": avg_it, "frames_counted": int(counters[4])},
            "kernels": kstats,
        }
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
