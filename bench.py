#!/usr/bin/env python3
"""Benchmark: decoded frames/s at N=64800, 50 BP iterations (BASELINE.json metric).

One process per GPU, torch.distributed over RCCL (qamr.dist).  Frames are
independent, so every rank decodes its own batch of B frames (weak scaling, no
collective on the data path); the only collectives are the all-reduce of the five
BER/FER counters and the max over ranks of the timed region.

Launch:
  python bench.py --gpus N ...            N > 1 without WORLD_SIZE: this process
                                          starts N fresh rank processes itself
                                          (before touching the GPU) and waits.
  torchrun --nproc-per-node N bench.py --gpus N ...
                                          WORLD_SIZE must equal --gpus.
  Rehearsal knobs (several ranks on one GPU, or on CPU): QAMR_BENCH_DEVICE=<d> binds
  every rank to GPU d, QAMR_BENCH_BACKEND=gloo replaces RCCL, QAMR_BENCH_STUB=1
  replaces the GPU work by a CPU stub (tests/test_dist.py).

A "step" = one pass of the hot path over one batch of B frames resident in HBM:
  --workload dvbs2_4pam   (default, configs[2]; configs[4] = the same at N=8):
                           batched Decoder._decode of B frames, max_iterations=50,
                           EsN0 3.0 dB (every frame runs all 50 iterations).
  --workload dvbs2_16pam  (configs[3]): fused NoiseMapper soft demap (16-PAM) ->
                           decode of B frames.
  --workload reg1008_4pam (configs[1]).
Inputs (symbols, AWGN, Bob's x_hat/n_hat/word/syndrome, and for the unfused
workloads the LAPPRs) are generated on the GPU before the timed region.

At N=1 the line also carries
  * roofline  -- the dominant kernel's algorithmic bytes / its hipEvent-timed launch
                 (on its launch stream, inside the timed region), the PMC traffic and
                 VALU issue fraction from profiles/pmc_traffic.json; "bound" names
                 the larger of the HBM and the fp64-VALU fractions;
  * secondary -- configs[1], configs[3] and the converging operating points
                 (4-PAM 4.0 dB, 16-PAM 14.5 dB), each timed separately;
  * cpu_baseline -- the oracle restatement (OpenMP over frames) on a bounded sample,
                 with its speed ratio to the Cython reference measured in the build
                 container (profiles/cpu_calibration.json).
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

from qamr import dist  # noqa: E402  (pure Python; touches no GPU)

METRIC = "decoded frames/sec @ N=64800, 50 BP iters; achieved HBM GB/s vs roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
GUIDE_COPY_GBS = 6290.0  # float4 streaming copy measured on MI355X (MI355X_MICROARCH.md: 79 % of spec)
# fp64 VALU: 78.6 TFLOP/s spec = 1024 SIMDs x 2.4 GHz x 16 fp64 FMA lanes: a wave64 fp64
# instruction occupies its SIMD 4 cycles, 32-bit VALU 2 cycles (MI355X_MICROARCH.md).
SIMDS, CLOCK_HZ = 1024, 2.4e9
# launches timed with hipEvents inside the timed region: the roofline's dominant kernel
# (k_check<7> under the default schedule, k_fused<7> under split = 2, k_resident<6> / k_iter<6> for
# configs[1]'s small code) and the fused demap
PRICED = ("check_d7", "fused_d7", "demap", "resident_d6", "iter_d6")

# (name, workload, snr, batch, steps, BASELINE.json config it measures, launches timed with hipEvents
#  in its kernel-stats pass, the one its roofline prices (or None), CPU leg)
SECONDARY = [
    ("configs1_reg1008_4pam", "reg1008_4pam", 3.0, 1024, 50, "configs[1]: reg-(3,6) N=1008, 4-PAM, B=1024",
     ("resident_d6", "iter_d6"), "resident_d6", False),
    ("configs3_dvbs2_16pam", "dvbs2_16pam", 13.0, 4096, 3,
     "configs[3]: N=64800 16-PAM, demap fused into the step, B=4096, 13 dB (all 50 iterations)",
     ("check_d7", "demap"), "demap", True),
    ("op_dvbs2_4pam_4.0dB", "dvbs2_4pam", 4.0, 4096, 3,
     "configs[2] code at its converging operating point 4.0 dB (frames stop early)",
     ("check_d7", "repack", "repack_out"), None, False),
    ("op_dvbs2_16pam_14.5dB", "dvbs2_16pam", 14.5, 4096, 3,
     "configs[3] at its converging operating point 14.5 dB (demap fused)",
     ("check_d7", "repack", "repack_out", "demap"), None, False),
]


def parse(argv=None):
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
    p.add_argument("--no-secondary", action="store_true", help="skip the secondary configs")
    p.add_argument("--graph", type=int, default=0, choices=[0, 1],
                   help="1: replay each step as a captured HIP graph (kernel timings then come from the "
                        "graph's event nodes, i.e. the last replay of the timed region)")
    return p.parse_args(argv)


# --------------------------------------------------------------------- bytes
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


def resident_bytes(w):
    """Algorithmic HBM bytes of one frame-resident decode (k_resident: messages and posteriors
    live in LDS): LAPPRs and syndrome bits in, posteriors, success flag and iteration count out
    per frame -- (16 V + C + 5) B."""
    return (16 * w.V + w.C + 5) * w.B


def demap_bytes(w):
    """Algorithmic HBM bytes of one demap launch: n_hat (8 B) and x_hat (8 B) in per symbol, bps
    LAPPRs (8 B each) out -- (16 + 8 bps) S B, S = V / bps symbols per frame."""
    return (16 + 8 * w.bps) * (w.V // w.bps) * w.B


def secondary_roofline(wl, w, ks, key, snr):
    """The roofline of a secondary config's priced kernel: its algorithmic bytes over its hipEvent
    launch time (HBM fraction) and its VALU issue fraction (PMC record of that config, at the clock
    its launches run at: in-kernel stamps of an unprofiled clock pass)."""
    if key not in ks:
        return None
    if key == "resident_d6":
        bytes_launch, kname = resident_bytes(w), "k_resident<6> (frame-resident decode of the batch: one launch)"
    elif key == "demap":
        bytes_launch, kname = demap_bytes(w), f"k_demap_wave<{w.bps}> (wave-private soft demap of the batch)"
    else:
        return None
    avg_s = ks[key]["avg_us"] / 1e6
    ach = bytes_launch / avg_s / 1e9
    t = pmc_entry(wl, w.B, key)
    valu = None
    if t and t.get("valu_insts_per_launch"):
        valu = valu_fraction(t, avg_s, kernel_clock(wl, w.B, key, snr))
    frac = ach / HBM_PEAK_GBS
    return {"bound": "valu" if valu and valu["frac"] > frac else "hbm", "achieved": round(ach, 2),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(frac, 5),
            "traffic": t.get("hbm_bytes_per_launch") if t else None, "kernel": kname,
            "bytes_per_launch": int(bytes_launch), "avg_launch_us": round(avg_s * 1e6, 1),
            "launches": ks[key]["launches"], "valu": valu}


# ----------------------------------------------------------------- rank body
def timed_region(step, sync, steps, warmup, before=None, after=None, device=None):
    """W untimed warmup steps, then EXACTLY K steps bracketed by a barrier + device
    sync on both sides; returns the max over ranks of the timed region [s].  The
    max-reduce runs on ``device`` (the rank's GPU under RCCL; qamr.dist stages a
    tensor any backend cannot reduce where it lives)."""
    import torch

    for _ in range(warmup):
        step()
    sync()
    if before:
        before()
    dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    timed_region.local = elapsed  # this rank's own timed region (the per-rank record of N > 1)
    if after:
        after()
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce_max(t)
    return float(t.item())


class StubWork:
    """CPU stand-in for the GPU step (QAMR_BENCH_STUB=1): exercises the launcher,
    the timed region and the counter reduction of the real rank body."""

    def __init__(self, args, rank, local):
        self.args, self.rank, self.local = args, rank, local
        self.B = args.batch
        self.V, self.C, self.E = 1008, 504, 3024
        self.dev = None  # host tensors (qamr.dist stages them for a GPU-only backend)

    def step(self):
        time.sleep(0.002)

    def sync(self):
        pass

    def counters(self):
        import torch

        r = self.rank
        return torch.tensor([10 * (r + 1), r + 1, self.B - r - 1, 7 * (self.B - r - 1), self.B], dtype=torch.int64)


class Work:
    """One workload on one GPU: code, softening pipeline, a batch resident in HBM."""

    def __init__(self, workload, snr, batch, max_iter, alpha, seed, rank, local):
        import torch

        import qamr
        from qamr import codes
        from qamr.pipeline import SofteningPipeline

        self.workload = workload
        if workload == "reg1008_4pam":
            self.vid, self.cid = codes.regular_code(1008)
            bps, snr = 2, (3.0 if snr is None else snr)
            self.code_name = "reg-(3,6) N=1008"
        else:
            self.vid, self.cid = codes.dvbs2_like_half()
            bps = 4 if workload == "dvbs2_16pam" else 2
            snr = snr if snr is not None else (13.0 if bps == 4 else 3.0)
            self.code_name = "DVB-S2-rate-1/2-profile IRA N=64800"
        self.bps, self.snr, self.max_iter, self.alpha = bps, snr, max_iter, alpha
        self.dev = torch.device("cuda", local)
        self.dec = qamr.Decoder(self.vid, self.cid, device=local)
        self.pipe = SofteningPipeline(self.dec, bps=bps, snr_db=snr, batch=batch, alpha=alpha,
                                      max_iterations=max_iter, device=local)
        gen = torch.Generator(device=self.dev).manual_seed(seed * 1000 + rank)
        self.batch = self.pipe.generate(gen)
        self.B = self.batch.B
        self.fused = workload == "dvbs2_16pam"
        self.lappr = self.pipe.demap(self.batch)  # input LAPPRs (re-computed inside each step when fused)
        self.final = torch.empty_like(self.lappr)
        self.succ = torch.empty(self.B, dtype=torch.uint8, device=self.dev)
        self.its = torch.empty(self.B, dtype=torch.int32, device=self.dev)
        self.V, self.C, self.E = self.dec.vnum, self.dec.cnum, self.dec.ednum
        torch.cuda.synchronize(self.dev)

    def step_eager(self):
        if self.fused:
            self.pipe.demap(self.batch, out=self.lappr)
        self.pipe.decode(self.lappr, self.batch, self.final, self.succ, self.its)

    def capture(self):
        """Capture one step (demap + the whole decode schedule, both streams) as a HIP
        graph; step() then replays it (no per-launch host overhead)."""
        import torch

        # The decode workspace is keyed by the launch stream (qamr.Decoder): warm up on the stream
        # the capture will use, so the captured step reuses that allocation instead of allocating
        # a second ~E x ld x 8 B workspace from the graph pool.
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):
            self.step_eager()
        torch.cuda.synchronize(self.dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=s):
            self.step_eager()
        torch.cuda.synchronize(self.dev)

    def step(self):
        if getattr(self, "graph", None) is not None:
            self.graph.replay()
        else:
            self.step_eager()

    def sync(self):
        import torch

        torch.cuda.synchronize(self.dev)

    def counters(self):
        self.pipe.counters.zero_()
        self.pipe.count(self.final, self.batch, self.succ, self.its)
        return self.pipe.counters.clone()

    def mean_iterations(self):
        return float(self.its.float().mean().item())

    def free(self):
        import torch

        for k in ("graph", "batch", "lappr", "final", "succ", "its", "pipe", "dec"):
            setattr(self, k, None)
        torch.cuda.empty_cache()


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


def probe_clock(w, n=16, ms=3.0):
    """Shader clock under the decode's load, unprofiled: one eager step is enqueued, then
    n one-wave clock probes (qr_clock_probe: shader cycles / 100 MHz realtime ticks over
    ~ms each) on a side stream, which the GPU schedules beside the step's kernels.
    Returns the median in GHz (None on failure)."""
    import ctypes

    import torch
    from qamr import _lib

    try:
        L = _lib.load()
        out = torch.zeros(2 * n, dtype=torch.int64, device=w.dev)
        side = torch.cuda.Stream(w.dev)
        torch.cuda.synchronize(w.dev)
        w.step_eager()
        time.sleep(0.05)  # let the step's first sweeps occupy the chip
        _lib.check(L.qr_clock_probe(ctypes.c_void_p(out.data_ptr()), n, int(ms * 1e5),
                                    ctypes.c_void_p(side.cuda_stream)))
        torch.cuda.synchronize(w.dev)
        o = out.cpu().numpy().reshape(n, 2)
        ghz = sorted(float(c) / float(r) * 0.1 for c, r in o if r > 0)
        probe_clock.spread = (round(ghz[0], 3), round(ghz[-1], 3)) if ghz else None
        return ghz[len(ghz) // 2] if ghz else None
    except Exception:
        return None


def kernel_clock(workload, batch, key="check_d7", snr=None):
    """The shader clock the chip holds DURING the launches of profile key `key` (check_d7,
    resident_d6 or demap), unprofiled: a child process runs the same workload for a few steps on
    libqamr_clock.so, the diagnostic twin of libqamr.so whose degree-7 check sweep, frame-resident
    decode and wave-private demapper stamp s_memtime / s_memrealtime around every workgroup
    (QR_EXPERIMENT_CLOCK; MI355X_MICROARCH.md 'DVFS give-back' item 6).  Returns its JSON
    {"clock_ghz", "launch_us", "workgroups", "steps"} or None."""
    import subprocess

    lib = os.path.join(ROOT, "qam-reconciliation_amd", "qamr", "libqamr_clock.so")
    if not os.path.exists(lib) or os.environ.get("QAMR_NO_CLOCK_PASS") == "1":  # (set under rocprofv3)
        return None
    cmd = [sys.executable, os.path.join(ROOT, "scripts", "diag", "clock_check.py"), "--json",
           "--workload", workload, "--batch", str(batch), "--key", key]
    if snr is not None:
        cmd += ["--snr", str(snr)]
    try:
        r = subprocess.run(cmd, env=dict(os.environ, QAMR_LIB=lib), capture_output=True, text=True, timeout=240)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        return d if d.get("clock_ghz", 0) > 0 else None
    except Exception:
        return None


def pmc_entry(workload, batch, key):
    """The PMC record (rocprofv3 --pmc passes, scripts/summarize_profile.py) of the launches of
    `key` in `workload` at `batch` frames: profiles/pmc_traffic.json (the headline's dominant
    kernel) or an entry of profiles/pmc_secondary.json (the secondary configs' priced kernels)."""
    recs = []
    for name in ("pmc_traffic.json", "pmc_secondary.json"):
        try:
            d = json.load(open(os.path.join(ROOT, "profiles", name)))
            recs += d if isinstance(d, list) else [d]
        except Exception:
            pass
    for t in recs:
        if t.get("workload") == workload and int(t.get("batch", -1)) == batch and t.get("kernel_key") == key \
                and t.get("math", 0) == 0:
            return t
    return None


def valu_fraction(t, avg_s, clk_kernel=None, clk_live=None):
    """SIMD issue time of a launch's VALU instructions (4 cycles per wave64 instruction -- fp64 or
    32-bit: SQ_ACTIVE_INST_VALU == SQ_INSTS_VALU in these kernels -- counts from the PMC record t)
    at the shader clock the launches run at, over the live launch time avg_s."""
    n_all, n64 = t["valu_insts_per_launch"], t.get("valu_f64_insts_per_launch", 0)
    clk_pmc = t.get("clock_ghz_pmc")
    clk_ghz = clk_kernel["clock_ghz"] if clk_kernel else None
    clk = clk_ghz or clk_live or clk_pmc or CLOCK_HZ / 1e9
    busy = 4 * n_all / SIMDS / (clk * 1e9)  # s of SIMD issue time
    return {"wave_insts_per_launch": int(n_all), "f64_wave_insts_per_launch": int(n64),
            "clock_ghz": round(clk, 3),
            "clock_source": "in-kernel stamps of the priced launches (libqamr_clock.so, unprofiled, same workload)"
            if clk_ghz else "live (qr_clock_probe beside an unprofiled step)" if clk_live
            else "profiled PMC pass" if clk_pmc else "spec",
            "clock_pass": clk_kernel,
            "clock_ghz_pmc": round(clk_pmc, 3) if clk_pmc else None,
            "issue_ms": round(busy * 1e3, 3),
            "frac": round(busy / avg_s, 4),
            "busy_pmc": round(t["valu_busy_pmc"], 4) if t.get("valu_busy_pmc") else None,
            "source": t.get("source"),
            "note": "SIMD issue time of the launch's VALU instructions (4 cycles per wave64 instruction, counts "
                    "from the rocprofv3 --pmc record) at the shader clock named by clock_source, over the live "
                    "launch time; clock_ghz_pmc = GRBM_GUI_ACTIVE per XCD / launch time of the profiled pass; "
                    "busy_pmc = rocprofv3 VALUBusy of the profiled launch"}


KERNEL_KEYS = ("check", "check_d7", "check_d6", "check1", "fused_d7", "var", "var_init", "parity", "status", "demap",
               "iter_d6", "resident_d6", "repack", "repack_out")


def kernel_stats(keys=KERNEL_KEYS):
    import qamr

    out = {}
    for k in keys:
        ms, n = qamr.profile_query(k)
        if n:
            out[k] = {"avg_us": 1e3 * ms / n, "launches": n, "total_ms": ms}
    return out


def roofline(args, w, kstats, dev, world=1):
    """The dominant kernel's algorithmic bytes per launch / its average launch time."""
    import qamr

    B, ld = w.B, w.batch.ld
    if "fused_d7" in kstats:
        # split = 2: one launch = check sweep of one frame half + variable sweep of the other
        half = ld // 2
        fr_c = min(B, half)
        fr_v = B - fr_c if B > half else 0
        bc0, _ = check_class_bytes(w.vid, w.cid, 7, fr_c)
        bc1, _ = check_class_bytes(w.vid, w.cid, 7, max(B - fr_c, 0))
        bytes_launch = (bc0 + bc1) / 2 + (var_sweep_bytes(w.V, w.E, fr_c) + var_sweep_bytes(w.V, w.E, fr_v)) / 2
        kname = f"k_fused<7,Normal> (check sweep of one frame half + variable sweep of the other)"
        kkey = "fused_d7"
    elif "check_d7" in kstats:
        if int(qamr._lib.tune_get("split")) >= 3 and ld % 512 == 0:
            # two-stream schedule: each launch = the check sweep of one frame half; the
            # variable sweep of the other half runs concurrently on a second stream
            half = ld // 2
            fr_c = min(B, half)
            bc0, _ = check_class_bytes(w.vid, w.cid, 7, fr_c)
            bc1, _ = check_class_bytes(w.vid, w.cid, 7, max(B - fr_c, 0))
            bytes_launch = (bc0 + bc1) / 2
            kname = ("k_check<7,Normal> (check sweep of one frame half; the variable sweep of the "
                     f"other half runs concurrently on a second stream)")
        else:
            bytes_launch, _ = check_class_bytes(w.vid, w.cid, 7, B)
            kname = "k_check<7,Normal> (degree-7 check-node sweep)"
        kkey = "check_d7"
    elif "resident_d6" in kstats:
        bytes_launch, kname = resident_bytes(w), "k_resident<6> (frame-resident decode: one launch per decode)"
        kkey = "resident_d6"
    else:
        return None
    avg_s = kstats[kkey]["avg_us"] / 1e6
    ach = bytes_launch / avg_s / 1e9
    traffic, valu = None, None
    t = pmc_entry(args.workload, B, kkey)
    if t:
        traffic = t.get("hbm_bytes_per_launch")
        if t.get("valu_insts_per_launch"):
            kc = kernel_clock(args.workload, B, kkey, args.snr) if (world == 1 and kkey in ("check_d7", "resident_d6")) \
                else None
            clk_live = None if kc else probe_clock(w)
            valu = valu_fraction(t, avg_s, kc, clk_live)
    copy_gbps = copy_bandwidth(dev)
    frac = ach / HBM_PEAK_GBS
    bound = "valu" if valu and valu["frac"] > frac else "hbm"
    return {"bound": bound, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(frac, 4), "traffic": traffic, "kernel": kname,
            "bytes_per_launch": int(bytes_launch), "avg_launch_us": round(avg_s * 1e6, 1),
            "launches": kstats[kkey]["launches"],
            "measured_copy_GBps": round(copy_gbps, 1), "frac_of_copy": round(ach / copy_gbps, 4),
            "guide_copy_GBps": GUIDE_COPY_GBS, "frac_of_guide_copy": round(ach / GUIDE_COPY_GBS, 4), "valu": valu}


def secondary(args, rank, local):
    """configs[1], configs[3] and the converging operating points, each on its own
    resident batch, timed separately from the headline (same step definition, no profiling in the
    timed region).  A second, untimed pass of as many steps records the hipEvent-timed average of
    its dominant launches (on their launch streams) so a kernel trace of the same config can be
    reconciled with its step; configs[1] and configs[3] carry a roofline of their priced kernel
    (k_resident<6>; the 16-PAM demapper), and the configs[3] line its CPU baseline (demap + decode
    on the host cores, SURVEY.md 8(d)'s demap leg)."""
    import types

    import qamr
    import torch

    out = {}
    for name, wl, snr, batch, steps, what, keys, priced, cpu_leg in SECONDARY:
        w = Work(wl, snr, batch, args.max_iter, args.alpha, args.seed, rank, local)
        el = timed_region(w.step, w.sync, steps, 1, device=w.dev)
        mean_it = round(w.mean_iterations(), 3)
        # kernel-stats pass (untimed): the same steps with events around the selected launches
        qamr.profile_reset()
        qamr.profile_select(keys)
        qamr.profile_enable(True)
        for _ in range(steps):
            w.step()
        w.sync()
        qamr.profile_enable(False)
        ks = kernel_stats(keys)
        if "repack" in ks:  # the device's repack count of the last decode: most decision points move nothing
            (r0, r1), (w0, w1) = w.dec.repack_stats(w.batch.ld, args.max_iter)
            ks["repack"].update(repacks_per_decode=r0 + r1, final_widths=[w0, w1],
                                note="k_repack_rows: every decision point (one before each variable sweep); "
                                     "only repacks_per_decode of them move columns")
        out[name] = {"frames_per_s": round(w.B * steps / el, 1), "ms_per_step": round(1e3 * el / steps, 3),
                     "steps": steps, "batch": w.B, "snr_db": w.snr, "mean_iterations": mean_it,
                     "what": what, "kernels": ks}
        if priced:
            out[name]["roofline"] = secondary_roofline(wl, w, ks, priced, snr)
        if cpu_leg and args.cpu_seconds > 0:
            out[name]["cpu_baseline"] = cpu_baseline(types.SimpleNamespace(workload=wl, max_iter=args.max_iter), w,
                                                     args.cpu_seconds)
        w.free()
        del w
        torch.cuda.empty_cache()
    return out


def cpu_calibration():
    p = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    try:
        return json.load(open(p))
    except Exception:
        return None


def cpu_baseline(args, w, budget_s):
    """Oracle restatement on the host cores for ~budget_s seconds of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count() or 1
    cores = max(1, min(aff, int(os.environ.get("OMP_NUM_THREADS", aff))))
    code = O.OracleCode(w.vid, w.cid)
    nfr = min(w.B, cores)
    synd = w.batch.synd[:, :nfr].cpu().numpy().T.copy()
    if w.fused:
        nm = O.OracleNoiseMapper(w.bps, 2.0, w.pipe.noise_var, np.array([0, 1] * (1 << w.bps >> 1), np.uint8))
        nh = w.batch.nhat[:, :nfr].cpu().numpy().T.copy()
        xs = w.batch.x[:, :nfr].cpu().numpy().T.copy()
    else:
        L = w.lappr[:, :nfr].cpu().numpy().T.copy()
    frames, t0, rounds, t_demap = 0, time.perf_counter(), 0, 0.0
    while True:
        if w.fused:
            td = time.perf_counter()
            L = np.stack([nm.demap_lappr_array(nh[f], xs[f], nthreads=cores) * w.alpha for f in range(nfr)])
            t_demap += time.perf_counter() - td
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
    value = frames / el
    out = {"value": value, "unit": "frames/s", "cores": cores, "kind": "port",
           "sample": f"{frames} frames ({rounds} rounds x {nfr}) of the same workload in {el:.1f} s, "
                     f"oracle/qamr_oracle.c (gcc -O2 -ffp-contract=off, OpenMP over frames) on {cpu_model}"}
    if w.fused:
        out["demap_s_per_frame"] = t_demap / frames
        out["decode_s_per_frame"] = (el - t_demap) / frames
        out["note"] = ("one step = NoiseMapper.demap_lappr_array (16-PAM, noisemapper.pyx:544-559) + Decoder._decode "
                       "per frame, frames in parallel over the cores; demap / decode split per frame of wall time")
    cal = cpu_calibration()
    if cal and args.workload in cal.get("workloads", {}):
        c = cal["workloads"][args.workload]
        if w.fused:
            out["demap_ratio_vs_cython"] = c.get("demap_ratio_port_over_cython")
        out["ratio_vs_cython"] = c["ratio_port_over_cython"]
        out["cython_equivalent_frames_per_s"] = value / c["ratio_port_over_cython"]
        out["calibration"] = (f"port/Cython speed ratio {c['ratio_port_over_cython']:.3f} measured on 1 core of the "
                              f"build container ({cal.get('cpu', '?')}) on the same frames: "
                              "profiles/cpu_calibration.json (scripts/cpu_calibrate.py)")
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if args.gpus < 1:
        raise SystemExit("bench: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # Start N fresh rank processes (this process has not touched the GPU) and wait.
        return dist.launch_local(args.gpus, [os.path.abspath(__file__)] + argv)
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    if env_world != args.gpus:
        raise SystemExit(f"bench: WORLD_SIZE={env_world} but --gpus {args.gpus}; they must agree")

    stub = os.environ.get("QAMR_BENCH_STUB") == "1"
    backend = os.environ.get("QAMR_BENCH_BACKEND") or ("gloo" if stub else None)
    dev_pin = os.environ.get("QAMR_BENCH_DEVICE")
    world, rank, local = dist.init(backend, None if dev_pin is None else int(dev_pin))
    local = int(dev_pin) if dev_pin is not None else local

    import torch

    if stub:
        w = StubWork(args, rank, local)
    else:
        import qamr

        if qamr.device_count() <= 0:
            raise SystemExit("bench: no HIP device")
        torch.cuda.set_device(local)
        w = Work(args.workload, args.snr, args.batch, args.max_iter, args.alpha, args.seed, rank, local)

    prof = not stub and not args.no_roofline
    graph = bool(args.graph) and not stub
    if graph:
        import qamr
        if prof:  # the captured launches carry their event pairs as graph nodes
            qamr.profile_reset()
            qamr.profile_select(PRICED)
            qamr.profile_enable(True)
        w.capture()
        if prof:
            qamr.profile_enable(False)

    def before():
        if prof and not graph:
            import qamr
            qamr.profile_reset()
            # only the kernel being priced carries events (timing every launch costs ~1.4 %)
            qamr.profile_select(PRICED)
            qamr.profile_enable(True)

    def after():
        if prof and not graph:
            import qamr
            qamr.profile_enable(False)

    elapsed = timed_region(w.step, w.sync, args.steps, args.warmup, before, after, device=w.dev)
    local_elapsed = timed_region.local
    counters = w.counters()
    dist.all_reduce_sum(counters)
    kstats = kernel_stats() if prof else {}
    # every rank's own timed region and its priced kernel's hipEvent average, gathered on rank 0
    # (N > 1: a slow rank, an imbalance or a slow barrier shows beside the max-reduced value)
    pkey = next((k for k in PRICED if k in kstats and k != "demap"), None)
    per = torch.zeros(2 * world, dtype=torch.float64, device=w.dev)
    per[rank] = 1e3 * local_elapsed / args.steps
    per[world + rank] = kstats[pkey]["avg_us"] if pkey else -1.0
    dist.all_reduce_sum(per)
    per = per.cpu().numpy()
    # the GPU each rank bound (LOCAL_RANK, or QAMR_BENCH_DEVICE in a rehearsal), gathered on rank 0
    bound = torch.zeros(world, dtype=torch.int64, device=w.dev)
    bound[rank] = 1 + (w.local if stub else torch.cuda.current_device())
    dist.all_reduce_sum(bound)
    rank_devices = [int(v) - 1 for v in bound.cpu().numpy()]
    total_frames = world * w.B * args.steps
    value = total_frames / elapsed

    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (GPU-generated AWGN softening frames, torch Philox RNG)" if not stub else "stub",
    }
    if stub:
        out["config"] = {"workload": "stub", "batch_per_gpu": w.B, "global_batch": world * w.B,
                         "parallelism": f"dp{world}", "backend": dist.backend(), "rank_devices": rank_devices}
        out["counters"] = [int(v) for v in counters]
    else:
        from qamr.pipeline import SofteningPipeline

        roof = roofline(args, w, kstats, w.dev, world) if (prof and rank == 0) else None
        it_mean = w.mean_iterations()
        # whole-decode algorithmic bandwidth (SURVEY.md 8(d) B_frame at the iterations actually run)
        B_frame = 16 * w.V + w.C + it_mean * (24 * w.E + 24 * w.V + w.C)
        cpu = None
        if rank == 0 and world == 1 and args.cpu_seconds > 0:
            cpu = cpu_baseline(args, w, args.cpu_seconds)
        snr_, ber, fer, avg_it = SofteningPipeline.summarize(counters.cpu().numpy(), w.pipe.K, w.snr)
        out["config"] = {"workload": args.workload, "code": w.code_name, "V": w.V, "C": w.C, "E": w.E,
                         "batch_per_gpu": w.B, "global_batch": world * w.B, "max_iterations": args.max_iter,
                         "snr_db": w.snr, "bps": w.bps, "fused_demap": w.fused, "parallelism": f"dp{world}",
                         "hip_graph": graph,
                         "backend": dist.backend() or "none", "rank_devices": rank_devices,
                         "arithmetic": "strict (glibc exp/log restated: outputs bit-identical to the reference)"}
        if dev_pin is not None:
            out["config"]["rehearsal"] = f"all {world} ranks on GPU {dev_pin}"
        out.update({
            "roofline": roof,
            "cpu_baseline": cpu,
            "decode_alg_GBps": round(B_frame * total_frames / elapsed / 1e9, 1),
            "mean_iterations": it_mean,
            "ber_fer": {"ber": ber, "fer": fer, "avg_iters_success": avg_it, "frames_counted": int(counters[4])},
            "kernels": kstats,
        })
        if world == 1 and not args.no_secondary:
            w.free()
            out["secondary"] = secondary(args, rank, local)
    if world > 1:
        out["per_rank"] = {"ms_per_step": [round(float(v), 3) for v in per[:world]],
                           "priced_kernel": pkey,
                           "avg_launch_us": [round(float(v), 1) if v >= 0 else None for v in per[world:]],
                           "note": "each rank's own timed region (the line's ms_per_step is their max) and the "
                                   "hipEvent average of its priced launches"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
