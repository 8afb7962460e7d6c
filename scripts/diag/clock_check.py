"""Diagnostic (MI355X): the shader clock the chip holds DURING the degree-7 check sweep,
unprofiled, from the in-kernel stamps of a QR_EXPERIMENT_CLOCK build (decoder.hip: every
workgroup adds its s_memtime / s_memrealtime spans to g_clk), beside the launch time from
hipEvents, for the default two-stream schedule and any QAMR_TUNE-style variants.

  make -C qam-reconciliation_amd/csrc   (builds qamr/libqamr_clock.so beside libqamr.so)
  QAMR_LIB=qam-reconciliation_amd/qamr/libqamr_clock.so python scripts/diag/clock_check.py "" "split=1"

Per variant: step ms, check_d7 launch us (events), effective clock GHz, and the VALU issue
fraction at that clock (1.585e9 wave-instructions x 4 cycles / 1024 SIMDs per 2048-frame
launch, scaled by the launch's frames).
  --json [--workload W --batch B --snr S --key K]: one JSON line {"clock_ghz", "launch_us",
"workgroups"} of the launches of profile key K (check_d7, resident_d6 or demap) for the default
tuning (QAMR_TUNE applies), read by bench.py's rooflines."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "qam-reconciliation_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from qamr import _lib  # noqa: E402

VALU_PER_FRAME = 1.585e9 / 2048  # wave-instructions of one check_d7 launch per frame (PMC, r03)


def run(variant, w, L, steps=4, quiet=False, key="check_d7"):
    for item in filter(None, variant.split(",")):
        k, v = item.split("=")
        _lib.tune_set(k.strip(), int(v))
    # the stamped kernels: degree-7 check sweep and frame-resident decode (qr_debug_clock), the
    # wave-private demapper (qr_debug_clock_demap)
    read = L.qr_debug_clock_demap if key == "demap" else L.qr_debug_clock
    w.step_eager()
    w.sync()
    out = (C.c_int64 * 3)()
    read(out)  # clear
    _lib.profile_enable(True)
    _lib.profile_select(key)
    _lib.profile_reset()
    t0 = time.perf_counter()
    for _ in range(steps):
        w.step_eager()
    w.sync()
    dt = (time.perf_counter() - t0) / steps
    ms, n = _lib.profile_query(key)
    read(out)
    _lib.profile_enable(False)
    cyc, ticks, blocks = out[0], out[1], out[2]
    ghz = cyc / ticks * 0.1 if ticks else float("nan")
    launch_us = ms / max(n, 1) * 1e3
    frames = w.B if _lib.tune_get("split") < 2 else w.B // 2
    issue_us = VALU_PER_FRAME * frames * 4 / 1024 / (ghz * 1e3)
    if quiet:
        return {"clock_ghz": round(ghz, 4), "launch_us": round(launch_us, 1), "workgroups": blocks, "steps": steps,
                "kernel_key": key}
    print(f"variant '{variant or 'default'}': step {dt * 1e3:.1f} ms, {w.B / dt:.0f} frames/s, check_d7 "
          f"{launch_us:.0f} us x {n}, clock {ghz:.3f} GHz ({blocks} workgroups), VALU issue {issue_us:.0f} us "
          f"= {issue_us / launch_us:.3f} of the launch", flush=True)


def wg_times(w, L, steps=2):
    """Occupancy of the last stamped check_d7 launch over time: how many of its workgroups are
    resident, and how long the drain at its end lasts."""
    import numpy as np

    for _ in range(steps):
        w.step_eager()
    w.sync()
    L.qr_debug_wg_times.argtypes = [C.c_void_p, C.c_int32]
    nb = 1 << 16
    buf = (C.c_int64 * (2 * nb))()
    L.qr_debug_wg_times(buf, nb)
    t = np.frombuffer(buf, dtype=np.int64).reshape(nb, 2)
    t = t[(t[:, 0] > 0) & (t[:, 1] >= t[:, 0])]
    t0 = t[:, 0].min()
    s, e = (t[:, 0] - t0) * 10e-3, (t[:, 1] - t0) * 10e-3  # us (100 MHz ticks)
    span = e.max()
    grid = np.linspace(0, span, 2001)
    active = np.array([np.count_nonzero((s <= x) & (e > x)) for x in grid])
    peak = np.percentile(active, 90)
    busy = (e - s).sum()
    below = grid[active < 0.9 * peak]
    drain = span - below[below > span / 2].min() if np.any(below > span / 2) else 0.0
    print(f"workgroups {len(t)}, span {span:.0f} us, workgroup duration median {np.median(e - s):.0f} us "
          f"(p10 {np.percentile(e - s, 10):.0f}, p90 {np.percentile(e - s, 90):.0f}), resident peak {peak:.0f}, "
          f"mean {busy / span:.0f} = {busy / span / peak:.3f} of peak; drain (below 90 % of peak) {drain:.0f} us; "
          f"first start spread {np.percentile(s, 5):.0f} us", flush=True)
    for q in (0.5, 0.8, 0.9, 0.95, 0.98):
        x = grid[int(q * 2000)]
        print(f"  t = {x:7.0f} us: {np.count_nonzero((s <= x) & (e > x))} resident", flush=True)


def main():
    L = _lib.load()
    L.qr_debug_clock.argtypes = [C.c_void_p]
    L.qr_debug_clock_demap.argtypes = [C.c_void_p]
    argv = sys.argv[1:]
    as_json = "--json" in argv
    opts = {"--workload": "dvbs2_4pam", "--batch": "4096", "--key": "check_d7", "--snr": ""}
    for k in opts:
        if k in argv:
            i = argv.index(k)
            opts[k] = argv[i + 1]
            del argv[i:i + 2]
    argv = [a for a in argv if a not in ("--json",)]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    w = bench.Work(opts["--workload"], float(opts["--snr"]) if opts["--snr"] else None, int(opts["--batch"]), 50, 1.0,
                   0, 0, 0)
    w.step_eager()
    w.sync()
    if as_json:
        import json
        print(json.dumps(run("", w, L, quiet=True, key=opts["--key"])), flush=True)
        return
    if "--wgtimes" in argv:
        wg_times(w, L)
        return
    defaults = {k: _lib.tune_get(k) for k in ("split", "check_per", "check_ft", "var_pace", "var_per", "var_ft", "nt", "compact",
                                             "side", "lds_pad_kb", "check_tail")}
    for variant in [a for a in argv if a != "--wgtimes"] or [""]:
        for k, v in defaults.items():
            _lib.tune_set(k, v)
        run(variant, w, L)


if __name__ == "__main__":
    main()
