"""Diagnostic (CPU, numpy): how often do the 64 frames of a wavefront take both
branches of glibc log inside h(t) = log(1 + exp(-t)) (near-1 branch iff t > 2.738)?
Decodes 64 softening frames of the N=64800 DVB-S2-profile code (oracle demap, numpy
flooding BP in the reference's order) and records, per box-plus call site of the
degree-7 check update, whether the wave's t+ = |a|+|b| / t- = ||a|-|b|| lanes are all
near-1, all table, or mixed.  Usage: python scripts/diag/branch_stats.py [snr_db] [bps]"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "qam-reconciliation_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from qamr import codes  # noqa: E402

snr = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
bps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
W = 64
THR = 2.738
vid, cid = codes.dvbs2_like_half()
V, C = int(vid.max()) + 1, int(cid.max()) + 1
M = 1 << bps
step = 2.0
a = (np.arange(M) - (M - 1) / 2) * step
Es = np.mean(a ** 2)
nv = Es * 10 ** (-snr / 10) / 2
nm = O.OracleNoiseMapper(bps, step, nv, np.array([i & 1 for i in range(M)], np.uint8))
rng = np.random.default_rng(1)
S = V // bps
L = np.empty((W, V))
for f in range(W):
    x = rng.integers(0, M, S)
    y = a[x] + rng.normal(0, np.sqrt(nv), S)
    xh = nm.hard_decide_index(y)
    n = nm.map_noise(y, xh)
    L[f] = nm.demap_lappr_array(n, x, nthreads=8)
# degree-7 checks as a [C7, 7] edge table (edges sorted by (cid, vid) -> ascending id)
order = np.argsort(cid, kind="stable")
deg = np.bincount(cid, minlength=C)
ptr = np.concatenate([[0], np.cumsum(deg)])
c7 = np.flatnonzero(deg == 7)
E7 = ptr[c7][:, None] + np.arange(7)[None, :]
ev = vid[order]
E = len(vid)


def h(t):
    return np.log1p(np.exp(-t))


def bp(x, y, rec):
    tp = np.abs(x) + np.abs(y)
    tm = np.abs(np.abs(x) - np.abs(y))
    rec.append((tp > THR, tm > THR))
    return np.sign(x) * np.sign(y) * np.minimum(np.abs(x), np.abs(y)) + h(np.abs(x + y)) - h(np.abs(x - y))


c2v = np.zeros((E, W))
post = L.T.copy()
stats = np.zeros((2, 3))  # [tp, tm] x [all near, all table, mixed]
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
for it in range(iters):
    m = post[ev[E7]] - c2v[E7]          # [C7, 7, W]
    rec = []
    F = [m[:, 0]]
    for i in range(1, 6):
        F.append(bp(F[-1], m[:, i], rec))
    Bn = m[:, 6]
    out = np.empty_like(m)
    out[:, 6] = F[5]
    for i in range(5, 0, -1):
        out[:, i] = bp(F[i - 1], Bn, rec)
        Bn = bp(Bn, m[:, i], rec)
    out[:, 0] = Bn
    c2v[E7] = out
    for tp, tm in rec:
        for k, z in enumerate((tp, tm)):
            allN = z.all(axis=1)
            allT = (~z).all(axis=1)
            stats[k] += [allN.sum(), allT.sum(), (~allN & ~allT).sum()]
    post = L.T.copy()
    np.add.at(post, ev, c2v)
    if it in (0, 4, 9, 19, 49):
        s = stats / stats.sum(axis=1, keepdims=True)
        print(f"it {it + 1}: t+ near/table/mixed {s[0].round(3)}  t- {s[1].round(3)}", flush=True)
