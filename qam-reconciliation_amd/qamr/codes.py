"""Parity-check matrices as edge lists (vid, cid): the reference's code format.

* ``load_edge_csv`` reads the reference's edge CSV convention: columns
  ``eid,cid,vid`` where the FIRST data row holds the counts (E, C, V) and is
  skipped (test/hamming_7-4.csv:2, test_decoder.py:227-228,
  sim_reconciliation.py:50-51,60: ``edge_df.vid[1:]``).
* ``regular_code`` / ``dvbs2_like_half`` are the synthetic codes of the
  benchmark configs; the DVB-S2 one is an IRA code with the
  DVB-S2 normal-frame rate-1/2 degree profile (the ETSI table is not part of
  the reference), E = 226 799, sha256(vid||cid as <i8) prefix 22c92f7d6f589b7d.
"""
from __future__ import annotations

import hashlib

import numpy as np


def load_edge_csv(path: str, counts_first_row: bool = True):
    """Return (vid, cid) int64 arrays from an edge CSV (header ``eid,cid,vid``)."""
    rows = []
    with open(path) as fh:
        header = [h.strip() for h in fh.readline().split(",")]
        iv, ic = header.index("vid"), header.index("cid")
        for line in fh:
            line = line.strip()
            if not line:
                continue
            parts = [p.strip() for p in line.split(",")]
            rows.append((int(parts[iv]), int(parts[ic])))
    arr = np.asarray(rows, dtype=np.int64).reshape(-1, 2)
    if counts_first_row:
        arr = arr[1:]
    return np.ascontiguousarray(arr[:, 0]), np.ascontiguousarray(arr[:, 1])


def save_edge_csv(path: str, vid, cid):
    """Write the reference's convention (counts row first)."""
    vid = np.asarray(vid, np.int64)
    cid = np.asarray(cid, np.int64)
    with open(path, "w") as fh:
        fh.write("eid,cid,vid\n")
        fh.write(f"{vid.size},{int(cid.max()) + 1},{int(vid.max()) + 1}\n")
        for e in range(vid.size):
            fh.write(f"{e},{int(cid[e])},{int(vid[e])}\n")


def regular_code(N: int, dv: int = 3, dc: int = 6, seed: int = 0):
    """Regular (dv, dc) code: variable sockets ``repeat(arange(N), dv)`` shuffled
    by ``default_rng(seed)``; checks ``repeat(arange(M), dc)`` (edges check-major).
    Parallel edges are kept, exactly as the reference would treat them."""
    rng = np.random.default_rng(seed)
    M = N * dv // dc
    s = np.repeat(np.arange(N), dv)
    rng.shuffle(s)
    return s.astype(np.int64), np.repeat(np.arange(M), dc).astype(np.int64)


def dvbs2_like_half(seed: int = 0, N: int = 64800):
    """IRA code with the DVB-S2 rate-1/2 normal-frame degree profile.

    Info nodes 0..12959 have degree 8, 12960..K-1 degree 3; their sockets are
    permuted by ``default_rng(seed).permutation`` and dealt 5 per check; the
    parity nodes form a staircase (K+j joins checks j and j+1; the last parity
    node has degree 1).  Edges sorted by (cid, vid).  Check degrees: 7 (x C-1)
    and 6 (x 1)."""
    rng = np.random.default_rng(seed)
    K = N // 2
    M = N - K
    dc = 7
    info_deg = np.concatenate([np.full(12960, 8), np.full(K - 12960, 3)])
    sockets = np.repeat(np.arange(K), info_deg)
    perm = rng.permutation(sockets.size)
    info_cid = np.repeat(np.arange(M), dc - 2)
    assert info_cid.size == sockets.size
    pj = np.arange(M)
    vid = np.concatenate([sockets[perm], K + pj, K + pj[:-1]]).astype(np.int64)
    cid = np.concatenate([info_cid, pj, pj[1:]]).astype(np.int64)
    o = np.lexsort((vid, cid))
    return np.ascontiguousarray(vid[o]), np.ascontiguousarray(cid[o])


def code_digest(vid, cid) -> str:
    h = hashlib.sha256()
    h.update(np.asarray(vid, "<i8").tobytes())
    h.update(np.asarray(cid, "<i8").tobytes())
    return h.hexdigest()
