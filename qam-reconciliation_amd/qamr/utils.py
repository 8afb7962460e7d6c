"""utils.pyx equivalents.  ``count_errors_from_lappr`` defines the BER counter
semantics (lappr >= 0 decides bit 0, utils.pyx:27-40) that the batched device
counter (qr_count_errors_device) and the RCCL reduction reproduce."""
from __future__ import annotations

import numpy as np


def dist_cut(x: float) -> float:
    """utils.pyx:18-23"""
    if x < 0:
        return 0
    if x > 1:
        return 1
    return x


def count_errors_from_lappr(lappr, word) -> int:
    """utils.pyx:27-40"""
    l = np.asarray(lappr, np.float64)
    w = np.asarray(word)
    if l.size != w.size:
        raise ValueError("Sizes do not match")
    w = w.astype(np.int64)
    return int(np.where(l >= 0, w, 1 - w).sum())
