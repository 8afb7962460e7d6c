"""PAM alphabet and BICM Gray labelling (host-side tables).

Mirrors qamreconciliation.alphabet.PAMAlphabet (alphabet.pyx:34-107) and
qamreconciliation.bicm.generate_table_s_to_b (bicm.pyx:26-41).  These are
O(M) host tables that feed the device demapper; the per-symbol work lives in
the HIP kernels (demap.hip).
"""
from __future__ import annotations

import numpy as np


def generate_table_s_to_b(log_order: int) -> np.ndarray:
    """Reflected-Gray symbol->bits table, column k = bit k (LSB first):
    ``s_to_b[i, k] = ((i ^ (i >> 1)) >> k) & 1`` -- the closed form of the
    recursive construction at bicm.pyx:26-41."""
    if log_order <= 0:
        raise ValueError(f"log_order ({log_order}) must be a positive integer")
    i = np.arange(1 << log_order)
    g = i ^ (i >> 1)
    return ((g[:, None] >> np.arange(log_order)[None, :]) & 1).astype(np.ubyte)


def generate_error_number_table(s_to_b) -> np.ndarray:
    """Hamming distance between the labels of symbols i and j (bicm.pyx:46-66,
    with the inner loop over the label length)."""
    s = np.asarray(s_to_b, dtype=np.ubyte)
    return (s[:, None, :] ^ s[None, :, :]).sum(axis=2).astype(np.int64)


class Alphabet:
    pass


class PAMAlphabet(Alphabet):
    """``PAMAlphabet(bit_per_symbol, step, probabilities=None)`` (alphabet.pyx:35-76)."""

    def __init__(self, bit_per_symbol: int, step: float, probabilities=None):
        bit_per_symbol = int(bit_per_symbol)
        if bit_per_symbol == 0:
            raise ValueError(f"Bit per symbol must be at least 1, got {bit_per_symbol}")
        if not (0 < bit_per_symbol < 256):
            raise OverflowError("value too large to convert to unsigned char")
        self.bit_per_symbol = bit_per_symbol
        self.order = 1 << bit_per_symbol
        self.step = float(step)
        if probabilities is None:
            self.probabilities = np.ones(self.order, dtype=np.double) / self.order
        else:
            p = np.asarray(probabilities, dtype=np.double)
            if p.size != self.order:
                raise ValueError("Probability vector does not match constellation size")
            tmp = 0.0
            for v in p:
                tmp += float(v)
            if abs(tmp - 1) > 1e-9:
                raise ValueError("Probabilities do not sum to 1")
            self.probabilities = p
        # alphabet.pyx:62
        self.constellation = (np.arange(self.order) - (self.order - 1) / 2) * self.step
        # alphabet.pyx:66-67
        var = 0.0
        for i in range(self.order):
            a = float(self.constellation[i])
            var += float(self.probabilities[i]) * (a * a)
        self.variance = var
        # alphabet.pyx:64, 69-73
        th = np.empty(self.order + 1, dtype=np.double)
        for i in range(1, self.order):
            th[i] = self.constellation[i] - self.step / 2
        th[0] = self.constellation[0] * 100
        th[-1] = self.constellation[-1] * 100
        self.thresholds = th
        self.s_to_b = generate_table_s_to_b(self.bit_per_symbol)

    def random_symbols(self, N: int, rng=None) -> np.ndarray:
        """alphabet.pyx:79-83 (numpy legacy global RNG unless ``rng`` is given)."""
        if rng is None:
            return np.array(np.random.choice(self.order, size=N, p=self.probabilities), dtype=np.int64)
        return np.asarray(rng.choice(self.order, size=N, p=self.probabilities), dtype=np.int64)

    def index_to_value(self, index) -> np.ndarray:
        """alphabet.pyx:86-95"""
        return self.constellation[np.asarray(index, dtype=np.int64)]

    def demap_symbols_to_bits(self, symbol_index) -> np.ndarray:
        """alphabet.pyx:98-107: bits[s*bps + k] = s_to_b[x[s], k]."""
        idx = np.asarray(symbol_index, dtype=np.int64)
        return np.ascontiguousarray(self.s_to_b[idx].reshape(-1))
