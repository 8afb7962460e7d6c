"""Batched, GPU-resident softening reconciliation (Monte-Carlo frame pipeline).

The reference runs one frame at a time on the CPU (sims/reconciliation.pyx:93-168,
``simulate_softening_snr_dB``).  Here a whole batch of B independent frames
lives in HBM in the frame-innermost layout ([node][ld], ld % 64 == 0) and each
stage is one HIP kernel of libqamr:

  Alice  x  ~ p (torch RNG)               reconciliation.pyx:129
  channel y = a[x] + sigma * n            :132
  Bob    x_hat, n_hat, word   (k_bob)     :135-138  noisemapper.pyx:349-388
  Bob    synd = H word        (k_syndrome) :139     matrix.pyx:55-60
  Alice  lappr = alpha * demap(n_hat, x)  :143-145  (k_demap, decoder layout)
  Alice  decode (k_check / k_status / k_var) :147
  count  BER/FER/iterations   (k_count_*)  :149-157

The RNG stream is torch's, not numpy's: parity is established on the fixtures
and the oracle, not on random streams.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from .alphabet import PAMAlphabet
from .decoder import Decoder
from .noisemapper import NoiseMapper


def noise_variance(pa: PAMAlphabet, snr_db: float) -> float:
    """N0 = Es * 10^(-snr/10) / 2 (reconciliation.pyx:109-110)."""
    return pa.variance * (10 ** (-snr_db / 10)) / 2


def alternating_config(order: int) -> np.ndarray:
    """Default sign configuration of sim_reconciliation.py:84-86."""
    cfg = np.zeros(order, np.uint8)
    cfg[1::2] = 1
    return cfg


def leading_dim(B: int) -> int:
    return ((B + 255) // 256) * 256 if B >= 256 else ((B + 63) // 64) * 64


@dataclass
class Batch:
    B: int
    ld: int
    x: object      # int64 [S, ld]   transmitted symbol index
    nhat: object   # float64 [S, ld] Bob's transformed noise
    word: object   # uint8 [V, ld]   Bob's hard bits
    synd: object   # uint8 [C, ld]   syndrome of word


class SofteningPipeline:
    """One GPU's share of ``simulate_softening_snr_dB`` for a batch of frames."""

    def __init__(self, decoder: Decoder, bps: int, snr_db: float, batch: int, alpha: float = 1.0,
                 max_iterations: int = 50, sign_config=None, step: float = 2.0, device: int = 0):
        import torch

        self.dec = decoder
        self.pa = PAMAlphabet(bps, step)
        self.snr_db = float(snr_db)
        self.noise_var = noise_variance(self.pa, snr_db)
        cfg = alternating_config(self.pa.order) if sign_config is None else np.asarray(sign_config, np.uint8)
        self.nm = NoiseMapper(self.pa, self.noise_var, cfg, device=device)
        self.alpha = float(alpha)
        self.max_iterations = int(max_iterations)
        self.V, self.C = decoder.vnum, decoder.cnum
        if self.V % bps:
            raise ValueError(f"V={self.V} is not a multiple of bit_per_symbol={bps}")
        self.S = self.V // bps
        self.K = self.V - self.C  # info bits = first K variable nodes (reconciliation.pyx:120-121)
        self.B = int(batch)
        self.ld = leading_dim(self.B)
        self.device = torch.device("cuda", device)
        self._a = torch.tensor(self.pa.constellation, dtype=torch.float64, device=self.device)
        self._p = torch.tensor(self.pa.probabilities, dtype=torch.float64, device=self.device)
        self._uniform = bool(np.all(self.pa.probabilities == self.pa.probabilities[0]))
        self.counters = torch.zeros(5, dtype=torch.int64, device=self.device)
        self._ferr = torch.empty(self.B, dtype=torch.int32, device=self.device)

    # -------------------------------------------------------------- inputs
    def generate(self, gen=None) -> Batch:
        import torch

        S, ld, dev = self.S, self.ld, self.device
        if self._uniform:
            x = torch.randint(0, self.pa.order, (S, ld), generator=gen, device=dev, dtype=torch.int64)
        else:
            x = torch.multinomial(self._p, S * ld, replacement=True, generator=gen).view(S, ld)
        y = self._a[x] + self.nm.noise_sigma * torch.randn((S, ld), generator=gen, device=dev, dtype=torch.float64)
        _, nhat, word = self.nm.bob_map_device(y, self.B)
        synd = self.dec_syndrome(word)
        return Batch(self.B, ld, x, nhat, word, synd)

    def dec_syndrome(self, word_fi):
        import torch

        out = torch.empty((self.C, self.ld), dtype=torch.uint8, device=self.device)
        st = torch.cuda.current_stream(self.device)
        _lib.check(_lib.load().qr_syndrome_device(self.dec.handle, self.B, self.ld, C.c_void_p(word_fi.data_ptr()),
                                                  C.c_void_p(out.data_ptr()), C.c_void_p(st.cuda_stream)),
                   "syndrome")
        return out

    # ---------------------------------------------------------- hot path
    def demap(self, batch: Batch, out=None):
        return self.nm.demap_device(batch.nhat, batch.x, batch.B, self.alpha, out=out)

    def decode(self, lappr_fi, batch: Batch, final=None, success=None, iters=None):
        return self.dec.decode_device(lappr_fi, batch.synd, batch.B, self.max_iterations, final, success, iters)

    def count(self, final_fi, batch: Batch, success, iters):
        """Accumulate {bit_errors, frame_errors, successes, iter_sum, frames}."""
        import torch

        st = torch.cuda.current_stream(self.device)
        _lib.check(_lib.load().qr_count_errors_device(
            batch.B, batch.ld, self.K, C.c_void_p(final_fi.data_ptr()), C.c_void_p(batch.word.data_ptr()),
            C.c_void_p(success.data_ptr()), C.c_void_p(iters.data_ptr()), C.c_void_p(self._ferr.data_ptr()),
            C.c_void_p(self.counters.data_ptr()), C.c_void_p(st.cuda_stream)), "count")
        return self.counters

    def run_batch(self, gen=None):
        b = self.generate(gen)
        l = self.demap(b)
        fin, succ, its = self.decode(l, b)
        self.count(fin, b, succ, its)
        return b, l, fin, succ, its

    @staticmethod
    def summarize(counters, K: int, snr_db: float):
        """(snr, ber, fer, avg_iters_of_successes) as reconciliation.pyx:163-168."""
        be, fe, su, it, fr = [int(v) for v in counters]
        ber = be / (fr * K) if fr else 0.0
        fer = fe / fr if fr else 0.0
        return snr_db, ber, fer, (0 if su == 0 else it / su)
