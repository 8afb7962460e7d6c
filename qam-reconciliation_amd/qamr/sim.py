"""Batched, GPU-resident Monte-Carlo reconciliation simulations.

GPU counterpart of sims/reconciliation.pyx:
  * ``simulate_softening_snr_dB``   (reconciliation.pyx:93-168)  -- the hot path
  * ``simulate_direct_snr_dB``      (reconciliation.pyx:173-249)
  * ``simulate_hard_reverse_snr_dB`` (reconciliation.pyx:253-329)
The reference decodes one frame at a time; here every batch of B independent
frames is generated, mapped, decoded and counted by libqamr kernels in HBM
(frame-innermost layout), and with several GPUs each rank takes its share of
every batch (frame sharding) and the five counters are all-reduced once per
batch (qamr.dist), so all ranks take the same ``ferr_count_min`` early-stop
decision.  The early stop is evaluated at batch granularity
(reconciliation.pyx:159-161 evaluates it per frame).  Returned tuples have the
reference's shape: (snr_dB, ber, fer, average iterations of successful frames).
RNG streams are torch's (per seed, rank and batch), not numpy's.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib, dist
from .alphabet import PAMAlphabet
from .decoder import Decoder
from .noisemapper import NoiseMapper
from .pipeline import alternating_config, leading_dim

MODES = ("softening", "direct", "hard")


class Simulator:
    def __init__(self, decoder: Decoder, bps: int, mode: str = "softening", max_iterations: int = 50,
                 alpha: float = 1.0, batch: int = 4096, configuration_base: bool = False, step: float = 2.0,
                 device: int = 0):
        import torch

        if mode not in MODES:
            raise ValueError(f"mode must be one of {MODES}")
        self.dec = decoder
        self.mode = mode
        self.pa = PAMAlphabet(bps, step)
        self.max_iterations = int(max_iterations)
        self.alpha = float(alpha)
        self.batch = int(batch)
        self.V, self.C = decoder.vnum, decoder.cnum
        if self.V % bps:
            raise ValueError(f"V={self.V} is not a multiple of bit_per_symbol={bps}")
        self.S = self.V // bps
        self.K = self.V - self.C  # reconciliation.pyx:120-121
        self.cfg = np.zeros(self.pa.order, np.uint8) if configuration_base else alternating_config(self.pa.order)
        self.device = torch.device("cuda", device)
        self._dev_index = device
        self._a = torch.tensor(self.pa.constellation, dtype=torch.float64, device=self.device)
        self._p = torch.tensor(self.pa.probabilities, dtype=torch.float64, device=self.device)
        self._uniform = bool(np.all(self.pa.probabilities == self.pa.probabilities[0]))

    # ---------------------------------------------------------------- pieces
    def _stream(self):
        import torch

        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _symbols(self, S, ld, gen):
        import torch

        if self._uniform:
            return torch.randint(0, self.pa.order, (S, ld), generator=gen, device=self.device, dtype=torch.int64)
        return torch.multinomial(self._p, S * ld, replacement=True, generator=gen).view(S, ld)

    def _bits(self, x, B, ld):
        import torch

        w = torch.empty((self.S * self.pa.bit_per_symbol, ld), dtype=torch.uint8, device=self.device)
        _lib.check(_lib.load().qr_symbols_to_bits_device(self.pa.bit_per_symbol, B, ld, self.S,
                                                         C.c_void_p(x.data_ptr()), C.c_void_p(w.data_ptr()),
                                                         self._stream()), "symbols_to_bits")
        return w

    def _synd(self, word, B, ld):
        import torch

        s = torch.empty((self.C, ld), dtype=torch.uint8, device=self.device)
        _lib.check(_lib.load().qr_syndrome_device(self.dec.handle, B, ld, C.c_void_p(word.data_ptr()),
                                                  C.c_void_p(s.data_ptr()), self._stream()), "syndrome")
        return s

    def frames(self, nm: NoiseMapper, B: int, gen, two_variance: float):
        """One batch of inputs for the selected mode: (lappr [V, ld], synd [C, ld], word [V, ld], ld)."""
        import torch

        ld = leading_dim(B)
        S = self.S
        x = self._symbols(S, ld, gen)
        y = self._a[x] + nm.noise_sigma * torch.randn((S, ld), generator=gen, device=self.device,
                                                      dtype=torch.float64)
        lappr = torch.empty((self.V, ld), dtype=torch.float64, device=self.device)
        if self.mode == "softening":                       # reconciliation.pyx:129-145
            _, nhat, word = nm.bob_map_device(y, B)
            synd = self._synd(word, B, ld)
            nm.demap_device(nhat, x, B, self.alpha, out=lappr)
        elif self.mode == "direct":                        # reconciliation.pyx:209-221
            word = self._bits(x, B, ld)
            synd = self._synd(word, B, ld)
            _lib.check(_lib.load().qr_direct_lappr_device(nm.handle, float(two_variance), B, ld, S,
                                                          C.c_void_p(y.data_ptr()), C.c_void_p(lappr.data_ptr()),
                                                          self._stream()), "direct_lappr")
        else:                                              # reconciliation.pyx:290-303
            xh, _, word = nm.bob_map_device(y, B)
            synd = self._synd(word, B, ld)
            table = torch.tensor(np.ascontiguousarray(nm.bare_llr_table), dtype=torch.float64, device=self.device)
            _lib.check(_lib.load().qr_bare_llr_device(self.pa.bit_per_symbol, C.c_void_p(table.data_ptr()), B, ld,
                                                      S, C.c_void_p(x.data_ptr()), C.c_void_p(lappr.data_ptr()),
                                                      self._stream()), "bare_llr")
        return lappr, synd, word, ld

    # ------------------------------------------------------------------ run
    def run_snr(self, snr_dB: float, simulation_loops: int, ferr_count_min: int, seed: int = 0):
        """Frames until `simulation_loops` or the early stop; returns
        (snr_dB, ber, fer, avg_iterations_of_successes)."""
        import torch

        world, rank, _ = dist.env_world()
        Es = self.pa.variance
        two_var = Es * (10 ** (-snr_dB / 10))          # reconciliation.pyx:191-192, 272-273
        N0 = Es * (10 ** (-snr_dB / 10)) / 2           # reconciliation.pyx:109-110
        cfg = self.cfg if self.mode == "softening" else None
        nm = NoiseMapper(self.pa, N0, cfg, device=self._dev_index)
        total = torch.zeros(5, dtype=torch.int64, device=self.device)
        ferr = torch.empty(max(1, self.batch), dtype=torch.int32, device=self.device)
        done, bidx = 0, 0
        while done < simulation_loops:
            n_global = min(self.batch * world, simulation_loops - done)
            _, B = dist.shard(n_global, world, rank)
            delta = torch.zeros(5, dtype=torch.int64, device=self.device)
            if B > 0:
                gen = torch.Generator(device=self.device).manual_seed(dist.rank_seed(seed, rank, bidx))
                lappr, synd, word, ld = self.frames(nm, B, gen, two_var)
                fin, succ, its = self.dec.decode_device(lappr, synd, B, self.max_iterations)
                if ferr.numel() < B:
                    ferr = torch.empty(B, dtype=torch.int32, device=self.device)
                _lib.check(_lib.load().qr_count_errors_device(
                    B, ld, self.K, C.c_void_p(fin.data_ptr()), C.c_void_p(word.data_ptr()),
                    C.c_void_p(succ.data_ptr()), C.c_void_p(its.data_ptr()), C.c_void_p(ferr.data_ptr()),
                    C.c_void_p(delta.data_ptr()), self._stream()), "count")
            dist.all_reduce_sum(delta)
            total += delta
            done += n_global
            bidx += 1
            if dist.early_stop(total.cpu().numpy(), ferr_count_min, simulation_loops):
                break
        be, fe, su, it, fr = [int(v) for v in total.cpu().numpy()]
        return (snr_dB, be / (fr * self.K), fe / fr, 0 if su == 0 else it / su)


def simulate_softening_snr_dB(snr_dB, dec, bps, nmconfig, decoder_iterations, simulation_loops, ferr_count_min,
                              alpha=1.0, batch=4096, seed=0):
    """reconciliation.pyx:93-168 (the Matrix is the decoder's own graph)."""
    sim = Simulator(dec, bps, "softening", decoder_iterations, alpha, batch)
    sim.cfg = np.ascontiguousarray(nmconfig, np.uint8)
    return sim.run_snr(snr_dB, simulation_loops, ferr_count_min, seed)


def simulate_direct_snr_dB(snr_dB, dec, bps, decoder_iterations, simulation_loops, ferr_count_min, batch=4096, seed=0):
    """reconciliation.pyx:173-249"""
    return Simulator(dec, bps, "direct", decoder_iterations, 1.0, batch).run_snr(
        snr_dB, simulation_loops, ferr_count_min, seed)


def simulate_hard_reverse_snr_dB(snr_dB, dec, bps, decoder_iterations, simulation_loops, ferr_count_min, batch=4096,
                                 seed=0):
    """reconciliation.pyx:253-329"""
    return Simulator(dec, bps, "hard", decoder_iterations, 1.0, batch).run_snr(
        snr_dB, simulation_loops, ferr_count_min, seed)
