"""Batched, GPU-resident Monte-Carlo reconciliation simulations.

GPU counterpart of sims/reconciliation.pyx:
  * ``simulate_softening_snr_dB``   (reconciliation.pyx:93-168)  -- the hot path
  * ``simulate_direct_snr_dB``      (reconciliation.pyx:173-249)
  * ``simulate_hard_reverse_snr_dB`` (reconciliation.pyx:253-329)
The reference decodes one frame at a time; here every batch of B independent
frames is generated, mapped, decoded and counted by libqamr kernels in HBM
(frame-innermost layout), and with several GPUs each rank takes a contiguous
share of every batch (frame sharding: global frame order = batch order, then
rank order, then the frame's column).  The five counters are all-reduced once
per batch (qamr.dist).  The ``ferr_count_min`` early stop is the reference's
per-frame rule (reconciliation.pyx:159-161): when it holds at the end of a
batch, the first global frame at which it held is located from the per-frame
error counts of every rank (``first_stop_frame``) and every counter is cut
there, so the returned tuple is the one the reference's sequential loop
returns for the same frames (tests/test_gpu_sim.py).  Returned tuples have the
reference's shape: (snr_dB, ber, fer, average iterations of successful frames).
RNG streams are torch's (per seed, rank and batch), not numpy's.
"""
from __future__ import annotations

import ctypes as C
import math

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
    def batch_results(self, nm: NoiseMapper, B: int, gen, two_var: float, hook=None):
        """Generate, map, decode and count one shard of B frames: (ferr int32[B], succ uint8[B],
        its int32[B], delta int64[5]) on the GPU.  hook(lappr, synd, word, B) sees the inputs."""
        import torch

        lappr, synd, word, ld = self.frames(nm, B, gen, two_var)
        if hook is not None:
            hook(lappr, synd, word, B)
        fin, succ, its = self.dec.decode_device(lappr, synd, B, self.max_iterations)
        ferr = torch.empty(B, dtype=torch.int32, device=self.device)
        delta = torch.zeros(5, dtype=torch.int64, device=self.device)
        _lib.check(_lib.load().qr_count_errors_device(
            B, ld, self.K, C.c_void_p(fin.data_ptr()), C.c_void_p(word.data_ptr()),
            C.c_void_p(succ.data_ptr()), C.c_void_p(its.data_ptr()), C.c_void_p(ferr.data_ptr()),
            C.c_void_p(delta.data_ptr()), self._stream()), "count")
        return ferr, succ[:B], its[:B], delta

    def run_snr(self, snr_dB: float, simulation_loops: int, ferr_count_min: int, seed: int = 0, hook=None):
        """Frames until `simulation_loops` or the early stop; returns
        (snr_dB, ber, fer, avg_iterations_of_successes).  hook(batch_index, lappr, synd, word, B):
        optional view of every shard's inputs (tests)."""
        world, rank, _ = dist.env_world()
        Es = self.pa.variance
        two_var = Es * (10 ** (-snr_dB / 10))          # reconciliation.pyx:191-192, 272-273
        N0 = Es * (10 ** (-snr_dB / 10)) / 2           # reconciliation.pyx:109-110
        cfg = self.cfg if self.mode == "softening" else None
        nm = NoiseMapper(self.pa, N0, cfg, device=self._dev_index)

        def frame_fn(bidx, start, B):
            import torch

            gen = torch.Generator(device=self.device).manual_seed(dist.rank_seed(seed, rank, bidx))
            h = None if hook is None else (lambda l, s, w, b: hook(bidx, l, s, w, b))
            return self.batch_results(nm, B, gen, two_var, h)

        be, fe, su, it, fr = run_frames(frame_fn, self.batch, simulation_loops, ferr_count_min, self.device)
        return (snr_dB, be / (fr * self.K), fe / fr, 0 if su == 0 else it / su)


def shard_counters(ferr, succ, its, n: int):
    """The five counters {bit_errors, frame_errors, successes, iteration_sum_of_successes,
    frames} of a shard's first n frames (reconciliation.pyx:149-157)."""
    import torch

    e = ferr[:n].to(torch.int64)
    s = succ[:n].to(torch.int64)
    return torch.stack([e.sum(), (e > 0).sum(), s.sum(), (its[:n].to(torch.int64) * s).sum(),
                        torch.tensor(n, dtype=torch.int64, device=ferr.device)])


def first_stop_frame(prev_frame_errors: int, ferr, start: int, done: int, ferr_count_min: int,
                     simulation_loops: int) -> int:
    """Global index of the first frame of this batch after which reconciliation.pyx:159-161
    holds: frame_error_count >= ferr_count_min and wordcount > simulation_loops / 20.  Both
    parts are monotone in the frame index, so it is max(first frame where the running frame-error
    count reaches the minimum, first index above loops / 20).  ferr: this rank's per-frame bit
    errors of its frames [done + start, done + start + len(ferr)); a collective over the ranks."""
    import torch

    world, rank, _ = dist.env_world()
    dev = ferr.device
    flags = (ferr > 0).to(torch.int64)
    per_rank = torch.zeros(world, dtype=torch.int64, device=dev)
    per_rank[rank] = flags.sum()
    dist.all_reduce_sum(per_rank)                               # frame errors of every rank's shard
    before = prev_frame_errors + int(per_rank[:rank].sum())     # shards are in rank order
    big = 1 << 62
    g_fe = big
    if flags.numel():
        hit = torch.nonzero(before + torch.cumsum(flags, 0) >= ferr_count_min)
        if hit.numel():
            g_fe = done + start + int(hit[0, 0])
    t = torch.tensor([g_fe], dtype=torch.int64, device=dev)
    dist.all_reduce_min(t)
    g_w = math.floor(simulation_loops / 20) + 1                 # first wordcount > loops / 20
    return max(int(t.item()), g_w)


def run_frames(frame_fn, batch: int, simulation_loops: int, ferr_count_min: int, device=None):
    """The frame loop of reconciliation.pyx:127-168 over batches of batch * world frames,
    each rank taking its contiguous shard (dist.shard).  frame_fn(batch_index, start, B) ->
    (ferr, succ, its, delta) for this rank's B frames [done + start, done + start + B) of the
    batch (delta = their five counters).  Returns the five global counters at the reference's
    stopping frame: {bit_errors, frame_errors, successes, iteration_sum, frames = wordcount+1}."""
    import torch

    world, rank, _ = dist.env_world()
    total = torch.zeros(5, dtype=torch.int64, device=device)
    done, bidx = 0, 0
    while done < simulation_loops:
        n_global = min(batch * world, simulation_loops - done)
        start, B = dist.shard(n_global, world, rank)
        if B > 0:
            ferr, succ, its, delta = frame_fn(bidx, start, B)
        else:
            ferr = torch.zeros(0, dtype=torch.int32, device=device)
            succ = torch.zeros(0, dtype=torch.uint8, device=device)
            its = torch.zeros(0, dtype=torch.int32, device=device)
            delta = torch.zeros(5, dtype=torch.int64, device=device)
        dist.all_reduce_sum(delta)
        after = (total + delta).cpu().numpy()
        if dist.early_stop(after, ferr_count_min, simulation_loops):
            # the reference stopped at some frame of this batch: cut every counter there
            g = first_stop_frame(int(total[1]), ferr, start, done, ferr_count_min, simulation_loops)
            keep = min(max(g - (done + start) + 1, 0), B)
            part = shard_counters(ferr, succ, its, keep) if keep else torch.zeros(5, dtype=torch.int64,
                                                                                 device=device)
            dist.all_reduce_sum(part)
            total += part.to(total.device)
            break
        total += delta
        done += n_global
        bidx += 1
    return [int(v) for v in total.cpu().numpy()]


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
