"""Drop-in ``NoiseMapper`` whose soft demap runs on the gfx950 kernels.

Mirrors qamreconciliation.noisemapper.NoiseMapper (noisemapper.pyx:102-559):
constructor signature, read-only tables and the hot-path methods
``demap_lappr_array`` / ``demap_lappr`` (the north-star entry point), plus the
Bob-side ``hard_decide_index`` / ``map_noise`` that produce its inputs.
The hot-path tables (F_Y_thresholds, delta_F_Y) come from libqamr's host code
with the scipy-exact erf; the remaining O(M^2) tables (transition
probabilities, bare LLRs, erf table) are small host-side numpy constructions
of noisemapper.pyx:166-235.

Batched device methods (torch tensors in HBM, frame-innermost layout):
``demap_device`` (fused with the LLR scaling alpha of reconciliation.pyx:144-145,
writing the decoder's input layout directly) and ``bob_map_device``.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _lib
from ._lib import check, check_tensor, ptr
from .alphabet import PAMAlphabet


def _check_batch(B, ld, what):
    if ld % 64 or not 0 < int(B) <= ld:
        raise ValueError(f"{what}: need ld % 64 == 0 and 0 < B <= ld (B={B}, ld={ld})")


def F_Z(z, mu, sigma):
    """noisemapper.pyx:66-79: the Gaussian CDF 0.5 (1 + erf((z - mu) / (sqrt(2) sigma))) at every
    z, with scipy's erf as the reference.  Off the hot path (a host helper)."""
    from scipy.special import erf

    z = np.asarray(z)
    if z.dtype != np.float64:
        raise ValueError(f"Buffer dtype mismatch, expected 'double' but got '{z.dtype}'")
    z = np.ascontiguousarray(z.ravel())
    return 0.5 * (1 + erf((z - float(mu)) / (math.sqrt(2) * float(sigma))))


def view_dist_cut(x):
    """noisemapper.pyx:82-98 (``__view_dist_cut``): every x clipped to the probability range,
    0 below 0, 1 from 1 on (NaN stays NaN, as the reference's comparisons leave it)."""
    x = np.asarray(x)
    if x.dtype != np.float64:
        raise ValueError(f"Buffer dtype mismatch, expected 'double' but got '{x.dtype}'")
    x = np.ascontiguousarray(x.ravel())
    return np.where(x < 0, 0.0, np.where(x >= 1, 1.0, x))


def host_tables(a, th, p, sigma, bps):
    """The O(M^2) host tables of NoiseMapper.__cinit__ (noisemapper.pyx:166-235),
    with C erf/log semantics: (fwrd_transition_probability, back_transition_probability,
    bare_llr_table, inf_erf_table)."""
    M = len(a)
    tmp = math.sqrt(2) * sigma
    fw = np.empty((M, M))
    for j in range(M):
        fw[j, 0] = 0.5 * (math.erf((th[1] - a[j]) / tmp) + 1)
        fw[j, M - 1] = 0.5 * (1 - math.erf((th[M - 1] - a[j]) / tmp))
        for i in range(1, M - 1):
            fw[j, i] = 0.5 * (math.erf((th[i + 1] - a[j]) / tmp) - math.erf((th[i] - a[j]) / tmp))
    back = np.empty((M, M))
    for i in range(M):
        for j in range(M):
            t = 0.0
            for k in range(M):
                t += p[k] * fw[k, i]
            back[i, j] = p[j] * fw[j, i] / t
    bare = np.empty((M, bps))
    old = np.seterr(divide="ignore")
    try:
        for j in range(M):
            for k in range(bps):
                N = D = 0.0
                for i in range(M):
                    mi = i >> k
                    if (mi * (mi + 1)) & 3:
                        D += fw[j, i]
                    else:
                        N += fw[j, i]
                # C log semantics (log(0) = -inf) rather than math.log's ValueError
                bare[j, k] = 1e300 if D == 0 else float(np.log(np.float64(N) / np.float64(D)))
    finally:
        np.seterr(**old)
    ierf = np.empty((M, M))
    for j in range(M):
        ierf[0, j] = -1
        for i in range(1, M):
            ierf[i, j] = math.erf((th[i] - a[j]) / tmp)
    return fw, back, bare, ierf


class NoiseMapper:
    def __init__(self, pa: PAMAlphabet, noise_var: float, sign_config=None, trunkation_threshold: float = 1e-21,
                 n_intervals_per_step: int = 1000, device: int = 0):
        noise_var = float(noise_var)
        if noise_var <= 0:  # noisemapper.pyx:111-112
            raise ValueError(f"noise variance must be strictly positive, got {noise_var}")
        if sign_config is None:  # :115-120
            sc = np.zeros(pa.order, dtype=np.uint8)
        else:
            sc = np.asarray(sign_config)
            if sc.dtype == np.bool_:
                sc = sc.view(np.uint8)
            if sc.dtype != np.uint8:
                raise ValueError(f"Buffer dtype mismatch, expected 'unsigned char' but got '{sc.dtype}'")
            if sc.size < pa.order:
                raise ValueError("Not enough data for a monotonicity sign configuration")
            sc = np.ascontiguousarray(sc)
        self.sign_config = sc
        self.order = pa.order
        self.half_order = pa.order >> 1
        self.bit_per_symbol = pa.bit_per_symbol
        self.constellation = np.asarray(pa.constellation, np.float64)
        self.variance = pa.variance
        self.thresholds = np.asarray(pa.thresholds, np.float64)
        self.probabilities = np.ascontiguousarray(pa.probabilities, np.float64)
        self.noise_var = noise_var
        self.noise_sigma = math.sqrt(noise_var)
        self._device = int(device)
        self._trunc = float(trunkation_threshold)
        self._nips = int(n_intervals_per_step)
        self._step = pa.step

        a = np.ascontiguousarray(self.constellation)
        th = np.ascontiguousarray(self.thresholds)
        h = C.c_void_p()
        check(_lib.load().qr_demap_create(int(self.bit_per_symbol), ptr(a), ptr(self.probabilities), ptr(th),
                                          noise_var, ptr(sc), self._device, C.byref(h)), "NoiseMapper")
        self._h = h
        self.F_Y_thresholds = np.empty(self.order + 1, np.float64)
        self.delta_F_Y = np.empty(self.order, np.float64)
        check(_lib.load().qr_demap_tables(h, ptr(self.F_Y_thresholds), ptr(self.delta_F_Y)))
        self._host_tables()
        self._y_range = None
        self._F_Y = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib._lib.qr_demap_destroy(h)
            self._h = None

    # ------------------------------------------------- small host-side tables
    def _host_tables(self):
        (self.fwrd_transition_probability, self.back_transition_probability, self.bare_llr_table,
         self.inf_erf_table) = host_tables(self.constellation, self.thresholds, self.probabilities,
                                           self.noise_sigma, self.bit_per_symbol)

    def _grid(self):
        """Uniform-weighted F_Y on the interpolation grid (noisemapper.pyx:135-144,
        264-275); not on the hot path, built lazily with scipy's erf."""
        if self._y_range is None:
            from scipy.special import erf
            if self._trunc > 1.0:
                lo, hi = self.constellation[0] * 10, self.constellation[-1] * 10
            else:
                t = math.sqrt(-2.0 * math.log(self._trunc)) * self.noise_sigma
                hi, lo = self.constellation[-1] + t, self.constellation[0] - t
            n = int(math.ceil((hi - lo) * self._nips / self._step)) + 1
            y = np.linspace(lo, hi, n)
            den = math.sqrt(2) * self.noise_sigma
            res = 0.5 * (1 + erf((y - self.constellation[0]) / den))
            for i in range(1, self.order):
                res = res + 0.5 * (1 + erf((y - self.constellation[i]) / den))
            self._y_range, self._F_Y = y, res / self.order
        return self._y_range, self._F_Y

    @property
    def y_range(self):
        return np.array(self._grid()[0])

    @property
    def F_Y_values(self):
        return np.array(self._grid()[1])

    @property
    def handle(self):
        return self._h

    def bare_llr(self, symb):
        """noisemapper.pyx:423-432 (hard-reverse LLR table lookup)."""
        s = np.asarray(symb, np.int64)
        return np.ascontiguousarray(self.bare_llr_table[s].reshape(-1))

    def index_to_val(self, index):
        """noisemapper.pyx:362-370"""
        return self.constellation[np.asarray(index, np.int64)]

    # ------------------------------------- CDF and its inverse (GPU, scalar API)
    def F_Y(self, y):
        """noisemapper.pyx:264-275: the uniformly weighted mixture CDF at every y."""
        y = np.asarray(y)
        if y.dtype != np.float64:
            raise ValueError(f"Buffer dtype mismatch, expected 'double' but got '{y.dtype}'")
        y = np.ascontiguousarray(y.ravel())
        out = np.empty(y.size, np.float64)
        if y.size:
            check(_lib.load().qr_F_Y_host(self._h, y.size, ptr(y), ptr(out)), "F_Y")
        return out

    def g(self, y, i):
        """noisemapper.pyx:289-292: the transformed noise of sample y in decision region i."""
        return float(self.map_noise(np.array([float(y)]), np.array([int(i)], np.int64))[0])

    def g_inv_search(self, n_hat, i, y_accuracy=1e-9):
        """noisemapper.pyx:310-345: y with F_Y(y) = the target of (n_hat, i), by doubling
        bracket + bisection to width <= y_accuracy."""
        return float(self.demap_noise_search(np.array([float(n_hat)]), np.array([int(i)], np.int64),
                                             y_accuracy)[0])

    def demap_noise_search(self, n_hat, symb, y_accuracy=1e-9):
        """noisemapper.pyx:407-419: g_inv_search over arrays."""
        n_hat = np.asarray(n_hat)
        symb = np.asarray(symb)
        if n_hat.dtype != np.float64:
            raise ValueError(f"Buffer dtype mismatch, expected 'double' but got '{n_hat.dtype}'")
        if symb.dtype != np.int64:
            raise ValueError(f"Buffer dtype mismatch, expected 'long' but got '{symb.dtype}'")
        if n_hat.size != symb.size:
            raise ValueError("Sizes do not match")
        n_hat = np.ascontiguousarray(n_hat.ravel())
        symb = np.ascontiguousarray(symb.ravel())
        out = np.empty(n_hat.size, np.float64)
        if n_hat.size:
            check(_lib.load().qr_g_inv_search_host(self._h, n_hat.size, ptr(n_hat), ptr(symb), float(y_accuracy),
                                                   ptr(out)), "g_inv_search")
        return out

    # ------------------------------------------------------- hot path (GPU)
    def demap_lappr_array(self, n, j):
        """noisemapper.pyx:544-559: LAPPRs [S*bps], out[s*bps + k] = Gray bit k of symbol s."""
        n = np.asarray(n)
        j = np.asarray(j)
        if n.dtype != np.float64:
            raise ValueError(f"Buffer dtype mismatch, expected 'double' but got '{n.dtype}'")
        if j.dtype != np.int64:
            raise ValueError(f"Buffer dtype mismatch, expected 'long' but got '{j.dtype}'")
        if n.size != j.size:
            raise ValueError("Sizes of transformed noise vector and tx symbols do not match")
        n = np.ascontiguousarray(n.ravel())
        j = np.ascontiguousarray(j.ravel())
        out = np.empty(n.size * self.bit_per_symbol, np.float64)
        if n.size:
            check(_lib.load().qr_demap_host(self._h, n.size, ptr(n), ptr(j), ptr(out)), "demap_lappr_array")
        return out

    def demap_lappr(self, n, j):
        """noisemapper.pyx:450-540 for one symbol."""
        return self.demap_lappr_array(np.array([float(n)]), np.array([int(j)], np.int64))

    # ----------------------------------------------- Bob side (GPU, batched)
    # Single-frame (reference-style) calls: the per-symbol maps are elementwise, so one
    # frame of S symbols is laid out along the frame axis as ONE symbol row of S "frames"
    # (ld = S rounded up to 64): S lanes of work instead of 64 columns per symbol.
    def _bob_host(self, y):
        import torch

        y = np.ascontiguousarray(np.asarray(y, np.float64).ravel())
        S = y.size
        ld = max(64, -(-S // 64) * 64)
        dev = torch.device("cuda", self._device)
        yt = torch.zeros((1, ld), dtype=torch.float64, device=dev)
        yt[0, :S] = torch.from_numpy(y).to(dev)
        xh, nh, w = self.bob_map_device(yt, S)
        torch.cuda.synchronize(dev)
        # word rows k = Gray bit k of the row's symbol; symbol s's bits are s * bps + k
        return (xh[0, :S].cpu().numpy(), nh[0, :S].cpu().numpy(),
                np.ascontiguousarray(w[:, :S].cpu().numpy().T).ravel())

    def hard_decide_index(self, y_samples):
        """noisemapper.pyx:349-359"""
        return self._bob_host(y_samples)[0]

    def map_noise(self, y_samples, index):
        """noisemapper.pyx:373-388: n[j] = g(y[j], index[j])."""
        import torch

        idx = np.asarray(index)
        y = np.asarray(y_samples, np.float64)
        if y.size != idx.size:
            raise ValueError("Input vectors sizes do not match")
        S = y.size
        ld = max(64, -(-S // 64) * 64)  # one frame along the frame axis (see _bob_host)
        dev = torch.device("cuda", self._device)
        yt = torch.zeros((1, ld), dtype=torch.float64, device=dev)
        yt[0, :S] = torch.from_numpy(np.ascontiguousarray(y.ravel())).to(dev)
        it = torch.zeros((1, ld), dtype=torch.int64, device=dev)
        it[0, :S] = torch.from_numpy(np.ascontiguousarray(idx.ravel().astype(np.int64))).to(dev)
        nh = self.map_noise_device(yt, it, S)
        torch.cuda.synchronize(dev)
        return nh[0, :S].cpu().numpy()

    def map_noise_device(self, y_fi, index_fi, B: int, stream=None):
        """y_fi float64 [S, ld], index_fi int64 [S, ld] -> n_hat float64 [S, ld]."""
        import torch

        if not isinstance(y_fi, torch.Tensor) or y_fi.dim() != 2:
            raise ValueError("map_noise_device: y_fi must be a 2-D tensor [S, ld]")
        S, ld = y_fi.shape
        _check_batch(B, ld, "map_noise_device")
        check_tensor(y_fi, "y_fi", (S, ld), torch.float64, self._device)
        check_tensor(index_fi, "index_fi", (S, ld), torch.int64, self._device)
        nh = torch.empty((S, ld), dtype=torch.float64, device=y_fi.device)
        if stream is None:
            stream = torch.cuda.current_stream(y_fi.device)
        check(_lib.load().qr_map_noise_device(self._h, int(B), int(ld), int(S), C.c_void_p(y_fi.data_ptr()),
                                              C.c_void_p(index_fi.data_ptr()), C.c_void_p(nh.data_ptr()),
                                              C.c_void_p(stream.cuda_stream)), "map_noise_device")
        return nh

    # ------------------------------------------------- device (HBM) batches
    def demap_device(self, n_fi, j_fi, B: int, alpha: float = 1.0, out=None, stream=None):
        """n_fi float64 [S, ld], j_fi int64 [S, ld] -> LAPPRs float64 [S*bps, ld]
        (the decoder's frame-innermost input), scaled by alpha."""
        import torch

        if not isinstance(n_fi, torch.Tensor) or n_fi.dim() != 2:
            raise ValueError("demap_device: n_fi must be a 2-D tensor [S, ld]")
        S, ld = n_fi.shape
        _check_batch(B, ld, "demap_device")
        check_tensor(n_fi, "n_fi", (S, ld), torch.float64, self._device)
        check_tensor(j_fi, "j_fi", (S, ld), torch.int64, self._device)
        if out is None:
            out = torch.empty((S * self.bit_per_symbol, ld), dtype=torch.float64, device=n_fi.device)
        check_tensor(out, "out", (S * self.bit_per_symbol, ld), torch.float64, self._device)
        if stream is None:
            stream = torch.cuda.current_stream(n_fi.device)
        check(_lib.load().qr_demap_batch_device(self._h, int(B), int(ld), int(S), C.c_void_p(n_fi.data_ptr()),
                                                C.c_void_p(j_fi.data_ptr()), float(alpha),
                                                C.c_void_p(out.data_ptr()), C.c_void_p(stream.cuda_stream)),
              "demap_device")
        return out

    def bob_map_device(self, y_fi, B: int, stream=None):
        """y_fi float64 [S, ld] -> (x_hat int64 [S, ld], n_hat float64 [S, ld], word uint8 [S*bps, ld])."""
        import torch

        if not isinstance(y_fi, torch.Tensor) or y_fi.dim() != 2:
            raise ValueError("bob_map_device: y_fi must be a 2-D tensor [S, ld]")
        S, ld = y_fi.shape
        _check_batch(B, ld, "bob_map_device")
        check_tensor(y_fi, "y_fi", (S, ld), torch.float64, self._device)
        dev = y_fi.device
        xh = torch.empty((S, ld), dtype=torch.int64, device=dev)
        nh = torch.empty((S, ld), dtype=torch.float64, device=dev)
        w = torch.zeros((S * self.bit_per_symbol, ld), dtype=torch.uint8, device=dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        check(_lib.load().qr_bob_map_device(self._h, int(B), int(ld), int(S), C.c_void_p(y_fi.data_ptr()),
                                            C.c_void_p(xh.data_ptr()), C.c_void_p(nh.data_ptr()),
                                            C.c_void_p(w.data_ptr()), C.c_void_p(stream.cuda_stream)),
              "bob_map_device")
        return xh, nh, w


class NoiseDemapper(NoiseMapper):
    """Declared in noisemapper.pxd:89 with no extra behaviour."""
