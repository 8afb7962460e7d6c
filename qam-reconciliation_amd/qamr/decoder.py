"""Drop-in ``Decoder`` backed by the gfx950 sum-product kernels of libqamr.so.

Mirrors qamreconciliation.decoder.Decoder (decoder.pyx:92-455): same
constructor, properties, method names, argument order, return tuples and
exception types.  Differences (documented, stricter): input lengths are
validated (the reference reads out of bounds, decoder.pyx:441-455), and check
nodes of degree < 2 are rejected at construction (undefined behaviour in the
reference, decoder.pyx:135-141).

Besides the one-frame API, ``decode_batch`` (host arrays, frame-major) and
``decode_device`` (torch tensors resident in HBM, frame-innermost layout) decode
many independent frames per launch -- the path the benchmark measures.
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict

import numpy as np

from . import _lib
from ._lib import check, ptr


def _as_buffer(a, dtype, name, expected):
    """Cython typed-memoryview semantics: exact dtype, 1-D (decoder.pxd)."""
    arr = np.asarray(a)
    if arr.dtype == np.bool_ and dtype == np.uint8:
        arr = arr.view(np.uint8)
    if arr.dtype != dtype:
        raise ValueError(f"Buffer dtype mismatch, expected '{expected}' but got '{arr.dtype}' ({name})")
    if arr.ndim != 1:
        raise ValueError(f"Buffer has wrong number of dimensions (expected 1, got {arr.ndim}) ({name})")
    return np.ascontiguousarray(arr)


def _as_inout(a, dtype, name, expected):
    """In/out buffers must be written in place: exact dtype, 1-D, contiguous."""
    if not isinstance(a, np.ndarray):
        raise ValueError(f"{name} must be a numpy array (written in place)")
    if a.dtype != dtype:
        raise ValueError(f"Buffer dtype mismatch, expected '{expected}' but got '{a.dtype}' ({name})")
    if a.ndim != 1 or not a.flags.c_contiguous or not a.flags.writeable:
        raise ValueError(f"{name} must be a writeable 1-D C-contiguous array")
    return a


class Decoder:
    """``Decoder(e_to_v, e_to_c)`` -- Tanner graph given as an edge list."""

    def __init__(self, e_to_v, e_to_c, device: int = 0):
        vid = _as_buffer(e_to_v, np.int64, "e_to_v", "long")
        cid = _as_buffer(e_to_c, np.int64, "e_to_c", "long")
        L = _lib.load()
        h = C.c_void_p()
        check(L.qr_code_create(ptr(vid), ptr(cid), vid.size, cid.size, int(device), C.byref(h)), "Decoder")
        self._h = h
        self._device = int(device)
        v, c, e = C.c_int64(), C.c_int64(), C.c_int64()
        dc, dv = C.c_int32(), C.c_int32()
        check(L.qr_code_info(h, C.byref(v), C.byref(c), C.byref(e), C.byref(dc), C.byref(dv)))
        self._V, self._C, self._E = int(v.value), int(c.value), int(e.value)
        self.max_check_degree, self.max_var_degree = int(dc.value), int(dv.value)
        self._ws = OrderedDict()  # per-stream device workspaces of decode_device (LRU, capped)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib._lib.qr_code_destroy(h)
            self._h = None

    # ---------------------------------------------------------- properties
    @property
    def cnum(self):
        """Number of check nodes (decoder.pyx:157-160)"""
        return self._C

    @property
    def vnum(self):
        """Number of variable nodes (decoder.pyx:163-166)"""
        return self._V

    @property
    def ednum(self):
        """Number of edges (decoder.pyx:169-172)"""
        return self._E

    @property
    def handle(self):
        return self._h

    @property
    def device(self):
        return self._device

    # ------------------------------------------------------ syndrome checks
    def _check_word_flags(self, word, synd):
        w = _as_buffer(word, np.uint8, "word", "unsigned char")
        s = _as_buffer(synd, np.uint8, "synd", "unsigned char")
        if w.size != self._V:
            raise ValueError("Size of word does not match number of vnodes")
        if s.size != self._C:
            raise ValueError("Size of synd does not match number of cnodes")
        flags = np.empty(self._C, np.uint8)
        allok = C.c_uint8()
        check(_lib.load().qr_check_word_host(self._h, ptr(w), ptr(s), ptr(flags), C.byref(allok)), "check_word")
        return flags, int(allok.value)

    def check_synd_node(self, check_node_index, word, synd):
        """decoder.pyx:190-209: ``parity ^ 1`` of one check for a hard word."""
        flags, _ = self._check_word_flags(word, synd)
        return int(flags[int(check_node_index)])

    def check_word(self, word, synd):
        """decoder.pyx:220-232: 1 iff every check is satisfied by the hard word."""
        _, allok = self._check_word_flags(word, synd)
        return allok

    def check_lappr(self, lappr, synd):
        """decoder.pyx:260-281: 1 iff sign(lappr) (< 0 -> bit 1) satisfies synd."""
        l = _as_buffer(lappr, np.float64, "lappr", "double")
        s = _as_buffer(synd, np.uint8, "synd", "unsigned char")
        if l.size != self._V:
            raise ValueError("Size of lappr does not match number of vnodes")
        if s.size != self._C:
            raise ValueError("Size of synd does not match number of cnodes")
        flags = np.empty(self._C, np.uint8)
        allok = C.c_uint8()
        check(_lib.load().qr_check_lappr_host(self._h, ptr(l), ptr(s), ptr(flags), C.byref(allok)), "check_lappr")
        return int(allok.value)

    # ------------------------------------------------------ node processing
    def process_var_node(self, node_index, lappr_data, check_to_var, var_to_check, updated_lappr):
        """decoder.pyx:301-319 (writes var_to_check and updated_lappr in place)."""
        l = _as_buffer(lappr_data, np.float64, "lappr_data", "double")
        c2v = _as_buffer(check_to_var, np.float64, "check_to_var", "double")
        v2c = _as_inout(var_to_check, np.float64, "var_to_check", "double")
        upd = _as_inout(updated_lappr, np.float64, "updated_lappr", "double")
        if l.size < self._V or upd.size < self._V or c2v.size < self._E or v2c.size < self._E:
            raise ValueError("message/LAPPR arrays are shorter than the graph")
        nodes = np.array([int(node_index)], np.int64)
        check(_lib.load().qr_process_var_nodes_host(self._h, ptr(nodes), 1, ptr(l), ptr(c2v), ptr(v2c), ptr(upd)),
              "process_var_node")

    def process_check_node(self, node_index, synd, check_to_var, var_to_check):
        """decoder.pyx:372-388 (writes check_to_var in place); returns 0."""
        s = _as_buffer(synd, np.uint8, "synd", "unsigned char")
        c2v = _as_inout(check_to_var, np.float64, "check_to_var", "double")
        v2c = _as_buffer(var_to_check, np.float64, "var_to_check", "double")
        if s.size < self._C or c2v.size < self._E or v2c.size < self._E:
            raise ValueError("message/syndrome arrays are shorter than the graph")
        nodes = np.array([int(node_index)], np.int64)
        check(_lib.load().qr_process_check_nodes_host(self._h, ptr(nodes), 1, ptr(s), ptr(c2v), ptr(v2c)),
              "process_check_node")
        return 0

    # ---------------------------------------------------------------- decode
    def decode(self, lappr_data, synd, max_iterations):
        """decoder.pyx:441-455 -> (success, iterations, final_lappr)."""
        l = _as_buffer(lappr_data, np.float64, "lappr_data", "double")
        s = _as_buffer(synd, np.uint8, "synd", "unsigned char")
        if l.size != self._V:
            raise ValueError(f"lappr has {l.size} entries, the code has {self._V} variable nodes")
        if s.size != self._C:
            raise ValueError(f"synd has {s.size} entries, the code has {self._C} check nodes")
        succ, its, res = self.decode_batch(l[None, :], s[None, :], max_iterations)
        return int(succ[0]), int(its[0]), res[0]

    def decode_batch(self, lappr, synd, max_iterations):
        """Decode B independent frames from host memory.

        lappr: float64 [B, V]; synd: uint8/bool [B, C].
        Returns (success uint8[B], iterations int32[B], final float64[B, V])."""
        l = np.ascontiguousarray(lappr)
        s = np.asarray(synd)
        if s.dtype == np.bool_:
            s = s.view(np.uint8)
        s = np.ascontiguousarray(s)
        if l.dtype != np.float64 or s.dtype != np.uint8:
            raise ValueError("decode_batch expects float64 LAPPRs and uint8 syndromes")
        if l.ndim != 2 or s.ndim != 2 or l.shape[0] != s.shape[0]:
            raise ValueError("decode_batch expects lappr [B, V] and synd [B, C]")
        if l.shape[1] != self._V or s.shape[1] != self._C:
            raise ValueError("decode_batch: shape does not match the code")
        B = l.shape[0]
        out = np.empty_like(l)
        succ = np.empty(B, np.uint8)
        its = np.empty(B, np.int32)
        check(_lib.load().qr_decode_host(self._h, B, ptr(l), ptr(s), int(max_iterations), ptr(out), ptr(succ),
                                         ptr(its)), "decode")
        return succ, its, out

    # ------------------------------------------------------- device (HBM) API
    def workspace_bytes(self, ld: int, max_iterations: int) -> int:
        n = C.c_size_t()
        check(_lib.load().qr_decode_workspace_size(self._h, int(ld), int(max_iterations), C.byref(n)))
        return int(n.value)

    def decode_device(self, lappr_fi, synd_fi, B: int, max_iterations: int, final_fi=None, success=None,
                      iters=None, stream=None):
        """Decode B frames resident in HBM (torch tensors, frame-innermost).

        lappr_fi: float64 [V, ld]; synd_fi: uint8 [C, ld]; ld % 64 == 0, 0 < B <= ld.
        Returns (final_fi float64 [V, ld], success uint8 [B], iters int32 [B]).
        Every tensor must be contiguous and on this decoder's GPU (checked).
        Asynchronous on ``stream`` (default: torch's current stream).  The message
        workspace is kept per stream, so calls on different streams never share it."""
        import torch

        from ._lib import check_tensor

        dev = self._device
        if not isinstance(lappr_fi, torch.Tensor) or lappr_fi.dim() != 2:
            raise ValueError("decode_device: lappr_fi must be a 2-D tensor [V, ld]")
        V, ld = lappr_fi.shape
        if V != self._V:
            raise ValueError("decode_device: tensor shapes do not match the code")
        if ld % 64 or not 0 < int(B) <= ld:
            raise ValueError(f"decode_device: need ld % 64 == 0 and 0 < B <= ld (B={B}, ld={ld})")
        check_tensor(lappr_fi, "lappr_fi", (self._V, ld), torch.float64, dev)
        check_tensor(synd_fi, "synd_fi", (self._C, ld), torch.uint8, dev)
        tdev = lappr_fi.device
        if final_fi is None:
            final_fi = torch.empty_like(lappr_fi)
        if success is None:
            success = torch.empty(B, dtype=torch.uint8, device=tdev)
        if iters is None:
            iters = torch.empty(B, dtype=torch.int32, device=tdev)
        check_tensor(final_fi, "final_fi", (self._V, ld), torch.float64, dev)
        if success.numel() < B or iters.numel() < B:
            raise ValueError(f"decode_device: success/iters must hold at least B={B} entries")
        check_tensor(success, "success", (success.numel(),), torch.uint8, dev)
        check_tensor(iters, "iters", (iters.numel(),), torch.int32, dev)
        if stream is None:
            stream = torch.cuda.current_stream(tdev)
        ws = self._workspace(stream, self.workspace_bytes(ld, max_iterations))
        check(_lib.load().qr_decode_batch_device(
            self._h, int(B), int(ld), C.c_void_p(lappr_fi.data_ptr()), C.c_void_p(synd_fi.data_ptr()),
            int(max_iterations), C.c_void_p(final_fi.data_ptr()), C.c_void_p(success.data_ptr()),
            C.c_void_p(iters.data_ptr()), C.c_void_p(ws.data_ptr()), ws.numel(),
            C.c_void_p(stream.cuda_stream)), "decode_device")
        return final_fi, success, iters

    def repack_stats(self, ld: int, max_iterations: int, stream=None):
        """Column repack of the last decode_device on ``stream`` (same ld, max_iterations):
        ((repacks of range 0, repacks of range 1), (final width 0, final width 1)).  Waits
        for the device (a synchronous copy); call after the decode has completed."""
        import torch

        if stream is None:
            stream = torch.cuda.current_stream(torch.device("cuda", self._device))
        ws = self._ws.get(int(stream.cuda_stream))
        if ws is None:
            raise ValueError("repack_stats: no decode_device has run on this stream")
        out = (C.c_int32 * 4)()
        check(_lib.load().qr_decode_repack_stats(self._h, int(ld), int(max_iterations), C.c_void_p(ws.data_ptr()),
                                                 ws.numel(), out), "repack_stats")
        return (int(out[0]), int(out[1])), (int(out[2]), int(out[3]))

    #: how many per-stream workspaces a Decoder keeps (each is E*ld*8 bytes of messages)
    max_workspaces = 2

    def _workspace(self, stream, need: int):
        """Device workspace (c2v messages, flags) of the decodes issued on `stream`.
        Allocated on that stream, so torch's caching allocator orders its reuse after
        the work queued there; one per stream, so concurrent decodes never race.
        Keyed by the stream handle: torch's streams come from a per-device pool and
        live as long as the process, so a handle always names the same stream.  At
        most ``max_workspaces`` are kept (least recently used dropped first): a dropped
        workspace goes back to the caching allocator, which hands its memory out again
        only after the work already queued on its stream."""
        import torch

        key = int(stream.cuda_stream)
        ws = self._ws.pop(key, None)
        if ws is None or ws.numel() < need:
            ws = None  # free the smaller one before allocating
            while len(self._ws) >= max(1, int(self.max_workspaces)):
                self._ws.popitem(last=False)
            with torch.cuda.stream(stream):
                ws = torch.empty(need, dtype=torch.uint8, device=torch.device("cuda", self._device))
        self._ws[key] = ws
        return ws
