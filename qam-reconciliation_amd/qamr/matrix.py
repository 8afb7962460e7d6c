"""Drop-in ``Matrix`` (matrix.pyx:20-60): the syndrome producer of the
softening pipeline.  ``eval_syndrome`` runs the frame-innermost XOR kernel of
libqamr (bit-exact integer work); ``eval_syndrome_device`` does it for a
batch resident in HBM."""
from __future__ import annotations

import numpy as np

from .decoder import Decoder, _as_buffer


class Matrix:
    def __init__(self, vnode_array, cnode_array, device: int = 0):
        vid = _as_buffer(vnode_array, np.int64, "vnode_array", "long")
        cid = _as_buffer(cnode_array, np.int64, "cnode_array", "long")
        if vid.shape[0] != cid.shape[0]:
            raise ValueError("Incompatible sizes for input vectors")  # matrix.pyx:22-23
        self._code = Decoder(vid, cid, device=device)
        self.vnum = self._code.vnum
        self.cnum = self._code.cnum
        self.ednum = self._code.ednum

    @property
    def code(self) -> Decoder:
        return self._code

    def eval_syndrome(self, word):
        """matrix.pyx:55-60: synd[cid[e]] ^= word[vid[e]]."""
        w = _as_buffer(word, np.uint8, "word", "unsigned char")
        if w.size != self.vnum:
            raise ValueError("Size of word does not match number of vnodes")
        # one frame: lane = check node (the node-level surface, qr_check_word_host): against
        # an all-zero syndrome each check reports (XOR of its word bytes) ^ 1
        ok, _ = self._code._check_word_flags(w, np.zeros(self.cnum, np.uint8))
        return ok ^ np.uint8(1)

    def eval_syndrome_device(self, word_fi, B: int, stream=None):
        """word_fi uint8 [V, ld] -> synd uint8 [C, ld]."""
        import ctypes as C

        import torch

        from . import _lib

        if not isinstance(word_fi, torch.Tensor) or word_fi.dim() != 2:
            raise ValueError("eval_syndrome_device: word_fi must be a 2-D tensor [V, ld]")
        V, ld = word_fi.shape
        if ld % 64 or not 0 < int(B) <= ld:
            raise ValueError(f"eval_syndrome_device: need ld % 64 == 0 and 0 < B <= ld (B={B}, ld={ld})")
        _lib.check_tensor(word_fi, "word_fi", (self.vnum, ld), torch.uint8, self._code.device)
        out = torch.empty((self.cnum, ld), dtype=torch.uint8, device=word_fi.device)
        if stream is None:
            stream = torch.cuda.current_stream(word_fi.device)
        _lib.check(_lib.load().qr_syndrome_device(self._code.handle, int(B), int(ld), C.c_void_p(word_fi.data_ptr()),
                                                  C.c_void_p(out.data_ptr()), C.c_void_p(stream.cuda_stream)),
                   "eval_syndrome_device")
        return out
