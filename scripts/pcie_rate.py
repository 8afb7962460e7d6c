#!/usr/bin/env python3
"""PCIe-inclusive decode rate (the drop-in host path, qr_decode_host: pageable numpy
in/out, H2D + transposes + decode + D2H) next to the HBM-resident device path, for the
headline workload (N=64800, B=4096, 50 iterations, 3.0 dB)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qam-reconciliation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import qamr  # noqa: E402
from qamr import codes  # noqa: E402
from qamr.pipeline import SofteningPipeline  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
vid, cid = codes.dvbs2_like_half()
dec = qamr.Decoder(vid, cid)
pipe = SofteningPipeline(dec, 2, 3.0, batch=B, max_iterations=50)
b = pipe.generate(torch.Generator(device="cuda").manual_seed(0))
lap = pipe.demap(b)
L = lap[:, :B].T.contiguous().cpu().numpy()
S = b.synd[:, :B].T.contiguous().cpu().numpy()
dec.decode_batch(L[:64], S[:64], 50)                      # warm (scratch allocation)
fin, su, it = dec.decode_device(lap, b.synd, B, 50)
torch.cuda.synchronize()
t0 = time.perf_counter()
fin, su, it = dec.decode_device(lap, b.synd, B, 50)
torch.cuda.synchronize()
t_dev = time.perf_counter() - t0
t0 = time.perf_counter()
s2, i2, f2 = dec.decode_batch(L, S, 50)
t_host = time.perf_counter() - t0
assert np.array_equal(s2, su.cpu().numpy()) and np.array_equal(i2, it.cpu().numpy())
gb = (L.nbytes * 2 + S.nbytes) / 1e9
print(f"B={B}: device path {t_dev * 1e3:.1f} ms ({B / t_dev:.0f} frames/s); host path incl. PCIe "
      f"{t_host * 1e3:.1f} ms ({B / t_host:.0f} frames/s, {gb:.2f} GB moved over PCIe)")
