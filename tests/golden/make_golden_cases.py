"""Case tables shared by tests/golden/make_golden.py (which ran them through the reference)
and the tests that read the fixtures back (pure data; importable without the reference)."""
import numpy as np

NOISE_SEARCH_CASES = (  # (bps, snr dB, probabilities or None) of noise_search.npz
    (1, 2.0, None), (2, 3.0, None), (2, 9.5, None), (2, 4.0, (0.1, 0.4, 0.3, 0.2)), (3, 8.0, None),
    (4, 13.0, None), (4, 25.0, None))
NOISE_SEARCH_ACC = (1e-6, 1e-9, 1e-12)


def alternating(M):
    cfg = np.zeros(M, np.uint8)
    cfg[1::2] = 1  # sim_reconciliation.py:84-86
    return cfg
