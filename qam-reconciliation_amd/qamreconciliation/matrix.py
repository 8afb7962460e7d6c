"""qamreconciliation.matrix (matrix.pyx:20): parity-check matrix / syndrome."""
from qamr.matrix import Matrix  # noqa: F401

__all__ = ["Matrix"]
