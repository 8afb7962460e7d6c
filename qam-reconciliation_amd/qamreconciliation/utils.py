"""qamreconciliation.utils (utils.pyx:18-40)."""
from qamr.utils import count_errors_from_lappr, dist_cut  # noqa: F401

__all__ = ["dist_cut", "count_errors_from_lappr"]
