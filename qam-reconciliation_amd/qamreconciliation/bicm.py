"""qamreconciliation.bicm (bicm.pyx:26-66): reflected-Gray symbol -> bits tables."""
from qamr.alphabet import generate_error_number_table, generate_table_s_to_b  # noqa: F401

__all__ = ["generate_table_s_to_b", "generate_error_number_table"]
