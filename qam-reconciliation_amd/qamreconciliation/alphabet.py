"""qamreconciliation.alphabet (alphabet.pyx:25-107): PAM constellation tables."""
from qamr.alphabet import Alphabet, PAMAlphabet  # noqa: F401

__all__ = ["Alphabet", "PAMAlphabet"]
