"""qamreconciliation.decoder (decoder.pyx:92): the gfx950 sum-product decoder."""
from qamr.decoder import Decoder  # noqa: F401

__all__ = ["Decoder"]
