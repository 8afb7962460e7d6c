"""Drop-in import name: ``from qamreconciliation import Decoder, Matrix,
NoiseMapper, PAMAlphabet`` (the reference's qamreconciliation/__init__.py:1-4)
resolves to the MI355X implementation in ``qamr``."""
from qamr import Decoder, Matrix, NoiseDemapper, NoiseMapper, PAMAlphabet  # noqa: F401
from qamr.utils import count_errors_from_lappr  # noqa: F401
