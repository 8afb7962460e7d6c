"""Drop-in import name for the reference package (qamreconciliation/__init__.py:1-4):

    from qamreconciliation import Decoder, Matrix, NoiseMapper, PAMAlphabet
    from qamreconciliation.decoder import Decoder          # sims/sim_decode.py:11
    from qamreconciliation import bicm, alphabet           # sims/display_softened.py:20

all resolve to the MI355X implementation in ``qamr``.  The sign-flip NoiseMapper
variants are importable (the reference exports them) but out of scope (SURVEY.md
section 2): constructing one raises NotImplementedError."""
from .decoder import Decoder  # noqa: F401
from .matrix import Matrix  # noqa: F401
from .noisemapper import NoiseMapper, NoiseDemapper, NoiseMapperFlipSign, NoiseMapperAntiFlipSign  # noqa: F401
from .alphabet import PAMAlphabet  # noqa: F401
from . import alphabet, bicm, decoder, matrix, noisemapper, utils  # noqa: F401
from .utils import count_errors_from_lappr  # noqa: F401
