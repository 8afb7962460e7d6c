"""qamr -- MI355X-native (gfx950) LDPC syndrome decoder and PAM/BICM soft
demapper: a drop-in for the hot path of moriglia/qam-reconciliation
(``Decoder.decode`` and ``NoiseMapper.demap_lappr_array``) backed by
hand-written HIP kernels in libqamr.so (C-ABI: include/qamr.h).

There is no CPU fallback: constructing a Decoder/NoiseMapper/Matrix without a
HIP device raises.
"""
from . import codes
from ._lib import (QamrError, build, device_count, load, profile_enable, profile_query, profile_reset,
                   profile_select)
from .alphabet import Alphabet, PAMAlphabet, generate_table_s_to_b
from .decoder import Decoder
from .matrix import Matrix
from .noisemapper import NoiseDemapper, NoiseMapper
from .utils import count_errors_from_lappr

__all__ = ["Decoder", "Matrix", "NoiseMapper", "NoiseDemapper", "PAMAlphabet", "Alphabet", "codes",
           "count_errors_from_lappr", "generate_table_s_to_b", "build", "load", "device_count", "QamrError",
           "profile_enable", "profile_query", "profile_reset", "profile_select"]
