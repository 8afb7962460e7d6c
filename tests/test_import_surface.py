"""The drop-in import surface: the reference's own import lines resolve to the MI355X
implementation (no GPU needed to import; constructing the GPU classes needs one)."""
import pytest


def test_reference_package_init_names():
    # qamreconciliation/__init__.py:1-4
    from qamreconciliation.decoder import Decoder
    from qamreconciliation.matrix import Matrix
    from qamreconciliation.noisemapper import (NoiseMapper, NoiseDemapper, NoiseMapperFlipSign,
                                               NoiseMapperAntiFlipSign)
    from qamreconciliation.alphabet import PAMAlphabet
    import qamr

    assert Decoder is qamr.Decoder and Matrix is qamr.Matrix
    assert NoiseMapper is qamr.NoiseMapper and NoiseDemapper is qamr.NoiseDemapper
    assert PAMAlphabet is qamr.PAMAlphabet
    assert issubclass(NoiseMapperFlipSign, NoiseMapper) and issubclass(NoiseMapperAntiFlipSign, NoiseMapper)


def test_reference_caller_import_lines():
    from qamreconciliation import Decoder  # test/test_decoder.py:1
    from qamreconciliation.decoder import Decoder as CyDecoder  # sims/sim_decode.py:11, sim_direct.py:10
    from qamreconciliation import bicm, alphabet, NoiseMapper  # sims/display_softened.py:20
    from qamreconciliation.alphabet import PAMAlphabet  # sims/sim_montecarlo_information.py:7
    from qamreconciliation.noisemapper import NoiseMapper as NM  # sims/sim_montecarlo_information.py:8
    from qamreconciliation.utils import count_errors_from_lappr  # sims/reconciliation.pyx:18 (cimport)

    assert CyDecoder is Decoder and NM is NoiseMapper
    assert alphabet.PAMAlphabet is PAMAlphabet
    t = bicm.generate_table_s_to_b(2)
    assert t.tolist() == [[0, 0], [1, 0], [1, 1], [0, 1]]
    assert count_errors_from_lappr([1.0, -1.0, 0.0], [0, 0, 1]) == 2


def test_flip_sign_variants_are_out_of_scope():
    from qamreconciliation import NoiseMapperAntiFlipSign, NoiseMapperFlipSign, PAMAlphabet

    pa = PAMAlphabet(2, 2.0)
    for cls in (NoiseMapperFlipSign, NoiseMapperAntiFlipSign):
        with pytest.raises(NotImplementedError, match="out of scope"):
            cls(pa, 0.5)
