"""qamreconciliation.noisemapper (noisemapper.pyx:102-816).

``NoiseMapper`` / ``NoiseDemapper`` are the MI355X implementation.  The sign-flip
variants (noisemapper.pyx:775-816: they override ``g``/``g_inv`` with a half-order
flip rule, while ``demap_lappr`` still follows ``sign_config``) are not on the
reconciliation hot path and are out of scope: they import,
so ``from qamreconciliation import *`` works, but constructing one raises."""
from qamr.noisemapper import F_Z, NoiseDemapper, NoiseMapper, view_dist_cut  # noqa: F401

# the reference's module-level cpdef (noisemapper.pyx:90); no name mangling at module level
globals()["__view_dist_cut"] = view_dist_cut

__all__ = ["NoiseMapper", "NoiseDemapper", "NoiseMapperFlipSign", "NoiseMapperAntiFlipSign", "F_Z"]


class _OutOfScope(NoiseMapper):
    def __init__(self, *args, **kwargs):
        raise NotImplementedError(
            f"{type(self).__name__} (noisemapper.pyx:775-816) is out of scope of the MI355X build: "
            "only NoiseMapper's softening path (demap_lappr_array) is implemented")

    def __del__(self):
        pass


class NoiseMapperFlipSign(_OutOfScope):
    """noisemapper.pyx:775-795 -- out of scope (raises at construction)."""


class NoiseMapperAntiFlipSign(_OutOfScope):
    """noisemapper.pyx:798-816 -- out of scope (raises at construction)."""
