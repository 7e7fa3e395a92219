"""fgreg: MI355X-native per-pair registration forward of the fine-grained-fusion REGTR.

The compute path is libfgreg.so (HIP, gfx950) behind the C ABI in include/fgreg.h;
this package is the host-side mirror of the reference's model interface.
"""
from . import config, ops  # noqa: F401
from ._lib import FgrError, build, load  # noqa: F401
from .backbone import FixedMetaPreprocessor, KPFEncoder, PreprocessorHIP  # noqa: F401
from .pose import compute_rigid_transform, fast_compute_rigid_transform  # noqa: F401
from .regtr import RegTR  # noqa: F401

__all__ = ['RegTR', 'PreprocessorHIP', 'FixedMetaPreprocessor', 'KPFEncoder', 'ops', 'config',
           'fast_compute_rigid_transform', 'compute_rigid_transform', 'build', 'load', 'FgrError']
