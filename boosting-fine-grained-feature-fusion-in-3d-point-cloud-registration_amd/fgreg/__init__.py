"""fgreg: MI355X-native per-pair registration forward of the fine-grained-fusion REGTR.

The compute path is libfgreg.so (HIP, gfx950) behind the C ABI in include/fgreg.h;
this package is the host-side mirror of the reference's model interface.
"""
from . import config, ops  # noqa: F401
from ._lib import FgrError, build, load  # noqa: F401
from .backbone import FixedMetaPreprocessor, KPFEncoder, PreprocessorHIP  # noqa: F401
from .pose import compute_rigid_transform, fast_compute_rigid_transform  # noqa: F401
from .regtr import RegTR  # noqa: F401
from .pipeline import pipeline  # noqa: F401

PRECISIONS = ('fp32', 'bf16')


def set_precision(precision):
    """Compute mode of every dense product and the attention:
    'fp32' (default): fp32-accurate f16x3 split products on the fp16 matrix cores;
    'bf16': one bf16 MFMA product per fp32 product, fp32 accumulation and storage (BASELINE
    configs[4], 3DLoMatch; tolerance against the fp32 oracle in DESIGN.md). The Res2Net
    chains and everything outside the GEMMs / attention stay fp32-accurate in both modes."""
    from . import linear
    assert precision in PRECISIONS, precision
    linear.set_mode('f16x3' if precision == 'fp32' else 'bf16')
    ops.ATTN_MODE = 'f16x3' if precision == 'fp32' else 'bf16'


def precision():
    from . import linear
    return 'bf16' if linear.MODE == 'bf16' else 'fp32'

__all__ = ['RegTR', 'PreprocessorHIP', 'FixedMetaPreprocessor', 'KPFEncoder', 'ops', 'config',
           'fast_compute_rigid_transform', 'compute_rigid_transform', 'build', 'load', 'FgrError',
           'set_precision', 'precision']
