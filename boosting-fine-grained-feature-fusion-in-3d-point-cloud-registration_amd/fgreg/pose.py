"""Weighted Procrustes, the drop-in for utils/se3_torch.py's solvers (fgr_procrustes)."""
import torch

from . import ops

_EPS = 1e-6


def fast_compute_rigid_transform(a: torch.Tensor, b: torch.Tensor, weights: torch.Tensor = None,
                                 weights_threshold=0.85):
    """utils/se3_torch.py:226-273: T ([*,] 3, 4) with T*a = b.

    Like the reference, ``weights`` is thresholded IN PLACE (entries <= threshold
    become 0, :240-242) before the solve.
    """
    assert a.shape == b.shape and a.shape[-1] == 3
    if weights is None:
        weights = torch.ones(a.shape[:-1], dtype=a.dtype, device=a.device)
        return ops.procrustes(a, b, weights, threshold=None)
    assert a.shape[:-1] == weights.shape
    weights.masked_fill_(~(weights > weights_threshold), 0.0)
    return ops.procrustes(a, b, weights, threshold=None)


def compute_rigid_transform(a: torch.Tensor, b: torch.Tensor, weights: torch.Tensor = None):
    """utils/se3_torch.py:131-173 (no threshold; uniform weights when None)."""
    assert a.shape == b.shape and a.shape[-1] == 3
    if weights is None:
        weights = torch.ones(a.shape[:-1], dtype=a.dtype, device=a.device)
    return ops.procrustes(a, b, weights, threshold=None)
