"""TEST INFRASTRUCTURE ONLY (tests/): CPU restatement of the reference's overlap computation,
utils/pointcloud.py:8-66 (Open3D KDTreeFlann radius search, first = nearest hit), with scipy's
cKDTree: nearest neighbour within the radius in each direction, mutual correspondences with
the reference's `src_corr > 0` condition. Exact-distance ties (absent in random float data)
are the only case where Open3D's kd-tree order could differ."""
import numpy as np
from scipy.spatial import cKDTree


def _nearest_within(q, s, radius):
    d, i = cKDTree(s).query(q, k=1, distance_upper_bound=radius)
    # strict d < r as the GPU kernels (d^2 < r^2); cKDTree's bound is d <= r
    hit = np.isfinite(d) & (d * d < np.float32(radius) * np.float32(radius))
    return np.where(hit, i, -1)


def compute_overlap(src, tgt, radius):
    tgt_corr = _nearest_within(tgt, src, radius)
    src_corr = _nearest_within(src, tgt, radius)
    mutual = np.logical_and(tgt_corr[src_corr] == np.arange(len(src_corr)), src_corr > 0)
    src_tgt_corr = np.stack([np.nonzero(mutual)[0], src_corr[mutual]])
    return src_corr >= 0, tgt_corr >= 0, src_tgt_corr
