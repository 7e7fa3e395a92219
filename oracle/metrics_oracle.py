"""CPU restatement of the reference's ModelNet evaluation metrics -- TEST INFRASTRUCTURE ONLY.

Only tests/ may import this (it is the checker of fgreg/benchmark_modelnet.py). Pinned against
the reference itself: tests/golden/modelnet_metrics.npz holds the reference's own
compute_metrics / summarize_metrics outputs (tests/golden/make_golden.py make_modelnet_metrics),
checked by tests/test_oracle.py::test_metrics_oracle_matches_reference.

Restated (NumPy, float64; the Euler angles through scipy, the reference's own dependency):
* compute_metrics     benchmark/benchmark_modelnet.py:33-82
* summarize_metrics   benchmark/benchmark_modelnet.py:85-97
"""
import numpy as np
from scipy.spatial.transform import Rotation


def _euler_xyz(R):
    """dcm2euler(seq='xyz'), benchmark_modelnet.py:14-30."""
    return np.stack([Rotation.from_matrix(r).as_euler('xyz', degrees=True) for r in R])


def _inv(P):
    R, t = P[:, :, :3], P[:, :, 3:]
    Ri = np.transpose(R, (0, 2, 1))
    return np.concatenate([Ri, -Ri @ t], 2)


def _cat(A, B):
    return np.concatenate([A[:, :, :3] @ B[:, :, :3], A[:, :, :3] @ B[:, :, 3:] + A[:, :, 3:]], 2)


def _apply(P, x):
    return x @ np.transpose(P[:, :, :3], (0, 2, 1)) + P[:, None, :, 3]


def _min_sq(a, b):
    """min over b of |a_i - b_j|^2 (square_distance then min, :37-38, :68-69)."""
    out = np.empty(a.shape[:2])
    for i in range(a.shape[0]):
        d = ((a[i][:, None, :] - b[i][None, :, :]) ** 2).sum(-1)
        out[i] = d.min(1)
    return out


def compute_metrics(points_src, points_ref, points_raw, transform_gt, pred_transforms):
    """benchmark_modelnet.py:33-82 on arrays (B, N, 3), (B, N, 3), (B, R, 3), (B, 3, 4),
    (B, 3, 4) -> the same dict of per-pair arrays."""
    src, ref, raw = (np.asarray(a, np.float64)[..., :3] for a in (points_src, points_ref, points_raw))
    gt, pred = np.asarray(transform_gt, np.float32), np.asarray(pred_transforms, np.float32)
    r_gt, r_pred = _euler_xyz(gt[:, :3, :3]), _euler_xyz(pred[:, :3, :3])
    gt, pred = gt.astype(np.float64), pred.astype(np.float64)
    t_gt, t_pred = gt[:, :3, 3], pred[:, :3, 3]
    conc = _cat(_inv(gt), pred)
    tr = conc[:, 0, 0] + conc[:, 1, 1] + conc[:, 2, 2]
    err_r = np.degrees(np.arccos(np.clip(0.5 * (tr - 1), -1.0, 1.0)))
    err_t = np.linalg.norm(conc[:, :, 3], axis=-1)
    src_t = _apply(pred, src)
    src_clean = _apply(_cat(pred, _inv(gt)), raw)
    chamfer = _min_sq(src_t, raw).mean(1) + _min_sq(ref, src_clean).mean(1)
    return {'r_mse': np.mean((r_gt - r_pred) ** 2, axis=1),
            'r_mae': np.mean(np.abs(r_gt - r_pred), axis=1),
            't_mse': np.mean((t_gt - t_pred) ** 2, axis=1),
            't_mae': np.mean(np.abs(t_gt - t_pred), axis=1),
            'err_r_deg': err_r, 'err_t': err_t, 'chamfer_dist': chamfer}


def summarize_metrics(metrics):
    """benchmark_modelnet.py:85-97."""
    out = {}
    for k in metrics:
        if k.endswith('mse'):
            out[k[:-3] + 'rmse'] = np.sqrt(np.mean(metrics[k]))
        elif k.startswith('err'):
            out[k + '_mean'] = np.mean(metrics[k])
            out[k + '_rmse'] = np.sqrt(np.mean(metrics[k] ** 2))
        else:
            out[k] = np.mean(metrics[k])
    return out
