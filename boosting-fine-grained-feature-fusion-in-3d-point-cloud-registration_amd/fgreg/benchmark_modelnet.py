"""The ModelNet evaluation metrics of the test step on the GPU: a drop-in for the reference's
benchmark/benchmark_modelnet.py (compute_metrics :33-82, summarize_metrics :85-97,
print_metrics :100-121), which GenericRegModel.test_step calls on the last layer's pose
(models/generic_reg_model.py:138-147) and test_epoch_end summarises (:184-190).

compute_metrics runs fgr_modelnet_metrics (csrc/metrics.hip): the modified Chamfer distance's
two N x M row-minima over the raw cloud in one launch, the Euler / isotropic pose errors and the
per-pair means in a second. Same keys, shapes and dtypes as the reference (r_mse / r_mae
float64, the rest float32); GPU tensors only (no CPU path, like the rest of fgreg).
"""
import numpy as np
import torch

from . import _lib, ops
from .ops import _dev, _ptr, _stream

KEYS = ('r_mse', 'r_mae', 't_mse', 't_mae', 'err_r_deg', 'err_t', 'chamfer_dist')


def _xyz(t):
    return t[..., :3].float().contiguous()


def compute_metrics(data, pred_transforms):
    """benchmark_modelnet.py:33-82: data = {'points_src' (B, N, >=3), 'points_ref' (B, N, >=3),
    'points_raw' (B, R, >=3), 'transform_gt' (B, 3, 4)}, pred_transforms (B, 3, 4) -> dict of
    (B,) numpy arrays."""
    src, ref, raw = _xyz(data['points_src']), _xyz(data['points_ref']), _xyz(data['points_raw'])
    gt = data['transform_gt'][:, :3, :4].float().contiguous()
    pred = pred_transforms[:, :3, :4].float().contiguous()
    _dev(src, ref, raw, gt, pred)
    B, N = src.shape[0], src.shape[1]
    assert ref.shape == src.shape and raw.shape[0] == B and gt.shape == (B, 3, 4) \
        and pred.shape == (B, 3, 4), 'compute_metrics: inconsistent batch shapes'
    with torch.no_grad():
        out = torch.empty((B, 7), dtype=torch.float64, device=src.device)
        nb = _lib.ws_size('fgr_modelnet_metrics_workspace', B, N)
        ws = ops._workspace(src.device, nb)
        _lib.check(_lib.load().fgr_modelnet_metrics(
            _ptr(pred), _ptr(gt), _ptr(src), _ptr(ref), _ptr(raw), B, N, raw.shape[1], _ptr(ws),
            nb, _ptr(out), _stream()), 'fgr_modelnet_metrics')
        o = out.cpu().numpy()
    res = {}
    for j, k in enumerate(KEYS):
        res[k] = o[:, j] if k in ('r_mse', 'r_mae') else o[:, j].astype(np.float32)
    return res


def summarize_metrics(metrics):
    """benchmark_modelnet.py:85-97: means over all instances (rmse for the *mse keys, mean and
    rmse for the err* keys)."""
    out = {}
    for k, v in metrics.items():
        v = np.asarray(v)
        if k.endswith('mse'):
            out[k[:-3] + 'rmse'] = np.sqrt(np.mean(v))
        elif k.startswith('err'):
            out[k + '_mean'] = np.mean(v)
            out[k + '_rmse'] = np.sqrt(np.mean(v ** 2))
        else:
            out[k] = np.mean(v)
    return out


def print_metrics(logger, summary_metrics, losses_by_iteration=None, title='Metrics'):
    """benchmark_modelnet.py:100-121: the same log lines."""
    s = summary_metrics
    logger.info(title + ':')
    logger.info('=' * (len(title) + 1))
    if losses_by_iteration is not None:
        logger.info('Losses by iteration: ' + ' | '.join(f'{c:.5f}' for c in losses_by_iteration))
    logger.info(f"DeepCP metrics:{s['r_rmse']:.4f}(rot-rmse) | {s['r_mae']:.4f}(rot-mae) | "
                f"{s['t_rmse']:.4g}(trans-rmse) | {s['t_mae']:.4g}(trans-mae)")
    logger.info(f"Rotation error {s['err_r_deg_mean']:.4f}(deg, mean) | "
                f"{s['err_r_deg_rmse']:.4f}(deg, rmse)")
    logger.info(f"Translation error {s['err_t_mean']:.4g}(mean) | {s['err_t_rmse']:.4g}(rmse)")
    logger.info(f"Chamfer error: {s['chamfer_dist']:.7f}(mean-sq)")
