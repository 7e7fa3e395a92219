"""The ModelNet test-step metrics on the GPU (fgreg.benchmark_modelnet, fgr_modelnet_metrics;
benchmark/benchmark_modelnet.py:33-97) against the reference's own outputs
(tests/golden/modelnet_metrics.npz, written by the reference's compute_metrics /
summarize_metrics) and against oracle/metrics_oracle.py on larger batches: raw clouds of
2048 / 3000 / 5000 points (one or several 2048-point LDS stages), ragged poses incl. an exact
prediction and 180-degree-scale rotations."""
import logging

import numpy as np
import pytest
import torch

import metrics_oracle as mt
from conftest import golden
from test_oracle import check_modelnet_metrics

pytestmark = pytest.mark.gpu


def _run(gpu, src, ref, raw, gt, pred):
    from fgreg import benchmark_modelnet as bm
    data = {'points_src': torch.from_numpy(src).to(gpu), 'points_ref': torch.from_numpy(ref).to(gpu),
            'points_raw': torch.from_numpy(raw).to(gpu), 'transform_gt': torch.from_numpy(gt).to(gpu)}
    return bm.compute_metrics(data, torch.from_numpy(pred).to(gpu))


def test_metrics_vs_reference_fixture(gpu):
    from fgreg import benchmark_modelnet as bm
    g = golden('modelnet_metrics')
    m = _run(gpu, g['points_src'], g['points_ref'], g['points_raw'], g['transform_gt'],
             g['pred_transforms'])
    ref_m = {k[2:]: g[k] for k in g.files if k.startswith('m_')}
    assert set(m) == set(ref_m)
    for k in m:
        assert m[k].dtype == ref_m[k].dtype, k
    check_modelnet_metrics(m, ref_m, rel=1e-4)
    # the Euler errors see the same fp32 matrices as scipy: far tighter than the bound
    for k in ('r_mse', 'r_mae'):
        assert np.allclose(m[k], ref_m[k], rtol=1e-9, atol=1e-9), k
    s = bm.summarize_metrics(m)
    for k in s:
        assert np.allclose(s[k], g['s_' + k], rtol=1e-4, atol=1e-4), k
    bm.print_metrics(logging.getLogger('test'), s)


@pytest.mark.parametrize('n_raw', [2048, 3000, 5000])
def test_metrics_vs_oracle(gpu, n_raw):
    from scipy.spatial.transform import Rotation
    rng = np.random.default_rng(n_raw)
    B, N = 5, 717
    gt = np.zeros((B, 3, 4), np.float32)
    pred = np.zeros((B, 3, 4), np.float32)
    for b in range(B):
        rg = Rotation.random(random_state=int(rng.integers(1 << 30)))
        gt[b, :, :3] = rg.as_matrix()
        gt[b, :, 3] = rng.uniform(-1, 1, 3)
        rp = Rotation.from_rotvec(rng.normal(size=3) * (0.05 if b < 3 else 1.0)) * rg
        pred[b, :, :3] = rp.as_matrix()
        pred[b, :, 3] = gt[b, :, 3] + rng.uniform(-0.1, 0.1, 3)
    pred[0] = gt[0]
    raw = rng.uniform(-1, 1, (B, n_raw, 3)).astype(np.float32)
    src = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    ref = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    m = _run(gpu, src, ref, raw, gt, pred)
    o = mt.compute_metrics(src, ref, raw, gt, pred)
    check_modelnet_metrics(m, o, rel=1e-4)
