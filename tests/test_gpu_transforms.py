"""GPU parity of the ModelNet crop test pipeline (fgreg/transforms_gpu.py on csrc/crop.hip,
SURVEY.md §8(f) row 3).

The checker is the host pipeline `fgreg.transforms.modelnet_crop_test`, itself pinned field
for field to the reference's transform objects (data_loaders/modelnet_transforms.py, chained
as data_loaders/modelnet.py:111-117) by tests/test_transforms.py. Every output field must be
EQUAL: coordinates bit for bit (the kernels repeat NumPy's float32 evaluation order), masks,
overlap flags and correspondences exactly. Cases: the reference's p = 0.7 two-cloud crop and
the p = 0.5 rule, raw clouds with normals (6 columns), ragged batches (1500 / 2048 / 4096-
point raw clouds in one call), duplicated points (equal projections: ties at the percentile),
and the size guards.
"""
import numpy as np
import pytest
import torch

from fgreg import transforms as T
from fgreg import transforms_gpu as TG
from fgreg.synthetic import _box_surface

pytestmark = pytest.mark.gpu


def _raw(i, n=2048, normals=False, dup=False):
    rng = np.random.default_rng(100 + i)
    p = _box_surface(rng, n).astype(np.float32)
    if dup:                                     # every point twice: ties everywhere
        p = np.concatenate([p[: n // 2], p[: n // 2]])
    if normals:
        nv = rng.normal(size=p.shape).astype(np.float32)
        p = np.concatenate([p, nv / np.linalg.norm(nv, axis=1, keepdims=True)], 1)
    return p


def _check(got, want):
    for k in ('src_xyz', 'tgt_xyz', 'tgt_raw', 'src_overlap', 'tgt_overlap', 'correspondences',
              'pose', 'idx'):
        g, w = got[k], want[k]
        assert g.dtype == w.dtype, (k, g.dtype, w.dtype)
        assert g.shape == w.shape, (k, g.shape, w.shape)
        assert torch.equal(g.cpu(), w), k
    assert got['src_xyz'].is_cuda and got['correspondences'].is_cuda


@pytest.mark.parametrize('normals', [False, True])
def test_crop_batch_equals_host(normals):
    idx = [0, 5, 42, 123, 7, 999, 31337, 2**31 - 1]
    raws = [_raw(i, normals=normals) for i in idx]
    got = TG.modelnet_crop_test_gpu(raws, idx)
    for r, i, g in zip(raws, idx, got):
        _check(g, T.modelnet_crop_test(r.copy(), i))


def test_crop_ragged_and_ties():
    idx = [3, 4, 5, 6]
    raws = [_raw(3, 1500), _raw(4, 4096), _raw(5, 2048, dup=True), _raw(6, 1100)]
    got = TG.modelnet_crop_test_gpu(raws, idx)
    for r, i, g in zip(raws, idx, got):
        _check(g, T.modelnet_crop_test(r.copy(), i))


def test_crop_half():
    idx = [11, 12]
    raws = [_raw(i) for i in idx]
    got = TG.modelnet_crop_test_gpu(raws, idx, p_keep=(0.5, 0.5))
    for r, i, g in zip(raws, idx, got):
        _check(g, T.modelnet_crop_test(r.copy(), i, p_keep=(0.5, 0.5)))


def test_crop_from_device_tensors_and_collate():
    idx = [1, 2]
    raws = [_raw(i) for i in idx]
    b = TG.modelnet_crop_batch_gpu([torch.from_numpy(r).cuda() for r in raws], idx)
    want = T.collate_pair([T.modelnet_crop_test(r.copy(), i) for r, i in zip(raws, idx)])
    assert torch.equal(b['pose'].cpu(), want['pose'])
    for k in ('src_xyz', 'tgt_xyz', 'correspondences'):
        for g, w in zip(b[k], want[k]):
            assert torch.equal(g.cpu(), w), k


def test_crop_guards():
    with pytest.raises(NotImplementedError):
        TG.modelnet_crop_test_gpu([_raw(0, 4097)], [0])
    with pytest.raises(NotImplementedError):          # crop keeps < 717 points
        TG.modelnet_crop_test_gpu([_raw(0, 900)], [0])
    with pytest.raises(NotImplementedError):
        TG.modelnet_crop_test_gpu([_raw(0)], [0], p_keep=(0.7,))
