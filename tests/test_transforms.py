"""Input side of the test step (fgreg.transforms).

Where the reference is mounted (this container), the ModelNet crop test pipeline is run
through the reference's own transform objects (data_loaders/modelnet_transforms.py, in the
order of data_loaders/modelnet.py:111-117) on the same raw clouds and sample indices, and
every output field must match exactly. Elsewhere only the shape / invariant checks run.
"""
import os
import sys

import numpy as np
import pytest
import torch

from fgreg import transforms as T
from fgreg.synthetic import _box_surface

REF = '/root/reference'


def _raw(i, normals=False):
    rng = np.random.default_rng(100 + i)
    p = _box_surface(rng, 2048).astype(np.float32)
    if normals:
        n = rng.normal(size=p.shape).astype(np.float32)
        p = np.concatenate([p, n / np.linalg.norm(n, axis=1, keepdims=True)], 1)
    return p


@pytest.mark.parametrize('i', [0, 7, 123])
def test_crop_pipeline_invariants(i):
    s = T.modelnet_crop_test(_raw(i), i)
    assert s['src_xyz'].shape == (717, 3) and s['tgt_xyz'].shape == (717, 3)
    assert s['pose'].shape == (3, 4) and s['tgt_raw'].shape == (2048, 3)
    c = s['correspondences'].numpy()
    assert c.shape[0] == 2 and (c >= 0).all() and c.shape[1] > 0
    # corresponding points agree up to the pose and the (clipped) jitter of both clouds
    R, t = s['pose'][:, :3].double(), s['pose'][:, 3].double()
    a = s['src_xyz'].double()[c[0]] @ R.T + t
    b = s['tgt_xyz'].double()[c[1]]
    assert float((a - b).abs().max()) < 0.1 + 1e-5
    # overlap flags: every corresponded point is in the overlap
    assert s['src_overlap'][c[0]].all() and s['tgt_overlap'][c[1]].all()
    # deterministic per index
    s2 = T.modelnet_crop_test(_raw(i), i)
    assert torch.equal(s['src_xyz'], s2['src_xyz'])


def test_collate_pair():
    batch = T.collate_pair([T.modelnet_crop_test(_raw(i), i) for i in range(3)])
    assert isinstance(batch['src_xyz'], list) and len(batch['src_xyz']) == 3
    assert batch['pose'].shape == (3, 3, 4)
    assert 'overlap_p' not in batch
    b2 = T.collate_pair([{'src_xyz': torch.zeros(2, 3), 'tgt_xyz': torch.zeros(3, 3),
                          'pose': torch.zeros(3, 4), 'overlap_p': 0.4, 'src_path': 'a'}])
    assert b2['overlap_p'].shape == (1,) and b2['src_path'] == ['a']


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, 'data_loaders')),
                    reason='reference checkout not mounted (GPU box)')
@pytest.mark.parametrize('i,normals', [(0, False), (5, False), (42, True)])
def test_crop_pipeline_matches_reference(i, normals, monkeypatch):
    monkeypatch.syspath_prepend(REF)
    sys.dont_write_bytecode = True
    import importlib.util
    # the file alone: data_loaders/__init__ pulls in h5py / torchvision (absent here)
    spec = importlib.util.spec_from_file_location(
        'ref_modelnet_transforms', os.path.join(REF, 'data_loaders', 'modelnet_transforms.py'))
    mt = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mt)
    steps = [mt.SetDeterministic(), mt.SplitSourceRef(), mt.RandomCrop([0.7, 0.7]),
             mt.RandomTransformSE3_euler(rot_mag=45.0, trans_mag=0.5), mt.Resampler(1024),
             mt.RandomJitter(), mt.ShufflePoints()]
    raw = _raw(i, normals)
    sample = {'points': raw.copy(), 'label': 0, 'idx': np.array(i, dtype=np.int32)}
    for st in steps:
        sample = st(sample)
    got = T.modelnet_crop_test(raw.copy(), i)
    np.testing.assert_array_equal(got['src_xyz'].numpy(), sample['points_src'][:, :3])
    np.testing.assert_array_equal(got['tgt_xyz'].numpy(), sample['points_ref'][:, :3])
    np.testing.assert_array_equal(got['tgt_raw'].numpy(), sample['points_raw'][:, :3])
    np.testing.assert_array_equal(got['pose'].numpy(), sample['transform_gt'])
    np.testing.assert_array_equal(got['correspondences'].numpy(), sample['correspondences'])
    np.testing.assert_array_equal(got['src_overlap'].numpy(), sample['src_overlap'])
    np.testing.assert_array_equal(got['tgt_overlap'].numpy(), sample['ref_overlap'])


@pytest.mark.parametrize('n', [2, 1100, 2048, 4096])
@pytest.mark.parametrize('p', [0.7, 0.55, 0.9])
def test_crop_rank_reproduces_percentile(n, p):
    """transforms_gpu._crop_rank: NumPy's own (k, gamma) of the 'linear' percentile, so the
    GPU threshold _lerp(s_k, s_k+1, gamma) equals np.percentile (with ties, too)."""
    from fgreg.transforms_gpu import _crop_rank
    rng = np.random.default_rng(n)
    p = np.float32(p)
    k, g = _crop_rank(n, p)
    for d in (rng.standard_normal(n), np.round(rng.standard_normal(n), 1)):
        s = np.sort(d)
        a, b = s[k], s[min(k + 1, n - 1)]
        diff = b - a
        th = b - diff * (1.0 - g) if g >= 0.5 else a + diff * g
        assert th == np.percentile(d, (1.0 - p) * 100)


def test_gpu_crop_upload_packing():
    """transforms_gpu._upload: several tables in one host-to-device copy, typed views intact
    (run on the CPU device here; the GPU tests use it on cuda)."""
    from fgreg.transforms_gpu import _upload
    rng = np.random.default_rng(0)
    arrs = (np.arange(5, dtype=np.int64), rng.random((2, 2, 3)), np.array([1, 2, 3], np.int32),
            rng.random((3, 3, 4)).astype(np.float32))
    out = _upload(torch.device('cpu'), *arrs)
    for o, a in zip(out, arrs):
        assert o.shape == a.shape and torch.equal(o, torch.from_numpy(a))
        assert o.data_ptr() % 16 == 0
