"""Input side on the GPU: compute_overlap (utils/pointcloud.py:8-66) and
the ThreeDMatchDataset-shaped pair loader (threedmatch.py:65-107) vs the CPU restatement
oracle/data_oracle.py on synthetic fragments."""
import os

import numpy as np
import pytest
import torch

import data_oracle as do

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('n,radius', [(2000, 0.05), (20000, 0.0375), (300, 0.2)])
def test_compute_overlap_vs_oracle(gpu, n, radius):
    from fgreg import data
    from fgreg.synthetic import lowoverlap_pair
    src, tgt, pose, _ = lowoverlap_pair(3, n_points=n)
    sw = (src.astype(np.float64) @ pose[:, :3].T.astype(np.float64) + pose[:, 3]).astype(np.float32)
    sm, tm, corr = data.compute_overlap(torch.from_numpy(sw).to(gpu), torch.from_numpy(tgt).to(gpu),
                                        radius)
    rsm, rtm, rcorr = do.compute_overlap(sw, tgt, radius)
    assert np.array_equal(sm.cpu().numpy(), rsm)
    assert np.array_equal(tm.cpu().numpy(), rtm)
    assert np.array_equal(corr.cpu().numpy(), rcorr)
    assert 0 < rsm.mean() < 1                        # a real partial overlap


def test_threedmatch_pairs_loader(gpu, tmp_path):
    from fgreg import data
    from fgreg.synthetic import lowoverlap_pair
    infos = {'rot': [], 'trans': [], 'src': [], 'tgt': [], 'overlap': []}
    raw = []
    for i in range(3):
        src, tgt, pose, f = lowoverlap_pair(i, n_points=4000)
        raw.append((src, tgt, pose))
        sp, tp = f'frag_{i}_a.pth', f'frag_{i}_b.npy'
        torch.save(src.astype(np.float64), os.path.join(tmp_path, sp))   # numpy in a .pth
        np.save(os.path.join(tmp_path, tp), tgt)
        infos['rot'].append(pose[:, :3].astype(np.float64))
        infos['trans'].append(pose[:, 3:].astype(np.float64))
        infos['src'].append(sp)
        infos['tgt'].append(tp)
        infos['overlap'].append(f)
    ds = data.ThreeDMatchPairs(str(tmp_path), infos, overlap_radius=0.0375, device=gpu)
    assert len(ds) == 3
    for i in range(3):
        s = ds[i]
        src, tgt, pose = raw[i]
        assert torch.equal(s['src_xyz'].cpu(), torch.from_numpy(src.astype(np.float64)).float())
        assert torch.equal(s['tgt_xyz'].cpu(), torch.from_numpy(tgt))
        assert torch.allclose(s['pose'], torch.from_numpy(pose), atol=1e-6)
        # the reference applies the float64 pose to the loaded points (threedmatch.py:80-84);
        # the loader does the same on the GPU and rounds once to float32 for the search
        sw32 = (src.astype(np.float64) @ pose[:, :3].T.astype(np.float64)
                + pose[:, 3].astype(np.float64)).astype(np.float32)
        rsm, rtm, rcorr = do.compute_overlap(sw32, tgt, 0.0375)
        assert np.array_equal(s['src_overlap'].cpu().numpy(), rsm)
        assert np.array_equal(s['tgt_overlap'].cpu().numpy(), rtm)
        assert np.array_equal(s['correspondences'].cpu().numpy(), rcorr)
        assert set(s) >= {'src_xyz', 'tgt_xyz', 'src_overlap', 'tgt_overlap', 'correspondences',
                          'pose', 'idx', 'src_path', 'tgt_path', 'overlap_p'}
