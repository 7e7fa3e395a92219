"""3DMatch Registration Recall host pipeline (fgreg.rr3dmatch).

* mat2quat: known answers (axis-angle rotations, identity, w >= 0 sign convention);
* est.log writer -> Redwood reader round trip (generic_reg_model.py:265-286 format);
* the benchmark on synthetic gt.log / gt.info scenes, against hand-counted recall;
* where the reference is mounted (this container only): evaluate_registration and
  benchmark of benchmark/benchmark_predator.py run on the same files, with nibabel (absent
  here) stubbed by fgreg's mat2quat -- this pins the parsing / masking / recall logic, not
  the quaternion (that is pinned by the known answers).
"""
import math
import os
import sys
import types

import numpy as np
import pytest
import torch

from fgreg import rr3dmatch as rr

REF = '/root/reference'


def _rot(axis, ang):
    axis = np.asarray(axis, dtype=np.float64)
    axis = axis / np.linalg.norm(axis)
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + math.sin(ang) * K + (1 - math.cos(ang)) * K @ K


def test_mat2quat_known_answers():
    np.testing.assert_allclose(rr.mat2quat(np.eye(3)), [1, 0, 0, 0], atol=1e-12)
    rng = np.random.default_rng(0)
    for _ in range(50):
        axis = rng.normal(size=3)
        axis /= np.linalg.norm(axis)
        ang = rng.uniform(0, math.pi * 0.999)
        q = rr.mat2quat(_rot(axis, ang))
        want = np.concatenate([[math.cos(ang / 2)], math.sin(ang / 2) * axis])
        np.testing.assert_allclose(q, want, atol=1e-9)
    q = rr.mat2quat(_rot([1, 0, 0], math.pi))          # w = 0: sign is free
    np.testing.assert_allclose(np.abs(q), [0, 1, 0, 0], atol=1e-9)


def _pose(rng, rot_deg=20.0, trans=0.5):
    T = np.eye(4)
    T[:3, :3] = _rot(rng.normal(size=3), math.radians(rng.uniform(0, rot_deg)))
    T[:3, 3] = rng.uniform(-trans, trans, 3)
    return T


def _write_scene(root, scene, n_frag, rng):
    """gt.log / gt.info for all pairs (i, j), j > i, of n_frag fragments."""
    d = os.path.join(root, scene)
    os.makedirs(d, exist_ok=True)
    pairs, poses = [], []
    with open(os.path.join(d, 'gt.log'), 'w') as fl, open(os.path.join(d, 'gt.info'), 'w') as fi:
        for i in range(n_frag):
            for j in range(i + 1, n_frag):
                T = _pose(rng)
                pairs.append((i, j))
                poses.append(T)
                fl.write(f'{i}\t{j}\t{n_frag}\n')
                for r in range(4):
                    fl.write('\t'.join(f'{v:.12f}' for v in T[r]) + '\n')
                A = rng.normal(size=(6, 6))
                info = A @ A.T + 6 * np.eye(6)
                fi.write(f'{i}\t{j}\t{n_frag}\n')
                for r in range(6):
                    fi.write('\t'.join(f'{v:.12f}' for v in info[r]) + '\n')
    return pairs, poses


def _make_benchmark(tmp_path, seed=0):
    rng = np.random.default_rng(seed)
    gt_root, est_root = str(tmp_path / 'gt'), str(tmp_path / 'est')
    expect = {}
    for s, scene in enumerate(['7-scenes-redkitchen', 'sun3d-home_at-home_at_scan1_2013_jan_1']):
        pairs, poses = _write_scene(gt_root, scene, 6 + s, rng)
        entries, good, n_gt = [], 0, 0
        for row, ((i, j), T) in enumerate(zip(pairs, poses)):
            counted = (j - i > 1) and row > 0       # reference: row 0 of gt.log never counts
            n_gt += counted
            ok = rng.uniform() < 0.6
            E = T.copy() if ok else T @ _pose(rng, rot_deg=40, trans=1.0)
            good += counted and ok
            entries.append((i, j, E))
        # est.log stores (tgt, src): the writer takes (src_idx, tgt_idx) = (j, i)
        rr.write_est_log(os.path.join(est_root, scene), [(j, i, E) for i, j, E in entries])
        expect[scene] = good / n_gt
    return gt_root, est_root, expect


def test_est_log_round_trip(tmp_path):
    rng = np.random.default_rng(1)
    poses = [_pose(rng) for _ in range(5)]
    rr.write_est_log(str(tmp_path / 's'), [(10 + k, k, P[:3]) for k, P in enumerate(poses)])
    pairs, traj = rr.read_trajectory(str(tmp_path / 's' / 'est.log'))
    assert pairs.shape == (5, 3) and [tuple(p) for p in pairs[:2]] == [('0', '10', '-1'),
                                                                       ('1', '11', '-1')]
    np.testing.assert_allclose(traj, np.stack(poses), atol=1e-12)


def test_save_3dmatch_log_dropin(tmp_path):
    """generic_reg_model._save_3DMatch_log naming: scene from src_path[1], indices from the
    cloud_bin file names, the last layer's pose."""
    pose = torch.zeros(6, 2, 3, 4)
    pose[..., :3, :3] = torch.eye(3)
    pose[-1, 1, :, 3] = torch.tensor([1., 2., 3.])
    batch = {'src_xyz': [None, None],
             'src_path': ['test/kitchen/cloud_bin_3.pth', 'test/kitchen/cloud_bin_7.pth'],
             'tgt_path': ['test/kitchen/cloud_bin_1.pth', 'test/kitchen/cloud_bin_2.pth']}
    rr.save_3dmatch_log(str(tmp_path), '3DMatch', batch, {'pose': pose})
    pairs, traj = rr.read_trajectory(str(tmp_path / '3DMatch' / 'kitchen' / 'est.log'))
    assert [tuple(p) for p in pairs] == [('1', '3', '-1'), ('2', '7', '-1')]
    np.testing.assert_allclose(traj[1, :3, 3], [1, 2, 3])


def test_benchmark_recall(tmp_path):
    gt_root, est_root, expect = _make_benchmark(tmp_path)
    report, mean_recall, per = rr.benchmark(est_root, gt_root)
    for scene, r in zip(per['scene'], per['recall']):
        assert r == pytest.approx(expect[scene])
    assert mean_recall == pytest.approx(np.mean(list(expect.values())))
    assert 'Weighted recall' in report
    assert os.path.exists(os.path.join(est_root, per['scene'][0], 'flag.npy'))


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, 'benchmark')),
                    reason='reference checkout not mounted (GPU box)')
def test_benchmark_matches_reference(tmp_path, monkeypatch):
    nib = types.ModuleType('nibabel')
    nq = types.ModuleType('nibabel.quaternions')
    nq.mat2quat = rr.mat2quat
    nib.quaternions = nq
    monkeypatch.setitem(sys.modules, 'nibabel', nib)
    monkeypatch.setitem(sys.modules, 'nibabel.quaternions', nq)
    monkeypatch.syspath_prepend(os.path.join(REF, 'benchmark'))
    monkeypatch.setenv('PYTHONDONTWRITEBYTECODE', '1')
    sys.dont_write_bytecode = True
    import importlib
    bp = importlib.import_module('benchmark_predator')
    gt_root, est_root, _ = _make_benchmark(tmp_path, seed=3)
    for scene in sorted(os.listdir(gt_root)):
        g = os.path.join(gt_root, scene)
        gp, gtr = bp.read_trajectory(os.path.join(g, 'gt.log'))
        n, info = bp.read_trajectory_info(os.path.join(g, 'gt.info'))
        ep, etr = bp.read_trajectory(os.path.join(est_root, scene, 'est.log'))
        want = bp.evaluate_registration(n, etr, ep, gp, gtr, info)
        got = rr.evaluate_registration(n, etr, ep, gp, gtr, info)
        assert got[0] == want[0] and got[1] == want[1] and list(got[2]) == list(want[2])
        np.testing.assert_allclose(got[3], want[3], rtol=1e-12, equal_nan=True)
    _, want_recall = bp.benchmark(est_root, gt_root)
    _, got_recall, _ = rr.benchmark(est_root, gt_root)
    assert got_recall == pytest.approx(want_recall, abs=1e-15)
