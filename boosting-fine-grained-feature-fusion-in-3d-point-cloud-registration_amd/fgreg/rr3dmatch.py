"""3DMatch / 3DLoMatch Registration Recall: the Redwood `est.log`
writer of `GenericRegModel._save_3DMatch_log` (models/generic_reg_model.py:265-286) and the
Predator-protocol evaluation of benchmark/benchmark_predator.py:96-378, restated.

Host code over ~1.6k pairs (text parsing, 6x6 quadratic forms): no GPU kernel is involved.
`mat2quat` restates nibabel.quaternions.mat2quat (nibabel is not installed here): the
Bar-Itzhack method -- the quaternion is the eigenvector of the symmetric 4x4 matrix K built
from the rotation with the largest eigenvalue, sign chosen so that w >= 0.

Behaviour kept from the reference on purpose:
* `evaluate_registration` stores the gt row index in `gt_mask[i, j]` and tests `> 0`, so the
  gt pair in row 0 of gt.log is never counted (benchmark_predator.py:247-253);
* only non-consecutive fragments (j - i > 1) are evaluated;
* the RMSE threshold is compared squared (err2 = 0.2 ** 2);
* recall is averaged over scenes (mean) and weighted by the number of valid gt pairs.
"""
import math
import os
from collections import defaultdict

import numpy as np

SHORT_NAMES = ['Kitchen', 'Home 1', 'Home 2', 'Hotel 1', 'Hotel 2', 'Hotel 3', 'Study',
               'MIT Lab']


def mat2quat(M):
    """(3,3) rotation -> (w, x, y, z), w >= 0 (nibabel.quaternions.mat2quat semantics)."""
    Qxx, Qyx, Qzx, Qxy, Qyy, Qzy, Qxz, Qyz, Qzz = np.asarray(M, dtype=np.float64).flat
    K = np.array([
        [Qxx - Qyy - Qzz, 0, 0, 0],
        [Qyx + Qxy, Qyy - Qxx - Qzz, 0, 0],
        [Qzx + Qxz, Qzy + Qyz, Qzz - Qxx - Qyy, 0],
        [Qyz - Qzy, Qzx - Qxz, Qxy - Qyx, Qxx + Qyy + Qzz]]) / 3.0
    vals, vecs = np.linalg.eigh(K)                 # lower triangle, as nibabel
    q = vecs[[3, 0, 1, 2], np.argmax(vals)]
    if q[0] < 0:
        q = -q
    return q


def transformation_error(trans, info):
    """Redwood RMSE approximation (benchmark_predator.py:66-85): e = [t, q_xyz],
    p = e^T info e / info[0, 0]."""
    t = trans[:3, 3]
    q = mat2quat(trans[:3, :3])
    er = np.concatenate([t, q[1:]])
    return float(er @ info @ er / info[0, 0])


def read_trajectory(filename, dim=4):
    """Redwood .log -> (pairs (n,3) str array, poses (n,4,4) f64) (benchmark_predator.py:88-126)."""
    with open(filename) as f:
        lines = f.readlines()
    keys = [ln.split('\t')[0:3] for ln in lines[0::dim + 1]]
    pairs = np.asarray([[k[0].strip(), k[1].strip(), k[2].strip()] for k in keys])
    traj = [ln.split('\t')[0:dim] for i, ln in enumerate(lines) if i % 5 != 0]
    return pairs, np.asarray(traj, dtype=np.float64).reshape(-1, dim, dim)


def read_trajectory_info(filename, dim=6):
    """Redwood .info -> (n_frames, (n,6,6) information matrices) (benchmark_predator.py:129-158)."""
    with open(filename) as f:
        contents = f.readlines()
    n_pairs = len(contents) // 7
    if len(contents) != 7 * n_pairs:
        raise ValueError(f'{filename}: {len(contents)} lines is not a multiple of 7')
    infos, n_frame = [], 0
    for i in range(n_pairs):
        _, _, n_frame = [int(v) for v in contents[i * 7].strip().split()]
        infos.append(np.stack([np.array(ln.split(), dtype=np.float64)
                               for ln in contents[i * 7 + 1:i * 7 + 7]]))
    return n_frame, np.asarray(infos, dtype=np.float64).reshape(-1, dim, dim)


def write_est_log(scene_folder, entries):
    """Appends (src_idx, tgt_idx, pose (3,4) or (4,4)) entries to <scene_folder>/est.log in
    the format of generic_reg_model.py:279-286 (tgt first, '-1' frame count, %.12f)."""
    os.makedirs(scene_folder, exist_ok=True)
    with open(os.path.join(scene_folder, 'est.log'), 'a') as fid:
        for src_idx, tgt_idx, pose in entries:
            pose = np.asarray(pose, dtype=np.float64)
            if pose.shape[0] == 3:
                pose = np.concatenate([pose, [[0., 0., 0., 1.]]], axis=0)
            fid.write('{}\t{}\t{}\n'.format(tgt_idx, src_idx, -1))
            for i in range(4):
                fid.write('\t'.join(map('{0:.12f}'.format, pose[i])) + '\n')


def save_3dmatch_log(log_root, benchmark, batch, pred):
    """Drop-in for GenericRegModel._save_3DMatch_log: batch['src_path'] / ['tgt_path'] are
    '<split>/<scene>/cloud_bin_<i>.pth'; pred['pose'] is (L,B,3,4) (last layer used) or (B,3,4)."""
    pose = pred['pose']
    pose = pose[-1] if pose.ndim == 4 else pose
    pose = pose.detach().cpu().numpy() if hasattr(pose, 'detach') else np.asarray(pose)
    for b in range(len(batch['src_xyz'])):
        scene = batch['src_path'][b].split(os.path.sep)[1]
        idx = lambda p: int(os.path.basename(p).split('_')[-1].replace('.pth', ''))
        write_est_log(os.path.join(log_root, benchmark, scene),
                      [(idx(batch['src_path'][b]), idx(batch['tgt_path'][b]), pose[b])])


def evaluate_registration(num_fragment, result, result_pairs, gt_pairs, gt, gt_info, err2=0.2):
    """-> (precision, recall, flags, errors) (benchmark_predator.py:224-282)."""
    err2 = err2 ** 2
    gt_mask = np.zeros((num_fragment, num_fragment), dtype=np.int64)
    for idx in range(gt_pairs.shape[0]):
        i, j = int(gt_pairs[idx, 0]), int(gt_pairs[idx, 1])
        if j - i > 1:
            gt_mask[i, j] = idx
    n_gt = np.sum(gt_mask > 0)
    errors = np.full(result_pairs.shape[0], np.nan)
    good, n_res, flags = 0, 0, []
    for idx in range(result_pairs.shape[0]):
        i, j = int(result_pairs[idx, 0]), int(result_pairs[idx, 1])
        if gt_mask[i, j] > 0:
            n_res += 1
            g = gt_mask[i, j]
            p = transformation_error(np.linalg.inv(gt[g]) @ result[idx], gt_info[g])
            errors[idx] = p
            if p <= err2:
                good += 1
                flags.append(0)
            else:
                flags.append(1)
        else:
            flags.append(2)
    if n_res == 0:
        n_res += 1e6
    return good / n_res, good / n_gt, flags, errors


def corresponding_gt(est_pairs, gt_pairs, gt_traj):
    """gt poses of the estimated pairs (benchmark_predator.py:161-180; the frame-count column
    of the estimate is replaced by the gt's)."""
    out = np.zeros((len(est_pairs), 4, 4))
    for e, pair in enumerate(est_pairs):
        pair = pair.copy()
        pair[2] = gt_pairs[0][2]
        out[e] = gt_traj[np.where((gt_pairs == pair).all(axis=1))[0]]
    return out


def rotation_error_deg(R1, R2):
    """arccos((tr(R1^T R2) - 1) / 2) in degrees, clamped (benchmark_predator.py:18-43)."""
    tr = np.einsum('bij,bij->b', R1, R2)
    return np.degrees(np.arccos(np.clip((tr - 1) / 2, -1, 1)))


def benchmark(est_folder, gt_folder):
    """Predator-protocol 3DMatch benchmark (benchmark_predator.py:285-378) -> (report str,
    mean recall over scenes, dict of per-scene numbers). Writes flag.npy / errors.npy per
    scene into est_folder like the reference."""
    scenes = sorted(os.listdir(gt_folder))
    re_med, te_med, precision, recall, n_valids = [], [], [], [], []
    report = 'Scene\t¦ prec.\t¦ rec.\t¦ re\t¦ te\t¦ samples\t¦\n'
    per_scene = defaultdict(list)
    for s_i, scene in enumerate(scenes):
        gdir = os.path.join(gt_folder, scene)
        gt_pairs, gt_traj = read_trajectory(os.path.join(gdir, 'gt.log'))
        n_valid = int(sum(abs(int(a) - int(b)) > 1 for a, b, _ in gt_pairs))
        n_valids.append(n_valid)
        n_frag, gt_info = read_trajectory_info(os.path.join(gdir, 'gt.info'))
        est_pairs, est_traj = read_trajectory(os.path.join(est_folder, scene, 'est.log'))
        p, r, flags, errors = evaluate_registration(n_frag, est_traj, est_pairs, gt_pairs,
                                                    gt_traj, gt_info)
        ext = corresponding_gt(est_pairs, gt_pairs, gt_traj)
        ok = np.array(flags) == 0
        re = rotation_error_deg(ext[:, :3, :3], est_traj[:, :3, :3])[ok]
        te = np.linalg.norm(ext[:, :3, 3] - est_traj[:, :3, 3], axis=1)[ok]
        re_med.append(np.median(re) if len(re) else math.nan)
        te_med.append(np.median(te) if len(te) else math.nan)
        precision.append(p)
        recall.append(r)
        per_scene['scene'].append(scene)
        per_scene['errors'].append(errors)
        name = SHORT_NAMES[s_i] if s_i < len(SHORT_NAMES) else scene
        report += '{}\t¦ {:.3f}\t¦ {:.3f}\t¦ {:.3f}\t¦ {:.3f}\t¦ {:3d}¦\n'.format(
            name, p, r, re_med[-1], te_med[-1], n_valid)
        np.save(os.path.join(est_folder, scene, 'flag.npy'), flags)
        np.save(os.path.join(est_folder, scene, 'errors.npy'), errors)
    w = np.array(n_valids, dtype=np.float64)
    report += 'Mean precision: {:.3f}: +- {:.3f}\n'.format(np.mean(precision), np.std(precision))
    report += 'Weighted precision: {:.3f}\n'.format((w * np.array(precision)).sum() / w.sum())
    report += 'Mean median RRE: {:.3f}: +- {:.3f}\n'.format(np.mean(re_med), np.std(re_med))
    report += 'Mean median RTE: {:.3F}: +- {:.3f}\n'.format(np.mean(te_med), np.std(te_med))
    report += 'Weighted recall (global recall): {:.3f}\n'.format(
        (w * np.array(recall)).sum() / w.sum())
    per_scene.update(precision=precision, recall=recall, n_valid=n_valids)
    return report, float(np.mean(recall)), dict(per_scene)
