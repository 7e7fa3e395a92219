"""Input side of the test step: the ModelNet "crop" *test* pipeline
(data_loaders/modelnet.py:111-117) and `collate_pair` (data_loaders/collate_functions.py:4-22).

The reference pipeline is a list of transform objects over a sample dict, each re-seeding
NumPy's global generator with the sample index when the sample is deterministic (test).
`modelnet_crop_test` reproduces its exact RNG stream and arithmetic in one function:

  SetDeterministic -> SplitSourceRef (modelnet_transforms.py:46-60)
  -> RandomCrop([p, p])            seed(idx); one S2 direction per cloud       (:176-246)
  -> RandomTransformSE3_euler       seed(idx); 3 angles, translation; src moved (:300-355)
  -> Resampler(n)                   seed(idx); 717 + 717 points ("Predator" size, :92-93)
  -> RandomJitter(0.01, 0.05)       stream continues                             (:151-173)
  -> ShufflePoints                  stream continues; ref permutation drawn first (:374-397)

and returns the dataset's sample dict (modelnet.py:160-185): src_xyz, tgt_xyz, tgt_raw,
src_overlap, tgt_overlap, correspondences, pose (3,4) = transform_gt (src -> tgt), idx.
Host-side numpy, as in the reference's DataLoader workers; `tests/test_transforms.py` pins it
element for element to the reference's own transform objects.
"""
import math

import numpy as np
import torch


def _uniform_s2():
    phi = np.random.uniform(0.0, 2 * np.pi)
    cos_theta = np.random.uniform(-1.0, 1.0)
    theta = np.arccos(cos_theta)
    return np.stack((np.sin(theta) * np.cos(phi), np.sin(theta) * np.sin(phi), np.cos(theta)),
                    axis=-1)


def _crop_mask(points, p_keep):
    d = np.dot(points[:, :3] - np.mean(points[:, :3], axis=0), _uniform_s2())
    if p_keep == 0.5:
        return d > 0
    return d > np.percentile(d, (1.0 - p_keep) * 100)


def _euler_se3(rot_mag, trans_mag):
    ax, ay, az = (np.random.uniform() * np.pi * rot_mag / 180.0 for _ in range(3))
    cx, cy, cz, sx, sy, sz = np.cos(ax), np.cos(ay), np.cos(az), np.sin(ax), np.sin(ay), np.sin(az)
    R = (np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
         @ np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
         @ np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]]))
    t = np.random.uniform(-trans_mag, trans_mag, 3)
    return np.concatenate((R, t[:, None]), axis=1).astype(np.float32)


def _apply(pose, xyz):
    return np.einsum('...ij,...bj->...bi', pose[:3, :3], xyz) + pose[:3, 3:4].transpose(-1, -2)


def _inv(pose):
    irot = pose[..., :3, :3].transpose(-1, -2)
    return np.concatenate([irot, -irot @ pose[..., :3, 3:4]], axis=-1)


def _resample(points, k):
    n = points.shape[0]
    if k <= n:
        idx = np.random.choice(n, k, replace=False)
    else:
        idx = np.concatenate([np.random.choice(n, n, replace=False),
                              np.random.choice(n, k - n, replace=True)])
    return points[idx, :], idx


def _remap(corr, src_map, ref_map):
    c = np.stack([src_map[corr[0]], ref_map[corr[1]]])
    return c[:, np.all(c >= 0, axis=0)]


def modelnet_crop_test(points, idx, p_keep=(0.7, 0.7), rot_mag=45.0, trans_mag=0.5,
                       num_points=1024, jitter=(0.01, 0.05)):
    """One deterministic test sample from a raw (N, 3 or 6) ModelNet cloud (see module doc)."""
    points = np.asarray(points)
    n = points.shape[0]
    src, ref = points.copy(), points.copy()
    corr = np.tile(np.arange(n), (2, 1))
    # RandomCrop (both clouds with p_keep[0], as the reference does)
    p_keep = np.array(p_keep, dtype=np.float32)
    if np.all(p_keep == 1.0):
        raise NotImplementedError('uncropped pipeline: use the "clean"/"jitter" variant')
    np.random.seed(idx)
    src_mask = _crop_mask(src, p_keep[0])
    ref_mask = (_crop_mask(ref, p_keep[0]) if len(p_keep) > 1
                else np.ones(n, dtype=np.bool_))
    src_ov = np.zeros(n, dtype=np.bool_)
    src_ov[corr[0][ref_mask[corr[1]]]] = 1
    ref_ov = np.zeros(n, dtype=np.bool_)
    ref_ov[corr[1][src_mask[corr[0]]]] = 1
    src_ov, ref_ov = src_ov[src_mask], ref_ov[ref_mask]
    sm, rm = np.full(n, -1), np.full(n, -1)
    sm[src_mask] = np.arange(src_mask.sum())
    rm[ref_mask] = np.arange(ref_mask.sum())
    corr = _remap(corr, sm, rm)
    src, ref = src[src_mask, :], ref[ref_mask, :]
    # RandomTransformSE3_euler on the source
    np.random.seed(idx)
    igt = _euler_se3(rot_mag, trans_mag)
    src_xyz = _apply(igt, src[:, :3])
    src = np.concatenate((src_xyz, _apply(np.concatenate([igt[:3, :3], np.zeros((3, 1), np.float32)], 1),
                                          src[:, 3:6])), axis=-1) if src.shape[1] == 6 else src_xyz
    transform_gt = _inv(igt)
    # Resampler
    np.random.seed(idx)
    if len(p_keep) == 1:
        src_size, ref_size = math.ceil(p_keep[0] * num_points), num_points
    else:
        src_size = ref_size = 717       # the reference's fixed "Predator" size (:92-93)
    src_size0, ref_size0 = src.shape[0], ref.shape[0]
    src, s_idx = _resample(src, src_size)
    ref, r_idx = _resample(ref, ref_size)
    sm, rm = np.full(src_size0, -1), np.full(ref_size0, -1)
    sm[s_idx] = np.arange(src_size)
    rm[r_idx] = np.arange(ref_size)
    corr = _remap(corr, sm, rm)
    src_ov, ref_ov = src_ov[s_idx], ref_ov[r_idx]
    # RandomJitter (stream continues)
    scale, clip = jitter
    for cloud in (src, ref):
        cloud[:, :3] += np.clip(np.random.normal(0.0, scale=scale, size=(cloud.shape[0], 3)),
                                a_min=-clip, a_max=clip)
    # ShufflePoints (reference permutation drawn first)
    r_perm = np.random.permutation(ref.shape[0])
    s_perm = np.random.permutation(src.shape[0])
    ref, src = ref[r_perm, :], src[s_perm, :]
    ref_ov, src_ov = ref_ov[r_perm], src_ov[s_perm]
    rm, sm = np.full(ref.shape[0], -1), np.full(src.shape[0], -1)
    rm[r_perm] = np.arange(ref.shape[0])
    sm[s_perm] = np.arange(src.shape[0])
    corr = np.stack([sm[corr[0]], rm[corr[1]]])
    return {
        'src_xyz': torch.from_numpy(src[:, :3]),
        'tgt_xyz': torch.from_numpy(ref[:, :3]),
        'tgt_raw': torch.from_numpy(points[:, :3]),
        'src_overlap': torch.from_numpy(src_ov),
        'tgt_overlap': torch.from_numpy(ref_ov),
        'correspondences': torch.from_numpy(corr),
        'pose': torch.from_numpy(transform_gt),
        'idx': torch.from_numpy(np.array(idx, dtype=np.int32)),
    }


_AS_LIST = ('src_xyz', 'tgt_xyz', 'tgt_raw', 'src_overlap', 'tgt_overlap', 'correspondences',
            'src_path', 'tgt_path', 'idx')


def collate_pair(samples):
    """collate_functions.py:4-22: variable-size fields stay per-sample lists; pose is stacked
    to (B, 3, 4); overlap_p (3DMatch) becomes a tensor."""
    out = {k: [s[k] for s in samples] for k in _AS_LIST if k in samples[0]}
    out['pose'] = torch.stack([s['pose'] for s in samples], dim=0)
    if 'overlap_p' in samples[0]:
        out['overlap_p'] = torch.tensor([s['overlap_p'] for s in samples])
    return out
