"""The ModelNet crop test pipeline with its geometry on the GPU.

`modelnet_crop_test_gpu(points_list, idx_list)` returns, for a batch of raw clouds, the same
sample dicts as `fgreg.transforms.modelnet_crop_test` (which restates
data_loaders/modelnet_transforms.py as data_loaders/modelnet.py:111-117 chains it), with the
tensors resident on the GPU and equal bit for bit. The work splits where the reference's
randomness allows:

- host, NumPy's global stream re-seeded per sample exactly as the reference re-seeds it:
  the two crop directions, the Euler pose, Resampler's choices, the jitter noise and the
  ShufflePoints permutations. None of them depends on the points, only on the seed and on
  the number of points each crop keeps;
- GPU (csrc/crop.hip): the crop projections, the percentile threshold and masks
  (`fgr_crop_pairs_mask`, one block per cloud), then moving the source, adding the noise,
  gathering the resampled / shuffled rows, the overlap flags and the correspondence list
  (`fgr_crop_pairs_assemble`, one block per pair).

Two small readbacks per batch: the crop counts (Resampler draws `choice(count, 717)`) and the
correspondence counts (the output shapes). Supported: the two-cloud crop the reference's
ModelNet configs use (`partial: [p, p]`, resampled to its fixed 717 points, p = 0.5 included);
other variants raise NotImplementedError. No CPU fallback: without the HIP library this raises.
"""
import numpy as np
import torch

from . import _lib
from .transforms import _euler_se3, _inv, _uniform_s2

_PREDATOR_SIZE = 717            # modelnet_transforms.py:92-93


def _ptr(t):
    return t.data_ptr()


def _upload(dev, *arrays):
    """One host-to-device copy for several small tables: packs the arrays (16-B aligned) into
    one byte buffer and returns typed device views of it."""
    offs, pos = [], 0
    for a in arrays:
        offs.append(pos)
        pos += (a.nbytes + 15) // 16 * 16
    buf = np.zeros(max(pos, 16), dtype=np.uint8)
    for a, o in zip(arrays, offs):
        buf[o:o + a.nbytes] = np.ascontiguousarray(a).view(np.uint8).ravel()
    dbuf = torch.from_numpy(buf).to(dev)
    return [dbuf[o:o + a.nbytes].view(_TORCH_DT[a.dtype]).view(a.shape)
            for a, o in zip(arrays, offs)]


_TORCH_DT = {np.dtype(np.int64): torch.int64, np.dtype(np.int32): torch.int32,
             np.dtype(np.float64): torch.float64, np.dtype(np.float32): torch.float32}


def _crop_rank(n, p_keep):
    """(k, gamma) of np.percentile(d, (1 - p) * 100) over n values, method 'linear': the
    threshold is NumPy's _lerp(s_k, s_k+1, gamma). Both come from NumPy itself on proxies, so
    the float32 virtual-index arithmetic is NumPy's own: over arange(n) the percentile is
    k + gamma, and over a 0/1 step at k it is _lerp(0, 1, gamma) = gamma exactly."""
    if p_keep == 0.5:
        return -1, 0.0
    q = (1.0 - p_keep) * 100
    k = int(np.floor(np.percentile(np.arange(n, dtype=np.float64), q)))
    k = min(max(k, 0), n - 1)
    step = np.zeros(n, dtype=np.float64)
    step[k + 1:] = 1.0
    g = float(np.percentile(step, q)) if k + 1 < n else 0.0
    return k, g


def modelnet_crop_test_gpu(points_list, idx_list, p_keep=(0.7, 0.7), rot_mag=45.0,
                           trans_mag=0.5, jitter=(0.01, 0.05), device='cuda'):
    """Batch form of fgreg.transforms.modelnet_crop_test with GPU-resident outputs.

    points_list: raw (N_b, 3 or 6) float32 clouds (numpy or torch, any device; all with the
    same column count); idx_list: the sample indices (the per-sample seeds)."""
    dev = torch.device(device)
    if dev.type != 'cuda':
        raise ValueError('modelnet_crop_test_gpu: a GPU device is required (no CPU fallback)')
    with torch.cuda.device(dev):                    # launches go to this device's stream
        return _crop_batch(points_list, idx_list, p_keep, rot_mag, trans_mag, jitter, dev)


def _crop_batch(points_list, idx_list, p_keep, rot_mag, trans_mag, jitter, dev):
    L = _lib.load()
    B = len(points_list)
    if B == 0 or B != len(idx_list):
        raise ValueError('need one index per raw cloud')
    p_keep = np.array(p_keep, dtype=np.float32)
    if len(p_keep) != 2:
        raise NotImplementedError('GPU crop pipeline: the two-cloud crop (partial: [p, p]) only')
    if np.all(p_keep == 1.0):
        raise NotImplementedError('uncropped pipeline: use the "clean"/"jitter" variant')
    raws = [torch.as_tensor(np.asarray(p) if not torch.is_tensor(p) else p) for p in points_list]
    ld = raws[0].shape[1]
    if any(r.dim() != 2 or r.shape[1] != ld or ld < 3 for r in raws):
        raise ValueError('raw clouds must be (N, C >= 3) with one column count')
    ns = [int(r.shape[0]) for r in raws]
    n_max = _lib.ctypes.c_int32()
    _lib.check(L.fgr_crop_max_points(_lib.ctypes.byref(n_max)), 'fgr_crop_max_points')
    if max(ns) > n_max.value or min(ns) < 1:
        raise NotImplementedError(f'GPU crop pipeline: 1..{n_max.value} points per raw cloud')
    raw = torch.cat([r.to(torch.float32) for r in raws]).to(dev).contiguous()
    off_h = np.concatenate([[0], np.cumsum(ns)]).astype(np.int64)
    ntot = int(off_h[-1])

    # RandomCrop draws (seed(idx); source direction, then reference: modelnet_transforms.py
    # :176-246 with the reference's p_keep[0] for both clouds)
    dirs = np.empty((B, 2, 3), dtype=np.float64)
    ranks = [_crop_rank(n, p_keep[0]) for n in ns]
    for b, idx in enumerate(idx_list):
        np.random.seed(idx)
        dirs[b, 0] = _uniform_s2()
        dirs[b, 1] = _uniform_s2()
    off, dirs_d, k_d, g_d = _upload(dev, off_h, dirs,
                                    np.array([r[0] for r in ranks], dtype=np.int32),
                                    np.array([r[1] for r in ranks], dtype=np.float64))
    mask = torch.empty((2, ntot), dtype=torch.uint8, device=dev)
    keep = torch.empty((2, ntot), dtype=torch.int32, device=dev)
    count = torch.empty((B, 2), dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(L.fgr_crop_pairs_mask(_ptr(raw), ld, _ptr(off), B, _ptr(dirs_d), _ptr(k_d),
                                     _ptr(g_d), _ptr(mask), _ptr(keep), _ptr(count), st),
               'fgr_crop_pairs_mask')
    cnt = count.cpu().numpy()                        # readback 1: Resampler needs the counts
    if (cnt < 0).any():
        raise _lib.FgrError('fgr_crop_pairs_mask: raw cloud size out of range')

    m = _PREDATOR_SIZE
    scale, clip = jitter
    sel = np.empty((B, 2, m), dtype=np.int32)
    noise = np.empty((B, 2, m, 3), dtype=np.float64)
    rt = np.empty((B, 3, 4), dtype=np.float32)
    poses = np.empty((B, 3, 4), dtype=np.float32)
    for b, idx in enumerate(idx_list):
        if cnt[b].min() < m:
            raise NotImplementedError('GPU crop pipeline: crop kept fewer points than the '
                                      'resampled size (Resampler would draw with replacement)')
        np.random.seed(idx)                          # RandomTransformSE3_euler (:300-355)
        igt = _euler_se3(rot_mag, trans_mag)
        rt[b] = igt
        poses[b] = _inv(igt)
        np.random.seed(idx)                          # Resampler (:92-148)
        s_idx = np.random.choice(int(cnt[b, 0]), m, replace=False)
        r_idx = np.random.choice(int(cnt[b, 1]), m, replace=False)
        nz = [np.clip(np.random.normal(0.0, scale=scale, size=(m, 3)), a_min=-clip, a_max=clip)
              for _ in range(2)]                     # RandomJitter (:151-173), source first
        r_perm = np.random.permutation(m)            # ShufflePoints (:374-397), ref first
        s_perm = np.random.permutation(m)
        sel[b, 0], sel[b, 1] = s_idx[s_perm], r_idx[r_perm]
        noise[b, 0], noise[b, 1] = nz[0][s_perm], nz[1][r_perm]
    sel_d, noise_d, rt_d, poses_d = _upload(dev, sel, noise, rt, poses)
    xyz = torch.empty((B, 2, m, 3), dtype=torch.float32, device=dev)
    ov = torch.empty((B, 2, m), dtype=torch.uint8, device=dev)
    corr = torch.empty((2, ntot), dtype=torch.int64, device=dev)
    n_corr = torch.empty(B, dtype=torch.int32, device=dev)
    _lib.check(L.fgr_crop_pairs_assemble(_ptr(raw), ld, _ptr(off), B, _ptr(mask), _ptr(keep),
                                         _ptr(sel_d), _ptr(noise_d), _ptr(rt_d), m, _ptr(xyz),
                                         _ptr(ov), _ptr(corr), _ptr(n_corr), st),
               'fgr_crop_pairs_assemble')
    nc = n_corr.cpu().numpy()                        # readback 2: correspondence counts
    if (nc < 0).any():
        raise _lib.FgrError('fgr_crop_pairs_assemble: raw cloud size out of range')
    ovb = ov.bool()
    out = []
    for b, idx in enumerate(idx_list):
        o = int(off_h[b])
        out.append({
            'src_xyz': xyz[b, 0],
            'tgt_xyz': xyz[b, 1],
            'tgt_raw': raw[o:o + ns[b], :3],
            'src_overlap': ovb[b, 0],
            'tgt_overlap': ovb[b, 1],
            'correspondences': corr[:, o:o + int(nc[b])],
            'pose': poses_d[b],
            'idx': torch.from_numpy(np.array(idx, dtype=np.int32)),
        })
    return out


def modelnet_crop_batch_gpu(points_list, idx_list, **kw):
    """modelnet_crop_test_gpu + collate_pair (collate_functions.py:4-22): the batch dict the
    model's forward / test_step take, GPU-resident."""
    from .transforms import collate_pair
    return collate_pair(modelnet_crop_test_gpu(points_list, idx_list, **kw))


__all__ = ['modelnet_crop_test_gpu', 'modelnet_crop_batch_gpu']
