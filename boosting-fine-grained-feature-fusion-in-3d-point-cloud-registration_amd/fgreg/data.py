"""Input side of the 3DMatch / 3DLoMatch test path on the GPU.

* ``compute_overlap(src, tgt, radius)`` restates ``utils/pointcloud.py:8-66`` (the reference
  computes it with Open3D's KD-tree when the pair's overlap masks are not precomputed,
  ``data_loaders/threedmatch.py:76-81``) on the GPU with fgr_radius_search in nanoflann mode,
  K = 1: for every point of one cloud the nearest point of the other within ``radius``
  (ties by index; Open3D's radius search returns distance-sorted hits, and exact-distance
  ties are the only place the two can differ). The reference's quirks are kept: a
  correspondence is mutual only if both directions agree AND the source's partner index is
  > 0 (``src_corr > 0``, pointcloud.py:57), so target point 0 never appears in it.
* ``ThreeDMatchPairs`` mirrors ``ThreeDMatchDataset.__getitem__`` (threedmatch.py:65-107)
  for the test phase: pose from the info dict's rot / trans (src -> tgt), the two fragment
  files, overlap masks and mutual correspondences (from a precomputed ``pairs`` mapping when
  given, else ``compute_overlap`` on the GPU), with the same keys. The info dict is passed in
  (the reference unpickles ``datasets/3dmatch/<phase>_<benchmark>_info.pkl``; reading that
  trusted file is the caller's choice). Fragments are read by ``load_fragment``: ``.npy`` /
  ``.npz`` with numpy's non-pickle loader, ``.pth`` with ``torch.load(weights_only=True)``
  and numpy's array types allow-listed (no arbitrary unpickling).
"""
import os

import numpy as np
import torch

from . import ops


def _safe_numpy_globals():
    g = [np.ndarray, np.dtype]
    for mod in ('numpy.core.multiarray', 'numpy._core.multiarray'):
        try:
            m = __import__(mod, fromlist=['_reconstruct'])
            g.append(m._reconstruct)
        except (ImportError, AttributeError):
            pass
    for t in (np.float32, np.float64, np.int64, np.int32):
        g.append(type(np.dtype(t)))
    return g


def load_fragment(path: str) -> np.ndarray:
    """(N, 3) float array of one fragment file (.pth as written by the reference's data
    preparation, or .npy / .npz)."""
    ext = os.path.splitext(path)[1]
    if ext == '.npy':
        return np.load(path, allow_pickle=False)
    if ext == '.npz':
        with np.load(path, allow_pickle=False) as z:
            return z[z.files[0]]
    with torch.serialization.safe_globals(_safe_numpy_globals()):
        obj = torch.load(path, map_location='cpu', weights_only=True)
    return obj.numpy() if isinstance(obj, torch.Tensor) else np.asarray(obj)


def _nearest_within(q: torch.Tensor, s: torch.Tensor, radius: float) -> torch.Tensor:
    """Index of the nearest point of s within radius for every point of q (-1: none)."""
    dev = q.device
    nq, ns = q.shape[0], s.shape[0]
    q_off = torch.tensor([0, nq], dtype=torch.int64, device=dev)
    s_off = torch.tensor([0, ns], dtype=torch.int64, device=dev)
    grid = ops.radius_grid(s, s_off, [ns], radius) if ns >= ops.GRID_MIN_SUPPORTS else None
    nb = ops.radius_search(q, q_off, [nq], s, s_off, [ns], radius, 1, mode=ops.NB_DIST, grid=grid)
    if nb.shape[1] == 0:
        return torch.full((nq,), -1, dtype=torch.int64, device=dev)
    idx = nb[:, 0]
    return torch.where(idx < ns, idx, torch.full_like(idx, -1))


def compute_overlap(src: torch.Tensor, tgt: torch.Tensor, radius: float):
    """-> (has_corr_src (Ns,) bool, has_corr_tgt (Nt,) bool, src_tgt_corr (2, n) int64),
    utils/pointcloud.py:8-66 on device tensors (src already in the target frame)."""
    tgt_corr = _nearest_within(tgt, src, radius)
    src_corr = _nearest_within(src, tgt, radius)
    ar = torch.arange(src.shape[0], device=src.device)
    back = tgt_corr[src_corr.clamp_min(0)]
    mutual = (back == ar) & (src_corr > 0)
    src_tgt_corr = torch.stack([torch.nonzero(mutual)[:, 0], src_corr[mutual]])
    return src_corr >= 0, tgt_corr >= 0, src_tgt_corr


class ThreeDMatchPairs(torch.utils.data.Dataset):
    """Test-phase 3DMatch / 3DLoMatch pairs with the keys of ThreeDMatchDataset
    (threedmatch.py:65-107). ``infos``: dict with lists 'rot' (3,3), 'trans' (3,1 or 3),
    'src', 'tgt' (paths relative to ``root``), 'overlap'; ``pairs``: optional mapping
    item -> (src_mask, tgt_mask, src_tgt_corr) (the precomputed h5 content)."""

    def __init__(self, root, infos, overlap_radius=0.0375, device='cuda', pairs=None):
        self.root, self.infos, self.radius = root, infos, float(overlap_radius)
        self.device = torch.device(device)
        self.pairs = pairs

    def __len__(self):
        return len(self.infos['rot'])

    def __getitem__(self, item):
        rot = np.asarray(self.infos['rot'][item], dtype=np.float64)
        trans = np.asarray(self.infos['trans'][item], dtype=np.float64).reshape(3, 1)
        pose = np.concatenate([rot, trans], 1)                 # se3_init: src -> tgt
        src_xyz = torch.from_numpy(load_fragment(os.path.join(self.root, self.infos['src'][item])))
        tgt_xyz = torch.from_numpy(load_fragment(os.path.join(self.root, self.infos['tgt'][item])))
        src = src_xyz.float().to(self.device)
        tgt = tgt_xyz.float().to(self.device)
        pose_t = torch.from_numpy(pose).float()
        if self.pairs is not None and item in self.pairs:
            sm, tm, corr = (torch.as_tensor(np.asarray(v)) for v in self.pairs[item])
        else:
            # the reference applies the float64 pose to the points before its (float64)
            # Open3D search (threedmatch.py:80-84, se3_numpy.se3_transform): same here, the
            # result rounded once to float32 for the radius kernel (whose d^2 < r^2 test is
            # float32 -- DESIGN.md "input side")
            p64 = torch.from_numpy(pose).to(self.device)
            src_w = (src_xyz.to(self.device, torch.float64) @ p64[:, :3].T + p64[:, 3]).float()
            sm, tm, corr = compute_overlap(src_w, tgt, self.radius)
        return {'src_xyz': src, 'tgt_xyz': tgt, 'src_overlap': sm, 'tgt_overlap': tm,
                'correspondences': corr, 'pose': pose_t, 'idx': item,
                'src_path': self.infos['src'][item], 'tgt_path': self.infos['tgt'][item],
                'overlap_p': self.infos['overlap'][item]}
