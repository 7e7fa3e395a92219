"""Synthetic registration pairs.

No dataset is reachable from this image, so the benchmark and the tests use
clouds of the same shape as the reference's test inputs:

* ``modelnet_reference_pair(i)`` (``make_batch('modelnet')``, the bench workload) -- the
  box-surface raw cloud below through the reference's exact crop test pipeline
  (fgreg/transforms.py, pinned to data_loaders/modelnet_transforms.py);

* ``modelnet_like_pair(i)`` -- a 2048-point raw cloud (uniform samples on the
  faces of a random box, normalised to max|p| = 1) pushed through the steps of
  the reference's ModelNet *test* transforms (data_loaders/modelnet.py:111-117):
  SplitSourceRef -> RandomCrop([0.7, 0.7]) -> RandomTransformSE3_euler(45 deg,
  0.5) -> Resampler(1024) which yields 717 points per cloud
  (data_loaders/modelnet_transforms.py:92-93) -> RandomJitter(0.01, clip 0.05)
  -> ShufflePoints. Every step is re-implemented here with a per-pair seeded
  generator; it reproduces the shapes and statistics, not the reference's RNG
  stream.
* ``indoor_like_pair(i)`` -- a 3DMatch-like fragment pair: points on the floor
  and four walls of a 3 x 3 x 2.5 m room with 5 mm noise; the second fragment
  is an independent sample under a random rotation <= 15 deg and translation
  <= 0.3 m.
* ``lowoverlap_pair(i)`` -- a 3DLoMatch-like pair (BASELINE configs[4]): two fragments cut
  from opposite ends of a 6 x 3 x 2.5 m room so that 10-30% of each fragment lies in the
  shared strip, each sampled independently with N points, plus the same random motion.
"""
import math

import numpy as np


def _euler_rotation(angles):
    ax, ay, az = angles
    cx, sx, cy, sy, cz, sz = (math.cos(ax), math.sin(ax), math.cos(ay), math.sin(ay),
                              math.cos(az), math.sin(az))
    rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return rx @ ry @ rz


def _box_surface(rng, n):
    ext = rng.uniform(0.3, 1.0, 3)
    face = rng.integers(0, 6, n)
    uv = rng.uniform(-0.5, 0.5, (n, 3))
    axis = face % 3
    side = np.where(face < 3, -0.5, 0.5)
    uv[np.arange(n), axis] = side
    p = uv * ext
    p /= np.max(np.linalg.norm(p, axis=1))
    return p


def _crop(rng, pts, p_keep):
    v = rng.normal(size=3)
    v /= np.linalg.norm(v)
    d = (pts - pts.mean(0)) @ v
    return pts[d > np.percentile(d, (1.0 - p_keep) * 100)]


def _resample(rng, pts, k):
    if k <= len(pts):
        idx = rng.choice(len(pts), k, replace=False)
    else:
        idx = np.concatenate([rng.permutation(len(pts)), rng.choice(len(pts), k - len(pts))])
    return pts[idx]


def modelnet_like_pair(i, n_raw=2048, n_keep=717, rot_mag=45.0, trans_mag=0.5):
    """Returns (src (n_keep,3) f32, tgt (n_keep,3) f32, pose (3,4) f32: src -> tgt)."""
    rng = np.random.default_rng(1000003 * (i + 1))
    raw = _box_surface(rng, n_raw)
    src = _crop(rng, raw, 0.7)
    tgt = _crop(rng, raw, 0.7)
    ang = np.deg2rad(rng.uniform(-rot_mag, rot_mag, 3))
    R = _euler_rotation(ang)
    t = rng.uniform(-trans_mag, trans_mag, 3)
    src = src @ R.T + t                       # transform applied to the source
    n_keep = min(n_keep, 717 if n_raw >= 1024 else n_keep)
    if n_raw < 1024:
        n_keep = min(n_keep, int(math.ceil(0.7 * n_raw)))
    src = _resample(rng, src, n_keep)
    tgt = _resample(rng, tgt, n_keep)
    jit = lambda p: p + np.clip(rng.normal(0.0, 0.01, p.shape), -0.05, 0.05)
    src, tgt = jit(src), jit(tgt)
    src = src[rng.permutation(len(src))]
    tgt = tgt[rng.permutation(len(tgt))]
    Rinv = R.T
    pose = np.concatenate([Rinv, (-Rinv @ t)[:, None]], 1)  # maps src back onto tgt frame
    return src.astype(np.float32), tgt.astype(np.float32), pose.astype(np.float32)


def _room(rng, n, size=(3.0, 3.0, 2.5)):
    sx, sy, sz = size
    areas = np.array([sx * sy, sx * sz, sx * sz, sy * sz, sy * sz])
    surf = rng.choice(5, n, p=areas / areas.sum())
    u, v = rng.uniform(0, 1, n), rng.uniform(0, 1, n)
    p = np.zeros((n, 3))
    f = surf == 0
    p[f] = np.stack([u[f] * sx, v[f] * sy, np.zeros(f.sum())], 1)
    f = surf == 1
    p[f] = np.stack([u[f] * sx, np.zeros(f.sum()), v[f] * sz], 1)
    f = surf == 2
    p[f] = np.stack([u[f] * sx, np.full(f.sum(), sy), v[f] * sz], 1)
    f = surf == 3
    p[f] = np.stack([np.zeros(f.sum()), u[f] * sy, v[f] * sz], 1)
    f = surf == 4
    p[f] = np.stack([np.full(f.sum(), sx), u[f] * sy, v[f] * sz], 1)
    p += rng.normal(0.0, 0.005, p.shape)
    return p - np.array([sx, sy, sz]) / 2


def indoor_like_pair(i, n_points=20000, max_rot_deg=15.0, max_trans=0.3):
    """Returns (src (N,3) f32, tgt (N,3) f32, pose (3,4) f32: src -> tgt)."""
    rng = np.random.default_rng(7919 * (i + 1))
    tgt = _room(rng, n_points)
    src0 = _room(rng, n_points)
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    ang = np.deg2rad(rng.uniform(0, max_rot_deg))
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    R = np.eye(3) + math.sin(ang) * K + (1 - math.cos(ang)) * K @ K
    t = rng.uniform(-max_trans, max_trans, 3)
    src = (src0 - t) @ R                         # src = R^T (x - t): pose maps src -> tgt
    pose = np.concatenate([R, t[:, None]], 1)
    return src.astype(np.float32), tgt.astype(np.float32), pose.astype(np.float32)


def _strip(rng, n, size, lo, hi):
    """n room-surface samples with lo <= x < hi (rejection sampling)."""
    out, have = [], 0
    while have < n:
        p = _room(rng, 3 * n, size)
        p = p[(p[:, 0] >= lo) & (p[:, 0] < hi)]
        out.append(p)
        have += len(p)
    return np.concatenate(out)[:n]


def lowoverlap_pair(i, n_points=20000, overlap=(0.1, 0.3), max_rot_deg=15.0, max_trans=0.3):
    """3DLoMatch-like pair: the target covers x in [-L/2, -L/2 + W) of an L = 6 m room, the
    source x in [L/2 - W, L/2), W = L / (2 - f) so a fraction f in ``overlap`` of each
    fragment's extent is shared. Returns (src (N,3) f32, tgt (N,3) f32, pose (3,4) f32:
    src -> tgt, overlap fraction f)."""
    rng = np.random.default_rng(104729 * (i + 1))
    size = (6.0, 3.0, 2.5)
    f = rng.uniform(*overlap)
    L = size[0]
    W = L / (2.0 - f)
    tgt = _strip(rng, n_points, size, -L / 2, -L / 2 + W)
    src0 = _strip(rng, n_points, size, L / 2 - W, L / 2)
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    ang = np.deg2rad(rng.uniform(0, max_rot_deg))
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    R = np.eye(3) + math.sin(ang) * K + (1 - math.cos(ang)) * K @ K
    t = rng.uniform(-max_trans, max_trans, 3)
    src = (src0 - t) @ R
    pose = np.concatenate([R, t[:, None]], 1)
    return src.astype(np.float32), tgt.astype(np.float32), pose.astype(np.float32), f


def modelnet_reference_pair(i, n_raw=2048):
    """A box-surface raw cloud (seeded by i) through the reference's exact ModelNet crop test
    pipeline (fgreg.transforms.modelnet_crop_test, sample index i): the bench workload.
    Returns (src (717,3) f32, tgt (717,3) f32, pose (3,4) f32: src -> tgt)."""
    from .transforms import modelnet_crop_test
    raw = _box_surface(np.random.default_rng(1000003 * (i + 1)), n_raw).astype(np.float32)
    smp = modelnet_crop_test(raw, i)
    return (smp['src_xyz'].numpy().astype(np.float32), smp['tgt_xyz'].numpy().astype(np.float32),
            smp['pose'].numpy().astype(np.float32))


def modelnet_raw_pair(i, n_raw=2048, rot_mag=45.0, trans_mag=0.5):
    """The raw-2048 stress input ("feed the 2048-pt clouds directly"):
    the box-surface raw cloud of pair i, uncropped and not resampled, as the target, and the
    same cloud under a random euler SE3 (45 deg, 0.5) plus jitter (0.01, clip 0.05) as the
    source. Returns (src (n_raw,3) f32, tgt (n_raw,3) f32, pose (3,4) f32: src -> tgt)."""
    rng = np.random.default_rng(1000003 * (i + 1))
    raw = _box_surface(rng, n_raw)
    ang = np.deg2rad(rng.uniform(-rot_mag, rot_mag, 3))
    R = _euler_rotation(ang)
    t = rng.uniform(-trans_mag, trans_mag, 3)
    jit = lambda p: p + np.clip(rng.normal(0.0, 0.01, p.shape), -0.05, 0.05)
    src = jit(raw @ R.T + t)[rng.permutation(n_raw)]
    tgt = jit(raw)
    pose = np.concatenate([R.T, (-R.T @ t)[:, None]], 1)
    return src.astype(np.float32), tgt.astype(np.float32), pose.astype(np.float32)


def make_batch(kind, batch_size, start=0, **kw):
    """List-of-clouds batch in the reference's collate_pair layout (collate_functions.py:4-22).
    'modelnet': the reference's crop test pipeline on synthetic raw clouds; 'modelnet_like':
    the seeded approximation above; 'modelnet_raw': the uncropped 2048-pt stress input;
    '3dlomatch': low-overlap fragments; otherwise 3DMatch-like fragments."""
    gen = {'modelnet': modelnet_reference_pair, 'modelnet_like': modelnet_like_pair,
           'modelnet_raw': modelnet_raw_pair, '3dlomatch': lowoverlap_pair}.get(kind, indoor_like_pair)
    pairs = [gen(start + b, **kw) for b in range(batch_size)]
    return ([p[0] for p in pairs], [p[1] for p in pairs],
            np.stack([p[2] for p in pairs]).astype(np.float32))
