#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ by running the REFERENCE itself.

TEST INFRASTRUCTURE ONLY. Runs in the build container (it needs /root/reference
and oracle/_ref/libkpconv_ref.so, built by `make -C oracle ref`); nothing on the
GPU box executes it. Only the .npz files it writes travel.

How the reference is run:
  * the reference Python modules are imported from /root/reference with
    import-only stand-ins for packages that are absent here and never executed on
    the CPU path (MinkowskiEngine, pytorch3d, tensorboard, nibabel, easydict,
    open3d-based visualisation);
  * KPConv preprocessing uses the reference's own CPU `Preprocessor`
    (models/backbone_kpconv/finegrained_kpconv.py:296-419) whose native calls
    (`cpp_neighbors.batch_query`, `cpp_subsampling.subsample_batch`) are served by
    the reference's unmodified C++ algorithms (oracle/_ref/libkpconv_ref.so) through
    ctypes instead of the reference's NumPy-1 CPython wrapper;
  * `fast_compute_rigid_transform` hard-codes `.to(device='cuda')`
    (utils/se3_torch.py:240); it is called unmodified with `Tensor.to('cuda')`
    redirected to CPU for the duration of the call.

Usage:  python tests/golden/make_golden.py        (writes tests/golden/*.npz)
"""
import contextlib
import ctypes
import os
import sys
import types

import numpy as np
import torch

REF = os.environ.get('FGREG_REFERENCE', '/root/reference')
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
LIBREF = os.path.join(REPO, 'oracle', '_ref', 'libkpconv_ref.so')
sys.dont_write_bytecode = True


# --------------------------------------------------------------------------------------
# Reference native calls via ctypes (reference algorithm code, our adaptor)
# --------------------------------------------------------------------------------------
_lib = ctypes.CDLL(LIBREF)
_fp = ctypes.POINTER(ctypes.c_float)
_ip = ctypes.POINTER(ctypes.c_int)
_lib.ref_neighbors_run.restype = ctypes.c_int
_lib.ref_neighbors_run.argtypes = [_fp, ctypes.c_int, _fp, ctypes.c_int, _ip, _ip, ctypes.c_int,
                                   ctypes.c_float]
_lib.ref_neighbors_fetch.argtypes = [_ip]
_lib.ref_subsample_run.restype = ctypes.c_int
_lib.ref_subsample_run.argtypes = [_fp, ctypes.c_int, _ip, ctypes.c_int, ctypes.c_float]
_lib.ref_subsample_fetch.argtypes = [_fp, _ip]


def _f32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _i32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.int32))


def _idx(a):
    """Index table for storage: int16 where every value fits (the loaders widen to int64)."""
    a = np.asarray(a)
    return a.astype(np.int16) if a.size and a.min() >= 0 and a.max() < 32767 else a.astype(np.int32)


def ref_batch_query(queries, supports, q_batches, s_batches, radius):
    q, s, qb, sb = _f32(queries), _f32(supports), _i32(q_batches), _i32(s_batches)
    w = _lib.ref_neighbors_run(q.ctypes.data_as(_fp), q.shape[0], s.ctypes.data_as(_fp), s.shape[0],
                               qb.ctypes.data_as(_ip), sb.ctypes.data_as(_ip), qb.shape[0],
                               ctypes.c_float(radius))
    out = np.empty((q.shape[0], w), dtype=np.int32)
    _lib.ref_neighbors_fetch(out.ctypes.data_as(_ip))
    return out


def ref_subsample_batch(points, batches, sampleDl=0.1, max_p=0, verbose=0):
    assert max_p == 0
    p, b = _f32(points), _i32(batches)
    m = _lib.ref_subsample_run(p.ctypes.data_as(_fp), p.shape[0], b.ctypes.data_as(_ip), b.shape[0],
                               ctypes.c_float(sampleDl))
    pts = np.empty((m, 3), dtype=np.float32)
    lens = np.empty((b.shape[0],), dtype=np.int32)
    _lib.ref_subsample_fetch(pts.ctypes.data_as(_fp), lens.ctypes.data_as(_ip))
    return pts, lens


# --------------------------------------------------------------------------------------
# Import the reference with import-only stand-ins
# --------------------------------------------------------------------------------------
def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


class _EasyDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


def _never(*a, **k):
    raise RuntimeError('stand-in called: this dependency is not available here')


def import_reference():
    _stub('MinkowskiEngine')
    _stub('pytorch3d')
    _stub('pytorch3d.ops', packed_to_padded=_never, ball_query=_never)

    class _SW:
        def __init__(self, *a, **k):
            pass

    _stub('torch.utils.tensorboard', SummaryWriter=_SW)
    _stub('nibabel')
    _stub('nibabel.quaternions', mat2quat=_never)
    _stub('easydict', EasyDict=_EasyDict)
    _stub('utils.viz', visualize_registration=_never)
    sys.path[:0] = [REF, os.path.join(REF, 'models'), os.path.join(REF, 'utils')]
    cwd = os.getcwd()
    os.chdir(REF)
    try:
        # same import order as the reference's entry points (train.py / test.py import
        # `models` first; models/__init__.py:18-21 then imports models/finegrained_regtr.py)
        import models  # noqa: F401,E402
        fr = sys.modules['models.finegrained_regtr']
        import backbone_kpconv.finegrained_kpconv as fk  # noqa: E402
    finally:
        os.chdir(cwd)
    fk.cpp_neighbors = types.SimpleNamespace(batch_query=ref_batch_query)
    fk.cpp_subsampling = types.SimpleNamespace(subsample_batch=ref_subsample_batch)
    return fr, fk


@contextlib.contextmanager
def cuda_to_cpu():
    """Redirect `tensor.to(device='cuda')` to CPU (utils/se3_torch.py:240 hard-codes it)."""
    orig = torch.Tensor.to

    def to(self, *args, **kwargs):
        dev = kwargs.get('device', args[0] if args else None)
        if isinstance(dev, str) and dev.startswith('cuda'):
            return self
        return orig(self, *args, **kwargs)

    torch.Tensor.to = to
    try:
        yield
    finally:
        torch.Tensor.to = orig


def load_cfg(name, **overrides):
    import yaml
    with open(os.path.join(REF, 'conf', name)) as f:
        raw = yaml.safe_load(f)
    cfg = _EasyDict()
    for sect in raw.values():
        for k, v in sect.items():
            cfg[k] = v
    cfg.update(overrides)
    return cfg


# --------------------------------------------------------------------------------------
# Synthetic inputs (our own generator; same recipe the package uses)
# --------------------------------------------------------------------------------------
sys.path.insert(0, os.path.join(REPO, 'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
from fgreg.synthetic import modelnet_like_pair, indoor_like_pair  # noqa: E402


def save(name, **arrays):
    path = os.path.join(HERE, name + '.npz')
    np.savez_compressed(path, **arrays)
    print(f'wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)')


# --------------------------------------------------------------------------------------
# Geometry fixtures: reference C++ grid subsampling and radius search
# --------------------------------------------------------------------------------------
def make_geometry():
    cases = {}
    # ModelNet-like pair, B=2 (4 clouds packed src0, src1, tgt0, tgt1)
    pairs = [modelnet_like_pair(i) for i in range(2)]
    clouds = [p[0] for p in pairs] + [p[1] for p in pairs]
    cases['modelnet'] = (clouds, 0.03 * 2.75, 50)
    # indoor-like fragment pair, downsized
    src, tgt, _ = indoor_like_pair(0, n_points=3000)
    cases['indoor'] = ([src, tgt], 0.025 * 2.5, 40)
    # edge cases: single point cloud, duplicated points, lattice points on voxel
    # boundaries (exact multiples of dl), negative coordinates
    rng = np.random.default_rng(7)
    lattice = (np.stack(np.meshgrid(np.arange(-3, 4), np.arange(-3, 4), np.arange(-2, 3),
                                    indexing='ij'), -1).reshape(-1, 3) * 0.06).astype(np.float32)
    dup = rng.uniform(-0.3, 0.3, (40, 3)).astype(np.float32)
    dup = np.concatenate([dup, dup[:10]], 0)
    single = np.array([[0.1, -0.2, 0.3]], np.float32)
    cases['edge'] = ([lattice, dup, single], 0.03 * 2.75, 50)

    for name, (clouds, r0, limit) in cases.items():
        pts = np.concatenate(clouds, 0).astype(np.float32)
        lens = np.array([len(c) for c in clouds], np.int32)
        dl1 = 2 * r0 / (2.75 if name != 'indoor' else 2.5)
        sub_pts, sub_lens = ref_subsample_batch(pts, lens, sampleDl=dl1)
        conv = ref_batch_query(pts, pts, lens, lens, r0)
        pool = ref_batch_query(sub_pts, pts, sub_lens, lens, r0)
        up = ref_batch_query(pts, sub_pts, lens, sub_lens, 2 * r0)
        conv1 = ref_batch_query(sub_pts, sub_pts, sub_lens, sub_lens, 2 * r0)
        save(f'geom_{name}', points=pts, lengths=lens, dl=np.float64(dl1), r0=np.float64(r0),
             limit=np.int64(limit), sub_points=sub_pts, sub_lengths=sub_lens,
             conv=_idx(conv), pool=_idx(pool), up=_idx(up), conv1=_idx(conv1))

    # Exact-boundary radius case: supports at |d| == r exactly in float32 must be excluded
    # (strict d2 < r2, nanoflann.hpp:249-250).
    r = np.float32(0.25)
    q = np.zeros((1, 3), np.float32)
    s = np.array([[0.25, 0, 0], [0, -0.25, 0], [0, 0, 0.2499999], [0.1, 0.1, 0.1], [0.3, 0, 0]],
                 np.float32)
    nb = ref_batch_query(q, s, [1], [5], float(r))
    save('geom_boundary', queries=q, supports=s, radius=np.float64(r), nb=nb)


# --------------------------------------------------------------------------------------
# Module fixtures
# --------------------------------------------------------------------------------------
def make_modules(fr, fk):
    import backbone_kpconv.finegrained_kpconv_blocks as fb
    from transformer.transformers import TransformerCrossEncoderLayer
    from transformer.position_embedding import PositionEmbeddingCoordsSine
    import se3_torch

    g = np.load(os.path.join(HERE, 'geom_modelnet.npz'))
    pts, lens = g['points'], g['lengths']
    limit = int(g['limit'])
    neighb = g['conv'][:, :limit].astype(np.int64)
    pools = g['pool'][:, :limit].astype(np.int64)

    # ---- KPConv (rigid, linear influence, sum) on the real neighbour table
    torch.manual_seed(1)
    np.random.seed(1)
    cwd = os.getcwd()
    os.chdir(REF)
    try:
        kp = fb.KPConv(15, 3, 16, 24, KP_extent=0.06, radius=0.0825,
                       fixed_kernel_points='center', KP_influence='linear',
                       aggregation_mode='sum')
    finally:
        os.chdir(cwd)
    kp.eval()
    x = torch.randn(len(pts), 16)
    x[::7] = -x[::7].abs()  # rows whose feature sum is <= 0 do not count (blocks:395-399)
    # queries: the first NQ rows of each table (every support row stays, shadows = len(pts))
    NQ = 700
    with torch.no_grad():
        out = kp(torch.from_numpy(pts[:NQ]), torch.from_numpy(pts), torch.from_numpy(neighb[:NQ]), x)
        sub = torch.from_numpy(g['sub_points'][:NQ])
        out_strided = kp(sub, torch.from_numpy(pts), torch.from_numpy(pools[:NQ]), x)
        mp = fb.max_pool(x, torch.from_numpy(pools[:NQ]))
    save('kpconv_block', q=pts[:NQ], s=pts, idx=_idx(neighb[:NQ]), x=x.numpy(), W=kp.weights.detach().numpy(),
         kp=kp.kernel_points.detach().numpy(), extent=np.float64(kp.KP_extent), out=out.numpy(),
         sub=g['sub_points'][:NQ], pools=_idx(pools[:NQ]), out_strided=out_strided.numpy(), maxpool=mp.numpy())

    # ---- InstanceNorm per cloud (BatchNormBlock, blocks:462-518)
    bn = fb.BatchNormBlock(12, True, 0.02)
    y = torch.randn(len(pts), 12) * 3 + 1
    with torch.no_grad():
        yn = bn(y, torch.from_numpy(lens.astype(np.int64)))
    save('instnorm', x=y.numpy(), lengths=lens, out=yn.numpy())

    # ---- Transformer cross-encoder layer (transformers.py:84-258), pre-norm, B=2 unequal
    torch.manual_seed(2)
    layer = TransformerCrossEncoderLayer(64, 8, 128, 0.0, activation='relu',
                                         normalize_before=True, sa_val_has_pos_emb=True,
                                         ca_val_has_pos_emb=True)
    layer.eval()
    with torch.no_grad():
        for m in (layer.norm1, layer.norm2, layer.norm3):
            m.weight.copy_(1 + 0.1 * torch.randn(m.weight.shape))
            m.bias.copy_(0.1 * torch.randn(m.bias.shape))
    ns, nt = [37, 29], [23, 41]
    S, T = max(ns), max(nt)
    src = torch.randn(S, 2, 64)
    tgt = torch.randn(T, 2, 64)
    spos = torch.randn(S, 2, 64)
    tpos = torch.randn(T, 2, 64)
    smask = torch.zeros(2, S, dtype=torch.bool)
    tmask = torch.zeros(2, T, dtype=torch.bool)
    for b in range(2):
        smask[b, ns[b]:] = True
        tmask[b, nt[b]:] = True
    with torch.no_grad():
        so, to = layer(src, tgt, src_key_padding_mask=smask, tgt_key_padding_mask=tmask,
                       src_pos=spos, tgt_pos=tpos)
    sd = {f'w.{k}': v.numpy() for k, v in layer.state_dict().items()}
    save('transformer_layer', src=src.numpy(), tgt=tgt.numpy(), src_pos=spos.numpy(),
         tgt_pos=tpos.numpy(), src_mask=smask.numpy(), tgt_mask=tmask.numpy(),
         src_out=so.numpy(), tgt_out=to.numpy(), **sd)

    # ---- Sine position embedding (position_embedding.py:8-49)
    pe = PositionEmbeddingCoordsSine(3, 256, scale=1.0)
    xyz = torch.from_numpy(pts[:32])
    pe512 = PositionEmbeddingCoordsSine(3, 512, scale=1.0)
    pe64 = PositionEmbeddingCoordsSine(3, 64, scale=1.0)
    save('pos_embed', xyz=xyz.numpy(), pe256=pe(xyz).numpy(), pe512=pe512(xyz).numpy(),
         pe64=pe64(xyz).numpy())

    # ---- Weighted Procrustes (se3_torch.py:131-173, 226-273)
    rng = np.random.default_rng(3)
    cases = {}
    # (a) regular: noisy rigid correspondences, weights partly above 0.85
    def rigid(n, seed, noise=0.01):
        r = np.random.default_rng(seed)
        a = r.uniform(-1, 1, (6, n, 3)).astype(np.float32)
        from scipy.spatial.transform import Rotation
        R = Rotation.from_rotvec(r.normal(size=3) * 0.6).as_matrix().astype(np.float32)
        t = r.normal(size=3).astype(np.float32) * 0.3
        b = a @ R.T + t + r.normal(scale=noise, size=a.shape).astype(np.float32)
        return a, b.astype(np.float32)
    a, b = rigid(200, 4)
    w = rng.uniform(0.5, 1.0, (6, 200)).astype(np.float32)
    cases['regular'] = (a, b, w)
    # (b) reflection: b is a mirrored copy of a -> det(V U^T) < 0 branch
    a2 = rng.uniform(-1, 1, (6, 50, 3)).astype(np.float32)
    b2 = a2 * np.array([1, 1, -1], np.float32)
    w2 = rng.uniform(0.9, 1.0, (6, 50)).astype(np.float32)
    cases['reflection'] = (a2, b2, w2)
    # (c) all weights <= 0.85 -> zero covariance -> identity rotation
    a3, b3 = rigid(64, 5)
    w3 = rng.uniform(0.0, 0.85, (6, 64)).astype(np.float32)
    cases['allzero'] = (a3, b3, w3)
    # (d) weights exactly at the threshold (kept only if strictly greater)
    a4, b4 = rigid(32, 6)
    w4 = np.full((6, 32), 0.85, np.float32)
    w4[:, ::3] = 0.95
    cases['threshold'] = (a4, b4, w4)
    out = {}
    for name, (a_, b_, w_) in cases.items():
        with torch.no_grad(), cuda_to_cpu():
            fast = se3_torch.fast_compute_rigid_transform(
                torch.from_numpy(a_), torch.from_numpy(b_), torch.from_numpy(w_.copy()))
            full = se3_torch.compute_rigid_transform(
                torch.from_numpy(a_), torch.from_numpy(b_), torch.from_numpy(w_))
        out[f'{name}_a'], out[f'{name}_b'], out[f'{name}_w'] = a_, b_, w_
        out[f'{name}_fast'], out[f'{name}_full'] = fast.numpy(), full.numpy()
    save('procrustes', **out)


# --------------------------------------------------------------------------------------
# End-to-end forward fixtures
# --------------------------------------------------------------------------------------
# 3 encoder layers instead of 6 (the losses on the last one, as the configs' [5]): a third of
# the stored per-layer features, the same layer structure
SMALL_LAYERS = dict(num_encoder_layers=3, overlap_loss_on=[2], feature_loss_on=[2], corr_loss_on=[2])
SMALL_MODELNET = dict(first_feats_dim=32, d_embed=32, d_feedforward=64, **SMALL_LAYERS)
sys.path.insert(0, HERE)
from named_weights import named_state_dict  # noqa: E402


def run_forward(fr, fk, cfg, clouds_src, clouds_tgt, bias=4.0, seed=0):
    torch.manual_seed(seed)
    np.random.seed(seed)
    cwd = os.getcwd()
    os.chdir(REF)
    try:
        model = fr.RegTR(cfg)
    finally:
        os.chdir(cwd)
    model.preprocessor = fk.Preprocessor(cfg)  # the reference's own CPU preprocessor
    # weights from (key, shape, seed) only (named_weights.py), so the fixture need not store
    # them: non-trivial normalisation statistics and affine terms (BatchNorm folding and the
    # LayerNorm affine are exercised), the logits bias `bias`; the kernel points keep the
    # reference's own random rotation and are stored
    sd = model.state_dict()
    keys_shapes = [(k, tuple(v.shape)) for k, v in sd.items() if not k.startswith('feature_criterion')]
    stored = {k: v.numpy() for k, v in sd.items() if 'kernel_points' in k}
    vals = named_state_dict(keys_shapes, seed, bias, stored)
    missing, unexpected = model.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()},
                                                strict=False)
    assert not unexpected and all(k.startswith('feature_criterion') for k in missing), missing
    model.sd_keys_shapes, model.sd_seed = keys_shapes, seed
    model.eval()
    batch = {'src_xyz': [torch.from_numpy(c) for c in clouds_src],
             'tgt_xyz': [torch.from_numpy(c) for c in clouds_tgt]}
    with torch.no_grad(), cuda_to_cpu():
        out = model(batch)
    meta = batch['kpconv_meta']
    return model, meta, out


def pack_forward(model, meta, out, cfg_over, clouds_src, clouds_tgt, bias):
    arrays = {}
    B = len(clouds_src)
    for b in range(B):
        arrays[f'in.src_xyz.{b}'] = clouds_src[b]
        arrays[f'in.tgt_xyz.{b}'] = clouds_tgt[b]
    for key in ('points', 'neighbors', 'pools', 'upsamples', 'stack_lengths'):
        for l, t in enumerate(meta[key]):
            a = t.numpy()
            if a.dtype == np.int64:      # index tables: int16 where they fit (loaders widen)
                a = a.astype(np.int16 if a.size and a.max() < 32767 and a.min() >= 0 else np.int32)
            arrays[f'meta.{key}.{l}'] = a
    for k in ('src_feat_un', 'tgt_feat_un', 'src_feat', 'tgt_feat', 'src_kp', 'src_kp_warped',
              'tgt_kp', 'tgt_kp_warped', 'src_overlap', 'tgt_overlap'):
        for b, t in enumerate(out[k]):
            arrays[f'out.{k}.{b}'] = t.numpy()
    arrays['out.pose'] = out['pose'].numpy()
    # the state_dict is rebuilt by the tests from (key, shape, seed): named_weights.py; only
    # the reference's own random kernel points are stored
    arrays['sd_keys'] = np.bytes_(repr([(k, list(sh)) for k, sh in model.sd_keys_shapes]))
    arrays['sd_seed'] = np.int64(model.sd_seed)
    for k, v in model.state_dict().items():
        if 'kernel_points' in k:
            arrays[f'sd.{k}'] = v.numpy()
    arrays['cfg_overrides'] = np.array(repr(cfg_over))
    arrays['bias'] = np.float64(bias)
    return arrays


def make_forward(fr, fk):
    # (1) reduced-width ModelNet config (same architecture/semantics, small state_dict)
    cfg = load_cfg('modelnet.yaml', **SMALL_MODELNET)
    pairs = [modelnet_like_pair(i, n_raw=512) for i in range(2)]
    src = [p[0] for p in pairs]
    tgt = [p[1] for p in pairs]
    model, meta, out = run_forward(fr, fk, cfg, src, tgt)
    save('forward_modelnet_small', **pack_forward(model, meta, out, SMALL_MODELNET, src, tgt, 4.0))

    # (2) reduced-width 3DMatch config (4 levels, limits 40, d_embed 64)
    over = dict(first_feats_dim=16, d_embed=32, d_feedforward=64, **SMALL_LAYERS)
    cfg = load_cfg('3dmatch.yaml', **over)
    s, t, _ = indoor_like_pair(1, n_points=1500)
    model, meta, out = run_forward(fr, fk, cfg, [s], [t])
    save('forward_3dmatch_small', **pack_forward(model, meta, out, over, [s], [t], 4.0))


def make_forward_decoder(fr, fk):
    """(3) the soft-correspondence head: the reduced ModelNet config with
    direct_regress_coor: False, i.e. the reference's CorrespondenceDecoder
    (finegrained_regtr.py:312-408) instead of the regressor -- inactive in the shipped configs,
    pinned here for API completeness."""
    over = dict(SMALL_MODELNET, direct_regress_coor=False)
    cfg = load_cfg('modelnet.yaml', **over)
    pairs = [modelnet_like_pair(i + 5, n_raw=512) for i in range(2)]
    src = [p[0] for p in pairs]
    tgt = [p[1] for p in pairs]
    model, meta, out = run_forward(fr, fk, cfg, src, tgt, seed=7)
    save('forward_modelnet_decoder', **pack_forward(model, meta, out, over, src, tgt, 4.0))


def make_forward_postnorm(fr, fk):
    """(4) the post-norm transformer (pre_norm: False -> forward_post, transformers.py:109-181,
    and no final encoder norm, finegrained_regtr.py:56-58): the reduced ModelNet config,
    inactive in the shipped configs, pinned for API completeness."""
    over = dict(SMALL_MODELNET, pre_norm=False)
    cfg = load_cfg('modelnet.yaml', **over)
    pairs = [modelnet_like_pair(i + 9, n_raw=512) for i in range(2)]
    src = [p[0] for p in pairs]
    tgt = [p[1] for p in pairs]
    model, meta, out = run_forward(fr, fk, cfg, src, tgt, seed=11)
    save('forward_modelnet_postnorm', **pack_forward(model, meta, out, over, src, tgt, 4.0))


def make_decoder_topk(fr):
    """(5) CorrespondenceDecoder with num_neighbors > 0 (finegrained_regtr.py:312-408; the
    option is a constructor argument only, RegTR never passes it). The module is run as the
    reference runs it, its (L, N, B, D) inputs built here; cases:
      eq_k4    B = 1, three layers, 64 + 64 rows, k = 4: the union leaves a few NaN rows;
      eq_k24   B = 1, 64 + 64 rows, k = 24: a larger union;
      eq_k1    B = 1, one layer, 64 + 64 rows, k = 1: about a third of the rows NaN;
      b2_k6    B = 2, every cloud 48 rows (no padding), k = 6;
      ne_k8    B = 1, 40 src + 64 tgt rows, k = 8: records whether the reference raised
               (an index >= 40 into the src query dim);
      pad_k1   B = 2, one layer, src 24 / 48 and tgt 48 / 20 rows, k = 1: a padded batch, whose
               padded query rows (random features here) feed the union;
      pad_k2   B = 2, two layers, src 30 / 48 and tgt 48 / 26 rows, k = 2;
      pad_ix   B = 2, two layers, src 30 / 48 and tgt 44 / 26 rows, k = 2: the reference raises
               IndexError (a tgt query's top-k src index >= 44).
    Weights: nn.Linear default init under torch.manual_seed(20 + case), stored."""
    from transformer.position_embedding import PositionEmbeddingCoordsSine
    arrays = {'cases': np.array(['eq_k4', 'eq_k24', 'eq_k1', 'b2_k6', 'ne_k8', 'pad_k1',
                                 'pad_k2', 'pad_ix'])}
    D = 32
    for ci, (name, L, ns, nt, k) in enumerate([('eq_k4', 3, [64], [64], 4),
                                               ('eq_k24', 3, [64], [64], 24),
                                               ('eq_k1', 1, [64], [64], 1),
                                               ('b2_k6', 3, [48, 48], [48, 48], 6),
                                               ('ne_k8', 3, [40], [64], 8),
                                               ('pad_k1', 1, [24, 48], [48, 20], 1),
                                               ('pad_k2', 2, [30, 48], [48, 26], 2),
                                               ('pad_ix', 2, [30, 48], [44, 26], 2)]):
        torch.manual_seed(20 + ci)
        pe = PositionEmbeddingCoordsSine(3, D, scale=1.0)
        dec = fr.CorrespondenceDecoder(D, True, pe, num_neighbors=k).eval()
        B = len(ns)
        sx = [torch.rand(n, 3) for n in ns]
        tx = [torch.rand(n, 3) for n in nt]
        sf = torch.randn(L, max(ns), B, D)
        tf = torch.randn(L, max(nt), B, D)
        p = f'{name}.'
        try:
            with torch.no_grad():
                sc, tc, so, to = dec(sf, tf, sx, tx)
            for b in range(B):
                arrays[p + f'out.src_corr.{b}'] = sc[b].numpy()
                arrays[p + f'out.tgt_corr.{b}'] = tc[b].numpy()
                arrays[p + f'out.src_overlap.{b}'] = so[b].numpy()
                arrays[p + f'out.tgt_overlap.{b}'] = to[b].numpy()
            arrays[p + 'raised'] = np.bytes_(b'')
        except (IndexError, RuntimeError) as e:
            arrays[p + 'raised'] = np.bytes_(type(e).__name__.encode())
        arrays[p + 'k'] = np.int64(k)
        arrays[p + 'src_feats'] = sf.numpy()
        arrays[p + 'tgt_feats'] = tf.numpy()
        for b in range(B):
            arrays[p + f'src_xyz.{b}'] = sx[b].numpy()
            arrays[p + f'tgt_xyz.{b}'] = tx[b].numpy()
        for kk, v in dec.state_dict().items():
            arrays[p + 'w.' + kk] = v.numpy()
    save('decoder_topk', **arrays)


def make_loss(fr, fk):
    """Test-step tail fixture: the reference's own RegTR.compute_loss
    (finegrained_regtr.py:252-309) and GenericRegModel._compute_metrics
    (generic_reg_model.py:203-215) on the forward of forward_modelnet_small (same seeded
    model, inputs and kpconv_meta, so the forward outputs are that fixture's out.*), with the
    pairs' ground-truth poses and per-point overlap flags (nearest point of the other cloud,
    under the true pose, within 0.05)."""
    from scipy.spatial import cKDTree
    cfg = load_cfg('modelnet.yaml', **SMALL_MODELNET)
    pairs = [modelnet_like_pair(i, n_raw=512) for i in range(2)]
    src = [p[0] for p in pairs]
    tgt = [p[1] for p in pairs]
    pose = np.stack([p[2] for p in pairs]).astype(np.float32)
    model, meta, out = run_forward(fr, fk, cfg, src, tgt)
    ref = np.load(os.path.join(HERE, 'forward_modelnet_small.npz'))
    for b in range(2):          # same forward as the committed fixture
        assert np.array_equal(out['src_feat'][b].numpy(), ref[f'out.src_feat.{b}'])
    sov, tov = [], []
    for b in range(2):
        sw = src[b] @ pose[b][:, :3].T + pose[b][:, 3]
        sov.append((cKDTree(tgt[b]).query(sw)[0] < 0.05).astype(np.float32))
        tov.append((cKDTree(sw).query(tgt[b])[0] < 0.05).astype(np.float32))
    batch = {'src_xyz': [torch.from_numpy(c) for c in src],
             'tgt_xyz': [torch.from_numpy(c) for c in tgt],
             'kpconv_meta': meta, 'pose': torch.from_numpy(pose),
             'src_overlap': [torch.from_numpy(o) for o in sov],
             'tgt_overlap': [torch.from_numpy(o) for o in tov]}
    with torch.no_grad(), cuda_to_cpu():
        losses = model.compute_loss(out, batch)
        metrics = model._compute_metrics(out, batch)
    arrays = {'pose': pose, 'W': model.feature_criterion.W.detach().numpy(),
              'W_un': model.feature_criterion_un.W.detach().numpy()}
    for b in range(2):
        arrays[f'src_overlap.{b}'] = sov[b]
        arrays[f'tgt_overlap.{b}'] = tov[b]
    for k, v in batch['overlap_pyr'].items():
        arrays[f'overlap_pyr.{k}'] = v.numpy()
    for k, v in losses.items():
        arrays[f'loss.{k}'] = np.float32(v.item())
    for k, v in metrics.items():
        arrays[f'metric.{k}'] = v.numpy()
    save('loss_modelnet_small', **arrays)


def make_loss_circle(fr, fk):
    """The same test-step tail with `feature_loss_type: circle` (finegrained_regtr.py:86-88:
    CircleLossFull with Euclidean feature distances, feature_loss.py:160-243, for both the
    per-layer and the un-transformed feature losses): the reference's own compute_loss on the
    forward / loss inputs of loss_modelnet_small (that fixture's pose and overlap flags)."""
    cfg = load_cfg('modelnet.yaml', feature_loss_type='circle', **SMALL_MODELNET)
    pairs = [modelnet_like_pair(i, n_raw=512) for i in range(2)]
    src = [p[0] for p in pairs]
    tgt = [p[1] for p in pairs]
    model, meta, out = run_forward(fr, fk, cfg, src, tgt)
    ref = np.load(os.path.join(HERE, 'forward_modelnet_small.npz'))
    for b in range(2):          # same forward as the committed fixture
        assert np.array_equal(out['src_feat'][b].numpy(), ref[f'out.src_feat.{b}'])
    lf = np.load(os.path.join(HERE, 'loss_modelnet_small.npz'))
    batch = {'src_xyz': [torch.from_numpy(c) for c in src],
             'tgt_xyz': [torch.from_numpy(c) for c in tgt],
             'kpconv_meta': meta, 'pose': torch.from_numpy(lf['pose']),
             'src_overlap': [torch.from_numpy(lf[f'src_overlap.{b}']) for b in range(2)],
             'tgt_overlap': [torch.from_numpy(lf[f'tgt_overlap.{b}']) for b in range(2)]}
    with torch.no_grad(), cuda_to_cpu():
        losses = model.compute_loss(out, batch)
    arrays = {}
    for k, v in losses.items():
        arrays[f'loss.{k}'] = np.float32(v.item())
    save('loss_circle_modelnet_small', **arrays)


# parameters whose full gradient is stored (one of every kind on the path); every other
# parameter is pinned by its gradient's L2 norm and sum
TRAIN_FULL_GRADS = (
    'kpf_encoder.encoder_blocks.0.KPConv.weights',
    'kpf_encoder.encoder_blocks.1.KPConv.weights',
    'kpf_encoder.encoder_blocks.1.unary1.mlp.weight',
    'kpf_encoder.encoder_blocks.1.res2net.layer1.0.convs.3.weight',
    'kpf_encoder.encoder_blocks.1.res2net.layer1.0.bns.3.weight',
    'kpf_encoder.encoder_blocks.1.res2net.layer1.0.bn3.bias',
    'kpf_encoder.encoder_blocks.3.unary_shortcut.mlp.weight',
    'kpf_encoder.encoder_blocks.3.KPConv.weights',
    'feat_proj.weight',
    'transformer_encoder.layers.0.self_attn.in_proj_weight',
    'transformer_encoder.layers.2.multihead_attn.in_proj_bias',
    'transformer_encoder.layers.2.norm2.weight',
    'transformer_encoder.layers.2.linear1.weight',
    'transformer_encoder.norm.bias',
    'correspondence_decoder.coor_mlp.0.weight',
    'correspondence_decoder.conf_logits_decoder.weight',
)


def make_train(fr, fk):
    """Training-step fixture: the model of forward_modelnet_small switched
    to train() (Res2Net BatchNorm on batch statistics), the reference's own forward and
    compute_loss with the loss inputs of loss_modelnet_small, then losses['total'].backward()
    (trainer.py:110-125 without the optimizer step). Stores the losses, the gradient norm and
    sum of every parameter, the full gradient of TRAIN_FULL_GRADS and the updated running
    statistics of two BatchNorm layers."""
    cfg = load_cfg('modelnet.yaml', **SMALL_MODELNET)
    pairs = [modelnet_like_pair(i, n_raw=512) for i in range(2)]
    src = [p[0] for p in pairs]
    tgt = [p[1] for p in pairs]
    model, meta, out = run_forward(fr, fk, cfg, src, tgt)
    lf = np.load(os.path.join(HERE, 'loss_modelnet_small.npz'))
    model.feature_criterion.W.data.copy_(torch.from_numpy(lf['W']))
    model.feature_criterion_un.W.data.copy_(torch.from_numpy(lf['W_un']))
    model.train()
    batch = {'src_xyz': [torch.from_numpy(c) for c in src],
             'tgt_xyz': [torch.from_numpy(c) for c in tgt],
             'pose': torch.from_numpy(lf['pose']),
             'src_overlap': [torch.from_numpy(lf[f'src_overlap.{b}']) for b in range(2)],
             'tgt_overlap': [torch.from_numpy(lf[f'tgt_overlap.{b}']) for b in range(2)]}
    model.zero_grad()
    with cuda_to_cpu():
        pred = model(batch)
        losses = model.compute_loss(pred, batch)
        losses['total'].backward()
    ref = np.load(os.path.join(HERE, 'forward_modelnet_small.npz'))
    for l in range(len(meta['neighbors'])):     # same neighbour tables as the forward fixture
        assert np.array_equal(batch['kpconv_meta']['neighbors'][l].numpy(),
                              ref[f'meta.neighbors.{l}'].astype(np.int64))
    arrays = {}
    for k, v in losses.items():
        arrays[f'loss.{k}'] = np.float32(v.item())
    for k, p in model.named_parameters():
        if p.grad is None:
            continue
        g = p.grad.double()
        arrays[f'gnorm.{k}'] = np.float64(g.norm().item())
        arrays[f'gsum.{k}'] = np.float64(g.sum().item())
        if k in TRAIN_FULL_GRADS:
            arrays[f'grad.{k}'] = p.grad.numpy()
    for bn in ('kpf_encoder.encoder_blocks.1.res2net.layer1.0.bn1',
               'kpf_encoder.encoder_blocks.4.res2net.layer1.0.bns.6'):
        m = dict(model.named_modules())[bn]
        arrays[f'bn.{bn}.running_mean'] = m.running_mean.numpy()
        arrays[f'bn.{bn}.running_var'] = m.running_var.numpy()
    save('train_modelnet_small', **arrays)


def make_modelnet_metrics():
    """benchmark/benchmark_modelnet.py:33-82 compute_metrics -- the ModelNet test step's metrics
    (generic_reg_model.py:138-147) -- on synthetic pairs: 6 pairs of 717 src / ref points and
    2048 raw points, predicted poses 2-12 degrees / 1-5 cm off the ground truth (ModelNet's
    RandomTransformSE3_euler magnitudes for gt), one pair predicted exactly."""
    sys.path.insert(0, os.path.join(REF, 'benchmark'))
    import benchmark_modelnet as bm
    from scipy.spatial.transform import Rotation
    rng = np.random.default_rng(11)
    B, N, R = 6, 717, 2048

    def pose(rot, t):
        P = np.zeros((3, 4), np.float32)
        P[:, :3] = rot.as_matrix()
        P[:, 3] = t
        return P
    gt, pred = [], []
    for b in range(B):
        rg = Rotation.from_euler('zyx', rng.uniform(-45, 45, 3), degrees=True)
        tg = rng.uniform(-0.5, 0.5, 3)
        gt.append(pose(rg, tg))
        if b == 0:
            pred.append(gt[-1].copy())
            continue
        ax = rng.normal(size=3)
        dr = Rotation.from_rotvec(ax / np.linalg.norm(ax) * np.radians(rng.uniform(2, 12)))
        pred.append(pose(dr * rg, tg + rng.uniform(-0.05, 0.05, 3)))
    gt, pred = np.stack(gt), np.stack(pred)
    raw = rng.uniform(-1, 1, (B, R, 3)).astype(np.float32)
    src = (raw[:, :N] + 0.01 * rng.normal(size=(B, N, 3))).astype(np.float32)
    ref = (raw[:, R - N:] + 0.01 * rng.normal(size=(B, N, 3))).astype(np.float32)
    data = {'points_src': torch.from_numpy(src), 'points_ref': torch.from_numpy(ref),
            'points_raw': torch.from_numpy(raw), 'transform_gt': torch.from_numpy(gt)}
    m = bm.compute_metrics(data, torch.from_numpy(pred))
    s = bm.summarize_metrics(m)
    save('modelnet_metrics', points_src=src, points_ref=ref, points_raw=raw, transform_gt=gt,
         pred_transforms=pred, **{'m_' + k: np.asarray(v) for k, v in m.items()},
         **{'s_' + k: np.asarray(v) for k, v in s.items()})


if __name__ == '__main__':
    fr, fk = import_reference()
    if sys.argv[1:] == ['loss']:
        make_loss(fr, fk)
        sys.exit(0)
    if sys.argv[1:] == ['loss_circle']:
        make_loss_circle(fr, fk)
        sys.exit(0)
    if sys.argv[1:] == ['train']:
        make_train(fr, fk)
        sys.exit(0)
    if sys.argv[1:] == ['decoder']:
        make_forward_decoder(fr, fk)
        sys.exit(0)
    if sys.argv[1:] == ['postnorm']:
        make_forward_postnorm(fr, fk)
        sys.exit(0)
    if sys.argv[1:] == ['topk']:
        make_decoder_topk(fr)
        sys.exit(0)
    if sys.argv[1:] == ['metrics']:
        make_modelnet_metrics()
        sys.exit(0)
    make_geometry()
    make_modules(fr, fk)
    make_forward(fr, fk)
    make_forward_decoder(fr, fk)
    make_forward_postnorm(fr, fk)
    make_decoder_topk(fr)
    make_loss(fr, fk)
    make_loss_circle(fr, fk)
    make_train(fr, fk)
    make_modelnet_metrics()
