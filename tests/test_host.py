"""CPU: the C ABI library loads and exports what include/fgreg.h declares; argument
validation fails loudly without touching a GPU; host-side logic (config, synthetic
inputs, model construction / state_dict layout, no CPU fallback)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO, forward_fixture


def _header_symbols():
    src = open(os.path.join(REPO, 'include', 'fgreg.h')).read()
    return sorted(set(re.findall(r'\b(fgr_[a-z0-9_]+)\s*\(', src)))


def test_library_exports_every_header_symbol():
    import fgreg
    L = fgreg.load()
    syms = _header_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(L, s), s
    from fgreg import _lib
    assert L.fgr_abi_version() == _lib.ABI_VERSION == 2


def test_python_signatures_cover_header():
    from fgreg import _lib
    syms = set(_header_symbols()) - {'fgr_abi_version', 'fgr_last_error'}
    assert syms == set(_lib.SIGNATURES)


def test_argument_errors_are_reported_without_gpu():
    import fgreg
    L = fgreg.load()
    rc = L.fgr_radius_search(None, None, None, None, 0, 0, 0, 0, ctypes.c_float(0.1), 0, 8, None,
                             None)
    assert rc == -1
    assert b'fgr_radius_search' in L.fgr_last_error()
    rc = L.fgr_kpconv_gather(None, None, 10, 10, None, 4, None, 100, None, 15,
                             ctypes.c_float(1.0), None, None, None, 0, None)
    assert rc == -1 and b'kpconv' in L.fgr_last_error()
    rc = L.fgr_attention(None, 0, None, 0, None, 0, None, 0, None, None, None, 1, 1, 1, 32,
                         ctypes.c_float(1.0), None)
    assert rc == -1


def test_ops_refuse_cpu_tensors():
    import fgreg
    x = torch.zeros(4, 3)
    off = torch.tensor([0, 4])
    with pytest.raises(fgreg.FgrError):
        fgreg.ops.radius_search(x, off, [4], x, off, [4], 0.1, 8)
    with pytest.raises(fgreg.FgrError):
        fgreg.ops.max_pool(torch.zeros(4, 8), torch.zeros(4, 2, dtype=torch.int64))


def test_config_flatten(tmp_path):
    import fgreg.config as fc
    p = tmp_path / 'c.yaml'
    p.write_text('a:\n  x: 1\n  y: [2, 3]\nb:\n  z: foo\n')
    cfg = fc.load_config(str(p))
    assert cfg == {'x': 1, 'y': [2, 3], 'z': 'foo'} and cfg.z == 'foo'
    m = fc.get('modelnet')
    assert m.neighborhood_limits == [50, 50] and m.d_embed == 256 and len(m.architecture) == 6


def test_synthetic_shapes():
    from fgreg.synthetic import indoor_like_pair, make_batch, modelnet_like_pair
    s, t, pose = modelnet_like_pair(0)
    assert s.shape == (717, 3) and t.shape == (717, 3) and pose.shape == (3, 4)
    R = pose[:, :3]
    assert np.allclose(R @ R.T, np.eye(3), atol=1e-5)
    s2, _, _ = modelnet_like_pair(0)
    assert np.array_equal(s, s2)                       # deterministic per pair index
    src, tgt, poses = make_batch('modelnet', 3)
    assert len(src) == 3 and poses.shape == (3, 3, 4)
    a, b, _ = indoor_like_pair(0, n_points=1000)
    assert a.shape == (1000, 3)


@pytest.mark.parametrize('name', ['forward_modelnet_small', 'forward_3dmatch_small'])
def test_state_dict_layout_matches_reference(name):
    import fgreg
    cfg, sd, *_ = forward_fixture(name)
    m = fgreg.RegTR(cfg)
    mine = m.state_dict()
    ref_keys = set(sd)
    assert ref_keys <= set(mine)
    assert set(mine) - ref_keys == {'feature_criterion.W', 'feature_criterion_un.W'}
    for k in ref_keys:
        assert tuple(mine[k].shape) == tuple(sd[k].shape), k


def test_full_config_parameter_counts():
    """18,799,602 (ModelNet) / 33,403,635 (3DMatch) parameters."""
    import fgreg
    for name, n in (('modelnet', 18799602), ('3dmatch', 33403635)):
        m = fgreg.RegTR(fgreg.config.get(name))
        assert sum(p.numel() for p in m.parameters()) == n


def test_kernel_disposition():
    from fgreg.backbone import kernel_disposition
    kp = kernel_disposition(15)
    assert kp.shape == (15, 3) and np.allclose(kp[0], 0)
    r = np.linalg.norm(kp[1:], axis=1)
    assert abs(r.mean() - 0.66) < 1e-6 and r.min() > 0.3


def test_res2net_fragments3_layout():
    """The bf16x6 weight image of fgr_res2net_chain6: three exact bf16 terms per value
    (sum within 2^-24 relative), zero K padding, [i][jt][ks][t][g][c][e] order."""
    from fgreg import ops
    g = torch.Generator().manual_seed(3)
    for w in (112, 224):
        W = torch.randn(7, w, w, generator=g)
        img = ops.res2net_fragments3(W)
        ks = (w + 31) // 32
        assert img.shape == (7, w // 16, ks, 3, 4, 16, 8) and img.dtype == torch.bfloat16
        tot = img.float().sum(3)                               # h + m + l
        i, jt, kk, gg, c, e = 5, 3, ks - 1, 2, 9, 6
        k = 32 * kk + 8 * gg + e
        want = W[i, 16 * jt + c, k] if k < w else torch.tensor(0.)
        assert torch.allclose(tot[i, jt, kk, gg, c, e], want, rtol=2 ** -23, atol=0)
        full = tot.permute(0, 1, 4, 2, 3, 5).reshape(7, w, ks * 32)
        assert (full[..., :w] - W).abs().max() <= 2 ** -22 * W.abs().max()
        assert bool((full[..., w:] == 0).all())


def _f16x3_emulate(x, w):
    """numpy restatement of fgr_gemm_f16x3's arithmetic (csrc/gemm16.hip): W rows scaled to
    max in [2^14, 2^15); A rows scaled per row from the first non-zero 32-chunk (max in
    [2^7, 2^8)), lowered when a chunk would pass 2^15 (partial sums rescaled); fp16 pairs;
    products hh + hm + mh accumulated in fp32 per 32-chunk."""
    m, k = x.shape
    n = w.shape[0]
    ew = np.array([15 - np.frexp(np.abs(r).max())[1] if np.abs(r).max() > 0 else 0 for r in w])
    ws = w * np.ldexp(1.0, ew)[:, None]
    wh = ws.astype(np.float16)
    wl = (ws - wh.astype(np.float32)).astype(np.float16)
    out = np.zeros((m, n), np.float32)
    for i in range(m):
        sh, acc = None, np.zeros(n, np.float32)
        for k0 in range(0, k, 32):
            ch = x[i, k0:k0 + 32]
            cm = np.abs(ch).max()
            if cm > 0 and (sh is None or np.frexp(cm)[1] + sh > 15):
                new = min(8 - np.frexp(cm)[1], 127)
                if sh is not None:
                    acc = (acc * np.float32(np.ldexp(1.0, new - sh))).astype(np.float32)
                sh = new
            xs = (ch * np.float32(np.ldexp(1.0, sh or 0))).astype(np.float32)
            ah = xs.astype(np.float16)
            al = (xs - ah.astype(np.float32)).astype(np.float16)
            f = lambda a, b: a.astype(np.float32)[None, :] * b.astype(np.float32)[:, k0:k0 + 32]
            acc = (acc + (f(al, wh) + f(ah, wl) + f(ah, wh)).sum(1, dtype=np.float64)).astype(np.float32)
        if sh is not None:
            out[i] = acc * np.float32(np.ldexp(1.0, -sh)) * np.ldexp(1.0, -ew).astype(np.float32)
    return out


def test_f16x3_split_numerics():
    """The f16x3 scheme is fp32-accurate (per-row normwise <= 2e-6 vs fp64) across 30
    decades of row magnitude (outputs 1e-25 .. 1e25, inside fp32's range), zero rows and rows growing 2^40 along k."""
    rng = np.random.default_rng(0)
    m, n, k = 64, 24, 160
    x = rng.standard_normal((m, k)) * (10.0 ** np.linspace(-15, 15, m))[:, None]
    x[3] = 0
    x[7, :100] = 0
    x[10:20] *= 2.0 ** np.linspace(0, 40, k)
    x = x.astype(np.float32)
    w = (rng.standard_normal((n, k)) / np.sqrt(k)).astype(np.float32)
    w[2] *= 1e-10
    w[5] *= 1e10
    got = _f16x3_emulate(x, w)
    ref = x.astype(np.float64) @ w.astype(np.float64).T
    den = np.abs(x).astype(np.float64) @ np.abs(w).astype(np.float64).T + 1e-300
    assert (got[3] == 0).all()
    assert (np.abs(got - ref) / den).max() < 2e-6


def test_training_mode_refuses_host_tensors():
    """model.train() runs the training forward (fgreg/training.py); like the inference forward
    it has no CPU path: host tensors are refused with FgrError, with or without autograd."""
    import fgreg
    import fgreg.config as fc
    model = fgreg.RegTR(fc.get('modelnet')).train()
    batch = {'src_xyz': [torch.zeros(8, 3)], 'tgt_xyz': [torch.zeros(8, 3)]}
    with pytest.raises(fgreg.FgrError):
        model(batch)
    with torch.no_grad(), pytest.raises(fgreg.FgrError):
        model(batch)


@pytest.mark.parametrize('what', ['dropout', 'num_neighbors'])
def test_training_refuses_untrainable_configs(what):
    """Configurations the training forward does not restate raise NotImplementedError before
    any work: dropout > 0 with a head dim the dropout attention kernels do not take (both
    precision modes train with dropout at head dim 32 / 64, transformers.py:95-110,
    tests/test_gpu_train.py), and the decoder's num_neighbors > 0."""
    import fgreg
    import fgreg.config as fc
    prev = fgreg.precision()
    try:
        if what == 'dropout':
            model = fgreg.RegTR(fc.get('modelnet', dropout=0.1, nhead=16)).train()   # head dim 16
            fgreg.set_precision('bf16')
        else:
            model = fgreg.RegTR(fc.get('modelnet', direct_regress_coor=False)).train()
            model.correspondence_decoder.num_neighbors = 4
        batch = {'src_xyz': [torch.zeros(8, 3)], 'tgt_xyz': [torch.zeros(8, 3)]}
        with pytest.raises(NotImplementedError, match=what.replace('_', '.')):
            model(batch)
    finally:
        fgreg.set_precision(prev)
    model.eval()                     # inference has no dropout and restates num_neighbors
    with pytest.raises(fgreg.FgrError):
        model(batch)


def test_load_fragment_formats(tmp_path):
    """fgreg.data.load_fragment: numpy arrays in a .pth (the reference's fragment files, read
    with torch.load(weights_only=True) + numpy allow-list), .npy and .npz (no pickle)."""
    import os
    from fgreg.data import load_fragment
    a = np.random.default_rng(0).normal(size=(50, 3))
    torch.save(a, os.path.join(tmp_path, 'a.pth'))
    np.save(os.path.join(tmp_path, 'a.npy'), a)
    np.savez(os.path.join(tmp_path, 'a.npz'), xyz=a)
    for f in ('a.pth', 'a.npy', 'a.npz'):
        assert np.array_equal(load_fragment(os.path.join(tmp_path, f)), a)
