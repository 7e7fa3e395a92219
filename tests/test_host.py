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
    assert L.fgr_abi_version() == 1


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
