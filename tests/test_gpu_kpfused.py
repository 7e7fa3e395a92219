"""fgr_kpconv_fused (gather + weight GEMM in one launch) against an fp64 torch restatement of
KPConv (finegrained_kpconv_blocks.py:296-399) and against the unfused gather + GEMM."""
import numpy as np
import pytest
import torch

from conftest import elem_err, rel_err

pytestmark = pytest.mark.gpu


def _case(cin, cout, H, nq, ns, seed, shadow=0.6, scale=1.0):
    rng = np.random.default_rng(seed)
    s = rng.uniform(-1, 1, (ns, 3)).astype(np.float32)
    q = s[rng.choice(ns, nq, replace=nq > ns)] + rng.normal(0, 0.01, (nq, 3)).astype(np.float32)
    idx = rng.integers(0, ns, (nq, H))
    idx[rng.uniform(size=(nq, H)) < shadow] = ns            # shadow entries
    x = (rng.normal(size=(ns, cin)) * scale).astype(np.float32)
    kp = (rng.normal(size=(15, 3)) * 0.3).astype(np.float32)
    W = (rng.normal(size=(15, cin, cout)) / np.sqrt(15 * cin)).astype(np.float32)
    return q, s, idx, x, kp, W


def _reference(q, s, idx, x, kp, W, ext):
    """fp64 KPConv sum (no division) and the normaliser, as the reference computes them."""
    cin = x.shape[1]
    sp = torch.cat([torch.from_numpy(s).double(), torch.zeros(1, 3, dtype=torch.float64) + 1e6])
    nb = sp[torch.from_numpy(idx)] - torch.from_numpy(q).double().unsqueeze(1)
    d2 = ((nb.unsqueeze(2) - torch.from_numpy(kp).double()) ** 2).sum(3)
    w = torch.clamp(1 - torch.sqrt(d2) / ext, min=0).transpose(1, 2)        # (nq, K, H)
    xp = torch.cat([torch.from_numpy(x).double(), torch.zeros(1, cin, dtype=torch.float64)])
    nx = xp[torch.from_numpy(idx)]                                          # (nq, H, cin)
    wf = torch.matmul(w, nx)                                                # (nq, K, cin)
    out = wf.reshape(wf.shape[0], -1) @ torch.from_numpy(W).double().reshape(-1, W.shape[2])
    cnt = torch.clamp((nx.sum(-1) > 0).sum(-1), min=1).float()
    return out, cnt


@pytest.mark.parametrize('cin,cout,H,nq', [(32, 32, 40, 700), (64, 64, 40, 1000),
                                           (128, 128, 50, 777), (256, 256, 50, 515),
                                           (128, 256, 50, 300), (64, 48, 7, 130),
                                           (32, 128, 130, 65), (256, 64, 50, 64)])
def test_kpconv_fused_vs_fp64(gpu, cin, cout, H, nq):
    import fgreg.ops as ops
    from fgreg import _lib
    q, s, idx, x, kp, W = _case(cin, cout, H, nq, 900, cin + cout + H)
    T = lambda a: torch.from_numpy(a).to(gpu)
    Wt = T(W)
    out, nn_ = ops.kpconv_fused(T(q), T(s), T(idx), T(x), T(kp), 0.5, Wt, _lib.KPF_F16X3)
    ref, cnt = _reference(q, s, idx, x, kp, W, 0.5)
    assert rel_err(out, ref) < 2e-6
    assert elem_err(out, ref) < 1e-4
    assert torch.equal(nn_.cpu(), cnt)
    # the unfused pair (gather -> f16x3 GEMM) agrees within the same contract
    wf, nn2 = ops.kpconv_gather(T(q), T(s), T(idx), T(x), T(kp), 0.5)
    assert torch.equal(nn2, nn_)


@pytest.mark.parametrize('scale', [1e-12, 1e-3, 1e4, 1e12])
def test_kpconv_fused_row_scales(gpu, scale):
    """Feature magnitudes far from 1 and rows whose chunks differ by 2^20 (the per-query
    scale is set by the first non-zero chunk and lowered when a later chunk grows)."""
    import fgreg.ops as ops
    from fgreg import _lib
    q, s, idx, x, kp, W = _case(128, 64, 50, 400, 600, 7, scale=scale)
    x[:, :32] *= 2.0 ** -20                      # first chunk tiny, later chunks large
    x[::7, :64] = 0.0                            # rows whose first chunks are zero
    T = lambda a: torch.from_numpy(a).to(gpu)
    out, _ = ops.kpconv_fused(T(q), T(s), T(idx), T(x), T(kp), 0.5, T(W), _lib.KPF_F16X3)
    ref, _ = _reference(q, s, idx, x, kp, W, 0.5)
    assert rel_err(out, ref) < 2e-6
    assert elem_err(out, ref) < 1e-4


def test_kpconv_fused_all_shadow_and_empty(gpu):
    import fgreg.ops as ops
    from fgreg import _lib
    q, s, idx, x, kp, W = _case(64, 64, 20, 100, 300, 3)
    idx[:50] = 300                               # queries without a single valid neighbour
    T = lambda a: torch.from_numpy(a).to(gpu)
    out, nn_ = ops.kpconv_fused(T(q), T(s), T(idx), T(x), T(kp), 0.5, T(W), _lib.KPF_F16X3)
    assert torch.equal(out[:50].cpu(), torch.zeros(50, 64))
    assert torch.equal(nn_[:50].cpu(), torch.ones(50))
    ref, _ = _reference(q, s, idx, x, kp, W, 0.5)
    assert rel_err(out, ref) < 2e-6
    e = torch.empty((0, 3), device=gpu)
    out0, nn0 = ops.kpconv_fused(e, T(s), torch.empty((0, 20), dtype=torch.int64, device=gpu),
                                 T(x), T(kp), 0.5, T(W), _lib.KPF_F16X3)
    assert out0.shape == (0, 64) and nn0.shape == (0,)


@pytest.mark.parametrize('cin,cout', [(32, 32), (128, 128), (256, 256)])
def test_kpconv_fused_bf16(gpu, cin, cout):
    """bf16 mode: wf and W rounded to bf16 at the MFMA, fp32 accumulation."""
    import fgreg.ops as ops
    from fgreg import _lib
    q, s, idx, x, kp, W = _case(cin, cout, 40, 600, 900, 11)
    T = lambda a: torch.from_numpy(a).to(gpu)
    out, nn_ = ops.kpconv_fused(T(q), T(s), T(idx), T(x), T(kp), 0.5, T(W), _lib.KPF_BF16)
    ref, cnt = _reference(q, s, idx, x, kp, W, 0.5)
    assert rel_err(out, ref) < 1e-2
    assert torch.equal(nn_.cpu(), cnt)


def test_kpconv_module_fused_equals_unfused(gpu, monkeypatch):
    """backbone.KPConv with the fused dispatch on and off: same outputs within f16x3."""
    from fgreg import backbone
    q, s, idx, x, kp, W = _case(128, 128, 50, 900, 900, 5)
    conv = backbone.KPConv(15, 3, 128, 128, 0.5, 0.4).to(gpu)
    with torch.no_grad():
        conv.weights.copy_(torch.from_numpy(W))
        conv.kernel_points.copy_(torch.from_numpy(kp))
    T = lambda a: torch.from_numpy(a).to(gpu)
    monkeypatch.setattr(backbone, 'KPF', '1')
    a = conv(T(q), T(s), T(idx), T(x))
    monkeypatch.setattr(backbone, 'KPF', '0')
    b = conv(T(q), T(s), T(idx), T(x))
    assert rel_err(a, b) < 4e-6
