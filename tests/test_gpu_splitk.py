"""Split-K g5 GEMM (fgr_gemm_f16x3_ws / fgr_gemm_bf16_ws): the parts' ordered sum with the
epilogue equals the product within the unsplit contract, and is bit-reproducible."""
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('mode', ['f16x3', 'bf16'])
@pytest.mark.parametrize('cfg,ks', [('I', 2), ('I', 4), ('X', 8), ('W', 4), ('S', 2), ('B', 3),
                                    ('T', 2)])
@pytest.mark.parametrize('M,N,K,act', [(2120, 512, 1024, 2), (1871, 256, 3840, 0),
                                       (333, 130, 1000, 3), (2120, 1536, 512, 0)])
def test_splitk_matches_fp64(gpu, monkeypatch, mode, cfg, ks, M, N, K, act):
    from fgreg import linear as lin
    monkeypatch.setattr(lin, 'MODE', mode)
    monkeypatch.setenv('FGR_GEMM16_TILE' if mode == 'f16x3' else 'FGR_GEMM_BF16_TILE', cfg)
    monkeypatch.setenv('FGR_GEMM_KSPLIT', str(ks))
    g = torch.Generator(device=gpu).manual_seed(M + N + K)
    x = torch.randn(M, K, device=gpu, generator=g)
    w = torch.randn(N, K, device=gpu, generator=g) * 0.05
    b = torch.randn(N, device=gpu, generator=g)
    r = torch.randn(M, N, device=gpu, generator=g)
    kw = {'bias': b}
    if act == 3:
        kw['residual'] = r
    y = lin.linear(x, w, act=act, **kw)
    y2 = lin.linear(x, w, act=act, **kw)
    assert torch.equal(y, y2)                               # fixed summation order
    if mode == 'bf16':
        p = x.bfloat16().double() @ w.bfloat16().double().t() + b.double()
    else:
        p = x.double() @ w.double().t() + b.double()
    if act == 2:
        p = p.relu()
    elif act == 3:
        t = p.relu() + r.double()
        p = torch.where(t > 0, t, 0.1 * t)
    assert rel_err(y, p) < (1e-5 if mode == 'bf16' else 2e-6)
