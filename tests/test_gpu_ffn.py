"""The pre-norm feed-forward sub-layer in one launch (fgr_ffn_f16x3, ops.ffn;
transformers.py:231-238): x + linear2(ReLU(linear1(LayerNorm3(x)))) with the hidden
activations kept on chip.

Checked against a float64 restatement (error at fp32 level and no worse than a few times
torch's own fp32 LayerNorm + GEMMs), against the two-launch path it replaces (linear_ln then
linear), on ragged row counts (1, a partial 64-row block, the ModelNet bench size), hidden
widths 64 / 1024 / 2048, in place (out = x), with a linear1 row far larger than the rest (the
hidden values' scale comes from a bound set by the largest row) and with most hidden units
cut by the ReLU; the C-ABI's refusal of unsupported widths and the W2 image layout.
"""
import math

import numpy as np
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu


def _layer(d, f, seed, big_row=False, neg_bias=False):
    g = torch.Generator().manual_seed(seed)
    norm = torch.nn.LayerNorm(d)
    with torch.no_grad():
        norm.weight.copy_(1 + 0.2 * torch.randn(d, generator=g))
        norm.bias.copy_(0.2 * torch.randn(d, generator=g))
    w1 = torch.randn(f, d, generator=g) / math.sqrt(d)
    b1 = 0.5 * torch.randn(f, generator=g)
    w2 = torch.randn(d, f, generator=g) / math.sqrt(f)
    b2 = torch.randn(d, generator=g)
    if big_row:
        w1[3] *= 1e4                    # the bound ||a|| max_j ||W1_j|| is 1e4 x the typical row
    if neg_bias:
        b1 -= 3.0                       # most hidden units are cut by the ReLU
    return norm, w1, b1, w2, b2


def _ref64(x, norm, w1, b1, w2, b2):
    xd = x.double()
    mu = xd.mean(1, keepdim=True)
    var = ((xd - mu) ** 2).mean(1, keepdim=True)
    a = (xd - mu) / torch.sqrt(var + norm.eps) * norm.weight.double() + norm.bias.double()
    h = (a @ w1.double().t() + b1.double()).clamp_min(0)
    return xd + h @ w2.double().t() + b2.double()


def _run(gpu, x, norm, w1, b1, w2, b2, out=None):
    from fgreg import linear as fl
    from fgreg import ops
    W1, B1, W2, B2 = (t.to(gpu) for t in (w1, b1, w2, b2))
    bound = torch.stack([W1.norm(dim=1).max(), B1.abs().max()]).contiguous()
    return ops.ffn(x, norm.to(gpu), fl.weight_image(W1, mode='f16x3', cache=False), B1,
                   fl.weight_image(W2, mode='ffn2', cache=False), B2, bound, out=out)


@pytest.mark.parametrize('m,f', [(9544, 1024), (1, 1024), (65, 1024), (1000, 64), (777, 2048),
                                 (13000, 1024)])
@pytest.mark.parametrize('case', ['plain', 'big_row', 'neg_bias'])
def test_ffn_vs_fp64(gpu, m, f, case):
    from fgreg import ops
    d = 256
    assert ops.ffn_supported(m, d, f)
    norm, w1, b1, w2, b2 = _layer(d, f, m + f, big_row=case == 'big_row',
                                  neg_bias=case == 'neg_bias')
    g = torch.Generator().manual_seed(m)
    x = 3.0 + 2.0 * torch.randn(m, d, generator=g)
    if m > 8:
        x[7] = 0.0                      # a constant row: LayerNorm gives beta
    ref = _ref64(x, norm, w1, b1, w2, b2)
    X = x.to(gpu)
    out = _run(gpu, X, norm, w1, b1, w2, b2)
    # torch fp32 (the comparison baseline only)
    N = norm.to(gpu)
    a32 = torch.nn.functional.layer_norm(X, (d,), N.weight, N.bias, N.eps)
    h32 = torch.addmm(b1.to(gpu), a32, w1.to(gpu).t()).clamp_min(0)
    y32 = X + torch.addmm(b2.to(gpu), h32, w2.to(gpu).t())
    e32, e = rel_err(y32, ref), rel_err(out, ref)
    # the update alone (y - x): its error is not hidden by the residual's magnitude
    eu = rel_err(out - X, ref - x.double())
    eu32 = rel_err(y32 - X, ref - x.double())
    assert e < 1e-5 and e < 4 * e32 + 1e-6, (e, e32)
    assert eu < 1e-5 and eu < 4 * eu32 + 1e-6, (eu, eu32)


def test_ffn_equals_two_launch_path(gpu):
    """ops.ffn against linear_ln (ReLU) then linear (+ residual): the same f16x3 products in
    two launches with the hidden activations in HBM."""
    from fgreg import linear as fl
    from fgreg import ops
    m, d, f = 9544, 256, 1024
    norm, w1, b1, w2, b2 = _layer(d, f, 5)
    x = (3.0 + 2.0 * torch.randn(m, d, generator=torch.Generator().manual_seed(5))).to(gpu)
    out = _run(gpu, x, norm, w1, b1, w2, b2)
    N = norm.to(gpu)
    h = fl.linear_ln(x, N, w1.to(gpu), b1.to(gpu), act=ops.ACT_RELU)
    two = fl.linear(h, w2.to(gpu), b2.to(gpu), residual=x)
    assert rel_err(out - x, two - x) < 4e-6


def test_ffn_in_place(gpu):
    m, d, f = 300, 256, 1024
    norm, w1, b1, w2, b2 = _layer(d, f, 9)
    x = (3.0 + 2.0 * torch.randn(m, d, generator=torch.Generator().manual_seed(9))).to(gpu)
    ref = _run(gpu, x, norm, w1, b1, w2, b2)
    y = x.clone()
    out = _run(gpu, y, norm, w1, b1, w2, b2, out=y)
    assert out.data_ptr() == y.data_ptr() and torch.equal(out, ref)


def test_ffn_w2_image_layout(gpu):
    """fgr_split_weights_ffn2: unit (chunk cc, panel q, term t, g, i) holds the two fp16 terms
    of W2[16 q + i][32 cc + 16 (e / 4) + 4 g + e % 4] * 2^e_row, e = 0..7; then the per-row
    inverse scales."""
    from fgreg import linear as fl
    d, f = 256, 128
    w2 = torch.randn(d, f, generator=torch.Generator().manual_seed(1))
    img = fl.weight_image(w2.to(gpu), mode='ffn2', cache=False).img.cpu()
    nb = f * d * 4
    units = img[:nb].view(torch.float16).view(f // 32, d // 16, 2, 4, 16, 8).double()
    wsc = img[nb:].view(torch.float32)[:d].double()
    val = (units[:, :, 0] + units[:, :, 1]) * wsc.view(1, d // 16, 1, 16, 1)   # (cc, q, g, i, e)
    e = torch.arange(8)
    for cc in range(f // 32):
        for gg in range(4):
            cols = 32 * cc + 16 * (e // 4) + 4 * gg + e % 4
            exp = w2.double()[:, cols].view(d // 16, 16, 8)
            got = val[cc, :, gg]
            assert float((got - exp).abs().max()) <= 2 ** -21 * float(w2.abs().max())


def test_ffn_refuses_unsupported(gpu):
    import fgreg
    from fgreg import _lib
    L = _lib.load()
    assert not L.fgr_ffn_f16x3_supported(100, 512, 1024)    # d != 256 (3DMatch): two launches
    assert not L.fgr_ffn_f16x3_supported(100, 256, 96)      # hidden % 64 != 0
    assert not L.fgr_ffn_f16x3_supported(100, 256, 4096)
    with pytest.raises(fgreg.FgrError):
        _lib.check(L.fgr_ffn_f16x3(None, 0, None, None, 1e-5, None, None, None, None, None, None,
                                   0, 10, 256, 1024, None), 'fgr_ffn_f16x3')
