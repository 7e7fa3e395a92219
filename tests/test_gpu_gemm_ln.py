"""LayerNorm -> (+ pos) -> Linear in one launch (fgr_gemm_f16x3_ln; the pre-norm transformer
sub-layer inputs, transformers.py:193-196, :213-221, :231-232).

Checked: the fused op against a float64 LayerNorm + product (error at fp32 level and no worse
than a few times torch's own fp32 LayerNorm + GEMM), against the unfused path (ops.layernorm
then linear), the fallback below the supported shapes, the C-ABI's refusal of unsupported
shapes, and a full pre-norm encoder layer at the ModelNet bench size (9544 rows, where every
in_proj and linear1 takes the fused launch) against the oracle's restatement of forward_pre.
"""
import math

import numpy as np
import pytest
import torch

import model_oracle as mo
from conftest import rel_err

pytestmark = pytest.mark.gpu


def _inputs(m, k, n, seed, mean=3.0):
    g = torch.Generator().manual_seed(seed)
    x = mean + 2.0 * torch.randn(m, k, generator=g)
    x[7] = 0.0                                   # constant rows: var 0, output = beta (+ pos)
    x[8] = 5.0
    norm = torch.nn.LayerNorm(k)
    with torch.no_grad():
        norm.weight.copy_(1 + 0.2 * torch.randn(k, generator=g))
        norm.bias.copy_(0.2 * torch.randn(k, generator=g))
    pos = torch.randn(m, k, generator=g)
    w = torch.randn(n, k, generator=g) / math.sqrt(k)
    b = torch.randn(n, generator=g)
    return x, norm, pos, w, b


def _ref64(x, norm, pos, w, b, relu):
    xd = x.double()
    mu = xd.mean(1, keepdim=True)
    var = ((xd - mu) ** 2).mean(1, keepdim=True)
    h = (xd - mu) / torch.sqrt(var + norm.eps) * norm.weight.double() + norm.bias.double()
    if pos is not None:
        h = h + pos.double()
    y = h @ w.double().t() + b.double()
    return y.clamp_min(0) if relu else y


@pytest.mark.parametrize('m,n,k', [(9544, 768, 256), (9544, 1024, 256), (9000, 256, 128),
                                   (8001, 640, 64), (25003, 256, 256)])
@pytest.mark.parametrize('with_pos,relu', [(True, False), (False, True)])
def test_gemm_ln_vs_fp64(gpu, m, n, k, with_pos, relu):
    from fgreg import linear as fl
    from fgreg import ops
    assert fl.MODE == 'f16x3' and fl.ln_fusable(m, n, k)
    x, norm, pos, w, b = _inputs(m, k, n, m + n + k)
    if not with_pos:
        pos = None
    ref = _ref64(x, norm, pos, w, b, relu)
    act = ops.ACT_RELU if relu else ops.ACT_NONE
    X, W, B = x.to(gpu), w.to(gpu), b.to(gpu)
    P = pos.to(gpu) if pos is not None else None
    N = norm.to(gpu)
    out = fl.linear_ln(X, N, W, B, act=act, add=P)
    # torch fp32 LayerNorm + GEMM (the comparison baseline only)
    h32 = torch.nn.functional.layer_norm(X, (k,), N.weight, N.bias, N.eps)
    if P is not None:
        h32 = h32 + P
    y32 = torch.addmm(B, h32, W.t())
    e32 = rel_err(y32.clamp_min(0) if relu else y32, ref)
    e = rel_err(out, ref)
    assert e < 1e-5 and e < 4 * e32 + 1e-6, (e, e32)
    # the unfused path (ops.layernorm, then the GEMM): same arithmetic, two launches
    old = fl.LN_FUSE
    try:
        fl.LN_FUSE = False
        un = fl.linear_ln(X, N, W, B, act=act, add=P)
    finally:
        fl.LN_FUSE = old
    assert rel_err(out, un) < 4e-6
    # constant rows normalise to beta (+ pos) exactly as the LayerNorm kernel does
    assert rel_err(out[7:9], un[7:9]) < 4e-6


def test_gemm_ln_fallback_and_refusal(gpu):
    """Below the supported shapes linear_ln runs layernorm + linear; the C ABI refuses them."""
    from fgreg import _lib
    from fgreg import linear as fl
    m, n, k = 500, 768, 256
    assert not fl.ln_fusable(m, n, k)
    x, norm, pos, w, b = _inputs(m, k, n, 3)
    ref = _ref64(x, norm, pos, w, b, False)
    norm = norm.to(gpu)                          # (in place)
    out = fl.linear_ln(x.to(gpu), norm, w.to(gpu), b.to(gpu), add=pos.to(gpu))
    assert rel_err(out, ref) < 1e-5
    L = _lib.load()
    X, W = x.to(gpu), w.to(gpu)
    sw = fl.weight_image(W, mode='f16x3')
    o = torch.empty(m, n, device=gpu)
    rc = L.fgr_gemm_f16x3_ln(X.data_ptr(), k, norm.weight.data_ptr(), norm.bias.data_ptr(), 1e-5, None, 0, sw.img.data_ptr(),
                             o.data_ptr(), n, None, m, n, k, 0,
                             torch.cuda.current_stream().cuda_stream)
    assert rc == -1 and b'not supported' in L.fgr_last_error()


def test_prenorm_layer_bench_size_vs_oracle(gpu):
    """One pre-norm TransformerCrossEncoderLayer (d 256, 8 heads, ffn 1024, values with pos:
    the ModelNet config) on 8 pairs of 596-point clouds = 9536 rows: the in_proj and linear1
    GEMMs take the fused LayerNorm launch; against the oracle's forward_pre (fp32 CPU)."""
    from fgreg import linear as fl
    from fgreg.transformer import Segments, TransformerCrossEncoderLayer
    d, nhead, ff, B, L = 256, 8, 1024, 8, 596
    assert fl.ln_fusable(2 * B * L, 3 * d, d) and fl.ln_fusable(2 * B * L, ff, d)
    torch.manual_seed(5)
    layer = TransformerCrossEncoderLayer(d, nhead, ff, 0.0, normalize_before=True,
                                         sa_val_has_pos_emb=True, ca_val_has_pos_emb=True)
    with torch.no_grad():
        for nm in ('norm1', 'norm2', 'norm3'):
            getattr(layer, nm).weight.normal_(1.0, 0.2)
            getattr(layer, nm).bias.normal_(0.0, 0.2)
    sd = {f'l.{k}': v.clone() for k, v in layer.state_dict().items()}
    g = torch.Generator().manual_seed(6)
    src = torch.randn(L, B, d, generator=g) + 1.0
    tgt = torch.randn(L, B, d, generator=g) - 0.5
    spos = torch.randn(L, B, d, generator=g)
    tpos = torch.randn(L, B, d, generator=g)
    mask = torch.zeros(B, L, dtype=torch.bool)
    rs, rt = mo.cross_encoder_layer(sd, 'l', src, tgt, mask, mask, spos, tpos, nhead)
    pack = lambda a, c: torch.cat([a[:, b] for b in range(B)] + [c[:, b] for b in range(B)])  # noqa: E731
    x, pos = pack(src, tgt).to(gpu), pack(spos, tpos).to(gpu)
    ref = pack(rs, rt)
    layer = layer.to(gpu).eval()
    seg = Segments([L] * (2 * B), gpu)
    with torch.no_grad():
        y, pending = layer.forward_packed(x.clone(), pos, seg)
        if pending is not None:
            y = y + pending
    assert rel_err(y, ref) < 1e-4


@pytest.mark.parametrize('d', [64, 256, 512, 96, 1024])
def test_layernorm_dual_matches_two_passes(gpu, d):
    """fgr_layernorm_dual (the encoder's output norm of layer l and norm1 + pos of layer l + 1
    in one pass) == two fgr_layernorm launches, bit for bit (d 96 / 1024: the two-launch
    fallback inside the library)."""
    from fgreg import ops
    g = torch.Generator().manual_seed(d)
    x = (2.0 + 3.0 * torch.randn(777, d, generator=g)).to(gpu)
    pos = torch.randn(777, d, generator=g).to(gpu)
    na, nb = torch.nn.LayerNorm(d), torch.nn.LayerNorm(d)
    with torch.no_grad():
        for nm in (na, nb):
            nm.weight.copy_(1 + 0.3 * torch.randn(d, generator=g))
            nm.bias.copy_(0.3 * torch.randn(d, generator=g))
    na, nb = na.to(gpu), nb.to(gpu)
    x0 = x.clone()
    a, b = ops.layernorm_dual(x, na, nb, add_b=pos)
    ra = ops.layernorm(x, na.weight, na.bias, na.eps)
    rb = ops.layernorm(x, nb.weight, nb.bias, nb.eps, add=pos)
    assert torch.equal(x, x0)
    assert torch.equal(a, ra) and torch.equal(b, rb)
    ref = torch.nn.functional.layer_norm(x.double(), (d,), nb.weight.double(), nb.bias.double(), nb.eps) + pos.double()
    assert rel_err(b, ref) < 1e-5


def test_gemm_ln_side_output(gpu):
    """fgr_gemm_f16x3_ln_out2: the GEMM as fgr_gemm_f16x3_ln, plus out2 = LayerNorm(x) with a
    second affine (written once per row) == ops.layernorm to fp32 rounding."""
    from fgreg import linear as fl
    from fgreg import ops
    m, n, k = 9544, 768, 256
    x, norm, pos, w, b = _inputs(m, k, n, 11)
    norm2 = torch.nn.LayerNorm(k)
    with torch.no_grad():
        norm2.weight.normal_(1.0, 0.3)
        norm2.bias.normal_(0.0, 0.3)
    X, P, W, B = x.to(gpu), pos.to(gpu), w.to(gpu), b.to(gpu)
    N, N2 = norm.to(gpu), norm2.to(gpu)
    out2 = torch.full((m, k), float('nan'), device=gpu)
    y = fl.linear_ln(X, N, W, B, add=P, side=(N2, out2))
    assert rel_err(y, fl.linear_ln(X, N, W, B, add=P)) == 0.0
    ref2 = ops.layernorm(X, N2.weight, N2.bias, N2.eps)
    assert torch.isfinite(out2).all() and rel_err(out2, ref2) < 1e-6


def test_encoder_bench_size_vs_oracle(gpu):
    """TransformerCrossEncoder (3 pre-norm layers, return_intermediate, final norm) at the
    ModelNet bench size: every in_proj / linear1 takes the fused LayerNorm launch and each
    layer's output norm is written by the next layer's fused launch; the stacked outputs
    against the oracle's forward_pre + norm per layer (transformers.py:31-59)."""
    from fgreg import linear as fl
    from fgreg.transformer import (Segments, TransformerCrossEncoder,
                                   TransformerCrossEncoderLayer)
    d, nhead, ff, B, L, NL = 256, 8, 1024, 8, 596, 3
    assert fl.ln_fusable(2 * B * L, 3 * d, d)
    torch.manual_seed(9)
    layer = TransformerCrossEncoderLayer(d, nhead, ff, 0.0, normalize_before=True,
                                         sa_val_has_pos_emb=True, ca_val_has_pos_emb=True)
    enc = TransformerCrossEncoder(layer, NL, torch.nn.LayerNorm(d), return_intermediate=True)
    with torch.no_grad():
        for mod in enc.modules():
            if isinstance(mod, torch.nn.LayerNorm):
                mod.weight.normal_(1.0, 0.2)
                mod.bias.normal_(0.0, 0.2)
    sd = {f'e.{kk}': v.clone() for kk, v in enc.state_dict().items()}
    g = torch.Generator().manual_seed(10)
    src = torch.randn(L, B, d, generator=g)
    tgt = torch.randn(L, B, d, generator=g)
    spos = torch.randn(L, B, d, generator=g)
    tpos = torch.randn(L, B, d, generator=g)
    mask = torch.zeros(B, L, dtype=torch.bool)
    refs = []
    s_, t_ = src, tgt
    for i in range(NL):
        s_, t_ = mo.cross_encoder_layer(sd, f'e.layers.{i}', s_, t_, mask, mask, spos, tpos, nhead)
        refs.append((mo._ln(sd, 'e.norm', s_), mo._ln(sd, 'e.norm', t_)))
    pack = lambda a, c: torch.cat([a[:, b] for b in range(B)] + [c[:, b] for b in range(B)])  # noqa: E731
    enc = enc.to(gpu).eval()
    with torch.no_grad():
        out = enc.forward_packed(pack(src, tgt).to(gpu), pack(spos, tpos).to(gpu),
                                 Segments([L] * (2 * B), gpu))
    assert out.shape == (NL, 2 * B * L, d)
    for i in range(NL):
        assert rel_err(out[i], pack(*refs[i])) < 1e-4, i


@pytest.mark.parametrize('lens,side', [([717, 596, 1, 700, 64, 130, 5000, 2336], False),
                                       ([596] * 16, True), ([65, 63, 64, 1, 128], False),
                                       ([6000, 5999, 6001, 6000], False), ([3001] * 8, True)])
def test_ln_qkv_images_vs_two_launch_path(gpu, lens, side):
    """fgr_gemm_f16x3_ln_qkv (the in_proj writing q fp32 and the K / V images of every global
    64-row tile, head dim 32) + fgr_attention_f16x3_img vs the path it replaces (LN-fused in_proj
    -> fp32 q | k | v -> fgr_attention_f16x3 with per-segment images): segments starting
    anywhere inside a tile (incl. a 1-row cloud and tiles shared by three clouds), self- and
    cross-attention, the side output, 24000 rows (1125 blocks of the split in_proj, more than one
    round on the chip). Both are fp32-accurate: <= 2e-6 normwise apart and
    <= 1e-5 from a float64 LayerNorm -> in_proj -> softmax attention."""
    from fgreg import linear as lin
    from fgreg import ops
    n, d, nh = sum(lens), 256, 8
    x, norm, pos, w, b = _inputs(n, d, 3 * d, seed=len(lens))
    x, pos, w, b, norm = x.to(gpu), pos.to(gpu), w.to(gpu), b.to(gpu), norm.to(gpu)
    assert ops.ln_qkv_supported(n, d, nh) or n < 8000
    if not ops.ln_qkv_supported(n, d, nh):
        pytest.skip('shape not on the row-stationary path')
    off = ops.offsets(lens, gpu)
    B = len(lens) // 2
    for kv in (list(range(len(lens))), [(c + B) % len(lens) for c in range(len(lens))]
               if len(lens) % 2 == 0 else list(range(len(lens)))):
        kv_seg = torch.tensor(kv, dtype=torch.int32, device=gpu)
        norm2 = torch.nn.LayerNorm(d).to(gpu)
        out2 = torch.empty_like(x) if side else None
        o = ops.ln_qkv_attention(x, norm, lin.weight_image(w, mode='f16x3'), b, pos, off, kv_seg,
                                 max(lens), nh, side=(norm2, out2) if side else None)
        qkv = lin.linear_ln(x, norm, w, b, add=pos)
        o2 = ops.attention(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], off, off, kv_seg,
                           max(lens), nh)
        assert rel_err(o, o2) < 2e-6, rel_err(o, o2)
        h = torch.nn.functional.layer_norm(x.double(), (d,), norm.weight.double(),
                                           norm.bias.double(), norm.eps) + pos.double()
        qkv64 = h @ w.double().t() + b.double()
        offs = np.cumsum([0] + lens)
        outs = []
        for i in range(len(lens)):
            j = kv[i]
            q = qkv64[offs[i]:offs[i + 1], :d].reshape(-1, nh, 32).transpose(0, 1) / math.sqrt(32)
            k = qkv64[offs[j]:offs[j + 1], d:2 * d].reshape(-1, nh, 32).transpose(0, 1)
            v = qkv64[offs[j]:offs[j + 1], 2 * d:].reshape(-1, nh, 32).transpose(0, 1)
            outs.append((torch.softmax(q @ k.transpose(1, 2), -1) @ v).transpose(0, 1).reshape(-1, d))
        o64 = torch.cat(outs, 0)
        assert rel_err(o, o64) < 1e-5, rel_err(o, o64)
        if side:
            ref2 = torch.nn.functional.layer_norm(x.double(), (d,), norm2.weight.double(),
                                                  norm2.bias.double(), norm2.eps)
            assert rel_err(out2, ref2) < 1e-6


@pytest.mark.parametrize('lens', [[1060, 1060], [1100, 977, 64, 1, 3000, 130]])
def test_qkv_images_dh64_vs_two_launch_path(gpu, lens):
    """fgr_gemm_f16x3_qkv (in_proj without the LayerNorm prologue writing q fp32 and the head
    dim 64 K / V images of every global 64-row tile in the staged g5 epilogue: the 3DMatch
    transformer, d 512 / 8 heads) + fgr_attention_f16x3_img vs linear -> fgr_attention_f16x3
    (<= 2e-6 apart) and vs float64 (<= 1e-5), self- and cross-attention, segments starting
    inside tiles."""
    from fgreg import linear as lin
    from fgreg import ops
    n, d, nh = sum(lens), 512, 8
    g = torch.Generator().manual_seed(n)
    h = (torch.randn(n, d, generator=g) * 1.5).to(gpu)
    w = (torch.randn(3 * d, d, generator=g) / math.sqrt(d)).to(gpu)
    b = torch.randn(3 * d, generator=g).to(gpu)
    assert ops.qkv_supported(n, d, nh)
    off = ops.offsets(lens, gpu)
    B = len(lens) // 2
    for kv in (list(range(len(lens))), [(c + B) % len(lens) for c in range(len(lens))]):
        kv_seg = torch.tensor(kv, dtype=torch.int32, device=gpu)
        o = ops.qkv_attention(h, lin.weight_image(w, mode='f16x3'), b, off, kv_seg, max(lens), nh)
        qkv = lin.linear(h, w, b)
        o2 = ops.attention(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], off, off, kv_seg,
                           max(lens), nh)
        assert rel_err(o, o2) < 2e-6, rel_err(o, o2)
        qkv64 = h.double() @ w.double().t() + b.double()
        offs = np.cumsum([0] + lens)
        outs = []
        for i in range(len(lens)):
            j = kv[i]
            q = qkv64[offs[i]:offs[i + 1], :d].reshape(-1, nh, 64).transpose(0, 1) / 8.0
            k = qkv64[offs[j]:offs[j + 1], d:2 * d].reshape(-1, nh, 64).transpose(0, 1)
            v = qkv64[offs[j]:offs[j + 1], 2 * d:].reshape(-1, nh, 64).transpose(0, 1)
            outs.append((torch.softmax(q @ k.transpose(1, 2), -1) @ v).transpose(0, 1).reshape(-1, d))
        assert rel_err(o, torch.cat(outs, 0)) < 1e-5
