"""Training backward on the GPU: every differentiable op of
fgreg/autograd.py against torch autograd in fp64 on the same inputs, then whole training steps
(train() forward + loss + backward) against the reference's own gradients and the fp64 oracle.

Gradient tolerances. Each op's backward is checked at fp32-accuracy level (normwise 1e-5 / 1e-4
for the reductions over tens of thousands of rows). End to end the gradient of this network is
discontinuous wherever a ReLU / LeakyReLU input sits at its kink or two max-pool candidates
tie; on random models thousands of activations lie within 1e-7..1e-6 (relative) of a kink
(model_oracle.ACT_TRACE), so ANY two fp32 implementations take a few different branches: the
oracle computed with torch's fused BatchNorm / InstanceNorm and the same oracle with the
decomposed formulas differ by 0.7-1.9e-3 in the encoder gradients (Frobenius), although each
agrees with its own fp64 run elsewhere. The whole-step checks therefore bound the encoder /
transformer gradients at GRAD_TOL = 1e-2 relative Frobenius (a wiring or formula error is
O(1)), the losses at 1e-5, and print the measured errors.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import model_oracle as mo
from conftest import (forward_fixture, is_trainable, loss_fixture, oracle_train_grads,
                      rel_err, train_fixture)

pytestmark = pytest.mark.gpu

GRAD_TOL = 1e-2


def fro(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _leaf(t, gpu):
    return t.detach().to(gpu).float().requires_grad_(True), t.detach().double().requires_grad_(True)


# ------------------------------------------------------------------------------------------
# per-op backward vs torch fp64 autograd
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize('m,n,k', [(1000, 80, 96), (9544, 256, 128), (37, 3, 32), (2000, 1, 256)])
@pytest.mark.parametrize('act', ['none', 'relu', 'residual'])
def test_linear_backward(gpu, m, n, k, act):
    from fgreg import ops
    from fgreg.autograd import linear_t
    g = torch.Generator().manual_seed(m + n + k)
    x, x64 = _leaf(torch.randn(m, k, generator=g), gpu)
    w, w64 = _leaf(torch.randn(n, k, generator=g) / math.sqrt(k), gpu)
    b, b64 = _leaf(torch.randn(n, generator=g), gpu)
    r, r64 = _leaf(torch.randn(m, n, generator=g), gpu)
    R = torch.randn(m, n, generator=g)
    if act == 'relu':
        y = linear_t(x, w, b, act=ops.ACT_RELU)
        y64 = torch.relu(x64 @ w64.t() + b64)
    elif act == 'residual':
        y = linear_t(x, w, b, residual=r)
        y64 = x64 @ w64.t() + b64 + r64
    else:
        y = linear_t(x, w, b)
        y64 = x64 @ w64.t() + b64
    (y * R.to(gpu)).sum().backward()
    (y64 * R.double()).sum().backward()
    assert rel_err(y, y64) < 1e-5
    for t, t64, name in ((x, x64, 'dx'), (w, w64, 'dw'), (b, b64, 'db')):
        assert rel_err(t.grad, t64.grad) < 1e-5, (name, rel_err(t.grad, t64.grad))
    if act == 'residual':
        assert rel_err(r.grad, r64.grad) < 1e-6


def _kpconv_case(cin):
    gk = np.load(__import__('conftest').GOLDEN + '/kpconv_block.npz')
    q, s = torch.from_numpy(gk['q']), torch.from_numpy(gk['s'])
    idx = torch.from_numpy(gk['idx'].astype(np.int64))
    kp = torch.from_numpy(gk['kp'])
    extent = float(gk['extent'])
    g = torch.Generator().manual_seed(cin)
    x = torch.randn(s.shape[0], cin, generator=g)    # features of the support rows
    x[::5] = -x[::5].abs()                       # rows that do not count in the normaliser
    W = torch.randn(15, cin, 24, generator=g) / math.sqrt(15 * cin)
    return q, s, idx, kp, extent, x, W, gk


@pytest.mark.parametrize('cin', [1, 16, 32, 64, 128, 256])
@pytest.mark.parametrize('strided', [False, True])
def test_kpconv_backward(gpu, cin, strided):
    """kpconv_t (gather + weight GEMM, normalised by the returned nnorm) vs the oracle's KPConv
    (finegrained_kpconv_blocks.py:265-401 restated) in fp64: dx (fgr_kpconv_scatter) and dW."""
    from fgreg.autograd import kpconv_t
    q, s, idx, kp, extent, x0, W0, gk = _kpconv_case(cin)
    if strided:
        q = torch.from_numpy(gk['sub'])
        idx = torch.from_numpy(gk['pools'].astype(np.int64))

    class Conv:
        pass
    conv = Conv()
    x, x64 = _leaf(x0, gpu)
    W, W64 = _leaf(W0, gpu)
    conv.weights, conv.kernel_points, conv.KP_extent = W, kp.to(gpu), extent
    out, nnorm = kpconv_t(conv, q.to(gpu), s.to(gpu), idx.to(gpu), x)
    y = out / nnorm.unsqueeze(1)
    y64 = mo.kpconv(q.double(), s.double(), idx, x64, W64, kp.double(), extent)
    R = torch.randn(y64.shape, generator=torch.Generator().manual_seed(3))
    (y * R.to(gpu)).sum().backward()
    (y64 * R.double()).sum().backward()
    assert rel_err(y, y64) < 1e-5
    assert rel_err(x.grad, x64.grad) < 1e-5, rel_err(x.grad, x64.grad)
    assert rel_err(W.grad, W64.grad) < 1e-5, rel_err(W.grad, W64.grad)


def test_max_pool_backward(gpu):
    from fgreg.autograd import max_pool_t
    gk = np.load(__import__('conftest').GOLDEN + '/kpconv_block.npz')
    idx = torch.from_numpy(gk['pools'].astype(np.int64))
    x0 = torch.randn(gk['s'].shape[0], 48, generator=torch.Generator().manual_seed(1))
    x0[:, :8] = -x0[:, :8].abs()                 # channels where the shadow zero wins
    x, x64 = _leaf(x0, gpu)
    y = max_pool_t(x, idx.to(gpu))
    y64 = mo.max_pool(x64, idx)
    R = torch.randn(y64.shape, generator=torch.Generator().manual_seed(2))
    (y * R.to(gpu)).sum().backward()
    (y64 * R.double()).sum().backward()
    assert torch.equal(y.cpu().double(), y64.detach())
    assert rel_err(x.grad, x64.grad) < 1e-6


def _segnorm_ref(x, lens, row_div, gamma, beta, act, residual, post, eps=1e-5):
    v = x / row_div[:, None] if row_div is not None else x
    outs, o = [], 0
    for n in lens:
        seg = v[o:o + n]
        mu = seg.mean(0)
        var = ((seg - mu) ** 2).mean(0)
        outs.append((seg - mu) / torch.sqrt(var + eps))
        o += n
    z = torch.cat(outs, 0)
    if gamma is not None:
        z = z * gamma + beta
    fa = {'none': lambda t: t, 'relu': F.relu, 'leaky': lambda t: F.leaky_relu(t, 0.1)}
    y = fa[act](z)
    if residual is not None:
        y = fa[post](y + residual)
    return y


@pytest.mark.parametrize('case', ['instnorm', 'instnorm_rowdiv_leaky', 'instnorm_residual',
                                  'batchnorm_relu', 'batchnorm_residual_relu', 'long_segments',
                                  'batchnorm_large'])
@pytest.mark.parametrize('c', [72, 70])
def test_segnorm_backward(gpu, case, c):
    """segnorm_t: InstanceNorm per cloud (with the KPConv row divisor, LeakyReLU, the
    bottleneck's residual + LeakyReLU) and training BatchNorm (one segment, affine, ReLU,
    residual + ReLU) vs the same formulas in fp64; c = 72 runs the float4 kernels, 70 the
    scalar ones. Chunks of 256 rows per segment: <= 16 (merge fused in order), 47
    (batchnorm_large: the fused four-way merge), 79 (long_segments: separate merges)."""
    from fgreg import ops
    from fgreg.autograd import segnorm_t
    g = torch.Generator().manual_seed(len(case))
    lens = [700, 300, 1, 513] if case != 'long_segments' else [20000, 9000]
    if case.startswith('batchnorm'):
        lens = [sum(lens)] if case != 'batchnorm_large' else [12000]
    n = sum(lens)
    x, x64 = _leaf(torch.randn(n, c, generator=g) * 3 + 5, gpu)
    rd = (1 + torch.randint(0, 9, (n,), generator=g)).float() if 'rowdiv' in case else None
    affine = case.startswith('batchnorm')
    gm, gm64 = _leaf(1 + 0.2 * torch.randn(c, generator=g), gpu) if affine else (None, None)
    bt, bt64 = _leaf(0.1 * torch.randn(c, generator=g), gpu) if affine else (None, None)
    res = 'residual' in case
    r, r64 = _leaf(torch.randn(n, c, generator=g), gpu) if res else (None, None)
    act = {'instnorm': 'none', 'instnorm_rowdiv_leaky': 'leaky', 'instnorm_residual': 'none',
           'batchnorm_relu': 'relu', 'batchnorm_residual_relu': 'none', 'long_segments': 'leaky',
           'batchnorm_large': 'relu'}[case]
    post = 'relu' if case == 'batchnorm_residual_relu' else 'leaky'
    A = {'none': ops.ACT_NONE, 'relu': ops.ACT_RELU, 'leaky': ops.ACT_LEAKY}
    off = ops.offsets(lens, gpu)
    y = segnorm_t(x, off, lens, row_div=rd.to(gpu) if rd is not None else None, act=A[act],
                  residual=r, post_act=A[post], gamma=gm, beta=bt)
    y64 = _segnorm_ref(x64, lens, rd.double() if rd is not None else None, gm64, bt64, act, r64,
                       post)
    R = torch.randn(n, c, generator=g)
    (y * R.to(gpu)).sum().backward()
    (y64 * R.double()).sum().backward()
    assert rel_err(y, y64) < 1e-5
    assert rel_err(x.grad, x64.grad) < 1e-4, rel_err(x.grad, x64.grad)
    if affine:
        assert rel_err(gm.grad, gm64.grad) < 1e-5 and rel_err(bt.grad, bt64.grad) < 1e-5
    if res:
        assert rel_err(r.grad, r64.grad) < 1e-5


def test_segnorm_fused_bit_identical(gpu, tmp_path):
    """The fused merge + apply kernels (segments of <= 16 chunks: one launch per direction
    fewer) give bit-identical outputs and gradients to the separate merge kernels
    (FGR_SEG_FUSED=0 in a subprocess): InstanceNorm with row divisor + residual, BatchNorm
    with gamma / beta."""
    import os
    import subprocess
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import _segnorm_dump
    here = _segnorm_dump.run(gpu)
    f = tmp_path / 'unfused.npz'
    env = dict(os.environ, FGR_SEG_FUSED='0')
    subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), '_segnorm_dump.py'), str(f)],
                   env=env, check=True, timeout=240)
    ref = np.load(f)
    assert sorted(ref.files) == sorted(here)
    for k in ref.files:
        assert np.array_equal(ref[k], here[k]), k


def test_batchnorm_running_stats(gpu):
    """batchnorm_t updates running_mean / running_var / num_batches_tracked like
    nn.BatchNorm1d.train() (momentum, unbiased variance)."""
    from fgreg.autograd import batchnorm_t
    bn = torch.nn.BatchNorm1d(40).to(gpu)
    ref = torch.nn.BatchNorm1d(40)
    with torch.no_grad():
        for m in (bn, ref):
            m.running_mean.fill_(0.3)
            m.running_var.fill_(2.0)
    x = torch.randn(3001, 40) * 2 + 1
    for _ in range(2):
        y = batchnorm_t(bn, x.to(gpu))
        y_ref = ref.train()(x)
    assert rel_err(y, y_ref) < 1e-5
    assert rel_err(bn.running_mean, ref.running_mean) < 1e-6
    assert rel_err(bn.running_var, ref.running_var) < 1e-6
    assert int(bn.num_batches_tracked) == int(ref.num_batches_tracked) == 2


@pytest.mark.parametrize('d', [32, 256, 512, 96])
def test_layernorm_backward(gpu, d):
    from fgreg.autograd import layernorm_t
    n = 3000
    g = torch.Generator().manual_seed(d)
    norm = torch.nn.LayerNorm(d).to(gpu)
    with torch.no_grad():
        norm.weight.copy_(1 + 0.2 * torch.randn(d, generator=g))
        norm.bias.copy_(0.1 * torch.randn(d, generator=g))
    x, x64 = _leaf(torch.randn(n, d, generator=g) * 2 + 3, gpu)
    pos = torch.randn(n, d, generator=g)
    y = layernorm_t(x, norm, add=pos.to(gpu))
    w64 = norm.weight.detach().cpu().double().requires_grad_(True)
    b64 = norm.bias.detach().cpu().double().requires_grad_(True)
    y64 = F.layer_norm(x64, (d,), w64, b64, 1e-5) + pos.double()
    R = torch.randn(n, d, generator=g)
    (y * R.to(gpu)).sum().backward()
    (y64 * R.double()).sum().backward()
    assert rel_err(y, y64) < 1e-5
    assert rel_err(x.grad, x64.grad) < 1e-5
    assert rel_err(norm.weight.grad, w64.grad) < 1e-5
    assert rel_err(norm.bias.grad, b64.grad) < 1e-5


def _attn_ref(qkv, lens, kv_seg, nhead):
    d = qkv.shape[1] // 3
    dh = d // nhead
    off = np.cumsum([0] + lens)
    outs = []
    for i in range(len(lens)):
        j = kv_seg[i]
        q = qkv[off[i]:off[i + 1], :d].reshape(-1, nhead, dh).transpose(0, 1) / math.sqrt(dh)
        k = qkv[off[j]:off[j + 1], d:2 * d].reshape(-1, nhead, dh).transpose(0, 1)
        v = qkv[off[j]:off[j + 1], 2 * d:].reshape(-1, nhead, dh).transpose(0, 1)
        outs.append((torch.softmax(q @ k.transpose(1, 2), -1) @ v).transpose(0, 1).reshape(-1, d))
    return torch.cat(outs, 0)


_KV_SEG = {'self': [0, 1, 2, 3], 'cross': [2, 3, 0, 1], 'shared': [3, 3, 0, 0]}


@pytest.mark.parametrize('d,nhead', [(32, 8), (256, 8), (512, 8)])
@pytest.mark.parametrize('kind', ['self', 'cross', 'shared'])
def test_attention_backward(gpu, d, nhead, kind):
    """attention_t (fused QKV; self = every cloud to itself, cross = cloud c to (c + B) mod 2B,
    shared = two query clouds on one key cloud: its dK / dV sum over both) vs fp64 softmax
    attention: dq, dk, dv through fgr_attention_bwd (head dim 4) / fgr_attention_bwd_train
    (head dims 32 / 64: the f16x3 kernels), unequal lengths incl. a 1-row cloud and clouds past
    one 64-row tile."""
    from fgreg import ops
    from fgreg.autograd import attention_t
    lens = [130, 1, 65, 300]
    kv_seg = _KV_SEG[kind]
    g = torch.Generator().manual_seed(d)
    qkv, qkv64 = _leaf(torch.randn(sum(lens), 3 * d, generator=g), gpu)
    off = ops.offsets(lens, gpu)
    o = attention_t(qkv, off, torch.tensor(kv_seg, dtype=torch.int32, device=gpu), max(lens), nhead)
    o64 = _attn_ref(qkv64, lens, kv_seg, nhead)
    R = torch.randn(o64.shape, generator=g)
    (o * R.to(gpu)).sum().backward()
    (o64 * R.double()).sum().backward()
    assert rel_err(o, o64) < 1e-5
    for sl, name in ((slice(0, d), 'dq'), (slice(d, 2 * d), 'dk'), (slice(2 * d, 3 * d), 'dv')):
        e = rel_err(qkv.grad[:, sl], qkv64.grad[:, sl])
        assert e < 1e-5, (name, e)


def _attn_ref_drop(qkv, lens, kv_seg, nhead, seed, p):
    """_attn_ref with nn.MultiheadAttention's attention-weight dropout, the mask of
    fgr_attention_f16x3_drop restated (fgreg.autograd.attn_drop_mask, packed row indices)."""
    from fgreg.autograd import attn_drop_mask
    d = qkv.shape[1] // 3
    dh = d // nhead
    off = np.cumsum([0] + lens)
    outs = []
    for i in range(len(lens)):
        j = kv_seg[i]
        q = qkv[off[i]:off[i + 1], :d].reshape(-1, nhead, dh).transpose(0, 1) / math.sqrt(dh)
        k = qkv[off[j]:off[j + 1], d:2 * d].reshape(-1, nhead, dh).transpose(0, 1)
        v = qkv[off[j]:off[j + 1], 2 * d:].reshape(-1, nhead, dh).transpose(0, 1)
        P = torch.softmax(q @ k.transpose(1, 2), -1)
        keep = torch.stack([torch.from_numpy(~attn_drop_mask(seed, p, h, range(off[i], off[i + 1]),
                                                             range(off[j], off[j + 1])))
                            for h in range(nhead)]).to(P.dtype)
        outs.append(((P * keep / (1 - p)) @ v).transpose(0, 1).reshape(-1, d))
    return torch.cat(outs, 0)


@pytest.mark.parametrize('prec', ['fp32', 'bf16'])
@pytest.mark.parametrize('d,nhead', [(256, 8), (512, 8)])
@pytest.mark.parametrize('kind', ['self', 'cross', 'shared'])
def test_attention_dropout_forward_backward(gpu, d, nhead, kind, prec):
    """Training-mode attention-weight dropout (nn.MultiheadAttention(dropout=p),
    transformers.py:95-96): fgr_attention_f16x3_drop / fgr_attention_bwd_drop against fp64
    softmax attention with the SAME mask (the kernels' counter-based hash restated in numpy):
    output and dq / dk / dv; the dropped fraction is p; p = 0 is the plain path. In the bf16
    mode the dropout path runs the same fp32-accurate kernels (same mask, same bound); its
    p = 0 path is the bf16 attention (bf16 bound)."""
    import fgreg
    prev = fgreg.precision()
    fgreg.set_precision(prec)
    try:
        _attention_dropout_case(gpu, d, nhead, kind, prec)
    finally:
        fgreg.set_precision(prev)


def _attention_dropout_case(gpu, d, nhead, kind, prec):
    from fgreg import ops
    from fgreg.autograd import _AttentionFn, attn_drop_mask
    lens = [130, 1, 65, 300]
    kv_seg = _KV_SEG[kind]
    g = torch.Generator().manual_seed(d + 7)
    qkv, qkv64 = _leaf(torch.randn(sum(lens), 3 * d, generator=g), gpu)
    off = ops.offsets(lens, gpu)
    ks = torch.tensor(kv_seg, dtype=torch.int32, device=gpu)
    seed, p = 987654321, 0.3
    o = _AttentionFn.apply(qkv, off, ks, max(lens), nhead, p, seed)
    o64 = _attn_ref_drop(qkv64, lens, kv_seg, nhead, seed, p)
    R = torch.randn(o64.shape, generator=g)
    (o * R.to(gpu)).sum().backward()
    (o64 * R.double()).sum().backward()
    assert rel_err(o, o64) < 1e-5
    for sl, name in ((slice(0, d), 'dq'), (slice(d, 2 * d), 'dk'), (slice(2 * d, 3 * d), 'dv')):
        e = rel_err(qkv.grad[:, sl], qkv64.grad[:, sl])
        assert e < 1e-5, (name, e)
    m = attn_drop_mask(seed, p, 3, range(300), range(300))
    assert abs(float(m.mean()) - p) < 0.01
    o0 = _AttentionFn.apply(qkv.detach(), off, ks, max(lens), nhead, 0.0, seed)
    assert rel_err(o0, _attn_ref(qkv64.detach(), lens, kv_seg, nhead)) < (1e-5 if prec == "fp32" else 5e-2)


def test_train_step_with_dropout(gpu):
    """A ModelNet training step with dropout 0.1 (every transformer dropout of
    transformers.py:95-110): finite losses and gradients, bit-identical under the same
    torch seed, different under another; dropout 0 gives the round-4 step."""
    import fgreg
    import fgreg.config as fc
    from fgreg.loss import compute_loss_train
    from fgreg.synthetic import make_batch

    def step(drop, seed):
        torch.manual_seed(0)
        np.random.seed(0)                # kernel points and the synthetic crops draw from numpy
        model = fgreg.RegTR(fc.get('modelnet', dropout=drop)).to(gpu).train()
        src, tgt, pose = make_batch('modelnet', 2)
        batch = {'src_xyz': [torch.from_numpy(a).to(gpu) for a in src],
                 'tgt_xyz': [torch.from_numpy(b).to(gpu) for b in tgt],
                 'pose': torch.from_numpy(np.asarray(pose, np.float32)).to(gpu),
                 'src_overlap': [torch.ones(len(a), device=gpu) for a in src],
                 'tgt_overlap': [torch.ones(len(b), device=gpu) for b in tgt]}
        torch.manual_seed(seed)
        out = model(batch)
        loss = compute_loss_train(model, out, batch)['total']
        loss.backward()
        g = torch.cat([p.grad.flatten() for p in model.parameters() if p.grad is not None])
        return float(loss.detach()), g
    l1, g1 = step(0.1, 5)
    l2, g2 = step(0.1, 5)
    l3, g3 = step(0.1, 6)
    l0, g0 = step(0.0, 5)
    assert math.isfinite(l1) and bool(torch.isfinite(g1).all())
    assert l1 == l2 and torch.equal(g1, g2)
    assert l1 != l3 and l1 != l0
    # the bf16 mode trains with dropout too (round 6): reproducible under one seed, and close to
    # the fp32-accurate step with the same masks (the bf16 products' own error)
    prev = fgreg.precision()
    fgreg.set_precision('bf16')
    try:
        b1, h1 = step(0.1, 5)
        b2, h2 = step(0.1, 5)
    finally:
        fgreg.set_precision(prev)
    assert math.isfinite(b1) and bool(torch.isfinite(h1).all())
    assert b1 == b2 and torch.equal(h1, h2)
    assert abs(b1 - l1) < 5e-2 * abs(l1)


@pytest.mark.parametrize('d', [64, 256])
def test_corr_attention_backward(gpu, d):
    """corr_attention_t (CorrespondenceDecoder.simple_attention over the (layer, cloud)
    segments, finegrained_regtr.py:328-363) vs fp64 autograd of the reference formula: dq, dk
    through fgr_corr_attention_bwd; unequal clouds incl. a 1-row cloud, 2 layers."""
    from fgreg.autograd import corr_attention_t
    from fgreg.transformer import Segments
    lens = [130, 1, 65, 300]
    B, L = 2, 2
    N = sum(lens)
    g = torch.Generator().manual_seed(d)
    q, q64 = _leaf(torch.randn(L * N, d, generator=g), gpu)
    k, k64 = _leaf(torch.randn(L * N, d, generator=g), gpu)
    xyz = torch.randn(N, 3, generator=g)
    seg = Segments(lens, gpu, n_layers=L)
    corr = corr_attention_t(q, k, xyz.to(gpu), seg, 1.0 / math.sqrt(d))
    off = np.cumsum([0] + lens)
    outs = []
    for l in range(L):
        for c in range(2 * B):
            p = (c + B) % (2 * B)
            qi = q64[l * N + off[c]:l * N + off[c + 1]] / math.sqrt(d)
            kj = k64[l * N + off[p]:l * N + off[p + 1]]
            outs.append(torch.softmax(qi @ kj.t(), -1) @ xyz[off[p]:off[p + 1]].double())
    corr64 = torch.cat(outs, 0)
    R = torch.randn(corr64.shape, generator=g)
    (corr * R.to(gpu)).sum().backward()
    (corr64 * R.double()).sum().backward()
    assert rel_err(corr, corr64) < 1e-5
    assert rel_err(q.grad, q64.grad) < 1e-5, rel_err(q.grad, q64.grad)
    assert rel_err(k.grad, k64.grad) < 1e-5, rel_err(k.grad, k64.grad)


@pytest.mark.parametrize('strided', [False, True])
def test_nbr_inverse(gpu, strided):
    """fgr_nbr_inverse: the CSR inverse of a neighbour table (the golden KPConv block's conv /
    pool tables with their shadow entries) equals the host's stable inverse."""
    from fgreg.autograd import nbr_inverse
    gk = np.load(__import__('conftest').GOLDEN + '/kpconv_block.npz')
    idx = gk['pools' if strided else 'idx'].astype(np.int64)
    ns = gk['s'].shape[0]
    start, pos, ent = (t.cpu().numpy() for t in nbr_inverse(torch.from_numpy(idx).to(gpu), ns))
    flat = idx.reshape(-1)
    valid = (flat >= 0) & (flat < ns)
    e = np.nonzero(valid)[0]
    order = e[np.argsort(flat[e], kind='stable')]
    cnt = np.bincount(flat[e], minlength=ns)
    assert np.array_equal(start, np.concatenate([[0], np.cumsum(cnt)]))
    assert np.array_equal(ent[:len(order)], order)
    want_pos = np.full(flat.shape, -1)
    want_pos[order] = np.arange(len(order))
    assert np.array_equal(pos[:flat.size], want_pos)


def test_backward_is_deterministic(gpu):
    """Two backward passes of one training step give bit-identical gradients (no floating-
    point atomics: the KPConv / max-pool scatters are gathers over the table's inverse)."""
    import fgreg
    import fgreg.config as fc
    from fgreg.synthetic import make_batch
    cfg = fc.get('modelnet')
    torch.manual_seed(7)
    model = fgreg.RegTR(cfg).to(gpu).train()
    src, tgt, _ = make_batch('modelnet', 2)
    batch = {'src_xyz': [torch.from_numpy(s).to(gpu) for s in src],
             'tgt_xyz': [torch.from_numpy(t).to(gpu) for t in tgt]}
    runs = []
    for _ in range(2):
        model.zero_grad(set_to_none=True)
        out = model(batch)
        loss = sum((t.square().sum() for t in out['src_kp_warped'] + out['tgt_kp_warped']),
                   torch.zeros((), device=gpu))
        loss = loss + sum(f.sum() for f in out['src_feat'] + out['tgt_feat_un'])
        loss.backward()
        runs.append({k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None})
    assert runs[0].keys() == runs[1].keys() and len(runs[0]) > 100
    diff = [k for k in runs[0] if not torch.equal(runs[0][k], runs[1][k])]
    assert not diff, diff[:5]


def test_colsum(gpu):
    from fgreg.autograd import colsum
    x = torch.randn(40001, 300, dtype=torch.float64)
    got = colsum(x.float().to(gpu)[:, 7:250])
    assert rel_err(got, x.float().double()[:, 7:250].sum(0)) < 1e-6


@pytest.mark.parametrize('rows,m,n', [(0, 64, 32), (1, 4, 4), (37, 12, 20), (1000, 132, 260),
                                      (5000, 1, 256), (5000, 3, 130), (777, 15, 24),
                                      (9544, 256, 256), (9544, 1024, 2048), (11472, 128, 1920),
                                      (20000, 3840, 256)])
@pytest.mark.parametrize('strided', [False, True])
def test_wgrad(gpu, rows, m, n, strided):
    """fgr_gemm_f16x3_wgrad (dW = dY^T X straight from the activations) vs fp64: every element
    within 1e-6 of its Cauchy-Schwarz scale |dY[:, i]| |X[:, j]| -- columns spanning twelve
    decades, so a per-tile (not per-column) scale would fail -- and bit-identical on a rerun."""
    from fgreg import autograd as ag
    from fgreg import linear as lin
    assert lin.MODE == 'f16x3'
    g = torch.Generator().manual_seed(rows + m + n)
    a = torch.randn(rows, m, generator=g) * 10.0 ** torch.empty(m).uniform_(-6, 6, generator=g)
    b = torch.randn(rows, n, generator=g) * 10.0 ** torch.empty(n).uniform_(-6, 6, generator=g)
    a[: rows // 3] *= 1e-3                        # rows of very different size in one chunk
    if strided:
        ag_, bg_ = torch.zeros(rows, m + 12, device=gpu), torch.zeros(rows, n + 8, device=gpu)
        ag_[:, 8:8 + m] = a.to(gpu)
        bg_[:, 4:4 + n] = b.to(gpu)
        ad, bd = ag_[:, 8:8 + m], bg_[:, 4:4 + n]
    else:
        ad, bd = a.to(gpu), b.to(gpu)
    got = ag.wgrad(ad, bd)
    assert torch.equal(got, ag.wgrad(ad, bd))
    got2, db = ag.wgrad(ad, bd, bias_grad=True)        # the fused bias gradient: same dW
    assert torch.equal(got, got2)
    db_want = a.double().sum(0)
    assert ((db.double().cpu() - db_want).abs() <= 1e-6 * a.double().abs().sum(0) + 1e-30).all()
    got = got.double().cpu()
    want = a.double().t() @ b.double()
    scale = a.double().norm(dim=0)[:, None] * b.double().norm(dim=0)[None, :]
    err = ((got - want).abs() / scale.clamp_min(1e-300)).max().item() if rows else got.abs().max().item()
    assert err < 1e-6, err


# ------------------------------------------------------------------------------------------
# whole training steps
# ------------------------------------------------------------------------------------------
def _gpu_train_step(cfg, sd, src, tgt, meta, batch, W, W_un, gpu):
    """fgreg.RegTR in train() on the given neighbour tables; the checker's loss
    (loss_oracle.compute_loss) evaluated in fp64 on the host from the GPU outputs (so its
    geometric masks are computed exactly as on the oracle side), backward through the GPU
    graph -> (losses, grads, model)."""
    import fgreg
    import loss_oracle as lo
    model = fgreg.RegTR(cfg)
    model.load_state_dict({k: v for k, v in sd.items()}, strict=False)
    model = model.to(gpu).train()
    model.preprocessor = fgreg.FixedMetaPreprocessor({k: [t.to(gpu) for t in v]
                                                      for k, v in meta.items()})
    xb = {'src_xyz': [torch.from_numpy(np.asarray(s)).to(gpu) for s in src],
          'tgt_xyz': [torch.from_numpy(np.asarray(t)).to(gpu) for t in tgt]}
    pred = model(xb)
    host = {k: ([t.cpu().double() for t in v] if isinstance(v, list) else v.cpu().double())
            for k, v in pred.items()}
    Wg = W.detach().cpu().double().requires_grad_(True)
    Wug = W_un.detach().cpu().double().requires_grad_(True)
    cv = lambda t: t.cpu().double() if t.is_floating_point() else t.cpu()
    b = {'pose': cv(batch['pose']),
         'kpconv_meta': {k: [cv(t) for t in v] for k, v in batch['kpconv_meta'].items()},
         'src_overlap': [cv(t) for t in batch['src_overlap']],
         'tgt_overlap': [cv(t) for t in batch['tgt_overlap']]}
    losses, _ = lo.compute_loss(cfg, Wg, Wug, host, b)
    losses['total'].backward()
    grads = {k: p.grad for k, p in model.named_parameters() if p.grad is not None}
    grads['feature_criterion.W'] = Wg.grad
    grads['feature_criterion_un.W'] = Wug.grad
    return losses, grads, model


def test_train_step_vs_reference(gpu):
    """The reference's own train() step (tests/golden/train_modelnet_small.npz: forward +
    compute_loss + backward on the model / inputs / neighbour tables of forward_modelnet_small)
    vs fgreg's: losses within 1e-5, every parameter's gradient norm and the full gradients of
    one parameter of every kind within GRAD_TOL (see the module docstring), the Res2Net
    BatchNorm running statistics after the step within 1e-5."""
    cfg, sd, src, tgt, meta, batch, W, W_un, ref = train_fixture()
    losses, grads, model = _gpu_train_step(cfg, sd, src, tgt, meta, batch, W, W_un, gpu)
    for k in ref.files:
        if k.startswith('loss.'):
            v = float(ref[k])
            assert abs(float(losses[k[5:]]) - v) <= 1e-5 * max(1.0, abs(v)), (k, float(losses[k[5:]]), v)
    norms = {k[6:] for k in ref.files if k.startswith('gnorm.')}
    assert norms == {k for k in grads if is_trainable(k)}, norms ^ set(grads)
    worst = (0.0, None)
    for k in norms:
        n_ref = float(ref['gnorm.' + k])
        e = abs(float(grads[k].double().norm()) - n_ref) / max(n_ref, 1e-12)
        worst = max(worst, (e, k))
        assert e < GRAD_TOL, (k, e)
    errs = {k[5:]: fro(grads[k[5:]], torch.from_numpy(ref[k])) for k in ref.files if k.startswith('grad.')}
    print('\nworst gradient-norm error', worst, '\nfull-gradient Frobenius errors',
          {k.split('.', 1)[1][-40:]: f'{v:.1e}' for k, v in errs.items()})
    for k, e in errs.items():
        assert e < GRAD_TOL, (k, e)
    mods = dict(model.named_modules())
    for k in ref.files:
        if k.startswith('bn.'):
            name, stat = k[3:].rsplit('.', 1)
            assert rel_err(getattr(mods[name], stat), ref[k]) < 1e-5, k


def test_compute_loss_train_vs_reference(gpu):
    """fgreg.loss.compute_loss_train (the differentiable compute_loss that bench.py --train
    backpropagates: the f16x3 GEMMs for the match logits, torch ops for the rest) on the GPU vs
    the reference's own train() step (train_modelnet_small.npz): losses within 1e-5, every
    parameter's gradient norm and the stored full gradients within GRAD_TOL, W / W_un included."""
    import fgreg
    from fgreg.loss import compute_loss_train
    cfg, sd, src, tgt, meta, batch, W, W_un, ref = train_fixture()
    model = fgreg.RegTR(cfg)
    model.load_state_dict({k: v for k, v in sd.items()}, strict=False)
    with torch.no_grad():
        model.feature_criterion.W.copy_(W)
        model.feature_criterion_un.W.copy_(W_un)
    model = model.to(gpu).train()
    model.preprocessor = fgreg.FixedMetaPreprocessor({k: [t.to(gpu) for t in v]
                                                      for k, v in meta.items()})
    xb = {'src_xyz': [torch.from_numpy(np.asarray(c)).to(gpu) for c in src],
          'tgt_xyz': [torch.from_numpy(np.asarray(c)).to(gpu) for c in tgt]}
    pred = model(xb)
    xb['pose'] = batch['pose'].to(gpu)
    xb['src_overlap'] = [t.to(gpu) for t in batch['src_overlap']]
    xb['tgt_overlap'] = [t.to(gpu) for t in batch['tgt_overlap']]
    losses = compute_loss_train(model, pred, xb)
    losses['total'].backward()
    for k in ref.files:
        if k.startswith('loss.'):
            v = float(ref[k])
            assert abs(float(losses[k[5:]]) - v) <= 1e-5 * max(1.0, abs(v)), (k, float(losses[k[5:]]), v)
    grads = {k: p.grad for k, p in model.named_parameters() if p.grad is not None}
    norms = {k[6:] for k in ref.files if k.startswith('gnorm.')}
    for k in norms:
        n_ref = float(ref['gnorm.' + k])
        e = abs(float(grads[k].double().norm()) - n_ref) / max(n_ref, 1e-12)
        assert e < GRAD_TOL, (k, e)
    for k in ref.files:
        if k.startswith('grad.'):
            e = fro(grads[k[5:]], torch.from_numpy(ref[k]))
            assert e < GRAD_TOL, (k, e)


@pytest.mark.parametrize('pre_norm,head', [(True, 'regressor'), (False, 'regressor'),
                                           (True, 'decoder')])
def test_train_step_vs_oracle_modelnet(gpu, pre_norm, head):
    """Full-width ModelNet config (d 256, head dim 32: the f16x3 attention and every GEMM path),
    B = 2 pairs of the bench workload: fgreg's train() step vs the fp64 oracle's on the same
    neighbour tables. Losses within 1e-5, every gradient within GRAD_TOL; the cosine of the
    whole gradient vector above 1 - 1e-6. pre_norm=False: the post-norm transformer
    (forward_post, transformers.py:109-181), whose gradients react more to rounding: the
    oracle's OWN fp32 step differs from its fp64 step by up to 2.6e-3 (median 7.4e-4, 1 - cos
    8.6e-7) there vs 1.8e-3 (1.3e-4, 3.8e-8) pre-norm (tools/grad_chaos.py), and the f16x3
    products perturb ~10x more than fp32 rounding, so post-norm is bounded at 3e-2 / 1 - 1e-4
    (a wiring or formula error stays O(1)). head='decoder': the CorrespondenceDecoder head
    (direct_regress_coor: False, finegrained_regtr.py:312-408: q / k projections and the
    softmax-weighted partner coordinates) trained through fgr_corr_attention_bwd."""
    import fgreg
    import fgreg.config as fc
    from fgreg.synthetic import make_batch
    cfg = fc.get('modelnet', pre_norm=pre_norm, direct_regress_coor=head == 'regressor')
    torch.manual_seed(5)
    np.random.seed(5)
    model = fgreg.RegTR(cfg)
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    src, tgt, pose = make_batch('modelnet', 2)
    meta = mo.preprocess(cfg, [np.asarray(c) for c in list(src) + list(tgt)])
    _, _, lb, _, _, _, W, W_un = loss_fixture()
    from scipy.spatial import cKDTree
    sov, tov = [], []
    for b in range(2):
        sw = src[b] @ pose[b][:, :3].T + pose[b][:, 3]
        sov.append(torch.from_numpy((cKDTree(tgt[b]).query(sw)[0] < 0.05).astype(np.float32)))
        tov.append(torch.from_numpy((cKDTree(sw).query(tgt[b])[0] < 0.05).astype(np.float32)))
    W = torch.randn(cfg.d_embed, cfg.d_embed, generator=torch.Generator().manual_seed(1)) * 0.1
    W_un = torch.randn(cfg.d_embed, cfg.d_embed, generator=torch.Generator().manual_seed(2)) * 0.1
    batch = {'pose': torch.from_numpy(pose), 'kpconv_meta': meta, 'src_overlap': sov,
             'tgt_overlap': tov}
    losses, grads, _ = _gpu_train_step(cfg, sd, src, tgt, meta, batch, W, W_un, gpu)
    l64, g64 = oracle_train_grads(cfg, sd, src, tgt, meta, batch, W, W_un)
    for k, v in l64.items():
        assert abs(float(losses[k]) - float(v)) <= 1e-5 * max(1.0, abs(float(v))), (k, float(losses[k]), float(v))
    # gradients that vanish mathematically (the decoder head's k_proj.bias shifts every score
    # of a query row equally, which the softmax cancels) are compared in absolute terms
    scale = max(float(g64[k].norm()) for k in g64)
    tiny = [k for k in g64 if float(g64[k].norm()) <= 1e-7 * scale]
    for k in tiny:
        assert float(grads[k].double().norm()) <= 1e-5 * scale, (k, float(grads[k].norm()), scale)
    errs = {k: fro(grads[k], g64[k]) for k in g64 if k not in tiny}
    worst = sorted(errs.items(), key=lambda kv: -kv[1])[:5]
    a = torch.cat([grads[k].detach().double().cpu().flatten() for k in errs])
    b = torch.cat([g64[k].detach().flatten() for k in errs])
    cos = float(a @ b / (a.norm() * b.norm()))
    print(f'\nworst Frobenius errors {worst}, median {np.median(list(errs.values())):.2e}, '
          f'cosine {cos:.10f}')
    tol, cos_tol = (GRAD_TOL, 1e-6) if pre_norm else (3e-2, 1e-4)
    assert cos > 1 - cos_tol
    for k, e in errs.items():
        assert e < tol, (k, e)


def _h3_image_ref(W):
    """The f16x3 weight image of fgr_split_weights_h3 restated in numpy: rows scaled by 2^e
    (max |w| in [2^14, 2^15)), two fp16 terms, units [panel][kstep][term][g][row][8]; then the
    per-row inverse scales (0 past n)."""
    n, k = W.shape
    npad, ks = -(-n // 16) * 16, -(-k // 64) * 2
    mx = np.abs(W).max(1)
    e = np.where(mx > 0, np.minimum(15 - np.frexp(mx)[1], 127), 0)
    wp = np.zeros((npad, ks * 32), np.float32)
    wp[:n, :k] = W * np.ldexp(np.float32(1), e).astype(np.float32)[:, None]
    hi = wp.astype(np.float16)
    lo = (wp - hi.astype(np.float32)).astype(np.float16)
    img = np.stack([hi, lo]).reshape(2, npad // 16, 16, ks, 4, 8).transpose(1, 3, 0, 4, 2, 5)
    wsc = np.zeros(npad, np.float32)
    wsc[:n] = np.ldexp(np.float32(1), -e)
    return np.ascontiguousarray(img).tobytes() + wsc.tobytes()


@pytest.mark.parametrize('shape,transpose', [((256, 256), False), ((1024, 256), False),
                                             ((37, 100), False), ((256, 1024), False),
                                             ((64, 2048), False), ((15, 16, 24), True),
                                             ((15, 64, 256), True), ((1024, 96), True),
                                             ((2048, 64), True)])
def test_weight_image_bits(gpu, shape, transpose):
    """Split weight images (the fused one-launch split for k <= 1024, the two-launch one beyond,
    row-major W and the transposed views the backward uses) equal their numpy restatement bit
    for bit."""
    from fgreg import linear as lin
    g = torch.Generator().manual_seed(sum(shape))
    w = torch.randn(shape, generator=g) * 10.0 ** torch.empty(shape[0]).uniform_(-3, 3, generator=g).view(
        -1, *([1] * (len(shape) - 1)))
    if transpose:                              # W = w.reshape(k, n).t(): column-major rows
        ent = lin.weight_image(w.to(gpu), transpose=True, mode='f16x3', cache=False)
        ref = _h3_image_ref(w.reshape(-1, shape[-1]).t().contiguous().numpy())
    else:
        ent = lin.weight_image(w.to(gpu), mode='f16x3', cache=False)
        ref = _h3_image_ref(w.numpy())
    got = ent.img.cpu().numpy().tobytes()
    assert len(got) == len(ref) and got == ref


def test_weight_image_batch_refresh(gpu):
    """After in-place updates (an optimizer step), the first weight_image call re-splits every
    stale cached image in one batched launch (fgr_split_weights_h3_batch): each image then
    equals its numpy restatement of the UPDATED weight, bit for bit, row-major, transposed and
    row-slice images alike."""
    from fgreg import linear as lin
    g = torch.Generator().manual_seed(5)
    ws = [torch.randn(s, generator=g).to(gpu) for s in [(256, 256), (1024, 96), (37, 100), (15, 16, 24)]]
    imgs = [lin.weight_image(ws[0], mode='f16x3'), lin.weight_image(ws[1], transpose=True, mode='f16x3'),
            lin.weight_image(ws[2], mode='f16x3'), lin.weight_image(ws[3], transpose=True, mode='f16x3'),
            lin.weight_image(ws[0], mode='f16x3', rows=(64, 192))]
    with torch.no_grad():
        for w in ws:
            w.mul_(-3.0).add_(0.25)
    got = [lin.weight_image(ws[0], mode='f16x3'), lin.weight_image(ws[1], transpose=True, mode='f16x3'),
           lin.weight_image(ws[2], mode='f16x3'), lin.weight_image(ws[3], transpose=True, mode='f16x3'),
           lin.weight_image(ws[0], mode='f16x3', rows=(64, 192))]
    assert all(a is b for a, b in zip(imgs, got))          # refreshed in place, not rebuilt
    w0, w1, w2, w3 = (w.cpu() for w in ws)
    refs = [_h3_image_ref(w0.numpy()), _h3_image_ref(w1.t().contiguous().numpy()),
            _h3_image_ref(w2.numpy()), _h3_image_ref(w3.reshape(-1, 24).t().contiguous().numpy()),
            _h3_image_ref(w0[64:192].contiguous().numpy())]
    for e, ref in zip(got, refs):
        assert e.img.cpu().numpy().tobytes() == ref
