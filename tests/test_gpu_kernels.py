"""GPU parity of the floating-point kernels against the reference's own outputs
(tests/golden/*.npz) and against plain PyTorch fp32 references of the same op.

Tolerance: normwise relative error max|a-b|/max|b| <= 1e-4 (fp32, SURVEY.md scope),
poses <= 1e-4 absolute on rotation entries and relative on translations.
"""
import math

import numpy as np
import pytest
import torch

import model_oracle as mo
from conftest import golden, rel_err

pytestmark = pytest.mark.gpu
TOL = 1e-4


def test_kpconv_block_vs_reference(gpu):
    """KPConv.forward (finegrained_kpconv_blocks.py:265-401) on the reference's own
    neighbour table, conv and strided (pool) variants, plus the max-pool shortcut."""
    from fgreg.backbone import KPConv
    import fgreg.ops as ops
    g = golden('kpconv_block')
    W = torch.from_numpy(g['W'])
    conv = KPConv(15, 3, W.shape[1], W.shape[2], float(g['extent']), 0.0825).to(gpu)
    with torch.no_grad():
        conv.weights.copy_(W.to(gpu))
        conv.kernel_points.copy_(torch.from_numpy(g['kp']).to(gpu))
    t = lambda a, dt=None: torch.from_numpy(a if dt is None else a.astype(dt)).to(gpu)
    out = conv(t(g['q']), t(g['s']), t(g['idx'], np.int64), t(g['x']))
    assert rel_err(out, g['out']) < TOL
    out_s = conv(t(g['sub']), t(g['s']), t(g['pools'], np.int64), t(g['x']))
    assert rel_err(out_s, g['out_strided']) < TOL
    mp = ops.max_pool(t(g['x']), t(g['pools'], np.int64))
    assert torch.equal(mp.cpu(), torch.from_numpy(g['maxpool']))


def _gather_case(cin, H, nq=700, ns=900, n_kp=15, seed=None):
    rng = np.random.default_rng(cin + H if seed is None else seed)
    s = rng.uniform(-1, 1, (ns, 3)).astype(np.float32)
    q = s[rng.choice(ns, nq, replace=False)] + rng.normal(0, 0.01, (nq, 3)).astype(np.float32)
    idx = rng.integers(0, ns, (nq, H))
    idx[rng.uniform(size=(nq, H)) < 0.6] = ns            # shadows
    if nq > 3:
        idx[3] = ns                                      # a query with no valid neighbour
    x = rng.normal(size=(ns, cin)).astype(np.float32)
    kp = (rng.normal(size=(n_kp, 3)) * 0.3).astype(np.float32)
    return q, s, idx, x, kp


@pytest.mark.parametrize('cin,H', [(1, 50), (1, 7), (3, 50), (16, 50), (32, 50), (64, 50),
                                   (128, 50), (256, 50), (256, 70), (64, 130), (32, 130),
                                   (32, 5), (16, 70)])
def test_kpconv_gather_vs_torch(gpu, cin, H):
    """Gather-weight stage vs the fp32 torch restatement (all channel widths in the configs;
    the cin = 1 stem kernel; the quad-lane kernel of cin 16 / 32 incl. widths past one
    64-neighbour chunk; the wide kernels)."""
    import fgreg.ops as ops
    q, s, idx, x, kp = _gather_case(cin, H)
    ns, ext = s.shape[0], 0.5
    T = lambda a: torch.from_numpy(a).to(gpu)
    wf, nn_ = ops.kpconv_gather(T(q), T(s), T(idx), T(x), T(kp), ext)
    # torch fp32 reference of the same op (blocks:296-381, 395-398)
    sp = torch.cat([torch.from_numpy(s), torch.zeros(1, 3) + 1e6])
    nb = sp[torch.from_numpy(idx)] - torch.from_numpy(q).unsqueeze(1)
    d2 = ((nb.unsqueeze(2) - torch.from_numpy(kp)) ** 2).sum(3)
    w = torch.clamp(1 - torch.sqrt(d2) / ext, min=0).transpose(1, 2)
    xp = torch.cat([torch.from_numpy(x), torch.zeros(1, cin)])
    nx = xp[torch.from_numpy(idx)]
    ref = torch.matmul(w, nx)
    assert rel_err(wf, ref) < TOL
    cnt = torch.clamp((nx.sum(-1) > 0).sum(-1), min=1).float()
    assert torch.equal(nn_.cpu(), cnt)


def test_instnorm_vs_reference(gpu):
    import fgreg.ops as ops
    g = golden('instnorm')
    lens = [int(v) for v in g['lengths']]
    out = ops.instnorm(torch.from_numpy(g["x"]).to(gpu), ops.offsets(lens, gpu), lens)
    assert rel_err(out, g['out']) < TOL


@pytest.mark.parametrize('lens,c,mu', [([700, 1, 33, 512], 72, 2.0), ([1024, 1000, 2], 72, 2.0),
                                       ([3000, 5, 1500, 1024, 1025], 72, 2.0),
                                       ([3000, 5, 1500, 1024, 1025], 64, 2.0),
                                       ([20000, 13389], 64, 50.0), ([5483, 1, 2000], 256, 2.0),
                                       ([1100, 4000], 1024, -30.0), ([596] * 16, 1024, 2.0),
                                       ([1, 1024, 300, 7] * 4, 576, -20.0)])
def test_instnorm_fusions_vs_torch(gpu, lens, c, mu):
    """Register path (segments <= 1024 rows, incl. ModelNet's 16 x 596 x 1024 and ragged
    16-cloud batches), the two-launch chunked path (C % 4 != 0) and
    the three-launch long-segment path (C / 4 divides 256), including 3DMatch-size clouds
    with |mean| >> std (the shifted sums must not cancel)."""
    import fgreg.ops as ops
    rng = np.random.default_rng(5)
    x = torch.from_numpy(rng.normal(mu, 3 if abs(mu) < 10 else 0.5, (sum(lens), c)).astype(np.float32))
    div = torch.from_numpy(rng.integers(1, 9, sum(lens)).astype(np.float32))
    res = torch.from_numpy(rng.normal(size=x.shape).astype(np.float32))
    ref = mo.instance_norm(x / div[:, None], torch.tensor(lens))
    ref_act = torch.nn.functional.leaky_relu(ref, 0.1)
    ref_res = torch.nn.functional.leaky_relu(ref + res, 0.1)
    off = ops.offsets(lens, gpu)
    X, D, R = x.to(gpu), div.to(gpu), res.to(gpu)
    assert rel_err(ops.instnorm(X, off, lens, row_div=D), ref) < TOL
    assert rel_err(ops.instnorm(X, off, lens, row_div=D, act=ops.ACT_LEAKY), ref_act) < TOL
    assert rel_err(ops.instnorm(X, off, lens, row_div=D, residual=R, post_act=ops.ACT_LEAKY),
                   ref_res) < TOL


@pytest.mark.parametrize('lens,c', [([20000, 13389], 64), ([1025, 30000, 2, 4097, 1500], 128),
                                    ([6000, 2100], 1024)])
def test_instnorm_long_repeat_and_graph(gpu, lens, c):
    """The long-segment path (shifted sums, fp64 merge): repeated eager calls and HIP-graph
    replays give the same bits and match the oracle; short segments beside long ones, 1024
    channels (one row per 256-thread iteration)."""
    import fgreg.ops as ops
    rng = np.random.default_rng(11)
    x = torch.from_numpy(rng.normal(7.0, 2.0, (sum(lens), c)).astype(np.float32))
    ref = torch.nn.functional.leaky_relu(mo.instance_norm(x, torch.tensor(lens)), 0.1)
    off = ops.offsets(lens, gpu)
    X = x.to(gpu)
    outs = [ops.instnorm(X, off, lens, act=ops.ACT_LEAKY) for _ in range(3)]
    assert rel_err(outs[0], ref) < TOL
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    out = torch.empty_like(X)
    with torch.cuda.stream(s):
        ops.instnorm(X, off, lens, act=ops.ACT_LEAKY, out=out)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.instnorm(X, off, lens, act=ops.ACT_LEAKY, out=out)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, outs[0])


@pytest.mark.parametrize('d', [32, 256, 512])
def test_sine_pos_embed_vs_reference(gpu, d):
    import fgreg.ops as ops
    g = golden('pos_embed')
    xyz = torch.from_numpy(g['xyz']).to(gpu)
    if d == 32:
        ref = mo.sine_pos_embed(torch.from_numpy(g['xyz']), 32)
    else:
        ref = torch.from_numpy(g[f'pe{d}'])
    assert rel_err(ops.sine_pos_embed(xyz, d), ref) < TOL


def test_layernorm_vs_torch(gpu):
    import fgreg.ops as ops
    rng = np.random.default_rng(1)
    for d in (32, 64, 96, 128, 192, 256, 512, 1024):
        x = torch.from_numpy(rng.normal(1, 2, (333, d)).astype(np.float32))
        w = torch.from_numpy(rng.normal(1, 0.1, d).astype(np.float32))
        b = torch.from_numpy(rng.normal(0, 0.1, d).astype(np.float32))
        a = torch.from_numpy(rng.normal(size=(333, d)).astype(np.float32))
        pb = torch.from_numpy(rng.normal(size=d).astype(np.float32))
        ref = torch.nn.functional.layer_norm(x, (d,), w, b, 1e-5) + a
        out = ops.layernorm(x.to(gpu), w.to(gpu), b.to(gpu), 1e-5, add=a.to(gpu))
        assert rel_err(out, ref) < TOL
        # pending residual bias: x += pre_bias in place, then normalised
        X = x.to(gpu)
        out = ops.layernorm(X, w.to(gpu), b.to(gpu), 1e-5, pre_bias=pb.to(gpu))
        ref = torch.nn.functional.layer_norm(x + pb, (d,), w, b, 1e-5)
        assert rel_err(out, ref) < TOL and rel_err(X, x + pb) < 1e-7


def _attn_ref(q, k, v, qlens, klens, kv_seg, nhead):
    """Per-segment fp32 softmax attention with torch (MHA core, scale sqrt(1/dh))."""
    d = q.shape[1]
    dh = d // nhead
    qo = np.cumsum([0] + qlens)
    ko = np.cumsum([0] + klens)
    out = torch.zeros_like(q)
    for i in range(len(qlens)):
        j = kv_seg[i]
        qs = q[qo[i]:qo[i + 1]].view(-1, nhead, dh).transpose(0, 1) * math.sqrt(1.0 / dh)
        ks = k[ko[j]:ko[j + 1]].view(-1, nhead, dh).transpose(0, 1)
        vs = v[ko[j]:ko[j + 1]].view(-1, nhead, dh).transpose(0, 1)
        a = torch.softmax(qs @ ks.transpose(1, 2), -1) @ vs
        out[qo[i]:qo[i + 1]] = a.transpose(0, 1).reshape(-1, d)
    return out


@pytest.mark.parametrize('nhead,d', [(8, 32), (8, 64), (8, 256), (8, 512), (1, 256), (2, 16)])
def test_attention_vs_torch(gpu, nhead, d):
    import fgreg.ops as ops
    rng = np.random.default_rng(d + nhead)
    lens = [575, 1, 64, 130, 300, 65]   # 3 "pairs": segment c attends to (c + 3) % 6
    n = sum(lens)
    qkv = torch.from_numpy(rng.normal(size=(n, 3 * d)).astype(np.float32)) * 2
    q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
    for kv_seg in ([0, 1, 2, 3, 4, 5], [3, 4, 5, 0, 1, 2]):
        ref = _attn_ref(q, k, v, lens, lens, kv_seg, nhead)
        g = qkv.to(gpu)
        off = ops.offsets(lens, gpu)
        seg = torch.tensor(kv_seg, dtype=torch.int32, device=gpu)
        out = ops.attention(g[:, :d], g[:, d:2 * d], g[:, 2 * d:], off, off, seg, max(lens), nhead)
        assert rel_err(out, ref) < TOL


def _attention_fp32(q, k, v, q_off, kv_off, kv_seg, max_q_len, n_head):
    """fgr_attention (fp32 MFMA, the any-head_dim kernel) called through the C ABI directly."""
    from fgreg import _lib
    d = q.shape[1]
    o = torch.empty_like(q)
    _lib.check(_lib.load().fgr_attention(
        q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0), v.data_ptr(), v.stride(0),
        o.data_ptr(), o.stride(0), q_off.data_ptr(), kv_off.data_ptr(), kv_seg.data_ptr(),
        kv_seg.numel(), max_q_len, n_head, d // n_head, math.sqrt(n_head / d),
        torch.cuda.current_stream().cuda_stream), 'fgr_attention')
    return o


@pytest.mark.parametrize('d', [256, 512])
@pytest.mark.parametrize('scale', [1.0, 6.0, 1e-6, 3e3])
def test_attention_split_is_fp32_accurate(gpu, scale, d):
    """The split attention (fgr_attention_f16x3, dh = 32 and 64) against a float64
    reference: error at fp32 level (<= 1e-5 normwise) and no worse than a few times the
    fp32-MFMA kernel's own error; separate key segmentation (kv lengths != q lengths,
    max_kv_len > max_q_len), partial and 1-key tiles, sharp softmax at scale 6, inputs far
    outside fp16's range (1e-6: subnormal in fp16 unscaled; 3e3: products past 65504).
    """
    import fgreg.ops as ops
    rng = np.random.default_rng(7)
    nhead = 8
    qlens = [300, 1, 64, 129]
    klens = [65, 700, 1, 128]
    kv_seg = [1, 0, 3, 2]
    q = torch.from_numpy(rng.normal(size=(sum(qlens), d))) * scale
    kv = torch.from_numpy(rng.normal(size=(sum(klens), 2 * d))) * scale
    if scale > 100:                 # large q and v, small k: scores stay O(1)
        kv[:, :d] /= scale * scale
    k, v = kv[:, :d], kv[:, d:]
    ref = _attn_ref(q, k, v, qlens, klens, kv_seg, nhead)            # float64
    qg, kvg = q.float().to(gpu), kv.float().to(gpu)
    qo, ko = ops.offsets(qlens, gpu), ops.offsets(klens, gpu)
    seg = torch.tensor(kv_seg, dtype=torch.int32, device=gpu)
    assert ops.ATTN_MODE == 'f16x3'
    out = ops.attention(qg, kvg[:, :d], kvg[:, d:], qo, ko, seg, max(qlens), nhead,
                        max_kv_len=max(klens))
    o32 = _attention_fp32(qg, kvg[:, :d], kvg[:, d:], qo, ko, seg, max(qlens), nhead)
    errs = {'f16x3': rel_err(out.double(), ref), 'fp32': rel_err(o32.double(), ref)}
    assert errs['f16x3'] < 1e-5, errs
    assert errs['f16x3'] < 4 * errs['fp32'] + 1e-7, errs


def test_transformer_layer_vs_reference(gpu):
    """One TransformerCrossEncoderLayer.forward_pre (transformers.py:183-244), B = 2 with
    unequal lengths, against the reference module's output (padded rows excluded)."""
    from fgreg.transformer import Segments, TransformerCrossEncoderLayer
    g = golden('transformer_layer')
    layer = TransformerCrossEncoderLayer(64, 8, 128, 0.0, normalize_before=True,
                                         sa_val_has_pos_emb=True, ca_val_has_pos_emb=True)
    sd = {k[2:]: torch.from_numpy(g[k]) for k in g.files if k.startswith('w.')}
    layer.load_state_dict(sd)
    layer = layer.to(gpu).eval()
    smask, tmask = g['src_mask'], g['tgt_mask']
    ns = [int((~smask[b]).sum()) for b in range(2)]
    nt = [int((~tmask[b]).sum()) for b in range(2)]
    rows = [g['src'][:ns[b], b] for b in range(2)] + [g['tgt'][:nt[b], b] for b in range(2)]
    prow = [g['src_pos'][:ns[b], b] for b in range(2)] + [g['tgt_pos'][:nt[b], b] for b in range(2)]
    x = torch.from_numpy(np.concatenate(rows)).to(gpu)
    pos = torch.from_numpy(np.concatenate(prow)).to(gpu)
    seg = Segments(ns + nt, gpu)
    with torch.no_grad():
        y, pending = layer.forward_packed(x.clone(), pos, seg)
        y = (y if pending is None else y + pending).cpu().numpy()
    ref = np.concatenate([g['src_out'][:ns[b], b] for b in range(2)] +
                         [g['tgt_out'][:nt[b], b] for b in range(2)])
    assert rel_err(y, ref) < TOL


@pytest.mark.parametrize('case', ['regular', 'reflection', 'allzero', 'threshold'])
def test_procrustes_vs_reference(gpu, case):
    from fgreg.pose import compute_rigid_transform, fast_compute_rigid_transform
    g = golden('procrustes')
    a, b, w = (torch.from_numpy(g[f'{case}_{k}']).to(gpu) for k in 'abw')
    w_copy = w.clone()
    fast = fast_compute_rigid_transform(a, b, w_copy)
    full = compute_rigid_transform(a, b, w)
    for got, want in ((fast, g[f'{case}_fast']), (full, g[f'{case}_full'])):
        got = got.cpu().numpy()
        assert np.abs(got[..., :3] - want[..., :3]).max() < TOL
        assert np.abs(got[..., 3] - want[..., 3]).max() < TOL * max(1.0, np.abs(want[..., 3]).max())
    # in-place thresholding, as the reference (se3_torch.py:240-242)
    thr = g[f'{case}_w'].copy()
    thr[~(thr > 0.85)] = 0
    assert np.array_equal(w_copy.cpu().numpy(), thr)


@pytest.mark.parametrize('cin,cout', [(128, 512), (256, 1024), (32, 128), (64, 256), (8, 32)])
def test_res2net_block_vs_oracle(gpu, cin, cout):
    """my_res2Net (res2net.py:84-159, 231-265) in eval: fused fgr_res2net_chain_h3 (widths
    28 / 56 / 112 -- 3DMatch's narrow blocks pad to whole 16-column tiles), fgr_res2net_chain6
    (the exact three-term bf16 split) at width 224, one linear() per step for the rest
    (width 7 here), vs the CPU restatement."""
    from fgreg.backbone import my_Bottle2neck, my_res2Net
    _res2net_case(gpu, cin, cout, my_Bottle2neck, my_res2Net)


@pytest.mark.parametrize('n', [1500, 9544])
def test_res2net_chain6_rows_bitexact(gpu, n, monkeypatch):
    """fgr_res2net_chain6 at width 224 picks 16- / 48-row blocks by row count (1500 -> 16,
    ModelNet's 9544 -> 48); every accumulator sees the same MFMA sequence as with the 32-row
    blocks (FGR_R2N_ROWS=32), so the outputs are bit-identical."""
    from fgreg.backbone import my_Bottle2neck, my_res2Net
    torch.manual_seed(3)
    m = my_res2Net(my_Bottle2neck, 256, 1024, baseWidth=14, scale=8).to(gpu).eval()
    assert m.layer1[0].width == 224            # the chain6 width
    x = torch.randn(n, 256, device=gpu)
    with torch.no_grad():
        a = m(x).clone()
        monkeypatch.setenv('FGR_R2N_ROWS', '32')
        b = m(x).clone()
    assert torch.equal(a, b)


@pytest.mark.parametrize('n', [1500, 9544])
def test_res2net_block_h3_width224(gpu, n, monkeypatch):
    """The f16x3 chain at width 224 (FGREG_R2N224=h3: 14-wave blocks of 32 rows at 1500
    rows, 48 rows at ModelNet's 9544) vs the CPU restatement; ragged last blocks."""
    from fgreg.backbone import my_Bottle2neck, my_res2Net
    monkeypatch.setenv('FGREG_R2N224', 'h3')
    _res2net_case(gpu, 256, 1024, my_Bottle2neck, my_res2Net, n=n)


def _res2net_case(gpu, cin, cout, my_Bottle2neck, my_res2Net, n=1500):
    torch.manual_seed(cout)
    m = my_res2Net(my_Bottle2neck, cin, cout, baseWidth=14, scale=8)
    g = torch.Generator().manual_seed(cin)
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.running_mean.copy_(0.1 * torch.randn(mod.running_mean.shape, generator=g))
                mod.running_var.copy_(0.75 + 0.5 * torch.rand(mod.running_var.shape, generator=g))
                mod.weight.copy_(1 + 0.1 * torch.randn(mod.weight.shape, generator=g))
                mod.bias.copy_(0.1 * torch.randn(mod.bias.shape, generator=g))
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.randn(n, cin, generator=g)
    ref = mo.res2net(sd, '', x) if False else mo.res2net({f'r.{k}': v for k, v in sd.items()}, 'r', x)
    m = m.to(gpu).eval()
    with torch.no_grad():
        out = m(x.to(gpu))
    assert rel_err(out, ref) < TOL


@pytest.mark.parametrize('m,n,k', [(11472, 128, 1920), (9200, 1024, 2048), (1000, 3, 256),
                                   (333, 896, 128), (64, 256, 36), (5000, 768, 256),
                                   (9544, 256, 256), (4097, 256, 256), (13000, 256, 256),
                                   (12300, 768, 256), (2120, 512, 512), (2120, 1024, 512),
                                   (1001, 512, 512), (300, 1024, 512), (9544, 1792, 256),
                                   (5000, 512, 256), (4100, 1024, 256), (20000, 256, 256),
                                   (40000, 1024, 256)])
def test_gemm_split_vs_fp64(gpu, m, n, k):
    """The f16x3 GEMM vs fp64, bias / ReLU / residual / ReLU-residual-LeakyReLU epilogues,
    strided A, the KPConv weight layout, a row slice of a cached weight: at fp32 level, no
    worse than 4x torch's own fp32 GEMM (the comparison baseline only)."""
    tol = 2e-6
    from fgreg import linear as fl
    from fgreg import ops
    g = torch.Generator().manual_seed(m + n + k)
    x = torch.randn(m, k + 4, generator=g)[:, :k]          # strided rows (lda = k + 4)
    w = torch.randn(n, k, generator=g) / math.sqrt(k)
    b = torch.randn(n, generator=g)
    r = torch.randn(m, n, generator=g)
    ref = x.double() @ w.double().t() + b.double()
    X, W, Bb, R = x.to(gpu), w.to(gpu), b.to(gpu), r.to(gpu)
    assert fl.MODE == 'f16x3'
    e32 = rel_err(torch.addmm(Bb, X, W.t()), ref)
    e = rel_err(fl.linear(X, W, Bb), ref)
    assert e < tol and e < 4 * e32 + 1e-7, (e, e32)
    assert rel_err(fl.linear(X, W, Bb, act=ops.ACT_RELU), ref.clamp_min(0)) < tol
    assert rel_err(fl.linear(X, W, residual=R), ref - b.double() + r.double()) < tol
    lk = torch.nn.functional.leaky_relu(ref.clamp_min(0) + r.double(), 0.1)
    assert rel_err(fl.linear(X, W, Bb, act=ops.ACT_RELU_RES_LEAKY, residual=R), lk) < tol
    # transposed (KPConv weight layout (K, Cin, Cout) used as (K*Cin, Cout))
    wt = w.t().contiguous().view(k, n)
    assert rel_err(fl.linear(X, wt.to(gpu), Bb, transpose=True), ref) < tol
    if n >= 2:          # row slice (the q|k / v blocks of an in_proj weight), cached per slice
        h = n // 2
        for _ in range(2):
            assert rel_err(fl.linear(X, W, Bb[h:], rows=(h, n)), ref[:, h:]) < tol
            assert rel_err(fl.linear(X, W, Bb[:h], rows=(0, h)), ref[:, :h]) < tol


@pytest.mark.parametrize('tile', ['', 'b', 'I', 'K', 'O', 'S', 'z'])
def test_gemm_f16x3_dynamic_range(gpu, tile, monkeypatch):
    """f16x3 row scaling (tile: '' the default dispatch, else FGR_GEMM16_TILE) under
    adversarial magnitudes: rows at 1e-15 .. 1e15 (far outside fp16's range), all-zero rows, rows whose first k chunks are zero, rows that grow by
    2^40 along k (forces the in-flight rescale of partial sums) and a weight matrix with
    rows at 1e-10 / 1e10 (outputs stay inside fp32's range). Every output row must match fp64 to 2e-6 of its own scale."""
    monkeypatch.setenv('FGR_GEMM16_TILE', tile)
    from fgreg import linear as fl
    g = torch.Generator().manual_seed(7)
    m, n, k = 700, 96, 256 if tile == 'z' else 320     # z: the K <= 256 row-stationary kernel
    x = torch.randn(m, k, generator=g, dtype=torch.float64)
    row_scale = torch.tensor([10.0 ** e for e in np.linspace(-15, 15, m)], dtype=torch.float64)
    x *= row_scale[:, None]
    x[5] = 0
    x[17, :200 if k > 256 else 160] = 0              # first nonzero chunk late
    ramp = torch.pow(2.0, torch.linspace(0, 40, k, dtype=torch.float64))
    x[30:60] *= ramp                                 # growing rows: rescales mid-k
    x[60:90] *= ramp.flip(0)                         # shrinking rows
    w = torch.randn(n, k, generator=g, dtype=torch.float64) / math.sqrt(k)
    w[3] *= 1e-10
    w[4] *= 1e10
    ref = x @ w.t()
    X, W = x.float().to(gpu), w.float().to(gpu)
    ref32 = X.double().cpu() @ W.double().cpu().t()     # fp32-rounded inputs, exact product
    old = fl.MODE
    try:
        fl.set_mode('f16x3')
        out = fl.linear(X, W).double().cpu()
    finally:
        fl.set_mode(old)
    assert torch.isfinite(out).all()
    assert (out[5] == 0).all()
    # per-row normwise error vs the exact product of the fp32 inputs
    den = (X.double().cpu().abs() @ W.double().cpu().abs().t()).clamp_min(1e-300)
    err = ((out - ref32).abs() / den).max()
    assert err < 2e-6, float(err)
    del ref


@pytest.mark.parametrize('n', [256, 512, 768, 1024])
def test_gemm_ws_dynamic_range(gpu, n):
    """The weight-split row-stationary kernel (gemm_ws.hip: K = 256, >= 4096 rows, one scale
    per row; N = 512 / 1024 as column parts over 2 / 4 blocks per row tile) under the adversarial magnitudes of test_gemm_f16x3_dynamic_range:
    every output row within 2e-6 of its own scale."""
    from fgreg import linear as fl
    from fgreg import _lib
    m, k = 4200, 256
    assert _lib.load().fgr_gemm_f16x3_ln_supported(m, n, k) == (n in (256, 768))
    g = torch.Generator().manual_seed(n)
    x = torch.randn(m, k, generator=g, dtype=torch.float64)
    x *= torch.tensor([10.0 ** e for e in np.linspace(-15, 15, m)], dtype=torch.float64)[:, None]
    x[5] = 0
    x[17, :160] = 0
    ramp = torch.pow(2.0, torch.linspace(0, 40, k, dtype=torch.float64))
    x[30:60] *= ramp
    x[60:90] *= ramp.flip(0)
    w = torch.randn(n, k, generator=g, dtype=torch.float64) / math.sqrt(k)
    w[3] *= 1e-10
    w[4] *= 1e10
    X, W = x.float().to(gpu), w.float().to(gpu)
    ref32 = X.double().cpu() @ W.double().cpu().t()
    out = fl.linear(X, W).double().cpu()
    assert torch.isfinite(out).all() and (out[5] == 0).all()
    den = (X.double().cpu().abs() @ W.double().cpu().abs().t()).clamp_min(1e-300)
    assert float(((out - ref32).abs() / den).max()) < 2e-6


@pytest.mark.parametrize('tile', list('abcdefghijklmnopqrstuvwxyz') + list('ABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789'))
def test_gemm_f16x3_tiles(gpu, tile, monkeypatch):
    """Every f16x3 tile / pipeline variant (FGR_GEMM16_TILE; A..R: the LDS-DMA g5 kernels of
    gemm5.hip) at fp32 accuracy on ragged shapes (M, N, K not multiples of the tiles; K % 64
    != 0, odd k32-step count; N = 3; K % 8 != 0 takes the register-staged fallback)."""
    from fgreg import linear as fl
    monkeypatch.setenv('FGR_GEMM16_TILE', tile)
    g = torch.Generator().manual_seed(11)
    old = fl.MODE
    try:
        fl.set_mode('f16x3')
        for m, n, k in ((1000, 200, 1000), (333, 3, 96), (130, 520, 40), (77, 50, 36),
                        (4099, 272, 264), (1000, 200, 256), (257, 1, 128), (4100, 33, 200),
                        (64, 16, 8)):
            x = torch.randn(m, k, generator=g)
            w = torch.randn(n, k, generator=g) / math.sqrt(k)
            b = torch.randn(n, generator=g)
            r = torch.randn(m, n, generator=g)
            ref = x.double() @ w.double().t() + b.double() + r.double()
            out = fl.linear(x.to(gpu), w.to(gpu), b.to(gpu), residual=r.to(gpu))
            assert rel_err(out, ref) < 2e-6, (tile, m, n, k)
    finally:
        fl.set_mode(old)


@pytest.mark.parametrize('m,d', [(57264, 256), (1000, 256), (333, 128), (97, 64), (4097, 32)])
def test_corr_head_fused_vs_fp64(gpu, m, d):
    """fgr_corr_head_f16x3 (CorrespondenceRegressor, finegrained_regtr.py:411-455, in two
    row-stationary launches: [coor_mlp[0] | conf_logits] over the stacked weight, then
    coor_mlp[2] -> ReLU -> coor_mlp[4] formed in the epilogue) vs the four Linear layers in fp64
    (per row within 1e-5 of the row's |.|-weighted magnitude) and vs the unfused per-Linear path
    of the same module (fgreg.regtr.FUSED_HEAD off) within 1e-5."""
    from fgreg import regtr
    from fgreg.regtr import CorrespondenceRegressor
    torch.manual_seed(m + d)
    head = CorrespondenceRegressor(d).to(gpu)
    f = torch.randn(2, m, d, device=gpu) * 0.7
    f[0, :7] = 0.0                                   # all-zero rows
    f[1, 3] *= 1e4                                   # a row far above the rest
    corr, logits = head.forward_packed(f)
    regtr.FUSED_HEAD = False
    try:
        corr_u, logits_u = head.forward_packed(f)
    finally:
        regtr.FUSED_HEAD = True
    x = f.reshape(-1, d).double().cpu()
    p = {k: v.detach().double().cpu() for k, v in head.state_dict().items()}
    h = torch.relu(x @ p['coor_mlp.0.weight'].t() + p['coor_mlp.0.bias'])
    h2 = torch.relu(h @ p['coor_mlp.2.weight'].t() + p['coor_mlp.2.bias'])
    c64 = h2 @ p['coor_mlp.4.weight'].t() + p['coor_mlp.4.bias']
    l64 = x @ p['conf_logits_decoder.weight'].t() + p['conf_logits_decoder.bias']
    den_c = (h2.abs() @ p['coor_mlp.4.weight'].abs().t()).max(1, keepdim=True).values + 1e-30
    den_l = (x.abs() @ p['conf_logits_decoder.weight'].abs().t()) + 1e-30
    ec = float(((corr.reshape(-1, 3).double().cpu() - c64).abs() / den_c).max())
    el = float(((logits.reshape(-1, 1).double().cpu() - l64).abs() / den_l).max())
    assert ec < 1e-5 and el < 1e-5, (ec, el)
    assert rel_err(corr, corr_u) < 1e-5 and rel_err(logits, logits_u) < 1e-6
