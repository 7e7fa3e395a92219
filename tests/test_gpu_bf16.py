"""The bf16 compute mode (BASELINE configs[4]: 3DLoMatch, "bf16 features with MFMA bf16
attention"; fgreg.set_precision('bf16')).

Kernels are checked twice: against a reference that rounds the same operands to bf16 and
accumulates in fp64 (the kernel must agree to fp32-accumulation level: the rounding points are
pinned, not just the error size), and against the exact fp64 product (the bf16 error bound).
The forward is checked against the fp32 CPU oracle on low-overlap pairs with the tolerance the
bf16 mode states (DESIGN.md "bf16 mode"): geometry bit-exact (it does not depend on the mode),
features and scores within BF16_FEAT_TOL normwise, poses within BF16_ROT_DEG / BF16_TRANS.
"""
import math

import numpy as np
import pytest
import torch

import model_oracle as mo
from conftest import rel_err

pytestmark = pytest.mark.gpu

# stated tolerances of the bf16 forward against the fp32 oracle (DESIGN.md "bf16 mode"), set
# from a sweep over 10 random models (profiles/r03_bf16_sweep.jsonl, tools/bf16_sweep.py: seeds
# 0-7 at 6k points, 20-21 at 20k): worst case measured 3.4e-2 normwise (a warped-keypoint
# tensor; features <= 2.2e-2, overlap scores <= 7.9e-3), rotation 2.85 deg, translation 7.4 mm.
# The pose bounds are half of the reference's own registration-success thresholds (conf
# reg_success_thresh_rot 10 deg / _trans 0.1 m is 5x the translation bound): with random-init
# weights the predicted correspondences collapse toward the centroids and the Procrustes rotation
# is ill-conditioned, so the ~2 % bf16 feature error shows up amplified there (the fp32-accurate
# mode stays at 1e-4 on the same cases).
BF16_FEAT_TOL = 5e-2        # normwise relative, every per-pair output tensor
BF16_ROT_DEG = 5.0          # rotation difference of the predicted poses, degrees
BF16_TRANS = 0.02           # translation difference, metres
KEYS = ['src_feat_un', 'tgt_feat_un', 'src_feat', 'tgt_feat', 'src_kp_warped', 'tgt_kp_warped',
        'src_overlap', 'tgt_overlap']


def _bf(t):
    return t.to(torch.bfloat16).double()


@pytest.fixture
def bf16_mode():
    import fgreg
    old = fgreg.precision()
    fgreg.set_precision('bf16')
    yield
    fgreg.set_precision(old)


@pytest.mark.parametrize('tile', ['', 'z', 'A', 'B', 'I', 'K', 'O', 'D', 'S', 'T', '0', '2', '5'])
@pytest.mark.parametrize('m,n,k', [(11472, 128, 1920), (9200, 1024, 2048), (1000, 3, 256),
                                   (333, 896, 128), (64, 256, 36), (5000, 768, 256), (1, 64, 7),
                                   (4097, 130, 1000)])
def test_gemm_bf16_rounding_points(gpu, bf16_mode, m, n, k, tile, monkeypatch):
    """fgr_gemm_bf16 = fp32 accumulation of bf16(A) bf16(W) products: vs the same rounded
    operands in fp64 within 1e-5 (accumulation order only); vs exact fp64 at bf16 level; bias /
    ReLU / residual / fused-leaky epilogues, strided A, the KPConv weight layout; every kernel
    variant (FGR_GEMM_BF16_TILE: '' default dispatch, 'z' register-staged, A..R the LDS-DMA g5)."""
    from fgreg import linear as fl
    monkeypatch.setenv('FGR_GEMM_BF16_TILE', tile)
    from fgreg import ops
    g = torch.Generator().manual_seed(m + n + k)
    x = torch.randn(m, k + 4, generator=g)[:, :k]
    w = torch.randn(n, k, generator=g) / math.sqrt(k)
    b = torch.randn(n, generator=g)
    r = torch.randn(m, n, generator=g)
    ref_bf = _bf(x) @ _bf(w).t() + b.double()
    ref = x.double() @ w.double().t() + b.double()
    X, W, Bb, R = x.to(gpu), w.to(gpu), b.to(gpu), r.to(gpu)
    y = fl.linear(X, W, Bb)
    assert rel_err(y.double(), ref_bf) < 1e-5
    assert rel_err(y.double(), ref) < 1e-2
    assert rel_err(fl.linear(X, W, Bb, act=ops.ACT_RELU).double(), ref_bf.clamp_min(0)) < 1e-5
    assert rel_err(fl.linear(X, W, residual=R).double(), ref_bf - b.double() + r.double()) < 1e-5
    lk = torch.nn.functional.leaky_relu(ref_bf.clamp_min(0) + r.double(), 0.1)
    assert rel_err(fl.linear(X, W, Bb, act=ops.ACT_RELU_RES_LEAKY, residual=R).double(), lk) < 1e-5
    wt = w.t().contiguous().view(k, n)
    assert rel_err(fl.linear(X, wt.to(gpu), Bb, transpose=True).double(), ref_bf) < 1e-5


def _attn_ref(q, k, v, qlens, klens, kv_seg, nhead):
    d = q.shape[1]
    dh = d // nhead
    qo, ko = np.cumsum([0] + qlens), np.cumsum([0] + klens)
    out = torch.zeros_like(q)
    for i in range(len(qlens)):
        j = kv_seg[i]
        qs = q[qo[i]:qo[i + 1]].view(-1, nhead, dh).transpose(0, 1) * math.sqrt(1.0 / dh)
        ks = k[ko[j]:ko[j + 1]].view(-1, nhead, dh).transpose(0, 1)
        vs = v[ko[j]:ko[j + 1]].view(-1, nhead, dh).transpose(0, 1)
        out[qo[i]:qo[i + 1]] = (torch.softmax(qs @ ks.transpose(1, 2), -1) @ vs).transpose(0, 1).reshape(-1, d)
    return out


@pytest.mark.parametrize('d', [256, 512])
@pytest.mark.parametrize('scale', [1.0, 4.0, 1e-6, 3e3])
def test_attention_bf16(gpu, bf16_mode, d, scale):
    """fgr_attention_bf16 (head_dim 32 / 64): separate key segmentation, partial and 1-key
    tiles, sharp softmax (scale 4: scores ~16), magnitudes far from 1 (bf16 shares fp32's
    exponent range, so no scaling is needed).
    * vs fp64 on the same bf16-rounded q * scale * log2(e), K and V: within 1e-2 (the
      remaining rounding is P's, ~2^-9 per weight) -- pins where the kernel rounds;
    * vs exact fp64: within 1e-2 where scores are O(1); a sharp softmax amplifies the bf16
      rounding of q and k (absolute score error ~ |s| 2^-8), so scale 4 is only reported;
    * clearly above the fp32-accurate path's error (the mode really is bf16)."""
    import fgreg.ops as ops
    rng = np.random.default_rng(11)
    nhead = 8
    dh = d // nhead
    qlens, klens, kv_seg = [300, 1, 64, 129], [65, 700, 1, 128], [1, 0, 3, 2]
    q = torch.from_numpy(rng.normal(size=(sum(qlens), d))) * scale
    kv = torch.from_numpy(rng.normal(size=(sum(klens), 2 * d))) * scale
    if scale > 100:
        kv[:, :d] /= scale * scale
    if scale < 1e-3:
        q /= scale * scale
    qg, kvg = q.float().to(gpu), kv.float().to(gpu)
    qo, ko = ops.offsets(qlens, gpu), ops.offsets(klens, gpu)
    seg = torch.tensor(kv_seg, dtype=torch.int32, device=gpu)
    out = ops.attention(qg, kvg[:, :d], kvg[:, d:], qo, ko, seg, max(qlens), nhead,
                        max_kv_len=max(klens)).double()
    sl2 = math.sqrt(1.0 / dh) * 1.4426950408889634
    q_r = _bf((q.float() * np.float32(sl2)).float()) / sl2       # what the kernel multiplies
    ref_r = _attn_ref(q_r, _bf(kv[:, :d].float()), _bf(kv[:, d:].float()), qlens, klens, kv_seg,
                      nhead)
    ref = _attn_ref(q, kv[:, :d], kv[:, d:], qlens, klens, kv_seg, nhead)
    e_r, e = rel_err(out, ref_r), rel_err(out, ref)
    print(f'\nd={d} scale={scale}: vs rounded-operand ref {e_r:.2e}, vs exact {e:.2e}')
    assert e_r < 1e-2, e_r
    if scale != 4.0:
        assert e < 1e-2, e
    assert e > 1e-5, e            # not silently the fp32-accurate path


def _random_model(cfg, seed):
    import fgreg
    torch.manual_seed(seed)
    np.random.seed(seed)          # init_kernel_points draws from numpy's global generator
    m = fgreg.RegTR(cfg)
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.running_mean.copy_(0.1 * torch.randn(mod.running_mean.shape, generator=g))
                mod.running_var.copy_(0.75 + 0.5 * torch.rand(mod.running_var.shape, generator=g))
        m.correspondence_decoder.conf_logits_decoder.bias.fill_(4.0)
    return m.eval()


def _rot_deg(a, b):
    r = a[:, :3] @ b[:, :3].T
    return math.degrees(math.acos(max(-1.0, min(1.0, (np.trace(r) - 1) / 2))))


# the sweep's cases (the bound was set from them) and HELD-OUT cases that did not enter the
# sweep (round 4: seeds 100-103 at 6k points, 110-111 at 20k), run against the same fixed bound
SWEEP_CASES = [(s, 6000) for s in range(8)] + [(20, 20000), (21, 20000)]
HELD_OUT_CASES = [(s, 6000) for s in range(100, 104)] + [(110, 20000), (111, 20000)]


@pytest.mark.parametrize('seed,n_points', SWEEP_CASES + HELD_OUT_CASES)
def test_bf16_forward_3dlomatch_vs_oracle(gpu, bf16_mode, seed, n_points):
    """The configs[4] forward in bf16 on low-overlap pairs against the fp32 CPU oracle, over
    16 random models and input pairs (seeded per case; no hand-picked seed; 6 of them held out
    of the sweep that set the bound): geometry bit-exact, outputs within the stated bf16
    tolerance."""
    import fgreg.config as fc
    from fgreg.synthetic import make_batch
    cfg = fc.get('3dlomatch')
    model = _random_model(cfg, seed)
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    src, tgt, _ = make_batch('3dlomatch', 1, start=seed, n_points=n_points)
    model = model.to(gpu)
    batch = {'src_xyz': [torch.from_numpy(s).to(gpu) for s in src],
             'tgt_xyz': [torch.from_numpy(t).to(gpu) for t in tgt]}
    out = model(batch)
    ref = mo.forward(cfg, sd, src, tgt, mode=mo.geom.INDEX)
    for lvl in range(len(ref['kpconv_meta']['points'])):
        for key in ('points', 'neighbors', 'pools', 'upsamples', 'stack_lengths'):
            assert torch.equal(batch['kpconv_meta'][key][lvl].cpu(), ref['kpconv_meta'][key][lvl])
    errs = {k: rel_err(out[k][0], ref[k][0]) for k in KEYS}
    p, pr = out['pose'].cpu().numpy()[-1, 0], ref['pose'].numpy()[-1, 0]
    rot, trans = _rot_deg(p, pr), float(np.linalg.norm(p[:, 3] - pr[:, 3]))
    print(f'\nbf16 3dlomatch seed={seed} n={n_points}: rel errs',
          {k: f'{v:.2e}' for k, v in errs.items()}, f'rot {rot:.3e} deg trans {trans:.3e} m')
    for k, v in errs.items():
        assert v < BF16_FEAT_TOL, (k, v)
    assert rot < BF16_ROT_DEG and trans < BF16_TRANS, (rot, trans)
    assert max(errs.values()) > 1e-4            # really the bf16 mode, not the fp32-accurate path


@pytest.mark.parametrize('lens', [[935, 936], [1100, 977, 64, 1, 3000, 130]])
def test_bf16_qkv_images_vs_two_launch_path(gpu, bf16_mode, lens):
    """fgr_gemm_bf16_qkv (the bf16 in_proj writing q fp32 and the bf16 K / V images of every
    global 64-row tile, head dim 64) + fgr_attention_bf16_img vs fgr_gemm_bf16 ->
    fgr_attention_bf16 (per-segment images): the images hold the same bf16 values and only the
    key tiling differs, which moves where the online softmax rounds P to bf16 -- so both are
    compared with the fp64 attention of the same q / k / v: the new path's error within 1.25x
    of the old one's (+ 1e-4) and below 1e-2; self- and cross-attention, segments starting
    inside tiles."""
    from fgreg import linear as lin
    from fgreg import ops
    n, d, nh = sum(lens), 512, 8
    g = torch.Generator().manual_seed(n + 1)
    h = (torch.randn(n, d, generator=g) * 1.5).to(gpu)
    w = (torch.randn(3 * d, d, generator=g) / math.sqrt(d)).to(gpu)
    b = torch.randn(3 * d, generator=g).to(gpu)
    assert ops.qkv_bf16_supported(n, d, nh)
    off = ops.offsets(lens, gpu)
    B = len(lens) // 2
    for kv in (list(range(len(lens))), [(c + B) % len(lens) for c in range(len(lens))]):
        kv_seg = torch.tensor(kv, dtype=torch.int32, device=gpu)
        o = ops.qkv_attention(h, lin.weight_image(w, mode='bf16'), b, off, kv_seg, max(lens), nh,
                              mode='bf16')
        qkv = lin.linear(h, w, b)
        o2 = ops.attention(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], off, off, kv_seg,
                           max(lens), nh)
        q64 = qkv.double().cpu()
        ref = _attn_ref(q64[:, :d], q64[:, d:2 * d], q64[:, 2 * d:], lens, lens, kv, nh)
        e_new, e_old = rel_err(o, ref), rel_err(o2, ref)
        print(f'\nlens {lens} kv {kv}: new {e_new:.2e} old {e_old:.2e} apart {rel_err(o, o2):.2e}')
        assert e_new < 1.25 * e_old + 1e-4 and e_new < 1e-2, (e_new, e_old)
