"""GPU parity of the test-step tail (fgreg/loss.py on libfgreg).

1. On the reference's own forward outputs and loss inputs (tests/golden/*): every loss and
   metric against the reference's compute_loss / _compute_metrics.
2. End to end from our forward on the reference's kpconv_meta.
3. Full ModelNet size (B = 8, random init) against the CPU oracle (oracle/loss_oracle.py,
   pinned to the reference by tests/test_oracle.py) on the same forward outputs.
4. Kernel edge cases: pool rows without a valid entry (NaN, as the reference), empty masks.
Tolerances: losses 1e-5 relative (fp32 reductions in a different order; the InfoNCE
threshold tests r_p / r_n use torch.cdist's matrix-multiply distance form, so a flip needs a
point within ~1e-7 of a threshold -- none in these inputs); rotation errors 1e-3 deg.
"""
import numpy as np
import pytest
import torch

import loss_oracle as lo
from conftest import loss_fixture

pytestmark = pytest.mark.gpu


class _Crit:
    def __init__(self, W):
        self.W = W


class _Model:
    def __init__(self, cfg, W, W_un):
        self.cfg = cfg
        self.feature_criterion = _Crit(W)
        self.feature_criterion_un = _Crit(W_un)


def _close(a, b, rel=1e-5):
    return abs(a - b) <= rel * max(1.0, abs(b))


def test_loss_on_reference_outputs(gpu):
    from fgreg import loss as fl
    cfg, pred, batch, ref_losses, ref_metrics, ref_pyr, W, W_un = loss_fixture(gpu)
    losses = fl.compute_loss(_Model(cfg, W, W_un), pred, batch)
    assert list(losses) == list(ref_losses), (list(losses), list(ref_losses))
    for k, v in ref_losses.items():
        assert _close(float(losses[k]), v), (k, float(losses[k]), v)
    for k, v in ref_pyr.items():
        np.testing.assert_allclose(batch['overlap_pyr'][k].cpu().numpy(), v, rtol=1e-6, atol=1e-7)
    metrics = fl.compute_metrics(pred, batch)
    np.testing.assert_allclose(metrics['rot_err_deg'].cpu().numpy(), ref_metrics['rot_err_deg'],
                               atol=1e-3)
    np.testing.assert_allclose(metrics['trans_err'].cpu().numpy(), ref_metrics['trans_err'],
                               rtol=1e-5, atol=1e-6)


def test_loss_end_to_end_on_reference_meta(gpu):
    """Our forward (reference kpconv_meta) -> our losses vs the reference's losses; the
    forward itself is within 1e-4, so the losses are compared at 1e-3."""
    import fgreg
    from fgreg import loss as fl
    from conftest import forward_fixture
    cfg, sd, src, tgt, meta, _ = forward_fixture('forward_modelnet_small')
    _, _, batch, ref_losses, _, _, W, W_un = loss_fixture(gpu)
    model = fgreg.RegTR(cfg)
    model.load_state_dict(sd, strict=False)
    with torch.no_grad():
        model.feature_criterion.W.copy_(W.cpu())
        model.feature_criterion_un.W.copy_(W_un.cpu())
    model = model.to(gpu).eval()
    model.preprocessor = fgreg.FixedMetaPreprocessor(batch['kpconv_meta'])
    out = model({'src_xyz': batch['src_xyz'], 'tgt_xyz': batch['tgt_xyz']})
    batch['kpconv_meta'] = {k: list(v) for k, v in batch['kpconv_meta'].items()}
    losses = fl.compute_loss(model, out, batch)
    for k, v in ref_losses.items():
        assert _close(float(losses[k]), v, 1e-3), (k, float(losses[k]), v)


def test_loss_full_size_vs_oracle(gpu):
    import fgreg
    import fgreg.config as fc
    from fgreg import loss as fl
    from fgreg.synthetic import make_batch
    cfg = fc.get('modelnet')
    torch.manual_seed(3)
    model = fgreg.RegTR(cfg).to(gpu).eval()
    src, tgt, pose = make_batch('modelnet', 8)
    rng = np.random.default_rng(0)
    batch = {'src_xyz': [torch.from_numpy(s).to(gpu) for s in src],
             'tgt_xyz': [torch.from_numpy(t).to(gpu) for t in tgt],
             'pose': torch.from_numpy(pose).to(gpu),
             'src_overlap': [torch.from_numpy((rng.uniform(size=len(s)) < 0.7).astype(np.float32))
                             .to(gpu) for s in src],
             'tgt_overlap': [torch.from_numpy((rng.uniform(size=len(t)) < 0.7).astype(np.float32))
                             .to(gpu) for t in tgt]}
    out = model(batch)
    losses = fl.compute_loss(model, out, batch)
    cpu = lambda v: [t.cpu() for t in v] if isinstance(v, list) else v.cpu()
    pred_c = {k: cpu(v) for k, v in out.items()}
    meta_keys = ('points', 'neighbors', 'pools', 'upsamples', 'stack_lengths')
    batch_c = {k: (cpu(v) if k != 'kpconv_meta' else {kk: cpu(v[kk]) for kk in meta_keys})
               for k, v in batch.items() if k != 'overlap_pyr'}
    ref, pyr = lo.compute_loss(cfg, model.feature_criterion.W.detach().cpu(),
                               model.feature_criterion_un.W.detach().cpu(), pred_c, batch_c)
    for k in ref:
        assert _close(float(losses[k]), float(ref[k])), (k, float(losses[k]), float(ref[k]))
    p = len(pyr) - 1
    torch.testing.assert_close(batch['overlap_pyr'][f'pyr_{p}'].cpu(), pyr[p], rtol=1e-6,
                               atol=1e-7, equal_nan=True)
    rot, trans = lo.pose_errors(pred_c['pose'], batch_c['pose'])
    m = fl.compute_metrics(out, batch)
    # near-identity rotations make acos ill-conditioned (d acos / dc ~ 1/sin): compare the
    # cosine instead of the angle
    np.testing.assert_allclose(np.cos(np.deg2rad(m['rot_err_deg'].cpu().numpy())),
                               np.cos(np.deg2rad(rot.numpy())), atol=2e-6)
    np.testing.assert_allclose(m['trans_err'].cpu().numpy(), trans.numpy(), rtol=1e-5, atol=1e-6)


def test_overlap_pool_edges(gpu):
    """Rows without a valid pool entry give NaN (0/0, the reference's behaviour); values are
    clamped to [0, 1]; shadow indices (>= n_prev) are skipped."""
    from fgreg import loss as fl
    prev = torch.tensor([0.0, 1.0, 1.0, 0.5], device=gpu)
    pools = torch.tensor([[0, 1, 4, 4], [4, 4, 4, 4], [1, 2, 3, 4], [3, 3, 3, 3]], device=gpu)
    out = fl.overlap_pool(prev, pools).cpu()
    assert out[0] == 0.5 and torch.isnan(out[1]) and abs(out[2] - 2.5 / 3) < 1e-7 and out[3] == 0.5


def test_infonce_empty_mask_is_nan(gpu):
    """No anchor within r_p of any positive -> sum(mask) = 0 -> NaN, as the reference."""
    from fgreg import loss as fl
    from fgreg import ops
    g = torch.Generator().manual_seed(0)
    A, P = torch.randn(40, 32, generator=g), torch.randn(30, 32, generator=g)
    axyz, pxyz = torch.randn(40, 3, generator=g), torch.randn(30, 3, generator=g) + 10.0
    W = torch.randn(32, 32, generator=g)
    out = fl.infonce(W.to(gpu), A.to(gpu), P.to(gpu), axyz.to(gpu), pxyz.to(gpu),
                     ops.offsets([40], gpu), ops.offsets([30], gpu), 0.12, 0.24)
    assert torch.isnan(out.cpu())
    ref = lo.infonce_pair(W, A, P, axyz, pxyz, 0.12, 0.24)
    assert torch.isnan(ref)


def _circle_cfg(cfg):
    c = type(cfg)(cfg)
    c['feature_loss_type'] = 'circle'
    return c


def test_circle_loss_on_reference_outputs(gpu):
    """feature_loss_type: circle (finegrained_regtr.py:86-88, CircleLossFull with Euclidean
    feature distances, feature_loss.py:160-243) on the reference's own forward outputs: the
    eval path (fgr_circle_loss) and the differentiable training path (compute_loss_train)
    against the reference's compute_loss with that option (loss_circle_modelnet_small.npz)."""
    from conftest import golden
    from fgreg import loss as fl
    cfg, pred, batch, _, _, _, _, _ = loss_fixture(gpu)
    cfg = _circle_cfg(cfg)
    g = golden('loss_circle_modelnet_small')
    ref = {k[5:]: float(g[k]) for k in g.files}
    losses = fl.compute_loss(_Model(cfg, None, None), pred, batch)
    assert list(losses) == list(ref)
    for k, v in ref.items():
        assert _close(float(losses[k]), v), (k, float(losses[k]), v)
    m = _Model(cfg, None, None)
    del m.feature_criterion, m.feature_criterion_un
    losses_t = fl.compute_loss_train(m, pred, batch)
    for k, v in ref.items():
        assert _close(float(losses_t[k]), v, 1e-4), (k, float(losses_t[k]), v)


def test_circle_loss_gradients_vs_oracle(gpu):
    """The training path's gradients of the circle feature losses w.r.t. the features against
    torch autograd of the oracle's restatement in fp64 (1e-3 relative Frobenius: the Gram-form
    distances on the f16x3 GEMM vs the explicit differences)."""
    from fgreg import loss as fl
    cfg, pred, batch, _, _, _, _, _ = loss_fixture(gpu)
    cfg = _circle_cfg(cfg)
    keys = ('src_feat', 'tgt_feat', 'src_feat_un', 'tgt_feat_un')
    pg = {k: [t.detach().clone().requires_grad_(True) for t in pred[k]] for k in keys}
    pred_g = dict(pred, **pg)
    m = _Model(cfg, None, None)
    del m.feature_criterion, m.feature_criterion_un
    losses = fl.compute_loss_train(m, pred_g, batch)
    (losses['feature_un'] + sum(losses[f'feature_{i}'] for i in cfg.feature_loss_on)).backward()
    B = len(pred['src_kp'])
    pose = batch['pose'].cpu().double()
    pc = {k: [t.detach().cpu().double().requires_grad_(True) for t in pred[k]] for k in keys}
    a_xyz = [lo.rigid_apply(pose[b], pred['src_kp'][b].cpu().double()) for b in range(B)]
    p_xyz = [t.cpu().double() for t in pred['tgt_kp']]
    tot = 0
    for i in cfg.feature_loss_on:
        tot = tot + torch.stack([lo.circle_pair(pc['src_feat'][b][i], pc['tgt_feat'][b][i],
                                                a_xyz[b], p_xyz[b], cfg.r_p, cfg.r_n)
                                 for b in range(B)]).mean()
    tot = tot + torch.stack([lo.circle_pair(pc['src_feat_un'][b], pc['tgt_feat_un'][b], a_xyz[b],
                                            p_xyz[b], cfg.r_p, cfg.r_n) for b in range(B)]).mean()
    tot.backward()
    for k in keys:
        for b in range(B):
            got, want = pg[k][b].grad.cpu().double(), pc[k][b].grad
            assert float((got - want).norm()) <= 1e-3 * float(want.norm()) + 1e-12, (k, b)


def test_circle_loss_full_size_vs_oracle(gpu):
    """ModelNet B = 8 sizes (random features of d = 256, ~600 keypoints per cloud) through
    fgr_circle_loss against the oracle; and a pair with no negative anywhere gives NaN."""
    from fgreg import loss as fl
    from fgreg import ops
    g = torch.Generator().manual_seed(1)
    B, d = 8, 256
    na = [590 + 7 * b for b in range(B)]
    npp = [600 - 5 * b for b in range(B)]
    A = [torch.randn(n, d, generator=g) * 0.1 for n in na]
    P = [torch.randn(n, d, generator=g) * 0.1 for n in npp]
    ax = [torch.rand(n, 3, generator=g) for n in na]
    px = [torch.rand(n, 3, generator=g) for n in npp]
    T = lambda L: torch.cat(L).to(gpu)
    out = fl.circle(T(A), T(P), T(ax), T(px), na, npp, ops.offsets(na, gpu), ops.offsets(npp, gpu),
                    0.12, 0.24)
    ref = torch.stack([lo.circle_pair(A[b], P[b], ax[b], px[b], 0.12, 0.24)
                       for b in range(B)]).mean()
    assert _close(float(out), float(ref)), (float(out), float(ref))
    # r_n beyond every distance: no negatives -> empty selections -> NaN, as the reference
    out = fl.circle(T(A[:1]), T(P[:1]), T(ax[:1]), T(px[:1]), na[:1], npp[:1],
                    ops.offsets(na[:1], gpu), ops.offsets(npp[:1], gpu), 0.12, 10.0)
    assert torch.isnan(out.cpu()) and torch.isnan(lo.circle_pair(A[0], P[0], ax[0], px[0], 0.12, 10.0))
