"""Test-step tail on libfgreg: the reference's ``compute_loss``
(models/finegrained_regtr.py:252-309) and ``_compute_metrics`` (generic_reg_model.py:203-215)
on the packed forward outputs, so ``GenericRegModel.test_step`` runs at GPU speed.

* ``compute_overlaps``  finegrained_kpconv.py:545-571      fgr_overlap_pool per level
* overlap loss          nn.BCEWithLogitsLoss (mean)          fgr_bce_logits_mean
* feature loss          InfoNCELossFull (feature_loss.py:246-314): the match logits
                        A W_sym P^T as two f16x3 GEMMs over all pairs at once (A W_sym, then
                        against every positive row), the masked log-sum-exp per anchor row
                        (fgr_infonce_rows) and the per-pair / batch means (fgr_infonce_reduce)
* correspondence loss   CorrCriterion('mae') both directions  fgr_corr_loss
* metrics               se3_compare of every layer's pose     fgr_se3_compare
Same keys, weights (finegrained_regtr.py:94-98) and reduction order as the reference; all
arithmetic in fp32 on the GPU (no CPU path: the ops raise on CPU tensors).
"""
import itertools

import torch

from . import _lib, ops
from .linear import linear
from .ops import _c, _dev, _ptr, _stream


def overlap_pool(prev: torch.Tensor, pools: torch.Tensor) -> torch.Tensor:
    """One compute_overlaps step: (N_prev,) overlaps, (N_q, H) pool table -> (N_q,)."""
    _dev(prev, pools)
    prev, pools = _c(prev, torch.float32), _c(pools, torch.int64)
    out = torch.empty((pools.shape[0],), dtype=torch.float32, device=prev.device)
    _lib.check(_lib.load().fgr_overlap_pool(_ptr(prev), prev.shape[0], _ptr(pools), pools.shape[0],
                                            pools.shape[1], _ptr(out), _stream()),
               'fgr_overlap_pool')
    return out


class _FeatCdistFn(torch.autograd.Function):
    """The reference's cdist(a, p, 'euclidean') of one pair (feature_loss.py:11-36: direct
    differences, sqrt(sum + 1e-12)) for the training CircleLoss: forward by fgr_pair_cdist,
    backward d fd_ij / d a_i = (a_i - p_j) / fd_ij as GEMMs of W = grad / fd:
    da = rowsum(W) a - W p, dp = colsum(W) p - W^T a (no Gram-form cancellation in either)."""

    @staticmethod
    def forward(ctx, a, pp):
        a, pp = _c(a, torch.float32), _c(pp, torch.float32)
        _dev(a, pp)
        na, npos, d = a.shape[0], pp.shape[0], a.shape[1]
        fd = torch.empty((na, npos), dtype=torch.float32, device=a.device)
        t = ops.to_device([0, na, 0, npos, 0], torch.int64, a.device)   # a_off, p_off, fd_off
        _lib.check(_lib.load().fgr_pair_cdist(_ptr(a), _ptr(pp), d, _ptr(t[0:2]), _ptr(t[2:4]),
                                              _ptr(t[4:5]), 1, na, npos, _ptr(fd), _stream()),
                   'fgr_pair_cdist')
        ctx.save_for_backward(a, pp, fd)
        return fd

    @staticmethod
    def backward(ctx, g):
        a, pp, fd = ctx.saved_tensors
        w = (g / fd).contiguous()
        da = dp = None
        if ctx.needs_input_grad[0]:
            da = a * w.sum(1, keepdim=True) - linear(w, pp.t().contiguous(), cache=False)
        if ctx.needs_input_grad[1]:
            dp = pp * w.sum(0)[:, None] - linear(w.t().contiguous(), a.t().contiguous(), cache=False)
        return da, dp


def compute_overlaps(batch):
    """finegrained_kpconv.py:545-571: {'pyr_0': cat(src_overlap + tgt_overlap), 'pyr_p': ...}."""
    meta = batch['kpconv_meta']
    pyr = {'pyr_0': torch.cat(list(batch['src_overlap']) + list(batch['tgt_overlap']),
                              dim=0).float()}
    for p in range(1, len(meta['points'])):
        pyr[f'pyr_{p}'] = overlap_pool(pyr[f'pyr_{p - 1}'], meta['pools'][p - 1])
    return pyr


def bce_with_logits_mean(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    _dev(x, y)
    assert x.dim() == 1 and y.shape == x.shape and x.dtype == torch.float32
    y = _c(y, torch.float32)
    out = torch.empty((), dtype=torch.float32, device=x.device)
    _lib.check(_lib.load().fgr_bce_logits_mean(_ptr(x), x.stride(0), _ptr(y), x.shape[0],
                                               _ptr(out), _stream()), 'fgr_bce_logits_mean')
    return out


def transform_points(xyz, seg_off, pose, inverse=False) -> torch.Tensor:
    """se3_transform_list over packed segments (pose (n_seg, 3, 4))."""
    _dev(xyz, seg_off, pose)
    xyz, pose = _c(xyz, torch.float32), _c(pose, torch.float32)
    out = torch.empty_like(xyz)
    _lib.check(_lib.load().fgr_transform_points(_ptr(xyz), xyz.shape[0], _ptr(seg_off),
                                                seg_off.numel() - 1, _ptr(pose), int(inverse),
                                                _ptr(out), _stream()), 'fgr_transform_points')
    return out


_WSYM = {}


def _w_sym(W: torch.Tensor) -> torch.Tensor:
    """triu(W) + triu(W)^T (feature_loss.py:280-281), kept per parameter version so its
    split image is cached by linear()."""
    key = id(W)
    ent = _WSYM.get(key)
    if ent is None or ent[0] is not W or ent[1] != W._version or ent[2] != W.data_ptr():
        with torch.no_grad():
            t = torch.triu(W.detach().float())
            ent = (W, W._version, W.data_ptr(), (t + t.t()).contiguous())
        _WSYM[key] = ent
    return ent[3]


def infonce(W, anchor_feat, positive_feat, anchor_xyz, positive_xyz, a_off, p_off, r_p, r_n):
    """InfoNCELossFull.forward over B pairs packed along rows (pair b: anchor rows
    a_off[b]..a_off[b+1], positive rows p_off[b]..p_off[b+1]) -> 0-d tensor."""
    _dev(anchor_feat, positive_feat, anchor_xyz, positive_xyz, a_off, p_off)
    A = _c(anchor_feat, torch.float32)
    P = _c(positive_feat, torch.float32)
    aw = linear(A, _w_sym(W))                          # A W_sym (W_sym symmetric)
    logits = linear(aw, P, cache=False)                # (N_a, N_p) over all pairs
    n_a, n_pairs = A.shape[0], a_off.numel() - 1
    row_loss = torch.empty((n_a,), dtype=torch.float32, device=A.device)
    row_mask = torch.empty_like(row_loss)
    L = _lib.load()
    axyz, pxyz = _c(anchor_xyz, torch.float32), _c(positive_xyz, torch.float32)
    _lib.check(L.fgr_infonce_rows(_ptr(logits), logits.stride(0), _ptr(axyz), _ptr(pxyz),
                                  _ptr(a_off), _ptr(p_off), n_pairs, n_a, float(r_p), float(r_n),
                                  _ptr(row_loss), _ptr(row_mask), _stream()), 'fgr_infonce_rows')
    out = torch.empty((), dtype=torch.float32, device=A.device)
    _lib.check(L.fgr_infonce_reduce(_ptr(row_loss), _ptr(row_mask), _ptr(a_off), n_pairs,
                                    _ptr(out), _stream()), 'fgr_infonce_reduce')
    return out


def circle(anchor_feat, positive_feat, anchor_xyz, positive_xyz, a_lens, p_lens, a_off, p_off,
           r_p, r_n):
    """CircleLossFull.forward (feature_loss.py:232-243, Euclidean feature distances as
    finegrained_regtr.py:87 builds it) over B pairs packed along rows -> 0-d tensor
    (fgr_circle_loss). a_lens / p_lens: host lengths of the pairs' anchor / positive rows."""
    _dev(anchor_feat, positive_feat, anchor_xyz, positive_xyz, a_off, p_off)
    A = _c(anchor_feat, torch.float32)
    P = _c(positive_feat, torch.float32)
    assert A.shape[1] == P.shape[1] and len(a_lens) == len(p_lens)
    sizes = [a * b for a, b in zip(a_lens, p_lens)]
    fd_off = torch.tensor([0] + list(itertools.accumulate(sizes)), dtype=torch.int64,
                          device=A.device)
    n_a, n_p, fd_elems = A.shape[0], P.shape[0], sum(sizes)
    L = _lib.load()
    nb = _lib._sz(0)
    _lib.check(L.fgr_circle_loss_workspace(fd_elems, n_a, n_p, nb), 'fgr_circle_loss_workspace')
    ws = torch.empty(nb.value, dtype=torch.uint8, device=A.device)
    out = torch.empty((), dtype=torch.float32, device=A.device)
    axyz, pxyz = _c(anchor_xyz, torch.float32), _c(positive_xyz, torch.float32)
    _lib.check(L.fgr_circle_loss(_ptr(A), _ptr(P), A.shape[1], _ptr(axyz), _ptr(pxyz),
                                 _ptr(a_off), _ptr(p_off), _ptr(fd_off), len(a_lens), n_a, n_p,
                                 max(a_lens), max(p_lens), fd_elems, float(r_p), float(r_n),
                                 _ptr(ws), nb.value, _ptr(out), _stream()), 'fgr_circle_loss')
    return out


def corr_loss(xyz, corr, w, seg_off, pose) -> torch.Tensor:
    """src (pose) + tgt (se3_inv(pose)) CorrCriterion('mae') with overlap weights."""
    _dev(xyz, corr, w, seg_off, pose)
    xyz, corr, w, pose = (_c(t, torch.float32) for t in (xyz, corr, w, pose))
    out = torch.empty((), dtype=torch.float32, device=xyz.device)
    _lib.check(_lib.load().fgr_corr_loss(_ptr(xyz), _ptr(corr), _ptr(w), _ptr(seg_off),
                                         pose.shape[0], _ptr(pose), _ptr(out), _stream()),
               'fgr_corr_loss')
    return out


def se3_compare(pred, gt):
    """pred (L, B, 3, 4), gt (B, 3, 4) -> {'rot_deg': (L, B), 'trans': (L, B)}."""
    _dev(pred, gt)
    pred, gt = _c(pred, torch.float32), _c(gt, torch.float32)
    n_layers, n_pairs = pred.shape[0], pred.shape[1]
    rot = torch.empty((n_layers, n_pairs), dtype=torch.float32, device=pred.device)
    trans = torch.empty_like(rot)
    _lib.check(_lib.load().fgr_se3_compare(_ptr(pred), _ptr(gt), n_layers, n_pairs, _ptr(rot),
                                           _ptr(trans), _stream()), 'fgr_se3_compare')
    return {'rot_deg': rot, 'trans': trans}


def weight_dict(cfg):
    """finegrained_regtr.py:94-98."""
    wd = {}
    for k in ['overlap', 'feature', 'corr']:
        for i in cfg.get(f'{k}_loss_on', [cfg.num_encoder_layers - 1]):
            wd[f'{k}_{i}'] = cfg.get(f'wt_{k}')
    wd['feature_un'] = cfg.wt_feature_un
    return wd


def compute_loss(model, pred, batch):
    """RegTR.compute_loss (finegrained_regtr.py:252-309) -> dict of 0-d tensors with the
    reference's keys; adds batch['overlap_pyr'] like the reference."""
    cfg = model.cfg
    ftype = cfg.get('feature_loss_type', 'infonce')
    if ftype not in ('infonce', 'circle'):
        raise NotImplementedError(f'feature_loss_type {ftype!r} (the reference builds infonce '
                                  'and circle, finegrained_regtr.py:83-90)')
    meta = batch['kpconv_meta']
    pose_gt = _c(batch['pose'].float(), torch.float32)           # (B, 3, 4)
    p = len(meta['stack_lengths']) - 1
    pyr = compute_overlaps(batch)
    batch['overlap_pyr'] = pyr
    ov = pyr[f'pyr_{p}']
    lens = [int(v) for v in meta['stack_lengths'][p].tolist()]
    B = len(lens) // 2
    dev = ov.device
    seg_off = ops.offsets(lens, dev)
    a_off, p_off = ops.offsets(lens[:B], dev), ops.offsets(lens[B:], dev)

    losses = {}
    logits = torch.cat(list(pred['src_overlap']) + list(pred['tgt_overlap']), dim=-2)
    for i in cfg.overlap_loss_on:
        losses[f'overlap_{i}'] = bce_with_logits_mean(logits[i, :, 0], ov)
    src_kp, tgt_kp = torch.cat(list(pred['src_kp'])), torch.cat(list(pred['tgt_kp']))
    axyz = transform_points(src_kp, a_off, pose_gt)
    if ftype == 'circle':        # CircleLossFull for both feature losses (:87-88, no weights)
        feat = lambda crit, a, pp: circle(a, pp, axyz, tgt_kp, lens[:B], lens[B:], a_off, p_off,
                                          cfg.r_p, cfg.r_n)
    else:
        feat = lambda crit, a, pp: infonce(crit.W, a, pp, axyz, tgt_kp, a_off, p_off, cfg.r_p,
                                           cfg.r_n)
    for i in cfg.feature_loss_on:
        losses[f'feature_{i}'] = feat(getattr(model, 'feature_criterion', None),
                                      torch.cat([s[i] for s in pred['src_feat']]),
                                      torch.cat([t[i] for t in pred['tgt_feat']]))
    losses['feature_un'] = feat(getattr(model, 'feature_criterion_un', None),
                                torch.cat(list(pred['src_feat_un'])),
                                torch.cat(list(pred['tgt_feat_un'])))
    xyz = torch.cat([src_kp, tgt_kp])
    for i in cfg.corr_loss_on:
        corr = torch.cat([w[i] for w in pred['src_kp_warped']] +
                         [w[i] for w in pred['tgt_kp_warped']])
        losses[f'corr_{i}'] = corr_loss(xyz, corr, ov, seg_off, pose_gt)
    wd = weight_dict(cfg)
    losses['total'] = torch.sum(torch.stack([losses[k] * wd[k] for k in losses]))
    return losses


def compute_metrics(pred, batch):
    """GenericRegModel._compute_metrics (generic_reg_model.py:203-215)."""
    metrics = {}
    for k in [k for k in pred.keys() if k.startswith('pose')]:
        err = se3_compare(pred[k], batch['pose'])
        metrics[f'rot_err_deg{k[4:]}'] = err['rot_deg']
        metrics[f'trans_err{k[4:]}'] = err['trans']
    return metrics


class _InfoNCEFn(torch.autograd.Function):
    """InfoNCELossFull over B pairs packed along rows (feature_loss.py:268-314) from the match
    logits over ALL pairs' positive rows, differentiable in the logits: forward
    fgr_infonce_rows + fgr_infonce_reduce (as the evaluation path), backward
    fgr_infonce_rows_bwd (softmax minus the positive's indicator, per row weight = kept /
    (pair's kept rows * pairs)). One launch each way for every pair of the batch."""

    @staticmethod
    def forward(ctx, logits, axyz, pxyz, a_off, p_off, pair_idx, r_p, r_n):
        n_a, n_p = logits.shape
        n_pairs = a_off.numel() - 1
        row_loss = torch.empty((n_a,), dtype=torch.float32, device=logits.device)
        row_mask = torch.empty_like(row_loss)
        L = _lib.load()
        _lib.check(L.fgr_infonce_rows(_ptr(logits), logits.stride(0), _ptr(axyz), _ptr(pxyz),
                                      _ptr(a_off), _ptr(p_off), n_pairs, n_a, float(r_p), float(r_n),
                                      _ptr(row_loss), _ptr(row_mask), _stream()), 'fgr_infonce_rows')
        out = torch.empty((), dtype=torch.float32, device=logits.device)
        _lib.check(L.fgr_infonce_reduce(_ptr(row_loss), _ptr(row_mask), _ptr(a_off), n_pairs,
                                        _ptr(out), _stream()), 'fgr_infonce_reduce')
        ctx.r_n = float(r_n)
        ctx.save_for_backward(logits, axyz, pxyz, a_off, p_off, pair_idx, row_mask)
        return out

    @staticmethod
    def backward(ctx, g):
        logits, axyz, pxyz, a_off, p_off, pair_idx, row_mask = ctx.saved_tensors
        n_a, n_p = logits.shape
        n_pairs = a_off.numel() - 1
        kept = torch.zeros((n_pairs,), dtype=torch.float32, device=logits.device)
        kept = kept.index_add_(0, pair_idx, row_mask)[pair_idx]
        # a pair with no kept row: the reference's empty selection passes no gradient on
        w = torch.where(kept > 0, row_mask / (kept * n_pairs), torch.zeros_like(row_mask))
        dl = torch.empty_like(logits)
        _lib.check(_lib.load().fgr_infonce_rows_bwd(
            _ptr(logits), logits.stride(0), _ptr(axyz), _ptr(pxyz), _ptr(a_off), _ptr(p_off),
            n_pairs, n_a, n_p, ctx.r_n, _ptr(w), _ptr(g.float().contiguous()), _ptr(dl), dl.stride(0),
            _stream()), 'fgr_infonce_rows_bwd')
        return dl, None, None, None, None, None, None, None


def compute_loss_train(model, pred, batch):
    """RegTR.compute_loss (finegrained_regtr.py:252-309) as a differentiable graph: the same
    keys, weights and reductions as compute_loss above, with the match logits of all pairs on
    the differentiable f16x3 GEMMs (fgreg.autograd.linear_t: A W_sym, then against the
    positives), InfoNCE over all pairs in one autograd Function (_InfoNCEFn: the evaluation
    kernels forward, fgr_infonce_rows_bwd backward), the BCE / CircleLoss / L1 terms as torch
    ops on the device, so that ``losses['total'].backward()`` reaches every parameter
    (trainer.py:110-125). The overlap pyramid and the warped keypoint targets carry no
    gradient (fgr_overlap_pool, fgr_transform_points as in compute_loss)."""
    import torch.nn.functional as F
    from .autograd import linear_t
    cfg = model.cfg
    ftype = cfg.get('feature_loss_type', 'infonce')
    if ftype not in ('infonce', 'circle'):
        raise NotImplementedError(f'feature_loss_type {ftype!r} (the reference builds infonce '
                                  'and circle, finegrained_regtr.py:83-90)')
    meta = batch['kpconv_meta']
    pose = batch['pose'].float()
    p = len(meta['stack_lengths']) - 1
    with torch.no_grad():
        pyr = compute_overlaps(batch)
    batch['overlap_pyr'] = pyr
    ov = pyr[f'pyr_{p}']
    host = meta.get('_host')          # the forward's host layout: no device read-back
    lens = list(host['lengths'][p]) if host else [int(v) for v in meta['stack_lengths'][p].tolist()]
    B = len(lens) // 2
    src_w, tgt_w = ov[:sum(lens[:B])], ov[sum(lens[:B]):]          # overlap weights (targets)

    def w_sym(W):
        t = torch.triu(W)
        return t + t.t()

    # the pairs packed along rows: anchors (src keypoints warped by the ground truth) and
    # positives (tgt keypoints), as the evaluation path packs them
    dev = pose.device
    a_off, p_off = ops.offsets(lens[:B], dev), ops.offsets(lens[B:], dev)
    with torch.no_grad():
        axyz_all = transform_points(torch.cat(list(pred['src_kp'])), a_off, pose)
        pxyz_all = torch.cat(list(pred['tgt_kp'])).float().contiguous()
    pair_idx = ops.to_device([b for b in range(B) for _ in range(lens[b])], torch.int64, dev)

    def infonce_all(W, A, P):
        # feature_loss.py:283-314 for every pair at once: the logits over all pairs' rows on
        # the differentiable f16x3 GEMMs (A W_sym P^T), each row's pair block read by
        # fgr_infonce_rows (the nearest positive within r_p is the target, every other
        # positive within r_n leaves the partition sum)
        # the positives padded with zero rows to a multiple of 8: the logits' extra columns
        # are read by no pair, and the backward GEMMs' contraction (K = positives) takes the
        # 16-B-aligned kernels
        if P.shape[0] % 8:
            P = F.pad(P, (0, 0, 0, (-P.shape[0]) % 8))
        logits = linear_t(linear_t(A, w_sym(W), cache=False), P, cache=False)
        return _InfoNCEFn.apply(logits, axyz_all, pxyz_all, a_off, p_off, pair_idx, cfg.r_p,
                                cfg.r_n)

    def circle_pair(a, pp, a_xyz, p_xyz):
        # CircleLossFull.get_circle_loss (feature_loss.py:191-230), Euclidean feature distances
        # by direct differences as the reference's cdist (_FeatCdistFn: the evaluation kernel's
        # first stage, its backward on the f16x3 GEMMs); non-positive / non-negative entries
        # contribute exp(0) = 1 as in the reference (its +-1e5 shift is multiplied by a zero
        # weight), the weights are detached as there
        fd = _FeatCdistFn.apply(a, pp)
        with torch.no_grad():
            cd = torch.cdist(a_xyz, p_xyz)
            pos, neg = cd < cfg.r_p, cd > cfg.r_n
            wp = torch.clamp_min(fd - 0.1, 0.0)
            wn = torch.clamp_min(1.4 - fd, 0.0)
        zero = torch.zeros_like(fd)
        tp = torch.where(pos, 10.0 * (fd - 0.1) * wp, zero)
        tn = torch.where(neg, 10.0 * (1.4 - fd) * wn, zero)
        row = F.softplus(torch.logsumexp(tp, 1) + torch.logsumexp(tn, 1)) / 10.0
        col = F.softplus(torch.logsumexp(tp, 0) + torch.logsumexp(tn, 0)) / 10.0
        # masked means without boolean indexing (no host sync); row / col are finite
        rm, cm = (pos.any(1) & neg.any(1)).float(), (pos.any(0) & neg.any(0)).float()
        return ((row * rm).sum() / rm.sum() + (col * cm).sum() / cm.sum()) / 2

    losses = {}
    pk = getattr(pred, 'packed', None)          # the packed outputs of RegTR's training forward
    if pk is not None:
        logits = pk['logits']
    else:
        logits = torch.cat(list(pred['src_overlap']) + list(pred['tgt_overlap']), dim=-2)
    for i in cfg.overlap_loss_on:
        losses[f'overlap_{i}'] = F.binary_cross_entropy_with_logits(logits[i, :, 0], ov)
    if ftype == 'circle':
        a_xyz = torch.split(axyz_all, lens[:B])
        for i in cfg.feature_loss_on:
            losses[f'feature_{i}'] = torch.stack([
                circle_pair(pred['src_feat'][b][i], pred['tgt_feat'][b][i], a_xyz[b], pred['tgt_kp'][b])
                for b in range(B)]).mean()
        losses['feature_un'] = torch.stack([
            circle_pair(pred['src_feat_un'][b], pred['tgt_feat_un'][b], a_xyz[b], pred['tgt_kp'][b])
            for b in range(B)]).mean()
    elif pk is not None:
        ns = pk['n_src']
        for i in cfg.feature_loss_on:
            f = pk['feats'][i]
            losses[f'feature_{i}'] = infonce_all(model.feature_criterion.W, f[:ns], f[ns:])
        losses['feature_un'] = infonce_all(model.feature_criterion_un.W, pk['both'][:ns],
                                           pk['both'][ns:])
    else:
        for i in cfg.feature_loss_on:
            losses[f'feature_{i}'] = infonce_all(
                model.feature_criterion.W, torch.cat([pred['src_feat'][b][i] for b in range(B)]),
                torch.cat([pred['tgt_feat'][b][i] for b in range(B)]))
        losses['feature_un'] = infonce_all(
            model.feature_criterion_un.W, torch.cat(list(pred['src_feat_un'])),
            torch.cat(list(pred['tgt_feat_un'])))

    def corr_mae(gt, warped, w):
        err = ((warped if torch.is_tensor(warped) else torch.cat(list(warped))) - gt).abs().sum(1)
        return (w * err).sum() / torch.clamp_min(w.sum(), 1e-6)

    with torch.no_grad():                 # the targets: keypoints under the ground-truth pose
        gt_src = axyz_all
        gt_tgt = transform_points(pxyz_all, p_off, pose, inverse=True)
    for i in cfg.corr_loss_on:
        if pk is not None:
            ns = pk['n_src']
            ws, wt = pk['corr'][i, :ns], pk['corr'][i, ns:]
        else:
            ws, wt = [w[i] for w in pred['src_kp_warped']], [w[i] for w in pred['tgt_kp_warped']]
        losses[f'corr_{i}'] = corr_mae(gt_src, ws, src_w) + corr_mae(gt_tgt, wt, tgt_w)
    wd = weight_dict(cfg)
    losses['total'] = torch.sum(torch.stack([losses[k] * wd[k] for k in losses]))
    return losses
