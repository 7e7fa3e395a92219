"""CPU restatement of the reference's test-step tail -- TEST INFRASTRUCTURE ONLY.

Only tests/ may import this (it is the checker of fgreg/loss.py, never the thing shipped).
Pinned against the reference itself: tests/golden/loss_modelnet_small.npz holds the
reference's own compute_loss / _compute_metrics outputs (tests/golden/make_golden.py
make_loss), checked by tests/test_oracle.py::test_loss_oracle_matches_reference.

Restated (PyTorch CPU, fp32 unless noted):
* compute_overlaps      models/backbone_kpconv/finegrained_kpconv.py:545-571
* RegTR.compute_loss    models/finegrained_regtr.py:252-309
* InfoNCELossFull       models/losses/feature_loss.py:246-314
* CircleLossFull        models/losses/feature_loss.py:160-243 (feature_loss_type: circle,
                        finegrained_regtr.py:86-88; pinned by loss_circle_modelnet_small.npz)
* CorrCriterion('mae')  models/losses/corr_loss.py:8-38
* se3_compare           utils/se3_torch.py:117-129 (via generic_reg_model.py:203-215)
"""
import math

import torch
import torch.nn.functional as F


def rigid_apply(pose, xyz):
    """R x + t for pose (3, 4), xyz (N, 3)."""
    return xyz @ pose[:, :3].t() + pose[:, 3]


def rigid_inverse(pose):
    rt = pose[:, :3].t()
    return torch.cat([rt, -(rt @ pose[:, 3:4])], 1)


def overlap_pyramid(src_overlap, tgt_overlap, pools, stack_lengths):
    """Level 0 = the per-point flags of all clouds; level p = mean of level p-1 over the
    valid entries (index < #points of level p-1) of pools[p-1], clamped to [0, 1]."""
    levels = [torch.cat(list(src_overlap) + list(tgt_overlap)).float()]
    for p in range(1, len(stack_lengths)):
        n_prev = int(stack_lengths[p - 1].sum())
        idx = pools[p - 1]
        valid = idx < n_prev
        vals = levels[-1][torch.where(valid, idx, torch.zeros_like(idx))] * valid
        levels.append(torch.clamp(vals.sum(1) / valid.sum(1), 0.0, 1.0))
    return levels


def infonce_pair(W, a_feat, p_feat, a_xyz, p_xyz, r_p, r_n):
    """Loss of one pair: rows whose nearest positive is within r_p; the nearest positive
    is the target, every other positive within r_n is excluded from the partition sum."""
    ws = torch.triu(W) + torch.triu(W).t()
    logits = (a_feat @ ws) @ p_feat.t()
    dist = torch.cdist(a_xyz, p_xyz)
    d1, j1 = dist.min(dim=1)
    keep = d1 < r_p
    excl = dist < r_n
    excl[torch.arange(len(j1)), j1] = False
    logits = logits.masked_fill(excl, -math.inf)
    per_row = torch.logsumexp(logits, dim=1) - logits[torch.arange(len(j1)), j1]
    return per_row[keep].sum() / keep.sum()


def circle_pair(a_feat, p_feat, a_xyz, p_xyz, r_p, r_n, log_scale=10.0, pos_margin=0.1,
                neg_margin=1.4):
    """CircleLossFull of one pair with Euclidean feature distances (sqrt(sum of squared
    differences + 1e-12)). Positives: point distance < r_p, negatives: > r_n. The reference masks
    by shifting the distances by -/+1e5 and then multiplies by a clamped weight that is 0 on the
    masked entries, so every non-positive (non-negative) entry adds exp(0) = 1 to the positive
    (negative) log-sum-exp. Rows / columns with at least one positive and one negative are
    averaged; the weights are constants for the gradient (detached)."""
    cd = torch.cdist(a_xyz, p_xyz)
    fd = torch.sqrt(((a_feat[:, None, :] - p_feat[None, :, :]) ** 2).sum(-1) + 1e-12)
    pos, neg = cd < r_p, cd > r_n
    wp = torch.clamp_min(fd - pos_margin, 0.0).detach()
    wn = torch.clamp_min(neg_margin - fd, 0.0).detach()
    zero = torch.zeros_like(fd)
    tp = torch.where(pos, log_scale * (fd - pos_margin) * wp, zero)
    tn = torch.where(neg, log_scale * (neg_margin - fd) * wn, zero)
    row = F.softplus(torch.logsumexp(tp, 1) + torch.logsumexp(tn, 1)) / log_scale
    col = F.softplus(torch.logsumexp(tp, 0) + torch.logsumexp(tn, 0)) / log_scale
    row_sel = pos.any(1) & neg.any(1)
    col_sel = pos.any(0) & neg.any(0)
    return (row[row_sel].mean() + col[col_sel].mean()) / 2


def corr_mae(kp, kp_warped, poses, weights):
    """sum_i w_i |warped_i - T(kp_i)|_1 / max(sum w, 1e-6) over all pairs' rows."""
    gt = torch.cat([rigid_apply(poses[b], kp[b]) for b in range(len(kp))])
    err = (torch.cat(list(kp_warped)) - gt).abs().sum(1)
    w = torch.cat(list(weights))
    return (w * err).sum() / torch.clamp_min(w.sum(), 1e-6)


def pose_errors(pred, gt):
    """pred (L, B, 3, 4), gt (B, 3, 4) -> rotation error (deg) and translation error."""
    L, B = pred.shape[:2]
    rot = torch.empty(L, B)
    trans = torch.empty(L, B)
    for l in range(L):
        for b in range(B):
            ig = rigid_inverse(gt[b])
            R = pred[l, b, :, :3] @ ig[:, :3]
            t = pred[l, b, :, :3] @ ig[:, 3] + pred[l, b, :, 3]
            c = torch.clamp(0.5 * (R.trace() - 1), -1.0, 1.0)
            rot[l, b] = torch.acos(c) * 180.0 / math.pi
            trans[l, b] = t.norm()
    return rot, trans


def compute_loss(cfg, W, W_un, pred, batch):
    """Losses dict with the reference's keys and weights, from per-cloud lists."""
    meta = batch['kpconv_meta']
    pose = batch['pose']
    p = len(meta['stack_lengths']) - 1
    pyr = overlap_pyramid(batch['src_overlap'], batch['tgt_overlap'], meta['pools'],
                          meta['stack_lengths'])
    ov = pyr[p]
    lens = [int(v) for v in meta['stack_lengths'][p]]
    B = len(lens) // 2
    n_src = sum(lens[:B])
    src_w = torch.split(ov[:n_src], lens[:B])
    tgt_w = torch.split(ov[n_src:], lens[B:])
    losses = {}
    logits = torch.cat(list(pred['src_overlap']) + list(pred['tgt_overlap']), dim=-2)
    for i in cfg.overlap_loss_on:
        losses[f'overlap_{i}'] = F.binary_cross_entropy_with_logits(logits[i, :, 0], ov)
    a_xyz = [rigid_apply(pose[b], pred['src_kp'][b]) for b in range(B)]
    if cfg.get('feature_loss_type', 'infonce') == 'circle':
        feat = lambda Wm, a, pp, b: circle_pair(a, pp, a_xyz[b], pred['tgt_kp'][b], cfg.r_p,
                                                cfg.r_n)
    else:
        feat = lambda Wm, a, pp, b: infonce_pair(Wm, a, pp, a_xyz[b], pred['tgt_kp'][b],
                                                 cfg.r_p, cfg.r_n)
    for i in cfg.feature_loss_on:
        losses[f'feature_{i}'] = torch.stack([
            feat(W, pred['src_feat'][b][i], pred['tgt_feat'][b][i], b) for b in range(B)]).mean()
    losses['feature_un'] = torch.stack([
        feat(W_un, pred['src_feat_un'][b], pred['tgt_feat_un'][b], b) for b in range(B)]).mean()
    inv = torch.stack([rigid_inverse(pose[b]) for b in range(B)])
    for i in cfg.corr_loss_on:
        losses[f'corr_{i}'] = (
            corr_mae(pred['src_kp'], [w[i] for w in pred['src_kp_warped']], pose, src_w) +
            corr_mae(pred['tgt_kp'], [w[i] for w in pred['tgt_kp_warped']], inv, tgt_w))
    wd = {}
    for k in ['overlap', 'feature', 'corr']:
        for i in cfg.get(f'{k}_loss_on', [cfg.num_encoder_layers - 1]):
            wd[f'{k}_{i}'] = cfg.get(f'wt_{k}')
    wd['feature_un'] = cfg.wt_feature_un
    losses['total'] = torch.stack([losses[k] * wd[k] for k in losses]).sum()
    return losses, pyr
