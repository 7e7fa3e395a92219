"""Drop-in replacement for the reference's models/finegrained_regtr.py.

Copy (or symlink) this file over models/finegrained_regtr.py of the reference checkout
and put this package directory on PYTHONPATH. `get_model(
'finegrained_regtr.RegTR')` (models/__init__.py:24-30) then returns this class, and
train.py / test.py run unchanged:

* the forward runs on the MI355X kernels of libfgreg.so (fgreg.RegTR.forward) with the
  reference's module / state_dict layout, so its checkpoints load as they are;
* the hooks (test_step, validation_step, metrics, 3DMatch logs) are the reference's own
  GenericRegModel, and the loss modules are the reference's (models/losses);
* compute_loss / compute_overlaps restate finegrained_regtr.py:252-309 and
  finegrained_kpconv.py:545-571 without importing MinkowskiEngine or PyTorch3D, which
  this path no longer needs.
"""
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

import fgreg  # noqa: E402
from fgreg.regtr import CorrespondenceDecoder, CorrespondenceRegressor  # noqa: E402,F401

# reference-side pieces that the forward does not replace (they exist in the reference tree)
from generic_reg_model import GenericRegModel  # noqa: E402
from losses.corr_loss import CorrCriterion  # noqa: E402
from losses.feature_loss import CircleLossFull, InfoNCELossFull  # noqa: E402
from utils.se3_torch import se3_inv, se3_transform_list  # noqa: E402
from utils.seq_manipulation import split_src_tgt  # noqa: E402


def compute_overlaps(batch):
    """Ground-truth overlap pyramid (finegrained_kpconv.py:545-571)."""
    overlaps = batch['src_overlap'] + batch['tgt_overlap']
    meta = batch['kpconv_meta']
    pyr = {'pyr_0': torch.cat(overlaps, dim=0).type(torch.float)}
    invalid = [s.sum() for s in meta['stack_lengths']]
    for p in range(1, len(meta['points'])):
        idx = meta['pools'][p - 1].clone()
        valid = idx < invalid[p - 1]
        idx[~valid] = 0
        g = pyr[f'pyr_{p - 1}'][idx] * valid
        g = torch.sum(g, dim=1) / torch.sum(valid, dim=1)
        pyr[f'pyr_{p}'] = torch.clamp(g, min=0, max=1)
    return pyr


class RegTR(GenericRegModel):
    """models/finegrained_regtr.py:23 with the forward on libfgreg (fgreg.RegTR)."""

    def __init__(self, cfg, *args, **kwargs):
        super().__init__(cfg, *args, **kwargs)
        fgreg.RegTR.build_modules(self, cfg, kwargs.get('neighbor_mode', 'ball_query'))
        # losses exactly as the reference sets them up (finegrained_regtr.py:82-98)
        self.overlap_criterion = nn.BCEWithLogitsLoss()
        if self.cfg.feature_loss_type == 'infonce':
            self.feature_criterion = InfoNCELossFull(cfg.d_embed, r_p=cfg.r_p, r_n=cfg.r_n)
            self.feature_criterion_un = InfoNCELossFull(cfg.d_embed, r_p=cfg.r_p, r_n=cfg.r_n)
        elif self.cfg.feature_loss_type == 'circle':
            self.feature_criterion = CircleLossFull(dist_type='euclidean', r_p=cfg.r_p, r_n=cfg.r_n)
            self.feature_criterion_un = self.feature_criterion
        else:
            raise NotImplementedError
        self.corr_criterion = CorrCriterion(metric='mae')
        self.weight_dict = {}
        for k in ['overlap', 'feature', 'corr']:
            for i in cfg.get(f'{k}_loss_on', [cfg.num_encoder_layers - 1]):
                self.weight_dict[f'{k}_{i}'] = cfg.get(f'wt_{k}')
        self.weight_dict['feature_un'] = cfg.wt_feature_un

    forward = fgreg.RegTR.forward

    def compute_loss(self, pred, batch):
        """finegrained_regtr.py:252-309."""
        losses = {}
        meta = batch['kpconv_meta']
        pose_gt = batch['pose']
        p = len(meta['stack_lengths']) - 1
        batch['overlap_pyr'] = compute_overlaps(batch)
        src_ov_p, tgt_ov_p = split_src_tgt(batch['overlap_pyr'][f'pyr_{p}'], meta['stack_lengths'][p])
        all_ov_pred = torch.cat(pred['src_overlap'] + pred['tgt_overlap'], dim=-2)
        all_ov_gt = batch['overlap_pyr'][f'pyr_{p}']
        for i in self.cfg.overlap_loss_on:
            losses[f'overlap_{i}'] = self.overlap_criterion(all_ov_pred[i, :, 0], all_ov_gt)
        for i in self.cfg.feature_loss_on:
            losses[f'feature_{i}'] = self.feature_criterion(
                [s[i] for s in pred['src_feat']], [t[i] for t in pred['tgt_feat']],
                se3_transform_list(pose_gt, pred['src_kp']), pred['tgt_kp'])
        losses['feature_un'] = self.feature_criterion_un(
            pred['src_feat_un'], pred['tgt_feat_un'],
            se3_transform_list(pose_gt, pred['src_kp']), pred['tgt_kp'])
        for i in self.cfg.corr_loss_on:
            s_l = self.corr_criterion(pred['src_kp'], [w[i] for w in pred['src_kp_warped']],
                                      batch['pose'], overlap_weights=src_ov_p)
            t_l = self.corr_criterion(pred['tgt_kp'], [w[i] for w in pred['tgt_kp_warped']],
                                      torch.stack([se3_inv(q) for q in batch['pose']]),
                                      overlap_weights=tgt_ov_p)
            losses[f'corr_{i}'] = s_l + t_l
        losses['total'] = torch.sum(torch.stack([(losses[k] * self.weight_dict[k]) for k in losses]))
        return losses
