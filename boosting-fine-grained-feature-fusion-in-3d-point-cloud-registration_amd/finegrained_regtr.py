"""Drop-in replacement for the reference's models/finegrained_regtr.py.

Copy (or symlink) this file over models/finegrained_regtr.py of the reference checkout
and put this package directory on PYTHONPATH. `get_model(
'finegrained_regtr.RegTR')` (models/__init__.py:24-30) then returns this class, and
train.py / test.py run unchanged:

* the forward runs on the MI355X kernels of libfgreg.so (fgreg.RegTR.forward) with the
  reference's module / state_dict layout, so its checkpoints load as they are;
* the hooks (test_step, validation_step, metrics, 3DMatch logs) are the reference's own
  GenericRegModel, and the loss modules are the reference's (models/losses);
* compute_loss / compute_overlaps / _compute_metrics (finegrained_regtr.py:252-309,
  finegrained_kpconv.py:545-571, generic_reg_model.py:203-215) run on libfgreg too
  (fgreg/loss.py), without MinkowskiEngine or PyTorch3D;
* train.py: in train() mode the forward is the differentiable training forward
  (fgreg/training.py, Res2Net BatchNorm on batch statistics, backward kernels in libfgreg) and
  compute_loss uses the reference's loss modules on it, so training_step -> backward ->
  clip_grad_norm_ -> optimizer.step (trainer.py:110-125) run unchanged.
"""
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

import fgreg  # noqa: E402
import fgreg.loss  # noqa: E402,F401
from fgreg.regtr import CorrespondenceDecoder, CorrespondenceRegressor  # noqa: E402,F401

# reference-side pieces that the forward does not replace (they exist in the reference tree)
from generic_reg_model import GenericRegModel  # noqa: E402
from losses.corr_loss import CorrCriterion  # noqa: E402
from losses.feature_loss import CircleLossFull, InfoNCELossFull  # noqa: E402


def compute_overlaps(batch):
    """Ground-truth overlap pyramid (finegrained_kpconv.py:545-571) on fgr_overlap_pool."""
    return fgreg.loss.compute_overlaps(batch)


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
    _prepare = fgreg.RegTR._prepare
    _forward = fgreg.RegTR._forward
    _core = fgreg.RegTR._core
    _segments = fgreg.RegTR._segments

    def _apply(self, fn, *args, **kwargs):
        fgreg.regtr._GRAPHS.pop(self, None)   # captured graphs point at the old weights
        return super()._apply(fn, *args, **kwargs)

    def compute_loss(self, pred, batch):
        """finegrained_regtr.py:252-309. Evaluation (test_step / validation_step, no autograd):
        on libfgreg (fgreg/loss.py): overlap BCE, InfoNCE (this module's feature_criterion W),
        CorrCriterion, same keys and weights. Training (train.py: autograd on, outputs of the
        train() forward): the reference's own loss modules on the differentiable outputs, so
        losses['total'].backward() reaches every parameter through fgreg's backward kernels."""
        if torch.is_grad_enabled() and pred['src_feat'][0].requires_grad:
            return self._compute_loss_autograd(pred, batch)
        return fgreg.loss.compute_loss(self, pred, batch)

    def _compute_loss_autograd(self, pred, batch):
        cfg = self.cfg
        meta = batch['kpconv_meta']
        pose_gt = batch['pose'].float()
        p = len(meta['stack_lengths']) - 1
        batch['overlap_pyr'] = compute_overlaps(batch)             # targets: no gradient
        ov = batch['overlap_pyr'][f'pyr_{p}']
        lens = [int(n) for n in meta['stack_lengths'][p].tolist()]
        B = len(lens) // 2
        ov_split = torch.split(ov, lens)
        src_ov, tgt_ov = list(ov_split[:B]), list(ov_split[B:])
        losses = {}
        all_pred = torch.cat(list(pred['src_overlap']) + list(pred['tgt_overlap']), dim=-2)
        for i in cfg.overlap_loss_on:
            losses[f'overlap_{i}'] = self.overlap_criterion(all_pred[i, :, 0], ov)
        with torch.no_grad():                                      # se3_transform_list(pose, src_kp)
            src_kp = torch.cat(list(pred['src_kp']))
            a_xyz = fgreg.loss.transform_points(src_kp, fgreg.ops.offsets(lens[:B], src_kp.device),
                                                pose_gt)
            a_xyz = list(torch.split(a_xyz, lens[:B]))
            rt = pose_gt[:, :, :3].transpose(1, 2)
            pose_inv = torch.cat([rt, -(rt @ pose_gt[:, :, 3:])], 2)   # se3_inv
        for i in cfg.feature_loss_on:
            losses[f'feature_{i}'] = self.feature_criterion(
                [s[i] for s in pred['src_feat']], [t[i] for t in pred['tgt_feat']], a_xyz,
                list(pred['tgt_kp']))
        losses['feature_un'] = self.feature_criterion_un(
            list(pred['src_feat_un']), list(pred['tgt_feat_un']), a_xyz, list(pred['tgt_kp']))
        for i in cfg.corr_loss_on:
            losses[f'corr_{i}'] = (
                self.corr_criterion(list(pred['src_kp']), [w[i] for w in pred['src_kp_warped']],
                                    pose_gt, overlap_weights=src_ov)
                + self.corr_criterion(list(pred['tgt_kp']), [w[i] for w in pred['tgt_kp_warped']],
                                      pose_inv, overlap_weights=tgt_ov))
        losses['total'] = torch.sum(torch.stack([losses[k] * self.weight_dict[k] for k in losses]))
        return losses

    def _compute_metrics(self, pred, batch):
        """generic_reg_model.py:203-215 (se3_compare of every pose output) on fgr_se3_compare."""
        with torch.no_grad():
            return fgreg.loss.compute_metrics(pred, batch)
