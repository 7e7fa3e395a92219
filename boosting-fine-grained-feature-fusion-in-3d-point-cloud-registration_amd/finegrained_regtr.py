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
  (fgreg/loss.py), without MinkowskiEngine or PyTorch3D.
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
        """finegrained_regtr.py:252-309 on libfgreg (fgreg/loss.py): overlap BCE, InfoNCE
        (this module's feature_criterion W), CorrCriterion, same keys and weights."""
        return fgreg.loss.compute_loss(self, pred, batch)

    def _compute_metrics(self, pred, batch):
        """generic_reg_model.py:203-215 (se3_compare of every pose output) on fgr_se3_compare."""
        with torch.no_grad():
            return fgreg.loss.compute_metrics(pred, batch)
