"""GPU: the drop-in models/finegrained_regtr.py (package file finegrained_regtr.py) replays
GenericRegModel.test_step's call sequence (generic_reg_model.py:128-132):

    pred = self.forward(batch); losses = self.compute_loss(pred, batch);
    metrics = self._compute_metrics(pred, batch)

on the reference's own forward fixture (its kpconv_meta, state_dict and loss inputs) and is
checked against the reference's compute_loss / _compute_metrics outputs
(tests/golden/loss_modelnet_small.npz). Also: train.py's training step (train() forward,
compute_loss, backward, clip_grad_norm_) against the reference's own training step
(tests/golden/train_modelnet_small.npz).

The reference tree does not exist on the GPU box, so the three reference modules the drop-in
imports (generic_reg_model, losses.corr_loss, losses.feature_loss) are given stand-ins here:
the base class only carries cfg and the call sequence above, and the loss modules their
parameters (InfoNCELossFull.W, feature_loss.py:246-266) and, for the training step, the
oracle's restatement of their forward (oracle/loss_oracle.py, pinned to the reference).
"""
import importlib.util
import os
import sys
import types

import numpy as np
import pytest
import torch
import torch.nn as nn

from conftest import PKG, forward_fixture, loss_fixture

pytestmark = pytest.mark.gpu


class _GenericRegModel(nn.Module):
    def __init__(self, cfg, *args, **kwargs):
        super().__init__()
        self.cfg = cfg

    def test_step(self, batch, batch_idx):
        """generic_reg_model.py:128-132 (the dataset-specific logging after it is host code)."""
        pred = self.forward(batch)
        losses = self.compute_loss(pred, batch)
        metrics = self._compute_metrics(pred, batch)
        return pred, losses, metrics


class _InfoNCELossFull(nn.Module):
    """Stand-in with the reference's parameter (feature_loss.py:246-266) and, for the
    training-step replay, its forward as restated by the oracle (loss_oracle.infonce_pair)."""

    def __init__(self, d_embed, r_p, r_n):
        super().__init__()
        self.W = nn.Parameter(torch.zeros(d_embed, d_embed))
        self.r_p, self.r_n = r_p, r_n

    def forward(self, src_feat, tgt_feat, src_xyz, tgt_xyz):
        import loss_oracle as lo
        return torch.stack([lo.infonce_pair(self.W, a, p, ax, px, self.r_p, self.r_n)
                            for a, p, ax, px in zip(src_feat, tgt_feat, src_xyz, tgt_xyz)]).mean()


class _CorrCriterion(nn.Module):
    """Stand-in for CorrCriterion('mae') (corr_loss.py:8-38) via loss_oracle.corr_mae."""

    def forward(self, kp_before, kp_warped_pred, pose_gt, overlap_weights=None):
        import loss_oracle as lo
        return lo.corr_mae(kp_before, kp_warped_pred, pose_gt, overlap_weights)


def _load_dropin():
    stubs = {'generic_reg_model': types.ModuleType('generic_reg_model'),
             'losses': types.ModuleType('losses'),
             'losses.corr_loss': types.ModuleType('losses.corr_loss'),
             'losses.feature_loss': types.ModuleType('losses.feature_loss')}
    stubs['generic_reg_model'].GenericRegModel = _GenericRegModel
    stubs['losses.corr_loss'].CorrCriterion = lambda metric='mae': _CorrCriterion()
    stubs['losses.feature_loss'].InfoNCELossFull = _InfoNCELossFull
    stubs['losses.feature_loss'].CircleLossFull = None
    saved = {k: sys.modules.get(k) for k in stubs}
    sys.modules.update(stubs)
    try:
        spec = importlib.util.spec_from_file_location('fgreg_dropin_gpu',
                                                      os.path.join(PKG, 'finegrained_regtr.py'))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return mod


def test_dropin_test_step_replay(gpu):
    import fgreg
    mod = _load_dropin()
    cfg, sd, src, tgt, meta, d = forward_fixture('forward_modelnet_small')
    _, _, batch, ref_losses, ref_metrics, _, W, W_un = loss_fixture(gpu)
    model = mod.RegTR(cfg)
    sd = dict(sd)
    sd['feature_criterion.W'] = W.cpu()
    sd['feature_criterion_un.W'] = W_un.cpu()
    model.load_state_dict(sd, strict=True)
    model = model.to(gpu).eval()
    model.preprocessor = fgreg.FixedMetaPreprocessor(batch['kpconv_meta'])
    batch['kpconv_meta'] = {k: list(v) for k, v in batch['kpconv_meta'].items()}
    with torch.no_grad():
        pred, losses, metrics = model.test_step(batch, 0)
    assert list(losses) == list(ref_losses)
    for k, v in ref_losses.items():     # forward within 1e-4 -> losses within 1e-3
        assert abs(float(losses[k]) - v) <= 1e-3 * max(1.0, abs(v)), (k, float(losses[k]), v)
    np.testing.assert_allclose(np.cos(np.deg2rad(metrics['rot_err_deg'].cpu().numpy())),
                               np.cos(np.deg2rad(ref_metrics['rot_err_deg'])), atol=1e-5)
    np.testing.assert_allclose(metrics['trans_err'].cpu().numpy(), ref_metrics['trans_err'],
                               rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(pred['pose'].cpu().numpy(), d['out.pose'], atol=1e-4)


def test_dropin_training_step(gpu):
    """train.py's step through the drop-in (trainer.py:110-125): model.train(),
    training_step's forward + compute_loss (the reference's loss modules on the differentiable
    outputs), backward, clip_grad_norm_: losses equal the reference's own training step
    (tests/golden/train_modelnet_small.npz) and every trainable parameter gets a finite
    gradient whose norm matches the reference's within 1e-2 (tests/test_gpu_train.py)."""
    import fgreg
    from conftest import golden, is_trainable
    mod = _load_dropin()
    cfg, sd, src, tgt, meta, d = forward_fixture('forward_modelnet_small')
    _, _, batch, _, _, _, W, W_un = loss_fixture(gpu)
    ref = golden('train_modelnet_small')
    model = mod.RegTR(cfg)
    sd = dict(sd)
    sd['feature_criterion.W'] = W.cpu()
    sd['feature_criterion_un.W'] = W_un.cpu()
    model.load_state_dict(sd, strict=True)
    model = model.to(gpu).train()
    model.preprocessor = fgreg.FixedMetaPreprocessor(batch['kpconv_meta'])
    batch['kpconv_meta'] = {k: list(v) for k, v in batch['kpconv_meta'].items()}
    pred = model(batch)
    losses = model.compute_loss(pred, batch)
    losses['total'].backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=0.1)
    for k in ref.files:
        if k.startswith('loss.'):
            v = float(ref[k])
            assert abs(float(losses[k[5:]]) - v) <= 1e-4 * max(1.0, abs(v)), (k, float(losses[k[5:]]), v)
    names = {k[6:] for k in ref.files if k.startswith('gnorm.')}
    got = {k: p.grad for k, p in model.named_parameters() if p.grad is not None}
    assert names == {k for k in got if is_trainable(k)}
    total = float(np.sqrt(sum(float(ref['gnorm.' + k]) ** 2 for k in names)))
    scale = min(1.0, 0.1 / (total + 1e-6))             # clip_grad_norm_ on the reference's norms
    for k in names:
        assert torch.isfinite(got[k]).all(), k
        n_ref = float(ref['gnorm.' + k]) * scale
        assert abs(float(got[k].double().norm()) - n_ref) <= 1e-2 * n_ref + 1e-9, k
