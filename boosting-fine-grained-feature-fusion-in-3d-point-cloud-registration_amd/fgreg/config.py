"""Configuration: the reference's flat conf-YAML dictionary.

``load_config`` flattens a two-level YAML exactly like the reference's
utils/misc.py:10-29, and ``Cfg`` gives the attribute access the reference gets from
EasyDict (train.py:64). ``MODELNET`` / ``THREEDMATCH`` restate the model-relevant
keys of conf/modelnet.yaml and conf/3dmatch.yaml, so tests and the benchmark need
no file from the reference.
"""
import copy

import yaml


class Cfg(dict):
    """dict with attribute access (EasyDict subset used by the model)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def get(self, k, default=None):
        return dict.get(self, k, default)


def load_config(path):
    """Two-level YAML -> flat dict (utils/misc.py:10-29)."""
    with open(path, 'r') as f:
        raw = yaml.safe_load(f)
    cfg = Cfg()
    for _, section in raw.items():
        for k, v in section.items():
            cfg[k] = v
    return cfg


_COMMON = dict(
    aggregation_mode='sum', fixed_kernel_points='center', in_feats_dim=1, in_points_dim=3,
    deform_radius=5.0, KP_extent=2.0, KP_influence='linear', use_batch_norm=True,
    batch_norm_momentum=0.02, modulated=False, num_kernel_points=15,
    model='finegrained_regtr.RegTR', attention_type='dot_prod', nhead=8, dropout=0.0,
    pre_norm=True, transformer_act='relu', num_encoder_layers=6,
    transformer_encoder_has_pos_emb=True, sa_val_has_pos_emb=True, ca_val_has_pos_emb=True,
    pos_emb_type='sine', corr_decoder_has_pos_emb=True, direct_regress_coor=True,
    wt_overlap=1.0, overlap_loss_pyr=3, overlap_loss_on=[5], wt_feature=0.1, wt_feature_un=0.0,
    feature_loss_on=[5], feature_loss_type='infonce', wt_corr=1.0, corr_loss_on=[5],
    reg_success_thresh_rot=10, reg_success_thresh_trans=0.1,
)

# conf/modelnet.yaml:35-105
MODELNET = Cfg(_COMMON, dataset='modelnet', num_layers=2, neighborhood_limits=[50, 50],
               first_subsampling_dl=0.03, first_feats_dim=512, conv_radius=2.75,
               overlap_radius=0.04,
               architecture=['simple', 'resnetb', 'resnetb', 'resnetb_strided', 'resnetb',
                             'resnetb'],
               d_embed=256, d_feedforward=1024, r_p=0.12, r_n=0.24)

# conf/3dmatch.yaml:26-100
THREEDMATCH = Cfg(_COMMON, dataset='3dmatch', num_layers=4, neighborhood_limits=[40, 40, 40, 40],
                  first_subsampling_dl=0.025, first_feats_dim=128, conv_radius=2.5,
                  overlap_radius=0.0375,
                  architecture=['simple', 'resnetb', 'resnetb_strided', 'resnetb', 'resnetb',
                                'resnetb_strided', 'resnetb', 'resnetb', 'resnetb_strided',
                                'resnetb', 'resnetb'],
                  d_embed=512, d_feedforward=1024, r_p=0.2, r_n=0.4)


def get(name, **overrides):
    # 3DLoMatch is the 3DMatch model on the low-overlap benchmark pairs (same conf/3dmatch.yaml)
    base = {'modelnet': MODELNET, '3dmatch': THREEDMATCH, '3dlomatch': THREEDMATCH}[name]
    cfg = Cfg(copy.deepcopy(dict(base)))
    cfg.update(overrides)
    return cfg
