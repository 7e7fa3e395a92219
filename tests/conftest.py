"""Shared test setup: markers, import paths, golden-fixture loaders.

`-m "not gpu"` tests run on any CPU host; `-m gpu` tests need an MI355X and call the
HIP path through the C ABI (libfgreg.so). The oracle (oracle/) is only ever used
here as the checker.
"""
import ast
import os
import sys

import numpy as np
import pytest
import torch

sys.dont_write_bytecode = True     # never leave bytecode next to /root/reference's sources
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, 'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd')
GOLDEN = os.path.join(REPO, 'tests', 'golden')
for p in (PKG, os.path.join(REPO, 'oracle'), GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an AMD MI355X GPU (HIP path through libfgreg.so)')


def golden(name):
    return np.load(os.path.join(GOLDEN, name + '.npz'), allow_pickle=False)


def forward_fixture(name):
    """-> (cfg, state_dict, src list, tgt list, meta dict of CPU tensors, fixture npz)."""
    import fgreg.config as fc
    d = golden(name)
    over = ast.literal_eval(str(d['cfg_overrides']))
    base = 'modelnet' if 'modelnet' in name else '3dmatch'
    cfg = fc.get(base, **over)
    sd = {k[3:]: torch.from_numpy(d[k]) for k in d.files if k.startswith('sd.')}
    if 'sd_keys' in d.files:      # weights rebuilt from (key, shape, seed): golden/named_weights.py
        from named_weights import named_state_dict
        raw = d['sd_keys'].item()
        keys = ast.literal_eval(raw.decode() if isinstance(raw, bytes) else str(raw))
        vals = named_state_dict(keys, int(d['sd_seed']), float(d['bias']),
                                {k: v.numpy() for k, v in sd.items()})
        sd = {k: torch.from_numpy(np.array(v)) for k, v in vals.items()}
    n_lvl = sum(1 for k in d.files if k.startswith('meta.points.'))
    meta = {}
    for key in ('points', 'neighbors', 'pools', 'upsamples', 'stack_lengths'):
        meta[key] = []
        for l in range(n_lvl):
            a = d[f'meta.{key}.{l}']
            meta[key].append(torch.from_numpy(a.astype(np.int64) if a.dtype in (np.int16, np.int32) else a))
    B = sum(1 for k in d.files if k.startswith('in.src_xyz.'))
    src = [d[f'in.src_xyz.{b}'] for b in range(B)]
    tgt = [d[f'in.tgt_xyz.{b}'] for b in range(B)]
    return cfg, sd, src, tgt, meta, d


def rel_err(a, b):
    """Normwise relative error max|a - b| / max|b| (the fp32 parity metric, <= 1e-4)."""
    a = a.detach().double().cpu() if torch.is_tensor(a) else torch.as_tensor(np.asarray(a, np.float64))
    b = b.detach().double().cpu() if torch.is_tensor(b) else torch.as_tensor(np.asarray(b, np.float64))
    assert a.shape == b.shape, (a.shape, b.shape)
    if b.numel() == 0:
        return 0.0
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def elem_err(a, b, floor=1e-2):
    """Elementwise relative error with an absolute floor:
    max_i |a_i - b_i| / max(|b_i|, floor * max|b|). Unlike rel_err it does not let a
    small-magnitude entry hide behind the tensor's largest one; the floor keeps entries
    that are ~0 by cancellation (where any fp32 path has only absolute accuracy) from
    dividing by ~0."""
    a = a.detach().double().cpu() if torch.is_tensor(a) else torch.as_tensor(np.asarray(a, np.float64))
    b = b.detach().double().cpu() if torch.is_tensor(b) else torch.as_tensor(np.asarray(b, np.float64))
    assert a.shape == b.shape, (a.shape, b.shape)
    if b.numel() == 0:
        return 0.0
    den = torch.clamp(b.abs(), min=max(floor * float(b.abs().max()), 1e-30))
    return float(((a - b).abs() / den).max())


@pytest.fixture(scope='session')
def gpu():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    import fgreg
    fgreg.load()
    return torch.device('cuda:0')


OUT_KEYS = ['src_feat_un', 'tgt_feat_un', 'src_feat', 'tgt_feat', 'src_kp', 'tgt_kp',
            'src_kp_warped', 'tgt_kp_warped', 'src_overlap', 'tgt_overlap']


def loss_fixture(device='cpu'):
    """-> (cfg, pred, batch, losses, metrics, pyr, W, W_un): the reference's forward outputs
    (forward_modelnet_small) as per-cloud tensors, the loss inputs and the reference's own
    compute_loss / _compute_metrics results (loss_modelnet_small)."""
    cfg, _, src, tgt, meta, d = forward_fixture('forward_modelnet_small')
    g = golden('loss_modelnet_small')
    B = len(src)
    T = lambda a: torch.from_numpy(np.asarray(a)).to(device)
    pred = {k: [T(d[f'out.{k}.{b}']) for b in range(B)] for k in OUT_KEYS}
    pred['pose'] = T(d['out.pose'])
    batch = {'src_xyz': [T(s) for s in src], 'tgt_xyz': [T(t) for t in tgt],
             'kpconv_meta': {k: [t.to(device) for t in v] for k, v in meta.items()},
             'pose': T(g['pose']),
             'src_overlap': [T(g[f'src_overlap.{b}']) for b in range(B)],
             'tgt_overlap': [T(g[f'tgt_overlap.{b}']) for b in range(B)]}
    losses = {k[5:]: float(g[k]) for k in g.files if k.startswith('loss.')}
    metrics = {k[7:]: g[k] for k in g.files if k.startswith('metric.')}
    pyr = {k[12:]: g[k] for k in g.files if k.startswith('overlap_pyr.')}
    return cfg, pred, batch, losses, metrics, pyr, T(g['W']), T(g['W_un'])


def is_trainable(key):
    """state_dict entries that are nn.Parameters with requires_grad in the reference (kernel
    points are requires_grad=False, blocks:250-263; BatchNorm running statistics are buffers)."""
    return not any(t in key for t in ('running_', 'num_batches', 'kernel_points'))


def train_fixture():
    """-> (cfg, sd, src, tgt, meta, loss batch (CPU), W, W_un, reference npz) for the training-
    step fixture (tests/golden/train_modelnet_small.npz: the reference's train() forward +
    compute_loss + backward on the model / inputs of forward_modelnet_small)."""
    cfg, sd, src, tgt, meta, _ = forward_fixture('forward_modelnet_small')
    _, _, batch, _, _, _, W, W_un = loss_fixture()
    return cfg, sd, src, tgt, meta, batch, W, W_un, golden('train_modelnet_small')


def oracle_train_grads(cfg, sd, src, tgt, meta, batch, W, W_un, dtype=torch.float64):
    """The oracle's training step on CPU in ``dtype`` (fp64 by default: the checker of an fp32
    implementation): forward_train + loss_oracle.compute_loss + backward -> (losses, {param
    key: grad})."""
    import loss_oracle as lo
    import model_oracle as mo
    cv = lambda t: t.detach().cpu().to(dtype) if t.is_floating_point() else t.cpu()
    sd = {k: (cv(v).requires_grad_(True) if (v.is_floating_point() and is_trainable(k))
              else cv(v)) for k, v in sd.items()}
    meta = {k: [cv(t) for t in v] for k, v in meta.items()}
    b = dict(batch)
    b['pose'] = cv(batch['pose'])
    b['src_overlap'] = [cv(t) for t in batch['src_overlap']]
    b['tgt_overlap'] = [cv(t) for t in batch['tgt_overlap']]
    b['kpconv_meta'] = {k: [cv(t) for t in v] for k, v in batch['kpconv_meta'].items()}
    Wg, Wug = cv(W).requires_grad_(True), cv(W_un).requires_grad_(True)
    pred = mo.forward_train(cfg, sd, [np.asarray(s) for s in src], tgt, meta=meta)
    losses, _ = lo.compute_loss(cfg, Wg, Wug, pred, b)
    losses['total'].backward()
    grads = {k: v.grad for k, v in sd.items() if v.requires_grad and v.grad is not None}
    grads['feature_criterion.W'] = Wg.grad
    grads['feature_criterion_un.W'] = Wug.grad
    return losses, grads
