"""CPU: the oracle (oracle/) is pinned against the reference's own outputs.

tests/golden/*.npz were produced by running the reference (its C++ preprocessing and
its Python model) in the build container -- see tests/golden/make_golden.py.
"""
import numpy as np
import pytest
import torch

import geom as og
import model_oracle as mo
from conftest import forward_fixture, golden, rel_err

CASES = ['modelnet', 'indoor', 'edge']


@pytest.mark.parametrize('case', CASES)
def test_oracle_grid_subsample_matches_reference(case):
    g = golden(f'geom_{case}')
    pts, lens = og.grid_subsample(g['points'], g['lengths'], float(g['dl']))
    assert lens.tolist() == g['sub_lengths'].tolist()
    o1 = o2 = 0
    for n in lens:
        a, b = pts[o1:o1 + n], g['sub_points'][o2:o2 + n]
        assert np.array_equal(a[np.lexsort(a.T[::-1])], b[np.lexsort(b.T[::-1])])
        o1 += n
        o2 += n


@pytest.mark.parametrize('case', CASES)
@pytest.mark.parametrize('which', ['conv', 'pool', 'up', 'conv1'])
def test_oracle_radius_matches_reference(case, which):
    g = golden(f'geom_{case}')
    P, PL, S, SL, r0 = g['points'], g['lengths'], g['sub_points'], g['sub_lengths'], float(g['r0'])
    q, ql, s, sl, r = {'conv': (P, PL, P, PL, r0), 'pool': (S, SL, P, PL, r0),
                       'up': (P, PL, S, SL, 2 * r0), 'conv1': (S, SL, S, SL, 2 * r0)}[which]
    ref = g[which].astype(np.int64)
    mine = og.radius_search(q, ql, s, sl, r, 0, og.DIST)      # uncapped, distance order
    assert mine.shape == ref.shape
    ns = len(s)
    # identical rows except for the order among exactly equal distances
    same = np.all(mine == ref, axis=1)
    for i in np.where(~same)[0]:
        v = ref[i][ref[i] < ns]
        assert np.array_equal(np.sort(mine[i]), np.sort(ref[i]))
        qv = q[i].astype(np.float32)
        dd = ((qv - s[v]).astype(np.float32) ** 2)
        d2 = ((dd[:, 0] + dd[:, 1]).astype(np.float32) + dd[:, 2]).astype(np.float32)
        assert np.all(np.diff(d2) >= 0)                       # reference sorted by distance
        mv = mine[i][mine[i] < ns]
        dm = ((qv - s[mv]).astype(np.float32) ** 2)
        d2m = ((dm[:, 0] + dm[:, 1]).astype(np.float32) + dm[:, 2]).astype(np.float32)
        assert np.array_equal(d2, d2m)                        # differs only inside ties
    # the mismatch rate is the tie rate: tiny except on the lattice / duplicate fixture
    if case != 'edge':
        assert same.mean() > 0.98


def test_oracle_radius_boundary():
    g = golden('geom_boundary')
    mine = og.radius_search(g['queries'], [1], g['supports'], [len(g['supports'])],
                            float(g['radius']), 0, og.DIST)
    assert np.array_equal(mine, g['nb'].astype(np.int64))


@pytest.mark.parametrize('name', ['forward_modelnet_small', 'forward_3dmatch_small',
                                  'forward_modelnet_decoder', 'forward_modelnet_postnorm'])
def test_oracle_forward_matches_reference(name):
    cfg, sd, src, tgt, meta, d = forward_fixture(name)
    out = mo.forward(cfg, sd, src, tgt, meta=meta)
    B = len(src)
    for k in ('src_feat_un', 'tgt_feat_un', 'src_feat', 'tgt_feat', 'src_kp_warped',
              'tgt_kp_warped', 'src_overlap', 'tgt_overlap'):
        for b in range(B):
            assert rel_err(out[k][b], d[f'out.{k}.{b}']) < 2e-5, (k, b)
    assert np.abs(out['pose'].numpy() - d['out.pose']).max() < 2e-5


@pytest.mark.parametrize('name', ['forward_modelnet_small', 'forward_3dmatch_small'])
def test_oracle_preprocess_stages_match_reference(name):
    """Every pyramid stage on identical inputs (the reference's own level-l points, in the
    reference's order): level l+1 barycentres bit-exact as a set, neighbour / pool /
    upsample tables bit-exact up to the order among exactly equal distances.

    End to end the reference's level-1 voxel order (std::unordered_map iteration) differs
    from ours (ascending key), and a barycentre sums its members in input order, so
    levels >= 2 agree to float rounding only -- see test_oracle_preprocess_end_to_end."""
    cfg, sd, src, tgt, meta, d = forward_fixture(name)
    limits = cfg['neighborhood_limits']
    r = cfg['first_subsampling_dl'] * cfg['conv_radius']
    n_lvl = len(meta['points'])
    for l in range(n_lvl):
        P, L = meta['points'][l].numpy(), meta['stack_lengths'][l].numpy()
        nb = og.radius_search(P, L, P, L, r, limits[l], og.DIST)
        _assert_same_up_to_ties(nb, meta['neighbors'][l].numpy(), P, P)
        if l + 1 < n_lvl:
            S, SL = meta['points'][l + 1].numpy(), meta['stack_lengths'][l + 1].numpy()
            sub, sl = og.grid_subsample(P, L, 2 * r / cfg['conv_radius'])
            assert sl.tolist() == SL.tolist()
            o1 = 0
            for n in sl:
                a, b = sub[o1:o1 + n], S[o1:o1 + n]
                assert np.array_equal(a[np.lexsort(a.T[::-1])], b[np.lexsort(b.T[::-1])])
                o1 += n
            pool = og.radius_search(S, SL, P, L, r, limits[l], og.DIST)
            _assert_same_up_to_ties(pool, meta['pools'][l].numpy(), S, P)
            up = og.radius_search(P, L, S, SL, 2 * r, limits[l], og.DIST)
            _assert_same_up_to_ties(up, meta['upsamples'][l].numpy(), P, S)
        r *= 2


def _assert_same_up_to_ties(mine, ref, q, s):
    assert mine.shape == ref.shape
    ns = len(s)
    for i in np.where(~np.all(mine == ref, axis=1))[0]:
        assert np.array_equal(np.sort(mine[i]), np.sort(ref[i])), i
        v = mine[i][mine[i] < ns]
        w = ref[i][ref[i] < ns]
        dv = ((q[i] - s[v]).astype(np.float32) ** 2)
        dw = ((q[i] - s[w]).astype(np.float32) ** 2)
        f = lambda x: ((x[:, 0] + x[:, 1]).astype(np.float32) + x[:, 2]).astype(np.float32)
        assert np.array_equal(f(dv), f(dw)), i


@pytest.mark.parametrize('name', ['forward_modelnet_small', 'forward_3dmatch_small'])
def test_oracle_preprocess_end_to_end(name):
    """Own pyramid from the raw clouds: level 0/1 bit-exact (as sets), deeper levels within
    float rounding of the reference's points, same lengths everywhere."""
    from scipy.spatial import cKDTree
    cfg, sd, src, tgt, meta, d = forward_fixture(name)
    m = mo.preprocess(cfg, list(src) + list(tgt), mode=og.DIST)
    assert np.array_equal(m['neighbors'][0].numpy(), meta['neighbors'][0].numpy())
    for l in range(len(meta['points'])):
        assert m['stack_lengths'][l].tolist() == meta['stack_lengths'][l].tolist()
        a, b = m['points'][l].numpy(), meta['points'][l].numpy()
        dist, _ = cKDTree(b).query(a)
        assert dist.max() <= (0.0 if l <= 1 else 1e-6)


def test_oracle_procrustes_matches_reference():
    g = golden('procrustes')
    for case in ('regular', 'reflection', 'allzero', 'threshold'):
        a, b, w = (torch.from_numpy(g[f'{case}_{k}']) for k in 'abw')
        assert np.abs(mo.weighted_procrustes(a, b, w).numpy() - g[f'{case}_fast']).max() < 1e-5
        assert np.abs(mo.weighted_procrustes(a, b, w, None).numpy() - g[f'{case}_full']).max() < 1e-5


def test_oracle_pos_embed_matches_reference():
    g = golden('pos_embed')
    for dm in (64, 256, 512):
        assert rel_err(mo.sine_pos_embed(torch.from_numpy(g['xyz']), dm), g[f'pe{dm}']) < 1e-6


def test_oracle_kpconv_and_instnorm_match_reference():
    g = golden('kpconv_block')
    T = torch.from_numpy
    out = mo.kpconv(T(g['q']), T(g['s']), T(g['idx'].astype(np.int64)), T(g['x']), T(g['W']),
                    T(g['kp']), float(g['extent']))
    assert rel_err(out, g['out']) < 1e-6
    assert torch.equal(mo.max_pool(T(g['x']), T(g['pools'].astype(np.int64))), T(g['maxpool']))
    n = golden('instnorm')
    assert rel_err(mo.instance_norm(T(n['x']), T(n['lengths'].astype(np.int64))), n['out']) < 1e-6


def test_circle_loss_oracle_matches_reference():
    """The oracle's CircleLossFull (feature_loss_type: circle) vs the reference's own
    compute_loss with that option on the same forward outputs and loss inputs
    (tests/golden/loss_circle_modelnet_small.npz)."""
    import loss_oracle as lo
    from conftest import loss_fixture, golden
    cfg, pred, batch, _, _, _, W, W_un = loss_fixture()
    cfg = type(cfg)(cfg)
    cfg['feature_loss_type'] = 'circle'
    g = golden('loss_circle_modelnet_small')
    ref = {k[5:]: float(g[k]) for k in g.files}
    losses, _ = lo.compute_loss(cfg, None, None, pred, batch)
    assert set(losses) == set(ref)
    for k, v in ref.items():
        assert abs(float(losses[k]) - v) <= 1e-5 * max(1.0, abs(v)), (k, float(losses[k]), v)


def test_loss_oracle_matches_reference():
    """oracle/loss_oracle.py vs the reference's own compute_loss / _compute_metrics on its
    own forward outputs (tests/golden/loss_modelnet_small.npz)."""
    import loss_oracle as lo
    from conftest import loss_fixture
    cfg, pred, batch, ref_losses, ref_metrics, ref_pyr, W, W_un = loss_fixture()
    losses, pyr = lo.compute_loss(cfg, W, W_un, pred, batch)
    assert set(losses) == set(ref_losses)
    for k, v in ref_losses.items():
        assert abs(float(losses[k]) - v) <= 1e-5 * max(1.0, abs(v)), (k, float(losses[k]), v)
    for p, lvl in enumerate(pyr):
        np.testing.assert_allclose(lvl.numpy(), ref_pyr[f'pyr_{p}'], rtol=1e-6, atol=1e-7)
    rot, trans = lo.pose_errors(pred['pose'], batch['pose'])
    np.testing.assert_allclose(rot.numpy(), ref_metrics['rot_err_deg'], atol=1e-3)
    np.testing.assert_allclose(trans.numpy(), ref_metrics['trans_err'], rtol=1e-5, atol=1e-6)


def test_train_oracle_matches_reference():
    """The oracle's training step (model_oracle.forward_train: Res2Net BatchNorm on batch
    statistics; loss_oracle.compute_loss; torch autograd) vs the reference's own train()
    forward + compute_loss + backward (tests/golden/train_modelnet_small.npz): losses, the
    gradient norm and sum of every parameter, full gradients of one parameter of every kind."""
    from conftest import oracle_train_grads, train_fixture
    cfg, sd, src, tgt, meta, batch, W, W_un, ref = train_fixture()
    losses, grads = oracle_train_grads(cfg, sd, src, tgt, meta, batch, W, W_un)
    for k in ref.files:
        if k.startswith('loss.'):
            v = float(ref[k])
            assert abs(float(losses[k[5:]]) - v) <= 1e-5 * max(1.0, abs(v)), (k, float(losses[k[5:]]), v)
    norms = [k[6:] for k in ref.files if k.startswith('gnorm.')]
    assert set(norms) == set(grads), set(norms) ^ set(grads)
    for k in norms:
        g = grads[k].double()
        n_ref = float(ref['gnorm.' + k])
        assert abs(float(g.norm()) - n_ref) <= 1e-4 * n_ref + 1e-12, (k, float(g.norm()), n_ref)
    for k in ref.files:
        if k.startswith('grad.'):
            assert rel_err(grads[k[5:]], ref[k]) < 1e-4, (k, rel_err(grads[k[5:]], ref[k]))


# fp32 floor of the reference's isotropic rotation error: acos of a value within a few fp32
# roundings of 1 (0.5 (trace - 1) with trace a 9-product fp32 sum) -- sqrt(2 * 8 * 2^-24) rad
ISO_ROT_FLOOR_DEG = float(np.degrees(np.sqrt(16 * 2.0 ** -24)))


def check_modelnet_metrics(got, ref_m, rel=1e-4):
    """compute_metrics outputs against the reference's (benchmark_modelnet.py:33-82): every
    value within `rel` relative (of the array's max) -- err_r_deg also within the fp32 floor
    of the reference's own acos near zero error."""
    for k, v in ref_m.items():
        g = np.asarray(got[k], np.float64)
        v = np.asarray(v, np.float64)
        assert g.shape == v.shape, k
        tol = rel * max(float(np.abs(v).max()), 1e-30) + (ISO_ROT_FLOOR_DEG if k == 'err_r_deg' else 0.0)
        assert float(np.abs(g - v).max()) <= tol, (k, g, v)


def test_metrics_oracle_matches_reference():
    """oracle/metrics_oracle.py against the reference's own benchmark_modelnet.compute_metrics
    and summarize_metrics (tests/golden/modelnet_metrics.npz)."""
    import metrics_oracle as mt
    g = golden('modelnet_metrics')
    m = mt.compute_metrics(g['points_src'], g['points_ref'], g['points_raw'], g['transform_gt'],
                           g['pred_transforms'])
    ref_m = {k[2:]: g[k] for k in g.files if k.startswith('m_')}
    check_modelnet_metrics(m, ref_m, rel=1e-5)
    s = mt.summarize_metrics({k[2:]: g[k] for k in g.files if k.startswith('m_')})
    for k in s:
        assert np.allclose(s[k], g['s_' + k], rtol=1e-6, atol=0), k
