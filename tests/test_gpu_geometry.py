"""GPU parity of the KPConv pyramid geometry (grid subsampling, radius search).

Integer outputs: bit-exact. Against the reference (tests/golden/geom_*.npz, produced by
the reference's own C++): grid barycentres bit-exact as sets per cloud (the reference
emits voxels in unordered_map order); ball_query rows = the reference's uncapped rows
re-sorted by index and truncated to K; nanoflann rows bit-exact after canonicalising
exact-distance ties by index (the reference's tie order is its kd-tree visit order).
Against the oracle (oracle/geom_oracle.c): bit-exact in every mode and order.
"""
import numpy as np
import pytest
import torch

import geom as og
from conftest import golden

pytestmark = pytest.mark.gpu

CASES = ['modelnet', 'indoor', 'edge']


def _d2(q, s):
    dx = (q[:, None, 0] - s[None, :, 0]).astype(np.float32)
    dy = (q[:, None, 1] - s[None, :, 1]).astype(np.float32)
    dz = (q[:, None, 2] - s[None, :, 2]).astype(np.float32)
    return ((dx * dx).astype(np.float32) + (dy * dy).astype(np.float32)).astype(np.float32) + \
        (dz * dz).astype(np.float32)


def _lens_off(lens, dev):
    import fgreg.ops as ops
    lens = [int(v) for v in lens]
    return lens, ops.offsets(lens, dev)


def _set_rows_equal(a_pts, a_lens, b_pts, b_lens):
    oa = ob = 0
    for na, nb in zip(a_lens, b_lens):
        a = a_pts[oa:oa + na]
        b = b_pts[ob:ob + nb]
        if not np.array_equal(a[np.lexsort(a.T[::-1])], b[np.lexsort(b.T[::-1])]):
            return False
        oa += na
        ob += nb
    return True


@pytest.mark.parametrize('case', CASES)
def test_grid_subsample_vs_reference_and_oracle(gpu, case):
    import fgreg.ops as ops
    g = golden(f'geom_{case}')
    pts = torch.from_numpy(g['points']).to(gpu)
    lens, off = _lens_off(g['lengths'], gpu)
    sub, sub_lens, keys = ops.grid_subsample(pts, off, lens, float(g['dl']), return_keys=True)
    sub = sub.cpu().numpy()
    # reference: same voxel counts, bit-identical barycentres as sets
    assert sub_lens == [int(v) for v in g['sub_lengths']]
    assert _set_rows_equal(sub, sub_lens, g['sub_points'], g['sub_lengths'])
    # oracle: identical order (ascending voxel key per cloud) and keys
    o_pts, o_lens, o_keys = og.grid_subsample(g['points'], g['lengths'], float(g['dl']),
                                              return_keys=True)
    assert np.array_equal(sub, o_pts)
    assert np.array_equal(keys.cpu().numpy(), o_keys)


def _canonical_dist_rows(table, q, s, ns_total):
    """Sort each row's valid entries by (d2, index) -- canonical nanoflann order."""
    out = table.copy()
    for i in range(table.shape[0]):
        row = table[i]
        valid = row[row < ns_total]
        if len(valid) < 2:
            continue
        d2 = _d2(q[i:i + 1], s[valid])[0]
        order = np.lexsort((valid, d2))
        out[i, :len(valid)] = valid[order]
    return out


@pytest.mark.parametrize('case', CASES)
@pytest.mark.parametrize('which', ['conv', 'pool', 'up', 'conv1'])
def test_radius_search_vs_reference(gpu, case, which):
    import fgreg.ops as ops
    g = golden(f'geom_{case}')
    P, PL = g['points'], g['lengths']
    S, SL = g['sub_points'], g['sub_lengths']
    r0 = float(g['r0'])
    q, ql, s, sl, r = {'conv': (P, PL, P, PL, r0), 'pool': (S, SL, P, PL, r0),
                       'up': (P, PL, S, SL, 2 * r0), 'conv1': (S, SL, S, SL, 2 * r0)}[which]
    ref = g[which].astype(np.int64)                     # uncapped, distance-sorted
    ns = len(s)
    qd, sd = torch.from_numpy(q).to(gpu), torch.from_numpy(s).to(gpu)
    qlens, qoff = _lens_off(ql, gpu)
    slens, soff = _lens_off(sl, gpu)
    K = int(g['limit'])

    # ball_query semantics: first K by index <- reference rows sorted by index
    mine = ops.radius_search(qd, qoff, qlens, sd, soff, slens, r, K, ops.NB_INDEX).cpu().numpy()
    want = np.full((len(q), K), ns, np.int64)
    for i in range(len(q)):
        v = np.sort(ref[i][ref[i] < ns])[:K]
        want[i, :len(v)] = v
    assert np.array_equal(mine, want)

    # nanoflann semantics: K nearest, width min(max_count, K)
    mine = ops.radius_search(qd, qoff, qlens, sd, soff, slens, r, K, ops.NB_DIST).cpu().numpy()
    # (ties canonicalised on the UNCAPPED rows, then truncated: equal distances that
    # straddle the K boundary are resolved by index, as the oracle documents)
    canon = _canonical_dist_rows(ref, q, s, ns)[:, :min(ref.shape[1], K)]
    assert mine.shape == canon.shape
    assert np.array_equal(mine, canon)
    # and bit-exact with the oracle in both modes
    for mode in (og.INDEX, og.DIST):
        o = og.radius_search(q, ql, s, sl, r, K, mode)
        m = ops.radius_search(qd, qoff, qlens, sd, soff, slens, r, K, mode).cpu().numpy()
        assert np.array_equal(m, o)


def test_radius_boundary_strict(gpu):
    """Supports at exactly |d| = r are excluded (strict d2 < r2, nanoflann.hpp:249-250)."""
    import fgreg.ops as ops
    g = golden('geom_boundary')
    q = torch.from_numpy(g['queries']).to(gpu)
    s = torch.from_numpy(g['supports']).to(gpu)
    ql, qo = _lens_off([1], gpu)
    sl, so = _lens_off([len(g['supports'])], gpu)
    mine = ops.radius_search(q, qo, ql, s, so, sl, float(g['radius']), 8, ops.NB_DIST)
    assert np.array_equal(mine.cpu().numpy(), g['nb'].astype(np.int64))


def test_radius_counts_and_empty_clouds(gpu):
    """Uncapped counts match the oracle; an empty cloud and 1-point clouds are handled."""
    import fgreg.ops as ops
    rng = np.random.default_rng(0)
    clouds = [rng.uniform(-1, 1, (n, 3)).astype(np.float32) for n in (300, 0, 1, 77)]
    P = np.concatenate(clouds)
    L = [len(c) for c in clouds]
    pd = torch.from_numpy(P).to(gpu)
    lens, off = _lens_off(L, gpu)
    counts, mx = ops.radius_count(pd, off, lens, pd, off, 0.3)
    oc, omx = og.radius_counts(P, L, P, L, 0.3)
    assert np.array_equal(counts.cpu().numpy().astype(np.int64), oc) and mx == omx
    for mode in (og.INDEX, og.DIST):
        m = ops.radius_search(pd, off, lens, pd, off, lens, 0.3, 24, mode).cpu().numpy()
        assert np.array_equal(m, og.radius_search(P, L, P, L, 0.3, 24, mode))
    sub, sl = ops.grid_subsample(pd, off, lens, 0.2)
    o_pts, o_lens = og.grid_subsample(P, L, 0.2)
    assert sl == o_lens.tolist() and np.array_equal(sub.cpu().numpy(), o_pts)


def test_geometry_at_3dmatch_scale(gpu):
    """Full 3DMatch-size level 0 (2 x 20k points, r = 0.0625, K = 40): properties on all
    rows (every kept index lies in the query's cloud, within r, ascending, no duplicates,
    shadow-padded) and exact oracle agreement on a subset of query rows."""
    import fgreg.ops as ops
    from fgreg.synthetic import indoor_like_pair
    src, tgt, _ = indoor_like_pair(3)
    P = np.concatenate([src, tgt])
    L = [len(src), len(tgt)]
    pd = torch.from_numpy(P).to(gpu)
    lens, off = _lens_off(L, gpu)
    r, K = 0.025 * 2.5, 40
    nb = ops.radius_search(pd, off, lens, pd, off, lens, r, K, ops.NB_INDEX).cpu().numpy()
    ns = len(P)
    rows = np.random.default_rng(1).choice(len(P), 400, replace=False)
    for i in rows:
        v = nb[i][nb[i] < ns]
        c = 0 if i < L[0] else 1
        lo, hi = (0, L[0]) if c == 0 else (L[0], ns)
        assert np.all((v >= lo) & (v < hi))
        assert np.all(np.diff(v) > 0)
        assert np.all(_d2(P[i:i + 1], P[v])[0] < np.float32(r) * np.float32(r))
        assert np.all(nb[i][len(v):] == ns)
    # exact agreement with the oracle on the selected rows (oracle run on those queries)
    sel = np.sort(rows)
    for c in range(2):
        lo, hi = (0, L[0]) if c == 0 else (L[0], ns)
        qi = sel[(sel >= lo) & (sel < hi)]
        o = og.radius_search(P[qi], [len(qi)], P[lo:hi], [hi - lo], r, K, og.INDEX)
        o = np.where(o < hi - lo, o + lo, ns)
        assert np.array_equal(nb[qi], o)
    sub, sl = ops.grid_subsample(pd, off, lens, 2 * r / 2.5)
    o_pts, o_lens = og.grid_subsample(P, L, 2 * r / 2.5)
    assert sl == o_lens.tolist() and np.array_equal(sub.cpu().numpy(), o_pts)


# ---- counting-sort paths (csrc/grid.hip) -----------------------------------------------------
def _grid_cases():
    """(name, points, lengths, radius): the golden inputs, a 3DMatch-size pair, a cloud with
    600 coincident points (600 hits per query: the LDS rank list overflows -> bisection path)
    and clouds of 0 / 1 points."""
    from fgreg.synthetic import indoor_like_pair
    out = []
    for case in CASES:
        g = golden(f'geom_{case}')
        out.append((case, g['points'], [int(v) for v in g['lengths']], float(g['r0'])))
    src, tgt, _ = indoor_like_pair(5)
    out.append(('3dmatch', np.concatenate([src, tgt]), [len(src), len(tgt)], 0.0625))
    rng = np.random.default_rng(2)
    dup = np.concatenate([np.full((600, 3), 0.25, np.float32),
                          rng.uniform(-1, 1, (900, 3)).astype(np.float32)])
    dup = dup[rng.permutation(len(dup))]
    one = rng.uniform(-1, 1, (1, 3)).astype(np.float32)
    out.append(('dup', np.concatenate([dup, one]), [len(dup), 0, 1], 0.2))
    return out


@pytest.mark.parametrize('mode', ['index', 'dist'])
def test_radius_grid_matches_bruteforce_and_oracle(gpu, mode):
    """Every row of the cell-grid search equals the brute-force scan (and the oracle) in both
    semantics, for conv (q = s), shifted queries partly outside the supports' bounding box,
    widths 40 and 256, and the uncapped counts."""
    import fgreg.ops as ops
    m = ops.NB_INDEX if mode == 'index' else ops.NB_DIST
    om = og.INDEX if mode == 'index' else og.DIST
    for name, P, L, r in _grid_cases():
        pd = torch.from_numpy(P).to(gpu)
        lens, off = _lens_off(L, gpu)
        grid = ops.RadiusGrid(pd, off, lens, r)
        Q = (P + np.float32(0.7 * r)).astype(np.float32)          # some queries leave the bbox
        qd = torch.from_numpy(Q).to(gpu)
        for q, qt in ((P, pd), (Q, qd)):
            for K in (40, 256):
                a = ops.radius_search(qt, off, lens, pd, off, lens, r, K, m, grid=grid)
                if a.shape[1] <= 64 or m == ops.NB_INDEX:   # brute-force DIST: width <= 64
                    b = ops.radius_search(qt, off, lens, pd, off, lens, r, K, m)
                    assert torch.equal(a, b), (name, K)
                if len(P) <= 5000:
                    assert np.array_equal(a.cpu().numpy(), og.radius_search(q, L, P, L, r, K, om))
            c1, m1 = ops.radius_count(qt, off, lens, pd, off, r, grid=grid)
            c2, m2 = ops.radius_count(qt, off, lens, pd, off, r)
            assert torch.equal(c1, c2) and m1 == m2, name


def test_grid_subsample_overflow_retry(gpu):
    """A key space past the histogram (tiny max_cells) is reported and the count redone with
    the needed capacity: the same voxels bit for bit (order, barycentres, keys) as the default
    capacity and as the oracle; max_cells < 0 (the removed radix path) is rejected."""
    import fgreg.ops as ops
    from fgreg._lib import FgrError
    for name, P, L, r in _grid_cases():
        pd = torch.from_numpy(P).to(gpu)
        lens, off = _lens_off(L, gpu)
        for dl in (0.4 * r, 0.8 * r):
            a = ops.grid_subsample(pd, off, lens, dl, return_keys=True)
            c = ops.grid_subsample(pd, off, lens, dl, return_keys=True, max_cells=16)
            assert c[1] == a[1] and torch.equal(c[0], a[0]) and torch.equal(c[2], a[2]), name
            o_pts, o_lens, o_keys = og.grid_subsample(P, L, dl, return_keys=True)
            assert a[1] == o_lens.tolist() and np.array_equal(a[0].cpu().numpy(), o_pts)
            assert np.array_equal(a[2].cpu().numpy(), o_keys)
    with pytest.raises(FgrError):
        ops.grid_subsample(pd, off, lens, 0.4 * r, max_cells=-1)


def test_grid_subsample_key_space_limit_raises(gpu):
    """Past 2^28 voxel cells (a 645-voxel cube per cloud) the dense path raises instead of
    allocating a larger histogram."""
    import fgreg.ops as ops
    from fgreg._lib import FgrError
    P = np.array([[0, 0, 0], [1000, 1000, 1000]], np.float32)
    pd = torch.from_numpy(P).to(gpu)
    lens, off = _lens_off([2], gpu)
    with pytest.raises(FgrError, match='key space'):
        ops.grid_subsample(pd, off, lens, 1.0)


@pytest.mark.parametrize('n', [0, 1, 2, 16, 64, 65, 300])
def test_lengths_to_offsets(gpu, n):
    """fgr_lengths_to_offsets (device lengths -> device row offsets, the per-level segment
    table of the preprocessing) equals the host prefix sum, across 64-entry chunk borders."""
    import fgreg.ops as ops
    rng = np.random.default_rng(n)
    lens = rng.integers(0, 5000, n).astype(np.int64)
    off = ops.lengths_to_offsets(torch.from_numpy(lens).to(gpu)).cpu().numpy()
    assert off.shape == (n + 1,)
    assert np.array_equal(off, np.concatenate([[0], np.cumsum(lens)]))
