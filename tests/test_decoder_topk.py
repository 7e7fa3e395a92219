"""CorrespondenceDecoder with num_neighbors > 0 (finegrained_regtr.py:312-408, :353-357).

The reference's masking indexes the query dimension with the top-k key indices, so a query
row keeps its plain softmax iff its index is in the union of every top-k index of its
direction, all other rows are NaN, and an index >= Q raises IndexError. The fixture
tests/golden/decoder_topk.npz is the reference module's own output
(tests/golden/make_golden.py make_decoder_topk). Checked here: the oracle's restatement
(CPU) and the HIP path (fgr_corr_attention + fgr_corr_topk_mask, gpu): NaN rows identical,
finite rows within 1e-4 normwise relative (the q / k projections are fp32-accurate f16x3
GEMMs on the GPU). Padded batches (pad_*): the reference's padded query rows feed the union;
the HIP path carries them as query-only phantom rows (transformer.Segments(phantoms=...)).
"""
import math

import numpy as np
import pytest
import torch

import model_oracle as mo
from conftest import golden, rel_err

FIX = 'decoder_topk'


def _case(d, c):
    B = sum(1 for k in d.files if k.startswith(f'{c}.src_xyz.'))
    sd = {k[len(c) + 3:]: torch.from_numpy(d[k]) for k in d.files if k.startswith(f'{c}.w.')}
    sx = [torch.from_numpy(d[f'{c}.src_xyz.{b}']) for b in range(B)]
    tx = [torch.from_numpy(d[f'{c}.tgt_xyz.{b}']) for b in range(B)]
    sf = torch.from_numpy(d[f'{c}.src_feats'])
    tf = torch.from_numpy(d[f'{c}.tgt_feats'])
    return B, sd, sx, tx, sf, tf, int(d[f'{c}.k']), d[f'{c}.raised'].item().decode()


def _check(mine, ref):
    mine = np.asarray(mine, np.float64)
    ref = np.asarray(ref, np.float64)
    assert mine.shape == ref.shape
    nan_m, nan_r = np.isnan(mine), np.isnan(ref)
    assert np.array_equal(nan_m, nan_r), (nan_m.any(-1).sum(), nan_r.any(-1).sum())
    if (~nan_r).any():
        assert rel_err(torch.from_numpy(np.where(nan_m, 0, mine)),
                       torch.from_numpy(np.where(nan_r, 0, ref))) < 1e-4


def test_fixture_has_nan_rows_and_a_raise():
    d = golden(FIX)
    cases = list(d['cases'])
    assert d['eq_k1.raised'].item() == b'' and d['ne_k8.raised'].item() == b'IndexError'
    assert np.isnan(d['eq_k1.out.src_corr.0']).any()


CASES = ['eq_k4', 'eq_k24', 'eq_k1', 'b2_k6', 'ne_k8', 'pad_k1', 'pad_k2', 'pad_ix']


@pytest.mark.parametrize('case', CASES)
def test_oracle_topk_matches_reference(case):
    d = golden(FIX)
    B, sd, sx, tx, sf, tf, k, raised = _case(d, case)
    pe = lambda x: mo.sine_pos_embed(x, sf.shape[-1])          # noqa: E731
    spe, _ = mo._pad([pe(x) for x in sx])
    tpe, _ = mo._pad([pe(x) for x in tx])
    sxp, smask = mo._pad(sx)
    txp, tmask = mo._pad(tx)
    p = ''

    def run():
        sc = mo.corr_simple_attention(sd, p, sf + spe, tf + tpe, txp, tmask, k)
        tc = mo.corr_simple_attention(sd, p, tf + tpe, sf + spe, sxp, smask, k)
        return sc, tc
    if raised:
        with pytest.raises(IndexError):
            run()
        return
    sc, tc = run()
    for b in range(B):
        n_s, n_t = len(sx[b]), len(tx[b])
        _check(sc[:, :n_s, b].numpy(), d[f'{case}.out.src_corr.{b}'])
        _check(tc[:, :n_t, b].numpy(), d[f'{case}.out.tgt_corr.{b}'])


def test_padded_rows_change_the_union():
    """pad_k1 discriminates: with the padded query rows left out of the union (what a packed
    layout without phantom rows would compute) the NaN rows differ from the reference's."""
    d = golden(FIX)
    B, sd, sx, tx, sf, tf, k, _ = _case(d, 'pad_k1')
    pe = lambda x: mo.sine_pos_embed(x, sf.shape[-1])          # noqa: E731
    spe, _ = mo._pad([pe(x) for x in sx])
    tpe, _ = mo._pad([pe(x) for x in tx])
    sxp, smask = mo._pad(sx)
    txp, tmask = mo._pad(tx)
    q = sf + spe
    q_real = q.clone()
    for b in range(B):       # padded rows of src cloud b: copy a real row's top-k onto them
        q_real[:, len(sx[b]):, b] = q[:, :1, b]
    sc = mo.corr_simple_attention(sd, '', q_real, tf + tpe, txp, tmask, k)
    differs = any(not np.array_equal(np.isnan(sc[:, :len(sx[b]), b].numpy()),
                                     np.isnan(d[f'pad_k1.out.src_corr.{b}'])) for b in range(B))
    assert differs


@pytest.mark.gpu
@pytest.mark.parametrize('case', CASES)
def test_gpu_topk_matches_reference(gpu, case):
    import fgreg
    from fgreg.regtr import CorrespondenceDecoder
    from fgreg.transformer import PositionEmbeddingCoordsSine, Segments
    d = golden(FIX)
    B, sd, sx, tx, sf, tf, k, raised = _case(d, case)
    L, D = sf.shape[0], sf.shape[-1]
    pe = PositionEmbeddingCoordsSine(3, D)
    dec = CorrespondenceDecoder(D, True, pe, num_neighbors=k)
    dec.load_state_dict(sd)
    dec = dec.to(gpu).eval()
    lens = [len(x) for x in sx] + [len(x) for x in tx]
    Qs, Qt = sf.shape[1], tf.shape[1]
    # the clouds' rows, then each padded cloud's padded rows as query-only phantom rows
    phantoms = [Qs - n for n in lens[:B]] + [Qt - n for n in lens[B:]]
    feats = torch.cat([sf[:, :len(sx[b]), b] for b in range(B)]
                      + [tf[:, :len(tx[b]), b] for b in range(B)]
                      + [sf[:, len(sx[b]):, b] for b in range(B)]
                      + [tf[:, len(tx[b]):, b] for b in range(B)], 1).contiguous().to(gpu)
    xyz = torch.cat(sx + tx, 0).contiguous().to(gpu)
    seg = Segments(lens, gpu, n_layers=L, phantoms=phantoms)
    with torch.no_grad():
        pos = pe(xyz)
        if raised:
            with pytest.raises(IndexError):
                dec.forward_packed(feats, xyz, pos, seg)
            return
        corr, logits = dec.forward_packed(feats, xyz, pos, seg)
    corr = corr.cpu().numpy()
    logits = logits.cpu().numpy()
    off = np.concatenate([[0], np.cumsum(lens)])
    for b in range(B):
        for side, c in (('src', b), ('tgt', B + b)):
            _check(corr[:, off[c]:off[c + 1]], d[f'{case}.out.{side}_corr.{b}'])
            assert rel_err(torch.from_numpy(logits[:, off[c]:off[c + 1]]),
                           d[f'{case}.out.{side}_overlap.{b}']) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize('k', [1, 3])
def test_gpu_forward_topk_padded_batch_vs_oracle(gpu, k):
    """A whole RegTR forward with the CorrespondenceDecoder's top-k masking on a padded batch
    (the decoder fixture's two ModelNet pairs, whose coarse clouds differ in length) against
    the oracle, which runs the reference's padded transformer and decoder: NaN rows
    identical, finite rows within 1e-4; an IndexError of the oracle is raised too."""
    import fgreg
    from conftest import forward_fixture
    cfg, sd, src, tgt, _, _ = forward_fixture('forward_modelnet_decoder')
    model = fgreg.RegTR(cfg)
    model.load_state_dict(sd, strict=False)
    model.correspondence_decoder.num_neighbors = k
    model = model.to(gpu).eval()
    batch = {'src_xyz': [torch.from_numpy(c).to(gpu) for c in src],
             'tgt_xyz': [torch.from_numpy(c).to(gpu) for c in tgt]}
    try:
        ref = mo.forward(cfg, sd, src, tgt, mode=mo.geom.INDEX, num_neighbors=k)
    except IndexError:
        with pytest.raises(IndexError):
            model(batch)
        return
    out = model(batch)
    lens = batch['kpconv_meta']['stack_lengths'][-1].tolist()
    B = len(src)
    assert len(set(lens[:B])) > 1 or len(set(lens[B:])) > 1, 'the batch must be padded'
    n_nan = 0
    for b in range(B):
        for side in ('src', 'tgt'):
            _check(out[f'{side}_kp_warped'][b].cpu().numpy(), ref[f'{side}_kp_warped'][b].numpy())
            n_nan += int(np.isnan(ref[f'{side}_kp_warped'][b].numpy()).any(-1).sum())
            assert rel_err(out[f'{side}_overlap'][b], ref[f'{side}_overlap'][b]) < 1e-4
            assert rel_err(out[f'{side}_feat'][b], ref[f'{side}_feat'][b]) < 1e-4
    print(f'\nk={k}: lengths {lens}, {n_nan} NaN rows in the reference restatement')
