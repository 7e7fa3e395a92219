"""RegTR (fine-grained fusion variant) on the MI355X kernels.

Mirrors models/finegrained_regtr.py: same constructor ``RegTR(cfg)``, same
submodule / state_dict names, same ``forward(batch) -> outputs`` keys and shapes
(:233-249), ``batch['kpconv_meta']`` filled as the reference does (:122). Inside,
the forward is re-laid out for the GPU:

* preprocessing on HIP kernels with one host sync per pyramid level (voxel counts);
* all 2B clouds kept packed end to end (no padding, no per-cloud Python loops);
* one launch per op for all clouds, self- and cross-attention included;
* pose for all (layer, pair) problems in one launch, straight from packed tensors.
The returned per-cloud lists are views into the packed tensors.
"""
import logging
import math
import os
import weakref
from collections import OrderedDict

import torch
import torch.nn as nn

from . import linear as lin
from . import ops
from .linear import linear
from .backbone import KPFEncoder, PreprocessorHIP, host_layout
from .transformer import (PositionEmbeddingCoordsSine, Segments, TransformerCrossEncoder,
                          TransformerCrossEncoderLayer)

_logger = logging.getLogger(__name__)

# compute mode of the correspondence head's GEMMs when the forward runs in bf16 (None: bf16
# like the rest); FGREG_BF16_HEAD=f16x3 keeps the pose-sensitive head fp32-accurate
HEAD_MODE = os.environ.get('FGREG_BF16_HEAD') or None
# the CorrespondenceRegressor head in two fused launches where supported (FGREG_FUSED_HEAD=0: one
# GEMM per Linear, for A/B)
FUSED_HEAD = os.environ.get('FGREG_FUSED_HEAD', '1') != '0'


class CorrespondenceRegressor(nn.Module):
    """finegrained_regtr.py:411-455 (direct_regress_coor: True, the shipped configs)."""

    def __init__(self, d_embed):
        super().__init__()
        self.coor_mlp = nn.Sequential(nn.Linear(d_embed, d_embed), nn.ReLU(),
                                      nn.Linear(d_embed, d_embed), nn.ReLU(),
                                      nn.Linear(d_embed, 3))
        self.conf_logits_decoder = nn.Linear(d_embed, 1)

    def _stacked(self):
        """[W0; Wc; 0] (d + 16, d) and [b0; bc; 0]: coor_mlp[0] and conf_logits_decoder as one
        product (fgr_corr_head_f16x3), rebuilt when a source tensor changes."""
        m = self.coor_mlp
        srcs = (m[0].weight, self.conf_logits_decoder.weight, m[0].bias,
                self.conf_logits_decoder.bias)
        key = tuple((t.data_ptr(), t._version) for t in srcs)
        st = getattr(self, '_stack_cache', None)
        if st is None or st[0] != key:
            d = m[0].weight.shape[1]
            with torch.no_grad():
                w = torch.zeros((d + 16, d), dtype=torch.float32, device=m[0].weight.device)
                w[:d] = m[0].weight
                w[d] = self.conf_logits_decoder.weight[0]
                b = torch.zeros((d + 16,), dtype=torch.float32, device=w.device)
                b[:d] = m[0].bias
                b[d] = self.conf_logits_decoder.bias[0]
            st = (key, w, b)
            object.__setattr__(self, '_stack_cache', st)     # not a parameter / buffer
            ops.note_state(w, b)
        return st[1], st[2]

    def forward_packed(self, feats):
        """feats (L, N, d) -> corr (L, N, 3), logits (L, N, 1). In the bf16 mode the head
        runs in ``HEAD_MODE`` (the pose reads its outputs directly; DESIGN.md "bf16 mode").
        f16x3 with d % 16 == 0, d <= 256 (ModelNet): two launches (fgr_corr_head_f16x3), else
        one GEMM per Linear."""
        L, N, d = feats.shape
        f = feats.reshape(L * N, d)
        m = self.coor_mlp
        mode = (HEAD_MODE or lin.MODE) if lin.MODE == 'bf16' else lin.MODE
        if FUSED_HEAD and mode == 'f16x3' and ops.corr_head_supported(L * N, d):
            w0c, b0c = self._stacked()
            corr, logits = ops.corr_head(f, lin.weight_image(w0c, mode='f16x3'), b0c,
                                         lin.weight_image(m[2].weight, mode='f16x3'), m[2].bias,
                                         m[4].weight, m[4].bias)
            return corr.view(L, N, 3), logits.view(L, N, 1)
        with lin.mode_scope(HEAD_MODE if lin.MODE == 'bf16' else None):
            h = linear(f, m[0].weight, m[0].bias, act=ops.ACT_RELU)
            h = linear(h, m[2].weight, m[2].bias, act=ops.ACT_RELU)
            corr = linear(h, m[4].weight, m[4].bias)
            logits = linear(f, self.conf_logits_decoder.weight, self.conf_logits_decoder.bias)
        return corr.view(L, N, 3), logits.view(L, N, 1)


class CorrespondenceDecoder(nn.Module):
    """finegrained_regtr.py:312-408 (direct_regress_coor: False): single-head attention
    whose values are the other cloud's coordinates. Parameter layout of the reference. The
    q / k projections run once over all L layers' rows (f16x3 GEMMs) and the attention of
    every (layer, cloud) segment is ONE fgr_corr_attention launch (values = the partner's 3
    coordinates, no padding to width d).

    num_neighbors > 0 reproduces the reference's masking as it executes (:353-357, see
    fgr_corr_topk_mask in include/fgreg.h): a query row keeps its plain softmax iff its index
    is in the union of all top-k key indices of its direction, else it is NaN; an index >= the
    padded query length raises IndexError like the reference's indexing. On padded batches the
    reference's padded query rows (its transformer's outputs at padded positions, queries of
    every attention and never keys) feed the union too: they are carried as query-only
    "phantom" rows after the clouds' rows (Segments(phantoms=...), RegTR._segments: one row per
    padded cloud, since all padded positions of a cloud compute the same row)."""

    def __init__(self, d_embed, use_pos_emb, pos_embed=None, num_neighbors=0):
        super().__init__()
        self.use_pos_emb = use_pos_emb
        self.pos_embed = pos_embed
        self.q_norm = nn.LayerNorm(d_embed)   # present in the reference, unused by its forward
        self.q_proj = nn.Linear(d_embed, d_embed)
        self.k_proj = nn.Linear(d_embed, d_embed)
        self.conf_logits_decoder = nn.Linear(d_embed, 1)
        self.num_neighbors = num_neighbors

    def forward_packed(self, feats, xyz, pos, seg: Segments):
        """feats (L, N + P, d): the clouds' rows, then seg's P phantom rows (whose positional
        embedding is the reference's zero padding); xyz / pos: the clouds' N rows."""
        L, N, d = feats.shape
        if self.use_pos_emb and pos.shape[0] < N:
            pos = torch.cat([pos, pos.new_zeros((N - pos.shape[0], d))])
        f = (feats + pos.unsqueeze(0) if self.use_pos_emb else feats).reshape(L * N, d)
        q = linear(f, self.q_proj.weight, self.q_proj.bias)
        k = linear(f, self.k_proj.weight, self.k_proj.bias)
        q_off, kv_seg, v_off = seg.layer_tables
        corr = ops.corr_attention(q, k, xyz, q_off, q_off, kv_seg, v_off, seg.max_len,
                                  1.0 / math.sqrt(d))        # q_proj(query) / sqrt(D) (:344)
        if self.num_neighbors > 0:
            self._topk_mask(corr, q, k, seg, d)
        logits = linear(feats.reshape(L * N, d), self.conf_logits_decoder.weight,
                        self.conf_logits_decoder.bias)
        return corr.view(L, N, 3), logits.view(L, N, 1)


    def _topk_mask(self, corr, q, k, seg: Segments, d):
        B = seg.B
        src_l, tgt_l = seg.lengths[:B], seg.lengths[B:]
        n_src, n_tgt = max(src_l), max(tgt_l)                # the padded Q / S of each direction
        if self.num_neighbors > min(n_src, n_tgt):
            raise RuntimeError('selected index k out of range')              # torch.topk
        if self.num_neighbors > min(src_l + tgt_l):
            # the top-k of a row would then rank -inf padded keys, whose order torch.topk
            # leaves unspecified
            raise NotImplementedError('num_neighbors > the shortest cloud of a padded batch')
        if (any(p > 0 for p in seg.phantoms[:B]) and len(set(src_l)) == 1) or \
                (any(p > 0 for p in seg.phantoms[B:]) and len(set(tgt_l)) == 1):
            raise ValueError('phantom rows for a direction without padding')
        for c in range(2 * B):
            if (len(set(src_l)) > 1 if c < B else len(set(tgt_l)) > 1) and \
                    seg.lengths[c] < (n_src if c < B else n_tgt) and seg.phantoms[c] == 0:
                raise ValueError(f'cloud {c} is padded in the reference but has no phantom row')
        q_off, kv_seg, _ = seg.layer_tables
        if seg.n_phantom == 0:
            flags = ops.corr_topk_mask(corr, q, k, q_off, q_off, kv_seg, 2 * B, seg.max_len,
                                       max(n_src, n_tgt), 1.0 / math.sqrt(d), self.num_neighbors)
        else:
            flags = self._topk_mask_phantoms(corr, q, k, seg, d, max(n_src, n_tgt))
        # src queries pick tgt key indices that index the src query dim, and vice versa
        for dir_, n_q, n_k in ((0, n_src, n_tgt), (1, n_tgt, n_src)):
            if n_k > n_q and bool(flags[dir_, n_q:n_k].any()):
                hi = int(flags[dir_, :n_k].nonzero().max())
                raise IndexError(f'index {hi} is out of bounds for dimension 2 with size {n_q}')

    def _topk_mask_phantoms(self, corr, q, k, seg: Segments, d, max_kv):
        """The mask with phantom rows: fgr_corr_topk_mask takes a segment's direction from its
        position in the layer ((s mod n) >= n / 2), so the rows are gathered per layer into
        [src clouds, src phantom groups, tgt clouds, tgt phantom groups] (empty groups for the
        clouds without padding), masked there, and scattered back."""
        B, n = seg.B, 2 * seg.B
        N = sum(seg.seg_lengths)
        L = q.shape[0] // N
        start = [0]
        for ln in seg.seg_lengths:
            start.append(start[-1] + ln)
        ph_start, j = {}, n
        for c in range(n):
            if seg.phantoms[c] > 0:
                ph_start[c] = start[j]
                j += 1
        rows, lens = [], []
        for l in range(L):
            for dir_ in (0, 1):
                for b in range(B):                                   # the clouds
                    c = dir_ * B + b
                    rows.append(torch.arange(start[c], start[c + 1]) + l * N)
                    lens.append(seg.lengths[c])
                for b in range(B):                                   # their phantom groups
                    c = dir_ * B + b
                    p = seg.phantoms[c]
                    rows.append(torch.arange(ph_start.get(c, 0), ph_start.get(c, 0) + p) + l * N)
                    lens.append(p)
        real = lambda c: c if c < B else 2 * B + (c - B)           # noqa: E731
        cloud = [b for b in range(B)] * 2 + [B + b for b in range(B)] * 2
        kv = [l * 4 * B + real((cloud[s] + B) % n) for l in range(L) for s in range(4 * B)]
        dev = q.device
        idx = torch.cat(rows).to(dev)
        off = ops.offsets(lens, dev)
        kv_seg = ops.to_device(kv, torch.int32, dev)
        cp = corr[idx].contiguous()
        flags = ops.corr_topk_mask(cp, q[idx].contiguous(), k[idx].contiguous(), off, off, kv_seg,
                                   4 * B, max(lens), max_kv, 1.0 / math.sqrt(d),
                                   self.num_neighbors)
        corr[idx] = cp
        return flags


class _LossParams(nn.Module):
    """Holds InfoNCELossFull's parameter W (models/losses/feature_loss.py:246-266) so that
    reference checkpoints load strictly; the loss itself is not part of the forward."""

    def __init__(self, d_embed):
        super().__init__()
        self.W = nn.Parameter(torch.zeros(d_embed, d_embed))
        nn.init.normal_(self.W, std=0.1)


class RegTR(nn.Module):
    """models/finegrained_regtr.py:23-250."""

    def __init__(self, cfg, *args, neighbor_mode='ball_query', **kwargs):
        super().__init__()
        self.build_modules(cfg, neighbor_mode)

    def build_modules(self, cfg, neighbor_mode='ball_query'):
        """Registers the submodules on ``self`` under the reference's names
        (finegrained_regtr.py:25-106). Usable on any nn.Module: the drop-in shim of
        INTEGRATION.md calls it on a GenericRegModel subclass."""
        self.cfg = cfg
        self.preprocessor = PreprocessorHIP(cfg, neighbor_mode=neighbor_mode)
        self.kpf_encoder = KPFEncoder(cfg, cfg.d_embed)
        self.feat_proj = nn.Linear(self.kpf_encoder.encoder_skip_dims[-1], cfg.d_embed, bias=True)
        if cfg.get('pos_emb_type', 'sine') != 'sine':
            raise NotImplementedError('pos_emb_type other than sine is not in the reference configs')
        self.pos_embed = PositionEmbeddingCoordsSine(3, cfg.d_embed,
                                                     scale=cfg.get('pos_emb_scaling', 1.0))
        layer = TransformerCrossEncoderLayer(
            cfg.d_embed, cfg.nhead, cfg.d_feedforward, cfg.dropout,
            activation=cfg.transformer_act, normalize_before=cfg.pre_norm,
            sa_val_has_pos_emb=cfg.sa_val_has_pos_emb, ca_val_has_pos_emb=cfg.ca_val_has_pos_emb,
            attention_type=cfg.attention_type)
        norm = nn.LayerNorm(cfg.d_embed) if cfg.pre_norm else None
        self.transformer_encoder = TransformerCrossEncoder(layer, cfg.num_encoder_layers, norm,
                                                           return_intermediate=True)
        if cfg.get('direct_regress_coor', False):
            self.correspondence_decoder = CorrespondenceRegressor(cfg.d_embed)
        else:
            self.correspondence_decoder = CorrespondenceDecoder(
                cfg.d_embed, cfg.corr_decoder_has_pos_emb, self.pos_embed)
        if cfg.get('feature_loss_type', 'infonce') == 'infonce':
            self.feature_criterion = _LossParams(cfg.d_embed)
            self.feature_criterion_un = _LossParams(cfg.d_embed)
        self.pose_threshold = 0.85   # hard-coded in fast_compute_rigid_transform (se3_torch.py:226)

    def forward(self, batch):
        """eval(): the inference forward (no autograd, HIP-graph replay of the core).
        train(): the training forward (fgreg/training.py): Res2Net BatchNorm on batch
        statistics and, with autograd enabled, differentiable end to end on libfgreg's forward
        and backward kernels (train.py's loss.backward())."""
        dev = batch['src_xyz'][0].device
        if self.training:
            from .training import check_trainable
            check_trainable(self)
            if dev.type != 'cuda':      # the ops raise FgrError on host tensors (no CPU path)
                return self._forward(batch, train=True)
            with torch.cuda.device(dev):
                return self._forward(batch, train=True)
        if dev.type != 'cuda':
            with torch.no_grad():
                return self._forward(batch)
        with torch.no_grad(), torch.cuda.device(dev):
            return self._forward(batch)

    def _prepare(self, batch):
        """The preprocessing (kpconv_meta, with every level's host lengths and device
        offsets): the eager part of the forward, with its host syncs."""
        meta = self.preprocessor(list(batch['src_xyz']) + list(batch['tgt_xyz']))
        for lvl in range(len(meta['points'])):       # device offsets of every level, eagerly
            host_layout(meta, lvl)
        return meta

    def _forward(self, batch, meta=None, train=False, slot=0):
        """meta: a kpconv_meta already prepared for this batch (fgreg.pipeline), else built
        here. train: the training-mode core (fgreg/training.py) instead of the inference one.
        slot: which of the shape signature's graph instances replays the core (fgreg.pipeline
        runs consecutive cores on different streams: each stream replays its own instance, so
        concurrent replays never share scratch buffers or static inputs)."""
        B = len(batch['src_xyz'])
        if meta is None:
            with torch.no_grad():
                meta = self._prepare(batch)
        batch['kpconv_meta'] = meta
        n_lvl = len(meta['points'])
        slens_c, _ = host_layout(meta, n_lvl - 1)
        xyz_c = meta['points'][-1]
        if train:
            from .training import core_train
            res = core_train(self, meta, self._segments(slens_c, xyz_c), B)
        else:
            core = (_graph_for(self, meta, slens_c, B, slot)
                    if GRAPHS and xyz_c.is_cuda and ops.TIMER is None else None)
            res = core.run(meta) if core is not None else self._core(
                meta, self._segments(slens_c, xyz_c), B)
        both, feats, corr, logits, pose = res

        offs = [0]
        for n in slens_c:
            offs.append(offs[-1] + n)
        rows = [(offs[c], offs[c + 1]) for c in range(2 * B)]
        outputs = {
            'src_feat_un': [both[b:e] for b, e in rows[:B]],
            'tgt_feat_un': [both[b:e] for b, e in rows[B:]],
            'src_feat': [feats[:, b:e] for b, e in rows[:B]],
            'tgt_feat': [feats[:, b:e] for b, e in rows[B:]],
            'src_kp': [xyz_c[b:e] for b, e in rows[:B]],
            'src_kp_warped': [corr[:, b:e] for b, e in rows[:B]],
            'tgt_kp': [xyz_c[b:e] for b, e in rows[B:]],
            'tgt_kp_warped': [corr[:, b:e] for b, e in rows[B:]],
            'src_overlap': [logits[:, b:e] for b, e in rows[:B]],
            'tgt_overlap': [logits[:, b:e] for b, e in rows[B:]],
            'pose': pose,
        }
        if train:
            # the packed tensors behind the per-cloud views (src clouds first), as an attribute
            # of the output dict (its keys stay the reference's): the training loss reads them
            # whole, so its backward sees one slice per tensor instead of a view per cloud
            # (fgreg.loss.compute_loss_train)
            outputs = _TrainOutputs(outputs)
            outputs.packed = {'both': both, 'feats': feats, 'corr': corr, 'logits': logits,
                              'n_src': offs[B]}
        return outputs

    def _segments(self, slens_c, xyz_c):
        dec = self.correspondence_decoder
        n_layers = 0 if isinstance(dec, CorrespondenceRegressor) else len(self.transformer_encoder.layers)
        phantoms = None
        if getattr(dec, 'num_neighbors', 0) > 0:
            # top-k masking on a padded batch: one query-only row per padded cloud
            B = len(slens_c) // 2
            mx = (max(slens_c[:B]), max(slens_c[B:]))
            phantoms = [int(n < mx[c >= B]) for c, n in enumerate(slens_c)]
        return Segments(slens_c, xyz_c.device, n_layers, phantoms=phantoms)

    def _core(self, meta, seg, B):
        """The post-preprocessing forward (finegrained_regtr.py:126-218): encoder, feat_proj,
        positional embedding, cross encoder, correspondence head, pose. Pure device work on
        the kpconv_meta tensors and their precomputed host layout -- no host sync, no host
        -> device copy -- so it can be captured in a HIP graph (_CoreGraph)."""
        pts0 = meta['points'][0]
        feats0 = torch.ones((pts0.shape[0], 1), dtype=torch.float32, device=pts0.device)
        feats_un, _ = self.kpf_encoder(feats0, meta)
        both = linear(feats_un, self.feat_proj.weight, self.feat_proj.bias)
        xyz_c = meta['points'][-1]
        pe = self.pos_embed(xyz_c)
        pos = pe if self.cfg.transformer_encoder_has_pos_emb else None
        if pos is None:
            pos = torch.zeros_like(both)
        if seg.n_phantom:
            # the reference's padded positions that feed the decoder's top-k union: input
            # features and positional embedding are its zero padding (finegrained_regtr.py:
            # 163-171)
            z = both.new_zeros((seg.n_phantom, both.shape[1]))
            feats = self.transformer_encoder.forward_packed(torch.cat([both, z]),
                                                            torch.cat([pos, z]), seg)
        else:
            feats = self.transformer_encoder.forward_packed(both, pos, seg)    # (L, N, d)
        if isinstance(self.correspondence_decoder, CorrespondenceRegressor):
            corr, logits = self.correspondence_decoder.forward_packed(feats)
        else:
            corr, logits = self.correspondence_decoder.forward_packed(feats, xyz_c, pe, seg)
        if seg.n_phantom:                  # drop the query-only phantom rows (_segments)
            feats, corr, logits = (t[:, :xyz_c.shape[0]].contiguous() for t in (feats, corr, logits))
        pose = ops.pair_pose(xyz_c, corr, logits[..., 0], seg.cloud_off, B, self.pose_threshold)
        return both, feats, corr, logits, pose

    def _apply(self, fn, *args, **kwargs):
        _GRAPHS.pop(self, None)        # .to() / .cuda() move the weights the graphs point at
        return super()._apply(fn, *args, **kwargs)


class _TrainOutputs(dict):
    """RegTR.forward's output dict in training mode, carrying the packed tensors (``packed``)
    beside the reference's keys."""
    packed = None


# ------------------------------------------------------------------------------------------
# HIP-graph replay of the post-preprocessing forward
# ------------------------------------------------------------------------------------------
# The preprocessing has one host sync per pyramid level (voxel counts) and data-dependent
# sizes, so it always runs eagerly. Everything after it is a fixed sequence of ~130-300
# launches whose shapes are set by the pyramid's per-cloud lengths: for a batch whose
# lengths (the "signature") were seen before, that sequence is captured once into a HIP graph
# (torch.cuda.CUDAGraph = hipGraph on ROCm) and replayed, removing the host launch cost
# (ctypes, Python) between kernels. The graph reads the kpconv_meta through static copies
# (refreshed by device copies before each replay) and its outputs are cloned, so callers
# never see a buffer that the next replay overwrites. Signatures are captured on their
# SECOND occurrence (one-off shapes stay eager), at most GRAPH_CACHE per model; a parameter
# update (version change), load_state_dict or .to() drops the model's graphs.
# FGREG_GRAPHS=0 disables the path (A/B).
GRAPHS = os.environ.get('FGREG_GRAPHS', '1') != '0'
GRAPH_CACHE = 16       # per model, over (stream slot, signature)
SEEN_CACHE = 4096        # signatures remembered for the capture-on-second-sighting rule (LRU)
_GRAPHS = weakref.WeakKeyDictionary()        # model -> {'ver', 'seen', 'graphs'}
_META_IN = ('points', 'neighbors', 'pools')  # what the core reads (upsamples: decoder only)


class _CoreGraph:
    def __init__(self, model, meta, slens_c, B):
        self.meta = {k: [t.clone() for t in meta[k]] for k in _META_IN}
        self.meta['stack_lengths'] = list(meta['stack_lengths'])
        self.meta['_host'] = {'lengths': meta['_host']['lengths'],
                              'offsets': [o.clone() for o in meta['_host']['offsets']]}
        self.seg = model._segments(slens_c, meta['points'][-1])
        # scratch buffers of this graph alone (split-K partials, attention K/V images, gather
        # flags): a replay never shares them with another graph or an eager launch, on
        # whatever stream it runs (replays of ONE graph are ordered by the caller's stream,
        # like its static inputs and outputs)
        self.ws = ops.PrivateWorkspace()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side), self.ws:       # warm-up outside the capture
            model._core(self.meta, self.seg, B)
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph), self.ws:
            self.out = model._core(self.meta, self.seg, B)

    def run(self, meta):
        srcs, dsts = [], []
        for k in _META_IN:
            for dst, src in zip(self.meta[k], meta[k]):
                srcs.append(src.contiguous())
                dsts.append(dst)
        ops.copy_batch(srcs, dsts)                  # one dispatch for all static inputs
        self.graph.replay()
        outs = [torch.empty_like(t) if t.is_contiguous() else t.clone() for t in self.out]
        pairs = [(t, o) for t, o in zip(self.out, outs) if t.is_contiguous()]
        ops.copy_batch([t for t, _ in pairs], [o for _, o in pairs])   # the clones, one dispatch
        return tuple(outs)


def _params_version(model):
    st = _GRAPHS.get(model)
    plist = st['params'] if st is not None else list(model.parameters()) + list(model.buffers())
    return sum(p._version for p in plist), plist


def _graph_for(model, meta, slens_c, B, slot=0):
    ver, plist = _params_version(model)
    st = _GRAPHS.get(model)
    if st is None or st['ver'] != ver:
        st = {'ver': ver, 'params': plist, 'seen': OrderedDict(), 'graphs': OrderedDict()}
        _GRAPHS[model] = st
    from . import linear as _lin
    sig = (slot, B, _lin.MODE, HEAD_MODE, ops.ATTN_MODE,
           tuple(tuple(l) for l in meta['_host']['lengths']),
           tuple(tuple(t.shape) for t in meta['neighbors']), tuple(tuple(t.shape) for t in meta['pools']))
    g = st['graphs'].get(sig)
    if g is not None:
        st['graphs'].move_to_end(sig)
        return g
    seen = st['seen']
    n = seen.pop(sig, 0)
    seen[sig] = n + 1                 # LRU of signatures: most recent last
    while len(seen) > SEEN_CACHE:
        seen.popitem(last=False)
    if n <= 0:
        return None
    dec = model.correspondence_decoder
    if getattr(dec, 'num_neighbors', 0) > 0:           # the top-k mask reads flags back: eager
        return None
    try:
        g = _CoreGraph(model, meta, slens_c, B)
    except RuntimeError as e:                          # capture unsupported here: stay eager
        _logger.warning('fgreg: HIP graph capture failed (%s); running eagerly', e)
        st['seen'][sig] = -(1 << 30)
        return None
    st['graphs'][sig] = g
    while len(st['graphs']) > GRAPH_CACHE:
        st['graphs'].popitem(last=False)
    return g
