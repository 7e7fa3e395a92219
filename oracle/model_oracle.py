"""CPU restatement of the reference's per-pair registration forward -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module. It is the checker (and the timed CPU baseline, kind "port"), never
the product: the product path is fgreg (HIP kernels) and fails loudly without
its extension.

Everything here is plain PyTorch-CPU fp32 written from the reference's
semantics, operating on a reference-layout state_dict; every function cites the
reference lines it restates. Pinned against tests/golden/forward_*.npz, which the
reference itself produced (tests/golden/make_golden.py).
"""
import math
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import geom  # noqa: E402

# Optional trace of the distance of every activation input to its kink (ReLU / LeakyReLU at 0,
# max-pool: gap between a row's two largest entries), relative to the tensor's max |value|:
# a list to append (site, margin) to, or None. Gradients are discontinuous at those points,
# so gradient parity between two fp32 implementations is only defined away from them
# (tests/test_gpu_train.py).
ACT_TRACE = None


def _trace(site, z):
    # exact zeros (an upstream ReLU's output, shadow rows) are excluded: every implementation
    # produces them exactly and takes the same branch there
    if ACT_TRACE is not None and z.numel():
        za = z.detach().abs()
        nz = za[za > 0]
        if nz.numel():
            ACT_TRACE.append((site, float(nz.min() / za.max())))


def _relu(z, site='relu'):
    _trace(site, z)
    return F.relu(z)


def _leaky(z, site='leaky'):
    _trace(site, z)
    return F.leaky_relu(z, 0.1)


# ----------------------------------------------------------------------------------------
# Preprocessing (models/backbone_kpconv/finegrained_kpconv.py:296-542)
# ----------------------------------------------------------------------------------------
def preprocess(cfg, clouds, mode=geom.INDEX):
    """List[(Ni,3)] -> kpconv_meta dict, per-level loop of finegrained_kpconv.py:455-532.

    mode INDEX: PreprocessorGPU semantics (ball_query first-K, width = limit);
    mode DIST:  Preprocessor (CPU/nanoflann) semantics (K nearest, width = min(max, limit)).
    Subsampled points come out in ascending voxel order (see oracle/geom_oracle.c).
    """
    limits = cfg['neighborhood_limits']
    r_normal = cfg['first_subsampling_dl'] * cfg['conv_radius']
    arch = cfg['architecture']
    pts = np.concatenate([np.asarray(c, np.float32) for c in clouds], 0)
    lens = np.array([len(c) for c in clouds], np.int64)
    out = {'points': [], 'neighbors': [], 'pools': [], 'upsamples': [], 'stack_lengths': []}
    layer_blocks, layer = [], 0
    for bi, block in enumerate(arch):
        if 'global' in block or 'upsample' in block:
            break
        if not ('pool' in block or 'strided' in block):
            layer_blocks.append(block)
            if bi < len(arch) - 1 and 'upsample' not in arch[bi + 1]:
                continue
        assert not any('deformable' in b for b in layer_blocks), 'deformable KPConv unsupported'
        r = r_normal
        if layer_blocks:
            conv_i = geom.radius_search(pts, lens, pts, lens, r, limits[layer], mode)
        else:
            conv_i = np.zeros((0, 1), np.int64)
        if 'pool' in block or 'strided' in block:
            dl = 2 * r_normal / cfg['conv_radius']
            pool_p, pool_b = geom.grid_subsample(pts, lens, dl)
            pool_i = geom.radius_search(pool_p, pool_b, pts, lens, r, limits[layer], mode)
            up_i = geom.radius_search(pts, lens, pool_p, pool_b, 2 * r, limits[layer], mode)
        else:
            pool_p, pool_b = np.zeros((0, 3), np.float32), np.zeros((0,), np.int64)
            pool_i = np.zeros((0, 1), np.int64)
            up_i = np.zeros((0, 1), np.int64)
        out['points'].append(torch.from_numpy(pts))
        out['neighbors'].append(torch.from_numpy(conv_i))
        out['pools'].append(torch.from_numpy(pool_i))
        out['upsamples'].append(torch.from_numpy(up_i))
        out['stack_lengths'].append(torch.from_numpy(lens))
        pts, lens = pool_p, pool_b
        r_normal *= 2
        layer += 1
        layer_blocks = []
    return out


# ----------------------------------------------------------------------------------------
# KPConv backbone (finegrained_kpconv_blocks.py, res2net.py)
# ----------------------------------------------------------------------------------------
def kpconv(q, s, idx, x, W, kp, extent):
    """Rigid KPConv, linear influence, sum aggregation (blocks:265-401)."""
    s = torch.cat([s, torch.zeros_like(s[:1]) + 1e6], 0)                     # :296
    nb = s[idx] - q.unsqueeze(1)                                               # :299-302
    diff = nb.unsqueeze(2) - kp                                                # :312-313
    sq = torch.sum(diff ** 2, dim=3)                                           # :316
    w = torch.clamp(1 - torch.sqrt(sq) / extent, min=0.0).transpose(1, 2)     # :355-356
    x = torch.cat([x, torch.zeros_like(x[:1])], 0)                             # :375
    nx = x[idx]                                                                # :378
    wf = torch.matmul(w, nx).permute(1, 0, 2)                                  # :381,388
    out = torch.matmul(wf, W).sum(0)                                           # :389-393
    nn_ = torch.sum(torch.gt(nx.sum(-1), 0.0), dim=-1)                        # :396-397
    nn_ = torch.max(nn_, torch.ones_like(nn_))                                 # :398
    return out / nn_.unsqueeze(1)                                              # :399


def max_pool(x, idx):
    """blocks:125-141: gather with an appended zero row, max over the row."""
    x = torch.cat([x, torch.zeros_like(x[:1])], 0)
    g = x[idx]
    if ACT_TRACE is not None and g.shape[1] > 1:
        # candidates: the real entries and ONE zero standing for all shadow entries (ties
        # among shadows carry no gradient); margin = gap between the two largest candidates
        real = idx < x.shape[0] - 1
        gd = g.detach()
        cand = torch.where(real.unsqueeze(-1), gd, torch.full_like(gd, -math.inf))
        shadow = torch.where((~real).any(1, keepdim=True), torch.zeros_like(gd[:, :1]),
                             torch.full_like(gd[:, :1], -math.inf))
        top = torch.cat([cand, shadow], 1).topk(2, dim=1)[0]
        gap = torch.nan_to_num(top[:, 0] - top[:, 1], nan=math.inf)
        gap = gap[gap > 0]                  # exact ties: the first entry wins everywhere
        if gap.numel():
            ACT_TRACE.append(('max_pool', float(gap.min() / gd.abs().max().clamp_min(1e-30))))
    return g.max(1)[0]


def instance_norm(x, lens, eps=1e-5):
    """nn.InstanceNorm1d(affine=False) per cloud (blocks:498-507)."""
    outs, o = [], 0
    for n in lens.tolist():
        seg = x[o:o + n]
        mu = seg.mean(0, keepdim=True)
        var = ((seg - mu) ** 2).mean(0, keepdim=True)
        outs.append((seg - mu) / torch.sqrt(var + eps))
        o += n
    return torch.cat(outs, 0)


def _bn(sd, p, x, eps=1e-5, train=False):
    """BatchNorm1d: eval on running statistics; train on the batch's (biased variance, all
    rows of all clouds -- nn.BatchNorm1d.train(), res2net.py:126-159 in train.py)."""
    if train:
        mu = x.mean(0)
        var = ((x - mu) ** 2).mean(0)
        return (x - mu) / torch.sqrt(var + eps) * sd[p + '.weight'] + sd[p + '.bias']
    return ((x - sd[p + '.running_mean']) / torch.sqrt(sd[p + '.running_var'] + eps)
            * sd[p + '.weight'] + sd[p + '.bias'])


def unary(sd, p, x, lens, relu=True):
    """UnaryBlock (blocks:521-555): Linear(no bias) -> InstanceNorm -> LeakyReLU(0.1)."""
    x = instance_norm(x @ sd[p + '.mlp.weight'].t(), lens)
    return _leaky(x, p) if relu else x


def res2net(sd, p, x, scale=8, train=False):
    """my_res2Net / my_Bottle2neck (res2net.py:126-159, 231-265); BatchNorm on running
    statistics (eval) or batch statistics (train)."""
    p = p + '.layer1.0'
    out = _relu(_bn(sd, p + '.bn1', x @ sd[p + '.conv1.weight'].t(), train=train), p + '.bn1')
    width = sd[p + '.convs.0.weight'].shape[0]
    spx = torch.split(out, width, 1)
    outs = []
    sp = None
    for i in range(scale - 1):
        sp = spx[i] if i == 0 else sp + spx[i]
        sp = _relu(_bn(sd, f'{p}.bns.{i}', sp @ sd[f'{p}.convs.{i}.weight'].t(), train=train),
                   f'{p}.bns.{i}')
        outs.append(sp)
    outs.append(spx[scale - 1])
    out = _bn(sd, p + '.bn3', torch.cat(outs, 1) @ sd[p + '.conv3.weight'].t(), train=train)
    res = _bn(sd, p + '.downsample.1', x @ sd[p + '.downsample.0.weight'].t(), train=train)
    return _relu(out + res, p + '.out')


def encoder(cfg, sd, meta, feats0, train=False):
    """KPFEncoder.forward (finegrained_kpconv.py:22-95) with block_decider's blocks."""
    r = cfg['first_subsampling_dl'] * cfg['conv_radius']
    layer = 0
    x = feats0
    for bi, block in enumerate(cfg['architecture']):
        p = f'kpf_encoder.encoder_blocks.{bi}'
        extent = r * cfg['KP_extent'] / cfg['conv_radius']
        strided = 'strided' in block
        if strided:
            q, s = meta['points'][layer + 1], meta['points'][layer]
            idx, lens_post = meta['pools'][layer], meta['stack_lengths'][layer + 1]
        else:
            q = s = meta['points'][layer]
            idx, lens_post = meta['neighbors'][layer], meta['stack_lengths'][layer]
        lens_pre = meta['stack_lengths'][layer]
        if block.startswith('simple'):                                         # blocks:620-634
            y = kpconv(q, s, idx, x, sd[p + '.KPConv.weights'], sd[p + '.KPConv.kernel_points'],
                       extent)
            x = _leaky(instance_norm(y, lens_post), p)
        elif block.startswith('resnetb'):                                      # blocks:692-727
            y = unary(sd, p + '.unary1', x, lens_pre) if p + '.unary1.mlp.weight' in sd else x
            y = kpconv(q, s, idx, y, sd[p + '.KPConv.weights'], sd[p + '.KPConv.kernel_points'],
                       extent)
            y = instance_norm(y, lens_post)
            y = _leaky(res2net(sd, p + '.res2net', y, train=train), p + '.res2net')
            sc = max_pool(x, idx) if strided else x
            if p + '.unary_shortcut.mlp.weight' in sd:
                sc = unary(sd, p + '.unary_shortcut', sc, lens_post, relu=False)
            x = _leaky(y + sc, p + '.out')
        else:
            raise NotImplementedError(block)
        if strided:
            layer += 1
            r *= 2
    return x


# ----------------------------------------------------------------------------------------
# Transformer (models/transformer/*.py)
# ----------------------------------------------------------------------------------------
def sine_pos_embed(xyz, d_model, temperature=10000, scale=1.0):
    """PositionEmbeddingCoordsSine.forward (position_embedding.py:29-49), n_dim=3."""
    npf = d_model // 3 // 2 * 2
    pad = d_model - npf * 3
    dim_t = torch.arange(npf, dtype=xyz.dtype)
    dim_t = temperature ** (2 * torch.div(dim_t, 2, rounding_mode='trunc') / npf)
    pd = (xyz * (scale * 2 * math.pi)).unsqueeze(-1) / dim_t
    emb = torch.stack([pd[..., 0::2].sin(), pd[..., 1::2].cos()], -1).reshape(*xyz.shape[:-1], -1)
    return F.pad(emb, (0, pad))


def mha(sd, p, q, k, v, kmask, nhead):
    """nn.MultiheadAttention forward (eval, no dropout) with a key padding mask.

    q (Lq,B,d), k/v (Lk,B,d), kmask (B,Lk) True = padded.
    """
    Lq, B, d = q.shape
    Lk = k.shape[0]
    dh = d // nhead
    W, b = sd[p + '.in_proj_weight'], sd[p + '.in_proj_bias']
    qp = q @ W[:d].t() + b[:d]
    kp_ = k @ W[d:2 * d].t() + b[d:2 * d]
    vp = v @ W[2 * d:].t() + b[2 * d:]
    qh = qp.reshape(Lq, B * nhead, dh).transpose(0, 1) * (1.0 / math.sqrt(dh))
    kh = kp_.reshape(Lk, B * nhead, dh).transpose(0, 1)
    vh = vp.reshape(Lk, B * nhead, dh).transpose(0, 1)
    mask = torch.zeros(B, Lk, dtype=q.dtype).masked_fill(kmask, float('-inf'))
    mask = mask.repeat_interleave(nhead, 0).unsqueeze(1)
    att = torch.softmax(torch.baddbmm(mask, qh, kh.transpose(1, 2)), -1)
    o = torch.bmm(att, vh).transpose(0, 1).reshape(Lq, B, d)
    return o @ sd[p + '.out_proj.weight'].t() + sd[p + '.out_proj.bias']


def _ln(sd, p, x):
    return F.layer_norm(x, x.shape[-1:], sd[p + '.weight'], sd[p + '.bias'], 1e-5)


def cross_encoder_layer(sd, p, src, tgt, smask, tmask, spos, tpos, nhead, pre_norm=True):
    """TransformerCrossEncoderLayer.forward_pre (transformers.py:183-244), values with pos;
    forward_post (:109-181) for pre_norm=False."""
    if not pre_norm:
        src = _ln(sd, p + '.norm1', src + mha(sd, p + '.self_attn', src + spos, src + spos,
                                              src + spos, smask, nhead))
        tgt = _ln(sd, p + '.norm1', tgt + mha(sd, p + '.self_attn', tgt + tpos, tgt + tpos,
                                              tgt + tpos, tmask, nhead))
        s2, t2 = src + spos, tgt + tpos
        s3 = mha(sd, p + '.multihead_attn', s2, t2, t2, tmask, nhead)
        t3 = mha(sd, p + '.multihead_attn', t2, s2, s2, smask, nhead)
        src, tgt = _ln(sd, p + '.norm2', src + s3), _ln(sd, p + '.norm2', tgt + t3)

        def ffn_post(x):
            h = _relu(x @ sd[p + '.linear1.weight'].t() + sd[p + '.linear1.bias'], p + '.ffn')
            return _ln(sd, p + '.norm3', x + h @ sd[p + '.linear2.weight'].t() + sd[p + '.linear2.bias'])
        return ffn_post(src), ffn_post(tgt)
    s2 = _ln(sd, p + '.norm1', src) + spos
    src = src + mha(sd, p + '.self_attn', s2, s2, s2, smask, nhead)
    t2 = _ln(sd, p + '.norm1', tgt) + tpos
    tgt = tgt + mha(sd, p + '.self_attn', t2, t2, t2, tmask, nhead)
    s2 = _ln(sd, p + '.norm2', src) + spos
    t2 = _ln(sd, p + '.norm2', tgt) + tpos
    s3 = mha(sd, p + '.multihead_attn', s2, t2, t2, tmask, nhead)
    t3 = mha(sd, p + '.multihead_attn', t2, s2, s2, smask, nhead)
    src, tgt = src + s3, tgt + t3

    def ffn(x):
        h = _relu(_ln(sd, p + '.norm3', x) @ sd[p + '.linear1.weight'].t() + sd[p + '.linear1.bias'],
                  p + '.ffn')
        return x + h @ sd[p + '.linear2.weight'].t() + sd[p + '.linear2.bias']
    return ffn(src), ffn(tgt)


def _pad(seqs):
    n = max(len(s) for s in seqs)
    out = torch.zeros(n, len(seqs), seqs[0].shape[-1], dtype=seqs[0].dtype)
    mask = torch.ones(len(seqs), n, dtype=torch.bool)
    for b, s in enumerate(seqs):
        out[:len(s), b] = s
        mask[b, :len(s)] = False
    return out, mask


def corr_simple_attention(sd, p, query, key, value, kmask, num_neighbors=0):
    """CorrespondenceDecoder.simple_attention (finegrained_regtr.py:328-363) on padded
    ([L,] N, B, D) inputs. num_neighbors > 0 restates the reference's masking as it executes:
    `neighbor_mask[:, :, topk_indices] = 0` indexes the QUERY dim (2) of the (L, B, Q, S) mask
    with the top-k KEY indices of every row, so query row j keeps its softmax iff j is among
    all top-k indices of every (layer, pair, row); other rows are all -inf (NaN softmax); an
    index >= Q raises IndexError."""
    q = (query @ sd[p + 'q_proj.weight'].t() + sd[p + 'q_proj.bias']) / math.sqrt(query.shape[-1])
    k = key @ sd[p + 'k_proj.weight'].t() + sd[p + 'k_proj.bias']
    attn = torch.einsum('...qbd,...sbd->...bqs', q, k)
    attn = attn.masked_fill(kmask[:, None, :], float('-inf'))
    if num_neighbors > 0:
        Q = attn.shape[-2]
        idx = torch.topk(attn, k=num_neighbors, dim=-1).indices.reshape(-1)
        if idx.numel() and int(idx.max()) >= Q:
            raise IndexError(f'index {int(idx.max())} is out of bounds for dimension 2 with size {Q}')
        keep = torch.zeros(Q, dtype=torch.bool)
        keep[idx] = True
        attn = attn.masked_fill(~keep[:, None], float('-inf'))
    return torch.einsum('...bqs,...sbd->...qbd', torch.softmax(attn, -1), value)


# ----------------------------------------------------------------------------------------
# Pose (utils/se3_torch.py)
# ----------------------------------------------------------------------------------------
def weighted_procrustes(a, b, w, threshold=0.85):
    """fast_compute_rigid_transform (se3_torch.py:226-273); threshold=None -> :131-173."""
    if threshold is not None:
        w = torch.where(w > threshold, w, torch.zeros_like(w))                 # :240-242
    wn = w[..., None] / torch.clamp_min(w.sum(-1, keepdim=True)[..., None], 1e-6)
    ca = (a * wn).sum(-2)
    cb = (b * wn).sum(-2)
    cov = (a - ca[..., None, :]).transpose(-2, -1) @ ((b - cb[..., None, :]) * wn)
    u, _, v = torch.svd(cov, some=False, compute_uv=True)
    rpos = v @ u.transpose(-1, -2)
    vneg = v.clone()
    vneg[..., 2] *= -1
    rneg = vneg @ u.transpose(-1, -2)
    rot = torch.where(torch.det(rpos)[..., None, None] > 0, rpos, rneg)
    t = -rot @ ca[..., :, None] + cb[..., :, None]
    return torch.cat([rot, t], -1)


# ----------------------------------------------------------------------------------------
# Whole forward (models/finegrained_regtr.py:108-250)
# ----------------------------------------------------------------------------------------
@torch.no_grad()
def forward(cfg, sd, src_xyz, tgt_xyz, meta=None, mode=geom.INDEX, num_neighbors=0):
    """The inference forward (eval(), no autograd). num_neighbors: the CorrespondenceDecoder's
    top-k masking (a constructor argument the reference's RegTR never passes; on padded
    batches its padded query rows take part as the reference computes them)."""
    return _forward(cfg, sd, src_xyz, tgt_xyz, meta, mode, train=False,
                    num_neighbors=num_neighbors)


def forward_train(cfg, sd, src_xyz, tgt_xyz, meta=None, mode=geom.INDEX):
    """The training-mode forward (model.train(), autograd on): Res2Net BatchNorm on batch
    statistics; differentiable in every state_dict tensor that requires grad (the pose is
    computed without gradients, as no loss reads it, finegrained_regtr.py:252-309)."""
    return _forward(cfg, sd, src_xyz, tgt_xyz, meta, mode, train=True)


def _forward(cfg, sd, src_xyz, tgt_xyz, meta, mode, train, num_neighbors=0):
    B = len(src_xyz)
    if meta is None:
        meta = preprocess(cfg, [np.asarray(c) for c in list(src_xyz) + list(tgt_xyz)], mode)
    slens_c = meta['stack_lengths'][-1].tolist()
    feats0 = torch.ones_like(meta['points'][0][:, :1])                         # :126
    feats_un = encoder(cfg, sd, meta, feats0, train=train)
    both = feats_un @ sd['feat_proj.weight'].t() + sd['feat_proj.bias']       # :149
    src_f, tgt_f = torch.split(both, slens_c)[:B], torch.split(both, slens_c)[B:]
    xyz_c = meta['points'][-1]
    src_xyz_c, tgt_xyz_c = torch.split(xyz_c, slens_c)[:B], torch.split(xyz_c, slens_c)[B:]
    pe = sine_pos_embed(xyz_c, cfg['d_embed'])                                 # :163
    src_pe, tgt_pe = torch.split(pe, slens_c)[:B], torch.split(pe, slens_c)[B:]
    spos, _ = _pad(src_pe)
    tpos, _ = _pad(tgt_pe)
    src, smask = _pad(src_f)
    tgt, tmask = _pad(tgt_f)
    nhead, L = cfg['nhead'], cfg['num_encoder_layers']
    s_int, t_int = [], []
    for l in range(L):                                                         # transformers.py:37-57
        pre = cfg.get('pre_norm', True)
        src, tgt = cross_encoder_layer(sd, f'transformer_encoder.layers.{l}', src, tgt, smask, tmask,
                                       spos, tpos, nhead, pre_norm=pre)
        # the final norm exists for pre_norm only (finegrained_regtr.py:56-58)
        s_int.append(_ln(sd, 'transformer_encoder.norm', src) if pre else src)
        t_int.append(_ln(sd, 'transformer_encoder.norm', tgt) if pre else tgt)
    s_cond, t_cond = torch.stack(s_int), torch.stack(t_int)

    def corr_mlp(x):                                                           # :411-455
        h = _relu(x @ sd['correspondence_decoder.coor_mlp.0.weight'].t()
                  + sd['correspondence_decoder.coor_mlp.0.bias'], 'coor_mlp.0')
        h = _relu(h @ sd['correspondence_decoder.coor_mlp.2.weight'].t()
                  + sd['correspondence_decoder.coor_mlp.2.bias'], 'coor_mlp.2')
        return h @ sd['correspondence_decoder.coor_mlp.4.weight'].t() + sd['correspondence_decoder.coor_mlp.4.bias']

    def conf(x):
        return (x @ sd['correspondence_decoder.conf_logits_decoder.weight'].t()
                + sd['correspondence_decoder.conf_logits_decoder.bias'])

    def simple_attention(query, key, value, kmask):                          # :328-363
        return corr_simple_attention(sd, 'correspondence_decoder.', query, key, value, kmask,
                                     num_neighbors)

    if cfg.get('direct_regress_coor', False):
        s_corr, t_corr = corr_mlp(s_cond), corr_mlp(t_cond)
    else:                                       # CorrespondenceDecoder (:312-408), pos emb on
        s2 = s_cond + spos if cfg.get('corr_decoder_has_pos_emb', True) else s_cond
        t2 = t_cond + tpos if cfg.get('corr_decoder_has_pos_emb', True) else t_cond
        sx, _ = _pad(src_xyz_c)
        tx, _ = _pad(tgt_xyz_c)
        s_corr = simple_attention(s2, t2, tx, tmask)
        t_corr = simple_attention(t2, s2, sx, smask)
    s_ov, t_ov = conf(s_cond), conf(t_cond)
    ns, nt = slens_c[:B], slens_c[B:]
    out = {
        'src_feat_un': list(src_f), 'tgt_feat_un': list(tgt_f),
        'src_feat': [s_cond[:, :ns[b], b] for b in range(B)],
        'tgt_feat': [t_cond[:, :nt[b], b] for b in range(B)],
        'src_kp': list(src_xyz_c), 'tgt_kp': list(tgt_xyz_c),
        'src_kp_warped': [s_corr[:, :ns[b], b] for b in range(B)],
        'tgt_kp_warped': [t_corr[:, :nt[b], b] for b in range(B)],
        'src_overlap': [s_ov[:, :ns[b], b] for b in range(B)],
        'tgt_overlap': [t_ov[:, :nt[b], b] for b in range(B)],
    }
    poses = []
    with torch.no_grad():
        for b in range(B):                                                     # :198-218
            a = torch.cat([src_xyz_c[b].expand(L, -1, -1), out['tgt_kp_warped'][b]], 1)
            bb = torch.cat([out['src_kp_warped'][b], tgt_xyz_c[b].expand(L, -1, -1)], 1)
            w = torch.cat([torch.sigmoid(out['src_overlap'][b][:, :, 0]),
                           torch.sigmoid(out['tgt_overlap'][b][:, :, 0])], 1)
            poses.append(weighted_procrustes(a, bb, w))
    out['pose'] = torch.stack(poses, 1)
    out['kpconv_meta'] = meta
    return out
