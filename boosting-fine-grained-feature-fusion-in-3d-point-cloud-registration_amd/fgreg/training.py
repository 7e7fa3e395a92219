"""The training-mode forward of RegTR, differentiable end to end.

``RegTR.forward`` routes here in ``train()`` mode: the same module tree, parameter names and
outputs as the inference forward (models/finegrained_regtr.py:108-250), with
* the Res2Net BatchNorm1d layers on batch statistics over all clouds of the batch, running
  statistics updated (res2net.py:126-159; nn.BatchNorm1d train semantics -- this couples the
  pairs of a batch, exactly as the reference);
* every op an autograd Function of fgreg.autograd (forward and backward on libfgreg), so
  ``loss.backward()`` of trainer.py:110-125 produces the gradients of every trainable
  parameter (kernel points stay fixed: requires_grad=False in the reference, blocks:250-263).
The pose is computed without gradients (the reference's losses never read it,
finegrained_regtr.py:252-309).
"""
import math

import torch
import torch.nn.functional as F

from . import ops
from . import linear as lin
from .autograd import (attention_t, batchnorm_t, corr_attention_t, kpconv_t, layernorm_t, leaky,
                       linear_t, max_pool_t, segnorm_t)
from .backbone import ResnetBottleneckBlock, SimpleBlock, UnaryBlock, _level_inputs, host_layout
from .ops import ACT_LEAKY, ACT_NONE, ACT_RELU


def unary_train(u: UnaryBlock, x, off, lens, residual=None, post_act=ACT_NONE):
    """Linear(no bias) -> InstanceNorm -> LeakyReLU (blocks:521-555)."""
    y = linear_t(x, u.mlp.weight)
    act = ACT_NONE if u.no_relu else ACT_LEAKY
    return segnorm_t(y, off, lens, act=act, residual=residual, post_act=post_act)


class _ColSplitFn(torch.autograd.Function):
    """torch.split(h, w, 1) whose backward is one concatenation of the chunk gradients (the
    generic split backward materialises a zero tensor of h's shape per chunk, copies the
    chunk's gradient into it and adds the chunks up)."""

    @staticmethod
    def forward(ctx, h, w, n):
        ctx.w = w
        return tuple(h.narrow(1, i * w, w) for i in range(n))

    @staticmethod
    def backward(ctx, *grads):
        ref = next(g for g in grads if g is not None)
        full = [g if g is not None else ref.new_zeros(ref.shape[0], ctx.w) for g in grads]
        return torch.cat(full, 1), None, None


def bottle2neck_train(m, x):
    """my_Bottle2neck.forward (res2net.py:126-159) with BatchNorm1d on batch statistics."""
    w = m.width
    h = batchnorm_t(m.bn1, linear_t(x, m.conv1.weight), act=ACT_RELU)
    chunks = _ColSplitFn.apply(h, w, h.shape[1] // w)
    outs, sp = [], None
    for i in range(m.nums):
        sp = chunks[i] if i == 0 else sp + chunks[i]
        sp = batchnorm_t(m.bns[i], linear_t(sp, m.convs[i].weight), act=ACT_RELU)
        outs.append(sp)
    if m.scale != 1:
        outs.append(chunks[m.nums])
    cat = torch.cat(outs, 1)
    if m.downsample is not None:
        res = batchnorm_t(m.downsample[1], linear_t(x, m.downsample[0].weight))
    else:
        res = x
    return batchnorm_t(m.bn3, linear_t(cat, m.conv3.weight), residual=res, post_act=ACT_RELU)


def block_train(block, x, meta):
    q, s, idx, post = _level_inputs(block.block_name, block.layer_ind, meta)
    if isinstance(block, SimpleBlock):                         # blocks:620-634
        lens, off = host_layout(meta, post)
        y, nnorm = kpconv_t(block.KPConv, q, s, idx, x)
        return segnorm_t(y, off, lens, row_div=nnorm, act=ACT_LEAKY)
    assert isinstance(block, ResnetBottleneckBlock)            # blocks:692-727
    lens_pre, off_pre = host_layout(meta, block.layer_ind)
    lens_post, off_post = host_layout(meta, post)
    x1 = unary_train(block.unary1, x, off_pre, lens_pre) if isinstance(block.unary1, UnaryBlock) else x
    y, nnorm = kpconv_t(block.KPConv, q, s, idx, x1)
    y = segnorm_t(y, off_post, lens_post, row_div=nnorm)
    # res2net ends in ReLU: the LeakyReLU at :715 is the identity, gradient included
    y = bottle2neck_train(block.res2net.layer1[0], y)
    shortcut = max_pool_t(x, idx) if 'strided' in block.block_name else x
    if isinstance(block.unary_shortcut, UnaryBlock):
        return unary_train(block.unary_shortcut, shortcut, off_post, lens_post, residual=y,
                           post_act=ACT_LEAKY)
    return leaky(y + shortcut)


def _residual(x, y_fn, lin, p):
    """x + dropout_p(lin(y)): the residual fused into the GEMM epilogue when p = 0, else the
    layer's dropout1/2/3 (transformers.py:108-110) between the product and the add."""
    if p > 0.0:
        return x + F.dropout(linear_t(y_fn, lin.weight, lin.bias), p, training=True)
    return linear_t(y_fn, lin.weight, lin.bias, residual=x)


def _ffn_hidden(layer, h, p):
    """activation(linear1(h)), then the FFN's own dropout (:102, :233) when p > 0."""
    h = linear_t(h, layer.linear1.weight, layer.linear1.bias, act=ACT_RELU)
    return F.dropout(h, p, training=True) if p > 0.0 else h


def layer_train(layer, x, pos, seg):
    """TransformerCrossEncoderLayer.forward_pre (transformers.py:183-244), both clouds packed;
    forward_post (:109-181) for pre_norm: False. With dropout p > 0 (the layer's
    nn.MultiheadAttention(dropout=p), dropout, dropout1/2/3, :95-110): attention-weight dropout
    in the attention kernels, torch dropout on the FFN hidden and the sub-layer outputs."""
    if not layer.normalize_before:
        return _layer_post_train(layer, x, pos, seg)
    p = float(layer.self_attn.dropout)
    for norm, mha, kv_seg in ((layer.norm1, layer.self_attn, seg.self_seg),
                              (layer.norm2, layer.multihead_attn, seg.cross_seg)):
        h = layernorm_t(x, norm, add=pos)
        qkv = linear_t(h, mha.in_proj_weight, mha.in_proj_bias)
        o = attention_t(qkv, seg.off, kv_seg, seg.max_len, layer.nhead, dropout=p)
        x = _residual(x, o, mha.out_proj, p)
    return _residual(x, _ffn_hidden(layer, layernorm_t(x, layer.norm3), p), layer.linear2, p)


def _layer_post_train(layer, x, pos, seg):
    p = float(layer.self_attn.dropout)
    for norm, mha, kv_seg in ((layer.norm1, layer.self_attn, seg.self_seg),
                              (layer.norm2, layer.multihead_attn, seg.cross_seg)):
        qkv = linear_t(x if pos is None else x + pos, mha.in_proj_weight, mha.in_proj_bias)
        o = attention_t(qkv, seg.off, kv_seg, seg.max_len, layer.nhead, dropout=p)
        x = layernorm_t(_residual(x, o, mha.out_proj, p), norm)
    return layernorm_t(_residual(x, _ffn_hidden(layer, x, p), layer.linear2, p), layer.norm3)


def check_trainable(model):
    """Raises NotImplementedError for configurations this training forward does not restate
    (checked before any work, so CPU and GPU callers see the same error)."""
    cfg = model.cfg
    if not (cfg.sa_val_has_pos_emb and cfg.ca_val_has_pos_emb):
        raise NotImplementedError('training with value-without-positional-embedding attention is '
                                  'not in the reference configs')
    if float(cfg.get('dropout', 0.0) or 0.0) > 0.0:
        # transformers.py:95-110: the attention-weight dropout runs in the f16x3 attention
        # kernels (head dim 32 / 64) in both precision modes (ops.attention)
        dh = cfg.d_embed // cfg.nhead
        if dh not in (32, 64):
            raise NotImplementedError(f'training with dropout {cfg.dropout} > 0 needs head dim '
                                      f'32 / 64 (head dim {dh})')
    if getattr(model.correspondence_decoder, 'num_neighbors', 0) > 0:
        raise NotImplementedError('training the CorrespondenceDecoder with num_neighbors > 0 (a '
                                  'constructor argument the reference RegTR never passes)')


def core_train(model, meta, seg, B):
    """RegTR._core in training mode -> (feats_un, feats (L, N, d), corr, logits, pose)."""
    from .regtr import HEAD_MODE, CorrespondenceRegressor
    cfg = model.cfg
    check_trainable(model)
    head = model.correspondence_decoder
    pts0 = meta['points'][0]
    x = torch.ones((pts0.shape[0], 1), dtype=torch.float32, device=pts0.device)
    for block in model.kpf_encoder.encoder_blocks:
        x = block_train(block, x, meta)
    both = linear_t(x, model.feat_proj.weight, model.feat_proj.bias)
    xyz_c = meta['points'][-1]
    with torch.no_grad():
        pe = model.pos_embed(xyz_c)
    pos = pe if cfg.transformer_encoder_has_pos_emb else None
    enc = model.transformer_encoder
    h = both
    inter = []
    for l, layer in enumerate(enc.layers):
        h = layer_train(layer, h, pos, seg)
        if enc.return_intermediate or l == len(enc.layers) - 1:
            inter.append(layernorm_t(h, enc.norm) if enc.norm is not None else h)
    feats = torch.stack(inter, 0)                                          # (L, N, d)
    L, N, d = feats.shape
    f = feats.reshape(L * N, d)
    if isinstance(head, CorrespondenceRegressor):                          # :411-455
        # the inference head's compute mode (regtr.py CorrespondenceRegressor.forward_packed)
        with lin.mode_scope(HEAD_MODE if lin.MODE == 'bf16' else None):
            m = head.coor_mlp
            t = linear_t(f, m[0].weight, m[0].bias, act=ACT_RELU)
            t = linear_t(t, m[2].weight, m[2].bias, act=ACT_RELU)
            corr = linear_t(t, m[4].weight, m[4].bias)
            logits = linear_t(f, head.conf_logits_decoder.weight, head.conf_logits_decoder.bias)
    else:                                                                  # :312-408
        fq = (feats + pe.unsqueeze(0) if head.use_pos_emb else feats).reshape(L * N, d)
        q = linear_t(fq, head.q_proj.weight, head.q_proj.bias)
        k = linear_t(fq, head.k_proj.weight, head.k_proj.bias)
        corr = corr_attention_t(q, k, xyz_c, seg, 1.0 / math.sqrt(d))     # q_proj(.) / sqrt(D)
        logits = linear_t(f, head.conf_logits_decoder.weight, head.conf_logits_decoder.bias)
    corr, logits = corr.view(L, N, 3), logits.view(L, N, 1)
    with torch.no_grad():
        pose = ops.pair_pose(xyz_c, corr.detach(), logits.detach()[..., 0], seg.cloud_off, B,
                             model.pose_threshold)
    return both, feats, corr, logits, pose
