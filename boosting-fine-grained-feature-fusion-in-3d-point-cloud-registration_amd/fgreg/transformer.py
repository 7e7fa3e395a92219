"""Cross-encoder transformer on packed, unpadded clouds.

Parameter names follow models/transformer/transformers.py (``layers.{i}.self_attn``,
``multihead_attn`` as nn.MultiheadAttention, ``linear1/2``, ``norm1-3``, final
``norm``), so reference checkpoints load unchanged. The compute differs in layout:
the reference pads src and tgt to (N_max, B, d) and runs every op twice (src, tgt)
with key padding masks (finegrained_regtr.py:164-179); here all 2B clouds stay
packed in one (N_tot, d) tensor in the encoder's cloud order
(src_0..src_{B-1}, tgt_0..tgt_{B-1}) and

* self-attention = one QKV GEMM over all rows + fgr_attention with every cloud
  attending to itself;
* cross-attention = one QKV GEMM over all rows + fgr_attention with cloud c
  attending to its partner (c + B) mod 2B -- both directions in one launch, reading
  the same pre-update activations exactly like the reference's simultaneous update
  (transformers.py:213-229);
* LayerNorm (+ positional embedding add) = fgr_layernorm.
Masked keys never exist, so no -inf masking is needed; padded query rows never exist,
so no work is wasted on them.
"""
import copy

import torch
import torch.nn as nn

import os

from . import linear as lin
from . import ops
from .linear import linear, linear_ln, ln_fusable

# the pre-norm in_proj writes the attention's K / V images itself where supported
# (fgr_gemm_f16x3_ln_qkv; FGREG_QKV_IMAGES=0: fp32 q | k | v and the attention's own image launch)
QKV_IMAGES = os.environ.get('FGREG_QKV_IMAGES', '1') != '0'


class Segments:
    """Device-side segment tables of one packed batch of 2B clouds (built before any graph
    capture: they are host -> device copies)."""

    def __init__(self, lengths, device, n_layers=0, phantoms=None):
        """``phantoms``: optional per-cloud counts of query-only rows appended after the 2B
        clouds' rows, grouped by cloud (the reference's padded positions, which it computes as
        queries of every attention and never as keys: CorrespondenceDecoder top-k masking on
        padded batches, finegrained_regtr.py:353-357). Each non-empty group is one more
        segment whose key segment is its cloud (self-attention) or the partner (cross);
        ``cloud_off`` = ``off[:2B + 1]`` is the clouds' own table."""
        self.lengths = [int(n) for n in lengths]
        n = len(self.lengths)
        assert n % 2 == 0
        self.B = n // 2
        self.phantoms = [int(p) for p in phantoms] if phantoms is not None else [0] * n
        assert len(self.phantoms) == n and min(self.phantoms, default=0) >= 0
        # segment -> the cloud it belongs to (the clouds first, then the phantom groups)
        self.seg_cloud = list(range(n)) + [c for c in range(n) if self.phantoms[c] > 0]
        self.seg_lengths = self.lengths + [p for p in self.phantoms if p > 0]
        self.n_phantom = sum(self.phantoms)
        self.off = ops.offsets(self.seg_lengths, device)
        self.cloud_off = self.off[:n + 1]
        self.self_seg = ops.to_device(self.seg_cloud, torch.int32, device)
        self.cross_seg = ops.to_device([(c + self.B) % n for c in self.seg_cloud], torch.int32,
                                       device)
        self.max_len = max(self.seg_lengths) if n else 0
        self.layer_tables = None
        if n_layers:
            # (layer, segment) segments of the L stacked layer outputs (L * N rows): segment
            # l * S + s attends to l * S + partner(cloud of s); value rows = the partner's xyz
            # rows, built from the host lengths (reading self.off back would sync the stream)
            N = sum(self.seg_lengths)
            S = len(self.seg_lengths)
            host_off = [0]
            for ln in self.seg_lengths[:-1]:
                host_off.append(host_off[-1] + ln)
            q_off = [l * N + o for l in range(n_layers) for o in host_off]
            q_off.append(n_layers * N)
            kv_seg = [l * S + (c + self.B) % n for l in range(n_layers) for c in self.seg_cloud]
            v_off = host_off * n_layers
            self.layer_tables = (ops.to_device(q_off, torch.int64, device),
                                 ops.to_device(kv_seg, torch.int32, device),
                                 ops.to_device(v_off, torch.int64, device))


class TransformerCrossEncoderLayer(nn.Module):
    """transformers.py:84-258: forward_pre (pre_norm: True, the shipped configs) and
    forward_post (pre_norm: False); dropout must be 0 at inference."""

    def __init__(self, d_model, nhead, dim_feedforward=2048, dropout=0.1, activation='relu',
                 normalize_before=False, sa_val_has_pos_emb=False, ca_val_has_pos_emb=False,
                 attention_type='dot_prod'):
        super().__init__()
        if attention_type != 'dot_prod':
            raise NotImplementedError(attention_type)
        if activation != 'relu':
            raise NotImplementedError('transformer_act other than relu is not in the configs')
        self.self_attn = nn.MultiheadAttention(d_model, nhead, dropout=dropout)
        self.multihead_attn = nn.MultiheadAttention(d_model, nhead, dropout=dropout)
        self.linear1 = nn.Linear(d_model, dim_feedforward)
        self.linear2 = nn.Linear(dim_feedforward, d_model)
        self.norm1 = nn.LayerNorm(d_model)
        self.norm2 = nn.LayerNorm(d_model)
        self.norm3 = nn.LayerNorm(d_model)
        self.nhead = nhead
        self.normalize_before = normalize_before
        self.sa_val_has_pos_emb = sa_val_has_pos_emb
        self.ca_val_has_pos_emb = ca_val_has_pos_emb

    def _attend(self, mha, h_pos, h_nopos, val_has_pos, seg, kv_seg, ln=None, side=None):
        """``ln`` = (x, norm, pos): h_pos = norm(x) + pos is formed inside the in_proj GEMM
        (linear_ln; val_has_pos only); ``side`` = (norm2, out2): out2 = norm2(x) as well."""
        W, b = mha.in_proj_weight, mha.in_proj_bias
        if ln is not None:
            x, norm, pos = ln
            d = x.shape[1]
            # the image path forms norm(x) + pos in its prologue: it needs the pos rows
            # (transformer_encoder_has_pos_emb False -> pos None -> linear_ln below)
            if (QKV_IMAGES and lin.MODE == 'f16x3' and ops.ATTN_MODE == 'f16x3' and pos is not None
                    and ops.ln_qkv_supported(x.shape[0], d, self.nhead)
                    and (side is None or side[0].eps == norm.eps)):
                # k / v straight into the attention's images (no fp32 k / v, no image launch)
                return ops.ln_qkv_attention(x, norm, lin.weight_image(W, mode='f16x3'), b, pos,
                                            seg.off, kv_seg, seg.max_len, self.nhead, side=side)
            qkv = linear_ln(x, norm, W, b, add=pos, side=side)        # (N, 3d): [q | k | v]
            q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
            return ops.attention(q, k, v, seg.off, seg.off, kv_seg, seg.max_len, self.nhead)
        d = h_pos.shape[1]
        if (val_has_pos and QKV_IMAGES and lin.MODE == 'f16x3' and ops.ATTN_MODE == 'f16x3'
                and ops.qkv_supported(h_pos.shape[0], d, self.nhead)):
            # head dim 64: the in_proj writes the attention's K / V images itself
            return ops.qkv_attention(h_pos, lin.weight_image(W, mode='f16x3'), b, seg.off, kv_seg,
                                     seg.max_len, self.nhead)
        if (val_has_pos and QKV_IMAGES and lin.MODE == 'bf16' and ops.ATTN_MODE == 'bf16'
                and ops.qkv_bf16_supported(h_pos.shape[0], d, self.nhead)):
            return ops.qkv_attention(h_pos, lin.weight_image(W, mode='bf16'), b, seg.off, kv_seg,
                                     seg.max_len, self.nhead, mode='bf16')
        if val_has_pos:
            qkv = linear(h_pos, W, b)                                 # (N, 3d): [q | k | v]
            q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
        else:
            qk = linear(h_pos, W, b[:2 * d], rows=(0, 2 * d))         # [q | k]
            q, k = qk[:, :d], qk[:, d:]
            v = linear(h_nopos, W, b[2 * d:], rows=(2 * d, 3 * d))
        o = ops.attention(q, k, v, seg.off, seg.off, kv_seg, seg.max_len, self.nhead)
        return o

    def takes_side(self, x, pos):
        """True if forward_packed can also write another LayerNorm of its input x (``side``)
        from its fused norm1 -> in_proj launch."""
        n, d = x.shape
        return (self.normalize_before and self.sa_val_has_pos_emb and pos is not None
                and ln_fusable(n, 3 * d, d))

    def wants_h1(self, x):
        """True if forward_packed takes a precomputed norm1(x) + pos (``h1``): pre-norm, values
        with pos, and norm1 not folded into the in_proj GEMM."""
        n, d = x.shape
        return (self.normalize_before and self.sa_val_has_pos_emb
                and not ln_fusable(n, 3 * d, d))

    def forward_packed(self, x, pos, seg: Segments, pending_bias=None, h1=None, side=None):
        """x (N_tot, d) packed clouds -> (x, pending bias) (forward_pre, transformers.py:183-244).

        Every residual GEMM adds its Linear's bias and the residual in its epilogue, so each
        LayerNorm only reads x (no in-place bias pass writing x back); ``pending_bias`` (a
        bias still to be added to x by the first LayerNorm) is accepted for callers that
        defer one, and the returned pending bias is None."""
        if not self.normalize_before:
            return self._forward_post(x, pos, seg, pending_bias), None
        n, d = x.shape
        # LayerNorm (+ pos) folded into the next GEMM where that GEMM supports it
        # (linear_ln): the norm output is never written
        fuse_in = ln_fusable(n, 3 * d, d)
        # self-attention, shared weights for src and tgt (:193-210)
        if fuse_in and self.sa_val_has_pos_emb and pending_bias is None:
            o = self._attend(self.self_attn, None, None, True, seg, seg.self_seg,
                             ln=(x, self.norm1, pos), side=side)
            side = None
        elif h1 is not None:              # norm1(x) + pos from the previous layer's output norm
            assert pending_bias is None and self.sa_val_has_pos_emb
            o = self._attend(self.self_attn, h1, None, True, seg, seg.self_seg)
        else:
            if side is not None:
                ops.layernorm(x, side[0].weight, side[0].bias, side[0].eps, out=side[1])
                side = None
            h = ops.layernorm(x, self.norm1.weight, self.norm1.bias, self.norm1.eps, add=pos,
                              pre_bias=pending_bias)
            h0 = None if self.sa_val_has_pos_emb else ops.layernorm(
                x, self.norm1.weight, self.norm1.bias, self.norm1.eps)
            o = self._attend(self.self_attn, h, h0, self.sa_val_has_pos_emb, seg, seg.self_seg)
        x = linear(o, self.self_attn.out_proj.weight, self.self_attn.out_proj.bias, residual=x)
        # cross-attention, both directions at once (:212-229)
        if fuse_in and self.ca_val_has_pos_emb:
            o = self._attend(self.multihead_attn, None, None, True, seg, seg.cross_seg,
                             ln=(x, self.norm2, pos))
        else:
            h = ops.layernorm(x, self.norm2.weight, self.norm2.bias, self.norm2.eps, add=pos)
            h0 = None if self.ca_val_has_pos_emb else ops.layernorm(
                x, self.norm2.weight, self.norm2.bias, self.norm2.eps)
            o = self._attend(self.multihead_attn, h, h0, self.ca_val_has_pos_emb, seg,
                             seg.cross_seg)
        x = linear(o, self.multihead_attn.out_proj.weight, self.multihead_attn.out_proj.bias,
                   residual=x)
        # position-wise feed-forward (:231-238): one launch where supported (ops.ffn: the
        # hidden activations stay on chip), else linear_ln (or layernorm + linear) then linear
        if lin.MODE == 'f16x3' and ops.ffn_supported(n, d, self.linear1.out_features):
            return ops.ffn(x, self.norm3, lin.weight_image(self.linear1.weight, mode='f16x3'),
                           self.linear1.bias, lin.weight_image(self.linear2.weight, mode='ffn2'),
                           self.linear2.bias, self._ffn_bound()), None
        h = linear_ln(x, self.norm3, self.linear1.weight, self.linear1.bias, act=ops.ACT_RELU)
        return linear(h, self.linear2.weight, self.linear2.bias, residual=x), None

    def _ffn_bound(self):
        """{max_j ||linear1.weight[j]||_2, max_j |linear1.bias[j]|} on the device (the fused
        feed-forward kernel's hidden-value scale, ops.ffn), rebuilt when either tensor changes."""
        w, b = self.linear1.weight, self.linear1.bias
        key = (w.data_ptr(), w._version, b.data_ptr(), b._version)
        st = self.__dict__.get('_ffn_bound_cache')
        if st is None or st[0] != key:
            with torch.no_grad():
                bound = torch.stack([w.detach().norm(dim=1).max(),
                                     b.detach().abs().max()]).float().contiguous()
            st = (key, bound)
            self.__dict__['_ffn_bound_cache'] = st          # not a parameter / buffer
            ops.note_state(bound)
        return st[1]

    def _forward_post(self, x, pos, seg: Segments, pending_bias=None):
        """forward_post (transformers.py:109-181): each sub-block's residual sum is formed in
        its output GEMM's epilogue, then LayerNorm'd; the norm1 output is also written with the
        positional embedding added (the cross-attention's q / k input, :139-147). Both
        directions of each attention run in one launch, reading the same pre-update rows
        like the reference's simultaneous src / tgt update."""
        assert pending_bias is None          # only the pre-norm path defers a bias
        h = ops.add(x, pos)                                       # with_pos_embed (:121-124)
        o = self._attend(self.self_attn, h, x, self.sa_val_has_pos_emb, seg, seg.self_seg)
        t = linear(o, self.self_attn.out_proj.weight, self.self_attn.out_proj.bias, residual=x)
        x = ops.layernorm(t, self.norm1.weight, self.norm1.bias, self.norm1.eps)       # :127
        h = ops.layernorm(t, self.norm1.weight, self.norm1.bias, self.norm1.eps, add=pos)
        o = self._attend(self.multihead_attn, h, x, self.ca_val_has_pos_emb, seg, seg.cross_seg)
        t = linear(o, self.multihead_attn.out_proj.weight, self.multihead_attn.out_proj.bias,
                   residual=x)
        x = ops.layernorm(t, self.norm2.weight, self.norm2.bias, self.norm2.eps)       # :163
        h = linear(x, self.linear1.weight, self.linear1.bias, act=ops.ACT_RELU)        # :167-169
        t = linear(h, self.linear2.weight, self.linear2.bias, residual=x)
        return ops.layernorm(t, self.norm3.weight, self.norm3.bias, self.norm3.eps)


class TransformerCrossEncoder(nn.Module):
    """transformers.py:18-59 with return_intermediate=True semantics."""

    def __init__(self, cross_encoder_layer, num_layers, norm=None, return_intermediate=False):
        super().__init__()
        self.layers = nn.ModuleList([copy.deepcopy(cross_encoder_layer) for _ in range(num_layers)])
        self.num_layers = num_layers
        self.norm = norm
        self.return_intermediate = return_intermediate

    def forward_packed(self, x, pos, seg: Segments):
        """-> (L, N_tot, d) normalised intermediates (or (1, N_tot, d))."""
        L = len(self.layers)
        n, d = x.shape
        inter = torch.empty((L if self.return_intermediate else 1, n, d), dtype=x.dtype,
                            device=x.device)
        x = x.clone()                      # the residual stream is updated in place
        pending = None
        h1 = side = None
        for l, layer in enumerate(self.layers):
            x, pending = layer.forward_packed(x, pos, seg, pending, h1=h1, side=side)
            h1 = side = None
            if self.return_intermediate or l == L - 1:
                nxt = self.layers[l + 1] if l + 1 < L else None
                if (nxt is not None and self.norm is not None and pending is None
                        and nxt.takes_side(x, pos) and self.norm.eps == nxt.norm1.eps):
                    # this layer's output norm is written by the next layer's fused
                    # norm1 -> in_proj launch (same rows, same statistics)
                    side = (self.norm, inter[l if self.return_intermediate else 0])
                elif (nxt is not None and self.norm is not None and pending is None
                        and nxt.wants_h1(x) and self.norm.eps == nxt.norm1.eps):
                    # this layer's output norm and the next layer's norm1 (+ pos): one pass
                    _, h1 = ops.layernorm_dual(x, self.norm, nxt.norm1, add_b=pos,
                                               out_a=inter[l if self.return_intermediate else 0])
                else:
                    self._norm(x, pending, inter[l if self.return_intermediate else 0])
                pending = None
        return inter

    def _norm(self, x, pending, out):
        if self.norm is None:
            if pending is not None:
                x.add_(pending)
            out.copy_(x)
            return out
        return ops.layernorm(x, self.norm.weight, self.norm.bias, self.norm.eps,
                             pre_bias=pending, out=out)


class PositionEmbeddingCoordsSine(nn.Module):
    """position_embedding.py:8-49 on fgr_sine_pos_embed."""

    def __init__(self, n_dim=1, d_model=256, temperature=10000, scale=None):
        super().__init__()
        if n_dim != 3:
            raise NotImplementedError('coordinates are 3-D in this path')
        self.n_dim, self.d_model, self.temperature = n_dim, d_model, temperature
        self.scale = 1.0 if scale is None else scale

    def forward(self, xyz):
        return ops.sine_pos_embed(xyz, self.d_model, self.temperature, self.scale)
