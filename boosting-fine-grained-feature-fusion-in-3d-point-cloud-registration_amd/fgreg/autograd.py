"""Differentiable ops of the training forward (train.py's
``training_step`` -> ``loss.backward()`` -> ``clip_grad_norm_``, trainer.py:110-125).

Each op is a ``torch.autograd.Function`` whose forward AND backward run in libfgreg:

* ``linear_t``      y = act(x W^T + b) (+ residual): forward on fgr_gemm_f16x3 (bf16 in the
                    bf16 mode); backward dX = dY W on the same GEMM with the transposed weight
                    image, dW = dY^T X on the GEMM with X as the (transposed) weight image,
                    db = fgr_colsum(dY);
* ``kpconv_t``      the KPConv gather-weight + weight product (finegrained_kpconv_blocks.py:
                    265-399 up to the division, which the following norm applies): backward
                    d_wf = dout W2^T (GEMM), dW = wf^T dout (GEMM; wf regathered, not kept),
                    dx = fgr_kpconv_scatter(d_wf) (the scatter-add of the reference's
                    ``gather(method=2)``, :66-97, as a gather over the table's inverse);
* ``segnorm_t``     per-(segment, channel) normalisation with batch statistics
                    (fgr_segnorm_*): InstanceNorm per cloud (BatchNormBlock, :462-518) and the
                    Res2Net BatchNorm1d in train() (res2net.py:126-159, one segment + affine,
                    running statistics updated like nn.BatchNorm1d);
* ``layernorm_t``   nn.LayerNorm (+ the positional add) -> fgr_layernorm / fgr_layernorm_bwd;
* ``attention_t``   the packed-segment MHA core on the fused QKV tensor -> fgr_attention_f16x3
                    forward, fgr_attention_bwd backward;
* ``max_pool_t``    max_pool (:125-141) -> fgr_max_pool / fgr_max_pool_bwd;
* ``corr_attention_t`` the CorrespondenceDecoder head's simple_attention (finegrained_regtr.py:
                    328-363) -> fgr_corr_attention / fgr_corr_attention_bwd.
Both scatters (KPConv dx, max-pool dx) read the neighbour table's CSR inverse (fgr_nbr_inverse,
built once per table): no floating-point atomics anywhere, so a backward pass is bit-for-bit
reproducible.
Elementwise glue between them (ReLU masks, the bottleneck's LeakyReLU(x + shortcut),
concatenation) is torch on the same device. No CPU path: every op raises on host tensors.
"""
import math
import os

import torch
import torch.nn.functional as F

from . import _lib, ops
from . import linear as lin
from .linear import linear
from .ops import ACT_LEAKY, ACT_NONE, ACT_RELU, _c, _dev, _ptr, _stream


def colsum(x: torch.Tensor) -> torch.Tensor:
    """Column sums of a (n, c) tensor with unit column stride (fgr_colsum, fp64 partials)."""
    _dev(x)
    assert x.dim() == 2 and x.stride(1) == 1 and x.dtype == torch.float32
    n, c = x.shape
    out = torch.empty((c,), dtype=torch.float32, device=x.device)
    L = _lib.load()
    nb = _lib.ws_size('fgr_colsum_workspace', n, c)
    ws = torch.empty(nb, dtype=torch.uint8, device=x.device)
    _lib.check(L.fgr_colsum(_ptr(x), n, c, max(x.stride(0), c), _ptr(out), _ptr(ws), nb,
                            _stream()), 'fgr_colsum')
    return out


_WGRAD = os.environ.get('FGREG_WGRAD', '1') != '0'     # 0: dW on the generic GEMM (A/B)
_ATTN_LSE = os.environ.get('FGREG_ATTN_LSE', '1') != '0'  # 0: the backward recomputes it (A/B)


def _wgrad_ok(t):
    return t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0


def wgrad(a: torch.Tensor, b: torch.Tensor, bias_grad=False):
    """a^T b (m, n) of row-major a (rows, m) and b (rows, n): the weight gradient dW = dY^T X
    (and with bias_grad, also the column sums of a: (dW, db)). f16x3 mode:
    fgr_gemm_f16x3_wgrad straight from both activations (widths padded to a multiple of 4),
    db in the same launches; otherwise the GEMM of the transposed copy of a with b as its
    (transposed) weight image, and fgr_colsum."""
    rows, m = a.shape
    n = b.shape[1]
    if not (_WGRAD and lin.MODE == 'f16x3'):
        dw = linear(a.t().contiguous(), b, transpose=True, cache=False)
        return (dw, colsum(a.contiguous())) if bias_grad else dw
    if m % 4 or n % 4:
        # narrow operands (a 1- or 3-output head, KPConv's first layer: 15 x 1 inputs): zero
        # columns up to a multiple of 4, then the kernel's result sliced (exact: zero columns
        # add nothing and the per-column scales are independent)
        pad = lambda t, k: t if k % 4 == 0 else F.pad(t, (0, (-k) % 4))      # noqa: E731
        r = wgrad(pad(a, m), pad(b, n), bias_grad)
        return (r[0][:m, :n].contiguous(), r[1][:m].contiguous()) if bias_grad else r[:m, :n].contiguous()
    _dev(a, b)
    if not _wgrad_ok(a):
        a = a.contiguous().clone() if a.is_contiguous() else a.contiguous()
    if not _wgrad_ok(b):
        b = b.contiguous().clone() if b.is_contiguous() else b.contiguous()
    out = torch.empty((m, n), dtype=torch.float32, device=a.device)
    db = torch.empty((m,), dtype=torch.float32, device=a.device) if bias_grad else None
    nb = _lib.ws_size('fgr_gemm_wgrad_workspace', rows, m, n, int(bias_grad))
    ws = ops._workspace(a.device, nb) if nb else None
    t0 = ops._begin('wgrad', (m, n, rows))       # (M, N, K) of the table: K = the rows
    _lib.check(_lib.load().fgr_gemm_f16x3_wgrad(
        _ptr(a), a.stride(0), _ptr(b), b.stride(0), rows, m, n, _ptr(out), out.stride(0), _ptr(db),
        _ptr(ws), nb, _stream()), 'fgr_gemm_f16x3_wgrad')
    ops._end('wgrad', t0, 2 * m * n * rows)
    return (out, db) if bias_grad else out


def _relu_mask(dy, y):
    """dy where the ReLU output y > 0, else 0 (one elementwise launch)."""
    return torch.ops.aten.threshold_backward(dy, y, 0)


# ------------------------------------------------------------------------------------------
# dense layers
# ------------------------------------------------------------------------------------------
class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, residual, act, cache=True):
        assert act in (ACT_NONE, ACT_RELU)
        y = linear(x, w, b, act=act, residual=residual, cache=cache)
        ctx.mode = lin.MODE          # the backward's products run in the forward's mode
        ctx.act, ctx.has_b, ctx.has_r, ctx.cache = act, b is not None, residual is not None, cache
        ctx.save_for_backward(x, w, y if act == ACT_RELU else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        dy = dy.contiguous()
        if ctx.act == ACT_RELU:
            dy = _relu_mask(dy, y)
        dx = dw = db = None
        want_db = ctx.has_b and ctx.needs_input_grad[2]
        with lin.mode_scope(ctx.mode):
            if ctx.needs_input_grad[0]:
                dx = linear(dy, w, transpose=True, tag='bwd_dx', cache=ctx.cache)   # dY W
            if ctx.needs_input_grad[1]:
                if want_db:                                     # dY^T X and the column sums
                    dw, db = wgrad(dy, x, bias_grad=True)
                else:
                    dw = wgrad(dy, x)                                               # dY^T X
        if want_db and db is None:
            db = colsum(dy)
        dres = dy if ctx.has_r and ctx.needs_input_grad[3] else None
        return dx, dw, db, dres, None, None


def linear_t(x, w, b=None, act=ACT_NONE, residual=None, cache=True):
    """act(x W^T + b) (+ residual after the activation is NOT supported: residual is added
    before, as the transformer's out-projection / FFN epilogues use it with act NONE).
    cache=False: w is an activation (a new tensor every step), its image is not cached."""
    assert residual is None or act == ACT_NONE
    return _LinearFn.apply(x, w, b, residual, act, cache)


# ------------------------------------------------------------------------------------------
# KPConv
# ------------------------------------------------------------------------------------------
def nbr_inverse(idx: torch.Tensor, ns: int):
    """-> (start (ns + 1,), pos (nq * width,), ent (nq * width,)) int32: the CSR inverse of the
    neighbour table idx over ns support rows (fgr_nbr_inverse: per support row, the entries
    q * width + h naming it in ascending order). Cached on the table tensor (a kpconv_meta
    table is shared by every conv / pool of its level and never written in place)."""
    _dev(idx)
    idx = _c(idx, torch.int64)
    cache = getattr(idx, '_fgr_inverse', None)
    if cache is not None and cache[0] == (ns, idx._version):
        return cache[1]
    nq, width = idx.shape
    dev = idx.device
    start = torch.empty(ns + 1, dtype=torch.int32, device=dev)
    pos = torch.empty(max(nq * width, 1), dtype=torch.int32, device=dev)
    ent = torch.empty_like(pos)
    L = _lib.load()
    nb = _lib._sz(0)
    _lib.check(L.fgr_nbr_inverse_workspace(nq, width, ns, nb), 'fgr_nbr_inverse_workspace')
    ws = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=dev)
    _lib.check(L.fgr_nbr_inverse(_ptr(idx), nq, width, ns, _ptr(start), _ptr(pos), _ptr(ent),
                                 _ptr(ws), nb.value, _stream()), 'fgr_nbr_inverse')
    res = (start, pos, ent)
    idx._fgr_inverse = ((ns, idx._version), res)
    return res


def kpconv_scatter(q, s, idx, dwf, kp, extent):
    """dx (ns, cin) of the KPConv gather from d_wf (nq, K * cin): fgr_kpconv_scatter over the
    table's inverse (deterministic: each support row adds its entries in CSR order)."""
    _dev(q, s, idx, dwf, kp)
    nq, width = idx.shape
    ns = s.shape[0]
    K = kp.shape[0]
    cin = dwf.shape[1] // K
    start, pos, _ = nbr_inverse(idx, ns)
    dx = torch.empty((ns, cin), dtype=torch.float32, device=dwf.device)
    L = _lib.load()
    nb = _lib.ws_size('fgr_kpconv_scatter_workspace', nq, width, cin)
    ws = ops._workspace(dwf.device, nb)         # grow-only scratch, not a fresh buffer per call
    _lib.check(L.fgr_kpconv_scatter(
        _ptr(_c(q, torch.float32)), _ptr(_c(s, torch.float32)), nq, ns, _ptr(_c(idx, torch.int64)),
        width, _ptr(dwf), cin, _ptr(_c(kp, torch.float32)), K, float(extent), _ptr(start),
        _ptr(pos), _ptr(dx), _ptr(ws), nb, _stream()), 'fgr_kpconv_scatter')
    return dx


class _KPConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, q, s, idx, kp, extent):
        wf, nnorm = ops.kpconv_gather(q, s, idx, x, kp, extent)
        out = linear(wf.view(wf.shape[0], -1), W, transpose=True)
        ctx.mode = lin.MODE
        ctx.extent = float(extent)
        ctx.save_for_backward(x, W, q, s, idx, kp)
        ctx.mark_non_differentiable(nnorm)
        return out, nnorm

    @staticmethod
    def backward(ctx, dout, _dnnorm):
        x, W, q, s, idx, kp = ctx.saved_tensors
        dout = dout.contiguous()
        nq = q.shape[0]
        K, cin, cout = W.shape
        dx = dW = None
        with lin.mode_scope(ctx.mode):
            if ctx.needs_input_grad[0]:
                dwf = linear(dout, W, transpose='flat', tag='bwd_dwf')       # (nq, K * cin)
                dx = kpconv_scatter(q, s, idx, dwf, kp, ctx.extent)
            if ctx.needs_input_grad[1]:
                wf, _ = ops.kpconv_gather(q, s, idx, x, kp, ctx.extent)      # regathered
                dW = wgrad(wf.view(nq, K * cin), dout).view(K, cin, cout)   # wf^T dout
        return dx, dW, None, None, None, None, None


def kpconv_t(conv, q, s, idx, x):
    """-> (sum_k WF_k W_k (Nq, Cout), nnorm (Nq,)) of a fgreg.backbone.KPConv, differentiable in
    x and the weights (kernel points are fixed, as requires_grad=False in the reference)."""
    return _KPConvFn.apply(x, conv.weights, q, s, idx, conv.kernel_points, conv.KP_extent)


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, idx):
        ctx.save_for_backward(x, idx)
        return ops.max_pool(x, idx)

    @staticmethod
    def backward(ctx, dy):
        x, idx = ctx.saved_tensors
        x, dy = x.contiguous(), dy.contiguous()
        ns, c = x.shape
        nq, width = idx.shape
        start, _, ent = nbr_inverse(idx, ns)
        dx = torch.empty_like(x)
        L = _lib.load()
        nb = _lib._sz(0)
        _lib.check(L.fgr_max_pool_bwd_workspace(nq, c, nb), 'fgr_max_pool_bwd_workspace')
        ws = torch.empty(nb.value, dtype=torch.uint8, device=x.device)
        _lib.check(L.fgr_max_pool_bwd(_ptr(x), ns, c, _ptr(idx.contiguous()), nq, width, _ptr(dy),
                                      _ptr(start), _ptr(ent), _ptr(dx), _ptr(ws), nb.value,
                                      _stream()), 'fgr_max_pool_bwd')
        return dx, None


def max_pool_t(x, idx):
    return _MaxPoolFn.apply(x, idx)


# ------------------------------------------------------------------------------------------
# normalisation
# ------------------------------------------------------------------------------------------
def _seg_ws(max_len, c, n_seg, extra=0, device=None):
    nb = _lib.ws_size('fgr_segnorm_workspace', max_len, c, n_seg)
    return torch.empty(nb + extra, dtype=torch.uint8, device=device)


class _SegNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, residual, row_div, seg_off, lengths, act, post_act, eps, stats):
        x = _c(x, torch.float32)
        _dev(x, gamma, beta, residual, row_div, seg_off)
        n, c = x.shape
        n_seg = len(lengths)
        max_len = max(lengths) if n_seg else 0
        assert seg_off.numel() == n_seg + 1 and sum(lengths) == n
        L = _lib.load()
        mean = torch.empty((n_seg, c), dtype=torch.float32, device=x.device)
        rstd, var = torch.empty_like(mean), torch.empty_like(mean)
        ws = _seg_ws(max_len, c, n_seg, device=x.device)
        rd = _c(row_div, torch.float32) if row_div is not None else None
        res = _c(residual, torch.float32) if residual is not None else None
        y = torch.empty_like(x)
        _lib.check(L.fgr_segnorm_fwd(_ptr(x), n, c, _ptr(seg_off), n_seg, max_len, _ptr(rd),
                                     float(eps), _ptr(mean), _ptr(rstd), _ptr(var), _ptr(gamma),
                                     _ptr(beta), act, _ptr(res), post_act, _ptr(y), _ptr(ws),
                                     ws.numel(), _stream()), 'fgr_segnorm_fwd')
        if stats is not None:
            stats.append((mean, var, n))
        ctx.meta = (n, c, n_seg, max_len, act, post_act, residual is not None, gamma is not None)
        ctx.save_for_backward(x, gamma, beta, rd, seg_off, mean, rstd, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma, beta, rd, seg_off, mean, rstd, y = ctx.saved_tensors
        n, c, n_seg, max_len, act, post_act, has_r, affine = ctx.meta
        dy = _c(dy, torch.float32)
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if has_r else None
        dg = torch.empty((c,), dtype=torch.float32, device=x.device) if affine else None
        db = torch.empty_like(dg) if affine else None
        ws = _seg_ws(max_len, c, n_seg, extra=8 * n_seg * c, device=x.device)
        _lib.check(_lib.load().fgr_segnorm_bwd(
            _ptr(x), n, c, _ptr(seg_off), n_seg, max_len, _ptr(rd), _ptr(mean), _ptr(rstd),
            _ptr(gamma), _ptr(beta), act, int(has_r), post_act, _ptr(y), _ptr(dy), _ptr(dx),
            _ptr(dres), _ptr(dg), _ptr(db), _ptr(ws), ws.numel(), _stream()), 'fgr_segnorm_bwd')
        return dx, dg, db, dres, None, None, None, None, None, None, None


def segnorm_t(x, off, lengths, row_div=None, act=ACT_NONE, residual=None, post_act=ACT_NONE,
              gamma=None, beta=None, eps=1e-5, stats=None):
    """post(act((x / row_div - mean) rstd (* gamma + beta)) + residual), statistics per segment
    of the current batch; ``stats`` (a list) receives (mean, biased var, rows)."""
    return _SegNormFn.apply(x, gamma, beta, residual, row_div, off, list(lengths), act, post_act,
                            eps, stats)


_BN_OFF = {}


def batchnorm_t(bn, x, act=ACT_NONE, residual=None, post_act=ACT_NONE):
    """nn.BatchNorm1d ``bn`` in training mode on (N, C) rows (batch statistics over all rows,
    running statistics updated in place as torch does: momentum, unbiased variance)."""
    n = x.shape[0]
    key = (n, x.device)
    off = _BN_OFF.get(key)
    if off is None:                       # [0, n] on the device, made once per row count
        if len(_BN_OFF) > 256:
            _BN_OFF.clear()
        off = _BN_OFF[key] = ops.offsets([n], x.device)
    stats = [] if bn.track_running_stats else None
    y = segnorm_t(x, off, [n], act=act, residual=residual, post_act=post_act, gamma=bn.weight,
                  beta=bn.bias, eps=bn.eps, stats=stats)
    if stats:
        mean, var, rows = stats[0]
        with torch.no_grad():
            bn.num_batches_tracked.add_(1)
            m = bn.momentum if bn.momentum is not None else 1.0 / float(bn.num_batches_tracked)
            unbiased = var[0] * (rows / max(rows - 1, 1))
            bn.running_mean.mul_(1 - m).add_(mean[0], alpha=m)
            bn.running_var.mul_(1 - m).add_(unbiased, alpha=m)
    return y


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, add, eps):
        x = _c(x, torch.float32)
        y = ops.layernorm(x, gamma, beta, eps, add=add)
        ctx.eps = float(eps)
        ctx.has_add = add is not None
        ctx.save_for_backward(x, gamma)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma = ctx.saved_tensors
        dy = _c(dy, torch.float32)
        n, d = x.shape
        dx = torch.empty_like(x)
        dgb = torch.empty((2 * d,), dtype=torch.float32, device=x.device)
        L = _lib.load()
        nb = _lib._sz(0)
        _lib.check(L.fgr_layernorm_bwd_workspace(n, d, nb), 'fgr_layernorm_bwd_workspace')
        ws = torch.empty(nb.value, dtype=torch.uint8, device=x.device)
        _lib.check(L.fgr_layernorm_bwd(_ptr(x), n, d, _ptr(gamma.contiguous()), ctx.eps, _ptr(dy),
                                       _ptr(dx), _ptr(dgb), _ptr(ws), nb.value, _stream()),
                   'fgr_layernorm_bwd')
        dadd = dy if ctx.has_add and ctx.needs_input_grad[3] else None
        return dx, dgb[:d], dgb[d:], dadd, None


def layernorm_t(x, norm, add=None):
    """nn.LayerNorm ``norm`` of x (+ add, e.g. the positional embedding)."""
    return _LayerNormFn.apply(x, norm.weight, norm.bias, add, norm.eps)


# ------------------------------------------------------------------------------------------
# attention
# ------------------------------------------------------------------------------------------
def attn_drop_mask(seed, p, head, q_rows, k_rows):
    """The attention-weight dropout mask of fgr_attention_f16x3_drop / fgr_attention_bwd_drop
    (common.h attn_drop_hash) for one head over packed query / key rows -> bool (len(q_rows),
    len(k_rows)), True = dropped. Restated with numpy uint32 arithmetic (tests)."""
    import numpy as np
    m32 = lambda v: v & np.uint64(0xFFFFFFFF)
    q = np.asarray(q_rows, dtype=np.uint64)[:, None]
    k = np.asarray(k_rows, dtype=np.uint64)[None, :]
    x = np.uint64(seed & 0xFFFFFFFF) ^ m32(np.uint64(head) * np.uint64(0x9E3779B9))
    x = x ^ m32(q * np.uint64(0x85EBCA6B))
    x = m32((x ^ (x >> np.uint64(16))) * np.uint64(0x7FEB352D))
    x = x ^ m32(k * np.uint64(0xC2B2AE35))
    x = m32((x ^ (x >> np.uint64(15))) * np.uint64(0x846CA68B))
    x = x ^ (x >> np.uint64(16))
    thresh = min(int(p * 4294967296.0), 4294967295)
    return x < np.uint64(thresh)


class _AttentionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, off, kv_seg, max_len, nhead, p=0.0, seed=0):
        qkv = _c(qkv, torch.float32)
        d = qkv.shape[1] // 3
        q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
        # the forward's log2-sum-exp per (row, head) for the backward (fgr_attention_*_train)
        lse = (torch.empty((qkv.shape[0], nhead), dtype=torch.float32, device=qkv.device)
               if _ATTN_LSE and ops.attention_lse_ok(q, k, v, nhead) else None)
        o = ops.attention(q, k, v, off, off, kv_seg, max_len, nhead,
                          dropout=(seed, p) if p > 0.0 else None, lse=lse)
        ctx.meta = (d, int(max_len), int(nhead), float(p), int(seed))
        ctx.save_for_backward(qkv, o, off, kv_seg, lse)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, off, kv_seg, lse = ctx.saved_tensors
        d, max_len, nhead, p_drop, seed = ctx.meta
        do = _c(do, torch.float32)
        n = qkv.shape[0]
        dh = d // nhead
        dqkv = torch.empty_like(qkv)
        L = _lib.load()
        nb = _lib._sz(0)
        n_seg = off.numel() - 1
        if lse is not None:
            # lse / D and the f16x3 kernels' tile images (fgr_attention_bwd_train)
            _lib.check(L.fgr_attention_bwd_train_workspace(n, n_seg, n, n_seg, nhead, dh, nb),
                       'fgr_attention_bwd_train_workspace')
        else:
            _lib.check(L.fgr_attention_bwd_workspace(n, nhead, nb), 'fgr_attention_bwd_workspace')
        ws = ops._workspace(qkv.device, nb.value)
        p, dp, ld = qkv.data_ptr(), dqkv.data_ptr(), qkv.stride(0)
        args = (p, ld, p + 4 * d, ld, p + 8 * d, ld, _ptr(o), o.stride(0), _ptr(do), do.stride(0),
                dp, ld, dp + 4 * d, ld, dp + 8 * d, ld, _ptr(off), _ptr(off), _ptr(kv_seg), n_seg,
                n_seg, n, max_len, max_len, nhead, dh, float(math.sqrt(1.0 / float(dh))),
                _ptr(ws), nb.value)
        if lse is not None:
            _lib.check(L.fgr_attention_bwd_train(*args, seed & 0xFFFFFFFF, p_drop, _ptr(lse), n,
                                                 _stream()), 'fgr_attention_bwd_train')
        elif p_drop > 0.0:
            _lib.check(L.fgr_attention_bwd_drop(*args, seed & 0xFFFFFFFF, p_drop, _stream()),
                       'fgr_attention_bwd_drop')
        else:
            _lib.check(L.fgr_attention_bwd(*args, _stream()), 'fgr_attention_bwd')
        return dqkv, None, None, None, None, None, None


def attention_t(qkv, off, kv_seg, max_len, nhead, dropout=0.0):
    """Packed-segment MHA core on a fused (N, 3d) [q | k | v] tensor: query segment i attends
    to key segment kv_seg[i] (self- or cross-attention over one segmentation). ``dropout`` > 0:
    nn.MultiheadAttention's attention-weight dropout in training, the mask seeded from torch's
    CPU generator (torch.manual_seed reproduces a step)."""
    if dropout > 0.0:
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
        return _AttentionFn.apply(qkv, off, kv_seg, max_len, nhead, float(dropout), seed)
    return _AttentionFn.apply(qkv, off, kv_seg, max_len, nhead)


class _CorrAttentionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, xyz, q_off, kv_seg, v_off, max_len, scale):
        q, k = _c(q, torch.float32), _c(k, torch.float32)
        corr = ops.corr_attention(q, k, xyz, q_off, q_off, kv_seg, v_off, max_len, scale)
        ctx.meta = (int(max_len), float(scale))
        ctx.save_for_backward(q, k, xyz, q_off, kv_seg, v_off)
        return corr

    @staticmethod
    def backward(ctx, dcorr):
        q, k, xyz, q_off, kv_seg, v_off = ctx.saved_tensors
        max_len, scale = ctx.meta
        dcorr = _c(dcorr, torch.float32)
        n, d = q.shape
        dq = torch.zeros_like(q)
        dk = torch.zeros_like(k)
        L = _lib.load()
        nb = _lib._sz(0)
        _lib.check(L.fgr_corr_attention_bwd_workspace(n, nb), 'fgr_corr_attention_bwd_workspace')
        ws = torch.empty(nb.value, dtype=torch.uint8, device=q.device)
        n_seg = q_off.numel() - 1
        _lib.check(L.fgr_corr_attention_bwd(
            _ptr(q), q.stride(0), _ptr(k), k.stride(0), _ptr(_c(xyz, torch.float32)), _ptr(dcorr),
            _ptr(dq), dq.stride(0), _ptr(dk), dk.stride(0), _ptr(q_off), _ptr(q_off), _ptr(kv_seg),
            _ptr(v_off), n_seg, n_seg, n, max_len, max_len, d, scale, _ptr(ws), nb.value,
            _stream()), 'fgr_corr_attention_bwd')
        return dq, dk, None, None, None, None, None, None


def corr_attention_t(q, k, xyz, seg, scale):
    """CorrespondenceDecoder.simple_attention (finegrained_regtr.py:328-363) over the (layer,
    cloud) segments of ``seg.layer_tables``: softmax(q.k scale) weighted partner coordinates,
    differentiable in q and k (fgr_corr_attention / fgr_corr_attention_bwd)."""
    q_off, kv_seg, v_off = seg.layer_tables
    return _CorrAttentionFn.apply(q, k, xyz, q_off, kv_seg, v_off, seg.max_len, scale)


def leaky(x):
    return F.leaky_relu(x, 0.1)
