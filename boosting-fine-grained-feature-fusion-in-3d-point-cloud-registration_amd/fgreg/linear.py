"""Dense layers of the forward (every Linear / KPConv-weight product goes through
``linear()``) on the GPU, in one of two precision modes (``set_mode``, or
``fgreg.set_precision``):

* ``f16x3`` (default): fgr_gemm_f16x3, the fp32-accurate scaled split-fp16 MFMA GEMM (operands
  scaled by per-row powers of two and split into two fp16 terms, three term products per
  step: <= ~3 * 2^-22 relative per product) -- meets the 1e-4 parity bar on every fixture.
* ``bf16``: fgr_gemm_bf16, one bf16 MFMA product per fp32 product (operands rounded to bf16,
  fp32 accumulation: ~2^-9 relative per product) -- the BASELINE configs[4] (3DLoMatch)
  compute mode, 3x fewer matrix-core cycles than f16x3; tolerance in DESIGN.md.
Weight images are built once and cached against the fp32 tensor's identity, data pointer
and version (a checkpoint load, .to() or in-place update invalidates the cache). There is no
library / PyTorch GEMM fallback: a shape the kernels reject raises.
"""
import os

import numpy as np
import torch

from . import _lib
from . import ops
from .ops import ACT_NONE, _begin, _dev, _end, _ptr, _stream

MODES = ('f16x3', 'bf16')
MODE = 'f16x3'


def set_mode(mode):
    global MODE
    assert mode in MODES, mode
    MODE = mode


class mode_scope:  # noqa: N801 -- used as a context manager
    """``with mode_scope('f16x3'):`` runs the enclosed linear() calls in another mode (e.g.
    the pose-sensitive correspondence head of the bf16 forward in f16x3, regtr.py)."""

    def __init__(self, mode):
        assert mode is None or mode in MODES, mode
        self.mode, self.prev = mode, None

    def __enter__(self):
        global MODE
        self.prev, MODE = MODE, (self.mode or MODE)
        return self

    def __exit__(self, *exc):
        global MODE
        MODE = self.prev
        return False


class _Image:
    """Split image of W (n, k), element (i, j) at w2[i * sn + j * sk]: fgr_split_weights_h3
    (f16x3: two fp16 terms, per-row power-of-two scales) or fgr_split_weights_bf16. ``view``
    keeps w2 when it is a view of the source's storage (so a stale f16x3 image can be
    re-split in place by the batched refresh)."""
    __slots__ = ('img', 'n', 'k', 'sn', 'sk', 'src', 'version', 'ptr', 'mode', 'view')
    # 'ffn2': the fused feed-forward kernel's linear2 image (chunk-major, k-permuted f16x3,
    # fgr_split_weights_ffn2; ops.ffn)
    FN = {'f16x3': 'fgr_split_weights_h3', 'bf16': 'fgr_split_weights_bf16',
          'ffn2': 'fgr_split_weights_ffn2'}

    def __init__(self, mode, w2: torch.Tensor, n, k, sn, sk, src: torch.Tensor):
        L = _lib.load()
        fn = self.FN[mode]
        nb = _lib.ws_size(fn + '_bytes', n, k)
        self.img = torch.empty(nb, dtype=torch.uint8, device=w2.device)
        _lib.check(getattr(L, fn)(_ptr(w2), n, k, sn, sk, _ptr(self.img), _stream()), fn)
        self.n, self.k, self.sn, self.sk, self.mode = n, k, sn, sk, mode
        self.src, self.version, self.ptr = src, src._version, src.data_ptr()
        shares = w2.untyped_storage().data_ptr() == src.untyped_storage().data_ptr()
        self.view = w2 if shares else None


_CACHE = {}


def _valid(ent, w):
    return (ent is not None and ent.src is w and ent.version == w._version
            and ent.ptr == w.data_ptr())            # .to() / load_state_dict swap .data


# fgr_split_desc (include/fgreg.h): w, img, stride_n, stride_k, panel0, n, k
_DESC = np.dtype([('w', '<u8'), ('img', '<u8'), ('sn', '<i8'), ('sk', '<i8'), ('panel0', '<i8'),
                  ('n', '<i4'), ('k', '<i4')])
BATCH_REFRESH = os.environ.get('FGREG_SPLIT_BATCH', '1') != '0'


def _refresh_stale(device):
    """Re-split, in one launch (fgr_split_weights_h3_batch), every cached f16x3 image on
    ``device`` whose weight was updated in place (same storage, new version) -- after an
    optimizer step that is every weight the training step is about to use, so the step pays
    one launch instead of one per image. Returns the number refreshed."""
    stale = [e for e in _CACHE.values()
             if e.mode == 'f16x3' and e.view is not None and e.src.device == device
             and e.src._version != e.version and e.src.data_ptr() == e.ptr]
    if len(stale) < 2:
        return 0
    d = np.zeros(len(stale), dtype=_DESC)
    p0 = 0
    for i, e in enumerate(stale):
        d[i] = (e.view.data_ptr(), e.img.data_ptr(), e.sn, e.sk, p0, e.n, e.k)
        p0 += (e.n + 15) // 16
    dd = torch.frombuffer(bytearray(d.tobytes()), dtype=torch.uint8)
    dd = dd.pin_memory().to(device, non_blocking=True)
    # the images are rewritten in place: forwards still in flight on other streams (a
    # pipeline's core streams) read them, so the refresh waits for those first
    ops.wait_state_readers()
    _lib.check(_lib.load().fgr_split_weights_h3_batch(_ptr(dd), len(stale), p0, _stream()),
               'fgr_split_weights_h3_batch')
    for e in stale:
        e.version = e.src._version
    ops.note_state(*[e.img for e in stale])
    return len(stale)


def weight_image(w: torch.Tensor, transpose=False, tag=None, mode=None, cache=True, rows=None):
    """Split image of w in ``mode`` (default: the current MODE), cached unless ``cache`` is
    False (operands that change every call, e.g. the backward's activations). ``rows`` =
    (r0, r1) takes the row slice w[r0:r1] (e.g. the q|k and v blocks of an in_proj weight),
    cached against the parent tensor."""
    mode = mode or MODE
    ck = (id(w), transpose, tag, mode, rows)
    ent = _CACHE.get(ck) if cache else None
    if (BATCH_REFRESH and ent is not None and mode == 'f16x3' and ent.src is w
            and ent.ptr == w.data_ptr() and ent.version != w._version and ent.view is not None):
        _refresh_stale(w.device)          # this image and every other stale one, one launch
    if not _valid(ent, w):
        src = w
        if rows is not None:
            w = w[rows[0]:rows[1]]
        if transpose == 'flat':          # (..., k) as W[n = leading index][k = last index]
            w2 = w.reshape(-1, w.shape[-1]).contiguous()
            ent = _Image(mode, w2, w2.shape[0], w2.shape[1], w2.shape[1], 1, src)
        elif transpose:                  # (K, Cin, Cout) as W[n = cout][k = K*Cin + cin]
            w2 = w.reshape(-1, w.shape[-1]).contiguous()
            ent = _Image(mode, w2, w2.shape[1], w2.shape[0], 1, w2.shape[1], src)
        else:
            w2 = w.contiguous()
            ent = _Image(mode, w2, w2.shape[0], w2.shape[1], w2.shape[1], 1, src)
        if cache:
            _CACHE[ck] = ent
            ops.note_state(ent.img)
    return ent


def linear(x: torch.Tensor, w: torch.Tensor, bias=None, act=ACT_NONE, residual=None,
           transpose=False, tag=None, out=None, cache=True, rows=None) -> torch.Tensor:
    """act(A @ W^T + bias (+ residual)) with A = x and W = w (n, k), or w[r0:r1] for ``rows``
    = (r0, r1), or W = w.reshape(k, n).t() if transpose (e.g. KPConv weights (K, Cin, Cout)
    used as (K*Cin, Cout)), or W = w.reshape(-1, w.shape[-1]) if transpose == 'flat' (the
    backward's d_wf = dout W2^T). ACT_RELU_RES_LEAKY applies the residual after the ReLU:
    LeakyReLU_0.1(ReLU(A @ W^T + bias) + residual)."""
    if transpose == 'flat':
        k = w.shape[-1]
        n = w.numel() // k
    else:
        n = w.shape[-1] if transpose else w.shape[0]
        k = w.numel() // n if transpose else w.shape[1]
    if rows is not None:
        assert not transpose and 0 <= rows[0] < rows[1] <= n
        n = rows[1] - rows[0]
    assert x.dim() == 2 and x.shape[1] == k and x.dtype == torch.float32
    if not (x.is_cuda and w.is_cuda):
        _dev(x, w)
    if residual is not None:
        assert residual.shape == (x.shape[0], n) and residual.stride(1) == 1
    if bias is not None:
        assert bias.numel() == n and bias.is_contiguous()
    if x.shape[0] == 1 and x.stride(1) == 1 and x.stride(0) != k:
        x = x.as_strided(x.shape, (k, 1))      # a 1-row view's row stride is arbitrary
    if not (x.stride(1) == 1 and (k % 8 != 0 or (x.stride(0) % 4 == 0
                                                 and x.data_ptr() % 16 == 0))):
        x = x.contiguous()                 # the split kernels need 16-B aligned rows
        if k % 8 == 0 and x.data_ptr() % 16 != 0:
            x = x.clone()
    sw = weight_image(w, transpose, tag, MODE, cache=cache, rows=rows)
    m = x.shape[0]
    if out is None:
        out = torch.empty((m, n), dtype=torch.float32, device=x.device)
    L = _lib.load()
    t0 = _begin('gemm', (m, n, k))
    # split-K workspace where the dispatcher wants one (few rows, long K)
    nb = _lib.ws_size('fgr_gemm_workspace', m, n, k, 0 if MODE == 'f16x3' else 1)
    ws = ops._workspace(x.device, nb) if nb else None
    _lib.check(getattr(L, 'fgr_gemm_' + MODE + '_ws')(
        _ptr(x), x.stride(0), _ptr(sw.img), _ptr(out), out.stride(0), _ptr(bias),
        _ptr(residual), residual.stride(0) if residual is not None else 0, m, n, k, act,
        _ptr(ws), nb, _stream()), 'fgr_gemm_' + MODE)
    _end('gemm', t0, 2 * m * n * k)
    return out


# fgr_gemm_f16x3_ln where supported (False, or FGR_LN_FUSE=0: layernorm, then linear)
LN_FUSE = os.environ.get('FGR_LN_FUSE', '1') != '0'


def ln_fusable(m, n, k) -> bool:
    """True if LayerNorm -> Linear of an (m, k) input to n outputs runs as one launch
    (fgr_gemm_f16x3_ln: f16x3 mode, the row-stationary kernel's shapes)."""
    return (LN_FUSE and MODE == 'f16x3'
            and bool(_lib.load().fgr_gemm_f16x3_ln_supported(m, n, k)))


def linear_ln(x: torch.Tensor, norm, w: torch.Tensor, bias=None, act=ACT_NONE, add=None,
              out=None, side=None) -> torch.Tensor:
    """act((LayerNorm(x) (+ add)) @ W^T + bias) with ``norm`` an nn.LayerNorm over x's
    features: the pre-norm sub-layer inputs of transformers.py:193-196, :213-221 (add = the
    positional embedding) and :231-232. One launch (fgr_gemm_f16x3_ln) where ln_fusable,
    else ops.layernorm then linear() -- the same arithmetic in two launches. ``side`` =
    (norm2, out2): also out2 = norm2(x) (the encoder's output norm of the previous layer; the
    fused launch writes it from the same statistics, fgr_gemm_f16x3_ln_out2; needs ``add``)."""
    m, k = x.shape
    n = w.shape[0]
    assert w.shape[1] == k and norm.weight.numel() == k
    if not ln_fusable(m, n, k) or (side is not None and (add is None or side[0].eps != norm.eps)):
        if side is not None:
            ops.layernorm(x, side[0].weight, side[0].bias, side[0].eps, out=side[1])
        return linear(ops.layernorm(x, norm.weight, norm.bias, norm.eps, add=add), w, bias,
                      act=act, out=out)
    _dev(x, w)
    x = x.contiguous()
    if add is not None:
        assert add.shape == x.shape
        add = add.contiguous()
    gamma, beta = norm.weight.contiguous(), norm.bias.contiguous()
    if bias is not None:
        assert bias.numel() == n and bias.is_contiguous()
    sw = weight_image(w, mode='f16x3')
    if out is None:
        out = torch.empty((m, n), dtype=torch.float32, device=x.device)
    t0 = _begin('gemm', (m, n, k))
    if side is None:
        _lib.check(_lib.load().fgr_gemm_f16x3_ln(
            _ptr(x), x.stride(0), _ptr(gamma), _ptr(beta), float(norm.eps), _ptr(add),
            add.stride(0) if add is not None else 0, _ptr(sw.img), _ptr(out), out.stride(0),
            _ptr(bias), m, n, k, act, _stream()), 'fgr_gemm_f16x3_ln')
    else:
        norm2, out2 = side
        assert out2.shape == x.shape and out2.stride(1) == 1
        _lib.check(_lib.load().fgr_gemm_f16x3_ln_out2(
            _ptr(x), x.stride(0), _ptr(gamma), _ptr(beta), float(norm.eps), _ptr(add),
            add.stride(0), _ptr(sw.img), _ptr(out), out.stride(0), _ptr(bias), m, n, k, act,
            _ptr(norm2.weight.contiguous()), _ptr(norm2.bias.contiguous()), _ptr(out2),
            out2.stride(0), _stream()), 'fgr_gemm_f16x3_ln_out2')
    _end('gemm', t0, 2 * m * n * k)
    return out
