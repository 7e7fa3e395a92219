"""Torch-facing wrappers of the libfgreg kernels.

Every function takes CUDA(HIP) tensors, validates shapes on the host (a kernel is
never launched on operands that do not match what it assumes), allocates the
outputs with the torch caching allocator and launches on torch's current stream.
There is deliberately no CPU path: on a tensor that is not on a GPU, or without
libfgreg.so, these raise.
"""
import ctypes
import math
import os
from typing import Sequence, Tuple

import torch

from . import _lib
from ._lib import ACT_LEAKY, ACT_NONE, ACT_RELU, ACT_RELU_RES_LEAKY, NB_DIST, NB_INDEX  # noqa: F401


def _ptr(t):
    return None if t is None else t.data_ptr()


class KernelTimer:
    """Optional per-op instrumentation for bench.py: HIP events recorded on the launch
    stream around each launch of the named ops, plus the algorithmic bytes / flops of
    every launch (computed only while ``count`` is on, outside any timed region)."""

    def __init__(self, names):
        self.names = set(names)
        self.events = {n: [] for n in names}
        self.work = {n: [] for n in names}
        self.labels = {n: [] for n in names}     # optional per-launch label (e.g. GEMM shape)
        self.count = False
        self.pool = []
        # lead_cycles > 0: a spin kernel of that many cycles (torch.cuda._sleep) goes on the
        # launch stream ahead of every timed call, so the GPU is still busy with it while the
        # host records the start event and submits the call's kernels: the start event then
        # fires right before the first kernel instead of a host launch latency earlier (an
        # eager replay is host-bound; without the lead each interval also holds the
        # submission gap, several us per launch against the kernel trace's durations)
        self.lead_cycles = 0

    def begin(self, name, label=None):
        """Creates the event pair of one launch and arms it in libfgreg
        (fgr_time_next_call), so the events are recorded on the launch stream by the entry
        point itself, immediately around its kernels: the interval excludes the Python /
        ctypes time before the launch, during which the GPU may sit idle."""
        if name not in self.names:
            return None
        if self.lead_cycles > 0:
            torch.cuda._sleep(self.lead_cycles)
        start, end = self.pool.pop() if self.pool else self._pair()
        _lib.check(_lib.load().fgr_time_next_call(start.cuda_event, end.cuda_event),
                   'fgr_time_next_call')
        self.labels[name].append(label)
        return start, end

    def end(self, name, pair, work=None):
        if pair is None:
            return
        _lib.load().fgr_time_next_call(None, None)   # disarm if the call launched nothing
        self.events[name].append(pair)
        if self.count and work is not None:
            self.work[name].append(work() if callable(work) else work)

    @staticmethod
    def _pair():
        start = torch.cuda.Event(enable_timing=True)
        end = torch.cuda.Event(enable_timing=True)
        start.record()            # materialise both events (re-recorded by the call)
        end.record()
        return start, end

    def prealloc(self, n):
        """Creates n event pairs up front, so a timed region pays only the arm call."""
        self.pool.extend(self._pair() for _ in range(n))

    def reset_events(self):
        self.events = {n: [] for n in self.names}
        self.labels = {n: [] for n in self.names}

    def per_label(self, name):
        """{label: [total ms, launches]} over the recorded launches of `name`."""
        out = {}
        for (a, b), lab in zip(self.events[name], self.labels[name]):
            ent = out.setdefault(lab, [0.0, 0])
            ent[0] += a.elapsed_time(b)
            ent[1] += 1
        return out

    def total_ms(self, name):
        return sum(a.elapsed_time(b) for a, b in self.events[name])


TIMER = None  # set to a KernelTimer to instrument


def _begin(name, label=None):
    return TIMER.begin(name, label) if TIMER is not None else None


def _end(name, start, work=None):
    if TIMER is not None:
        TIMER.end(name, start, work)


# the current stream's raw handle without building a torch.cuda.Stream object per launch (the
# eager training step calls this ~1500 times; FGREG_RAW_STREAM=0: torch.cuda.current_stream, A/B)
_raw_stream = (getattr(torch._C, '_cuda_getCurrentRawStream', None)
               if os.environ.get('FGREG_RAW_STREAM', '1') != '0' else None)
_cur_dev = getattr(torch._C, '_cuda_getDevice', None)


def _stream():
    if _raw_stream is not None:
        return _raw_stream(_cur_dev())
    return torch.cuda.current_stream().cuda_stream


# ------------------------------------------------------------------------------------------
# Lazily built model state (weight images, BN-folded weights, stacked head weights): built on
# the stream of the forward that first needs it, read by every later forward. fgreg.pipeline
# runs consecutive forwards on different streams, so it must order the forward after one that
# built state (STATE_EPOCH changed during its enqueue) and mark the new tensors as used by
# every core stream (take_new_state -> record_stream).
# ------------------------------------------------------------------------------------------
STATE_EPOCH = 0
_NEW_STATE = []
# streams on which forwards may still be reading cached state, stream -> the event recorded
# after their last enqueued forward (fgreg.pipeline registers its core streams here): an
# in-place refresh of a cached weight image waits for them first (linear._refresh_stale)
STATE_READERS = {}


def note_state(*tensors):
    """Called by the code that builds (or rewrites in place) cached model state."""
    global STATE_EPOCH
    STATE_EPOCH += 1
    _NEW_STATE.extend(t for t in tensors if torch.is_tensor(t))


def take_new_state():
    """The tensors noted since the last call (and forgets them)."""
    out = list(_NEW_STATE)
    _NEW_STATE.clear()
    return out


def wait_state_readers():
    """The current stream waits for every registered reader stream's last forward."""
    cur = torch.cuda.current_stream()
    for st, ev in list(STATE_READERS.items()):
        if st != cur and ev is not None:
            cur.wait_event(ev)


def _dev(*tensors):
    """Operands must be GPU tensors on the CURRENT device: launches go to that device's
    current stream (_stream), so a tensor on another device would hand foreign pointers
    to the kernels. RegTR.forward enters the inputs' device itself."""
    cur = None
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise _lib.FgrError('fgreg ops need GPU tensors (no CPU fallback by design)')
        if cur is None:
            cur = torch.cuda.current_device()
        if t.device.index != cur:
            raise _lib.FgrError(f'operand on {t.device} but the current device is cuda:{cur}: '
                                f'wrap the call in `with torch.cuda.device({t.device}):`')


def _c(t, dtype):
    if t.dtype != dtype:
        raise _lib.FgrError(f'expected {dtype}, got {t.dtype}')
    return t.contiguous()


def to_device(values, dtype, device) -> torch.Tensor:
    """A host list -> a device tensor without draining the stream: staged through pinned
    memory and copied asynchronously on the current stream (torch's caching host allocator
    keeps the staging block until that copy has run); a pageable torch.tensor(..., device=)
    would wait for all queued GPU work first."""
    t = torch.tensor(values, dtype=dtype)
    if torch.device(device).type != 'cuda':
        return t.to(device)
    return t.pin_memory().to(device, non_blocking=True)


def offsets(lengths: Sequence[int], device) -> torch.Tensor:
    """Host lengths -> device int64 row offsets (len + 1)."""
    o = [0]
    for n in lengths:
        o.append(o[-1] + int(n))
    return to_device(o, torch.int64, device)


# ------------------------------------------------------------------------------------------
# geometry
# ------------------------------------------------------------------------------------------
GRID_MAX_CELLS = 1 << 28     # dense voxel histogram ceiling (1 GiB of counters)


def grid_subsample(points: torch.Tensor, off: torch.Tensor, lengths: Sequence[int], dl: float,
                   return_keys=False, max_cells=None, device_layout=False):
    """Barycentre grid subsampling per cloud (grid_subsampling.cpp semantics).

    Returns (sub_points (M,3) f32, sub_lengths List[int][, keys (M,) int64]). One host
    sync (the voxel counts), as in the reference's own GPU path. ``max_cells``: the dense
    voxel-key histogram's capacity (None = the library default); a key space past it is
    reported by the count call and the count is redone with the needed capacity, up to
    GRID_MAX_CELLS (2^28 cells: a 645-voxel cube per cloud, 16 m at 3DMatch's 2.5 cm); past
    that it raises. ``device_layout``: also return
    the sub-clouds' lengths (nc,) and row offsets (nc + 1,) as device int64 tensors, built on
    the device from the counts (no host -> device copy): (sub, lengths, len_dev, off_dev).
    """
    _dev(points, off)
    pts = _c(points, torch.float32)
    n, nc = pts.shape[0], len(lengths)
    assert pts.dim() == 2 and pts.shape[1] == 3 and off.numel() == nc + 1
    L = _lib.load()
    cap = 0 if max_cells is None else int(max_cells)
    counts = torch.empty(nc + 1, dtype=torch.int64, device=pts.device)
    st = _stream()
    for _ in range(2):
        ws_bytes = _lib._sz(0)
        _lib.check(L.fgr_grid_subsample_workspace(n, nc, cap, ws_bytes),
                   'fgr_grid_subsample_workspace')
        ws = torch.empty(ws_bytes.value, dtype=torch.uint8, device=pts.device)
        t0 = _begin('grid_subsample')
        _lib.check(L.fgr_grid_subsample_count(_ptr(pts), _ptr(off), nc, n, float(dl), cap,
                                              _ptr(ws), ws_bytes.value, _ptr(counts), st),
                   'fgr_grid_subsample_count')
        _end('grid_subsample', t0)
        host = counts.cpu().tolist()  # host sync: output size is data-dependent
        if host[nc] >= 0:
            break
        need = -host[nc]           # dense key space past the histogram: retry once
        if need > GRID_MAX_CELLS:
            raise _lib.FgrError(f'grid subsampling: the clouds\' voxel key space ({need} cells at '
                                f'dl = {dl}) exceeds the dense histogram limit {GRID_MAX_CELLS}')
        cap = need
    m = host[nc]
    assert m >= 0, 'grid subsampling: key space overflow after retry'
    out = torch.empty((m, 3), dtype=torch.float32, device=pts.device)
    keys = torch.empty((m,), dtype=torch.int64, device=pts.device) if return_keys else None
    t0 = _begin('grid_subsample')
    _lib.check(L.fgr_grid_subsample_fill(n, nc, cap, m, _ptr(ws), ws_bytes.value, _ptr(pts),
                                         _ptr(out), _ptr(keys), st), 'fgr_grid_subsample_fill')
    _end('grid_subsample', t0, 12 * (n + m))   # D4: 12 (N_in + N_out) bytes
    if device_layout:
        assert not return_keys
        len_dev = counts[:nc]
        off_dev = lengths_to_offsets(len_dev)
        return out, host[:nc], len_dev, off_dev
    if return_keys:
        return out, host[:nc], keys
    return out, host[:nc]


def lengths_to_offsets(len_dev: torch.Tensor) -> torch.Tensor:
    """Device int64 lengths (n,) -> device row offsets (n + 1,), one launch, no host copy."""
    _dev(len_dev)
    assert len_dev.dtype == torch.int64 and len_dev.dim() == 1
    n = len_dev.numel()
    out = torch.empty(n + 1, dtype=torch.int64, device=len_dev.device)
    _lib.check(_lib.load().fgr_lengths_to_offsets(_ptr(len_dev.contiguous()), n, _ptr(out), _stream()),
               'fgr_lengths_to_offsets')
    return out


# Radius search over a cell grid for clouds of at least this many supports (below it the
# brute-force index-order scan is faster: fewer launches, the cloud stays in L1/L2).
GRID_MIN_SUPPORTS = int(os.environ.get('FGREG_RADIUS_GRID_MIN', '4096'))
GRID_MAX_WIDTH = 256


class RadiusGrid:
    """Supports of a packed batch binned into cells for one radius (fgr_radius_grid_build);
    serves every radius_search / radius_count over the same supports with radius <= that."""

    def __init__(self, s, s_off, s_lengths, radius):
        _dev(s, s_off)
        self.s = _c(s, torch.float32)
        self.s_off, self.s_lengths = s_off, list(s_lengths)
        self.radius = float(radius)
        nc = len(self.s_lengths)
        L = _lib.load()
        nb = _lib._sz(0)
        _lib.check(L.fgr_radius_grid_workspace(self.s.shape[0], nc, nb), 'fgr_radius_grid_workspace')
        self.ws = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=s.device)
        self.nbytes = nb.value
        t0 = _begin('radius_search')
        _lib.check(L.fgr_radius_grid_build(_ptr(self.s), _ptr(s_off), nc, self.s.shape[0],
                                           self.radius, _ptr(self.ws), self.nbytes, _stream()),
                   'fgr_radius_grid_build')
        _end('radius_search', t0, 12 * self.s.shape[0])

    def serves(self, s, radius):
        return s.data_ptr() == self.s.data_ptr() and float(radius) <= self.radius


def radius_grid(s, s_off, s_lengths, radius):
    """A RadiusGrid when the clouds are large enough for the cell path, else None."""
    if not len(s_lengths) or max(s_lengths) < GRID_MIN_SUPPORTS:
        return None
    return RadiusGrid(s, s_off, s_lengths, radius)


def radius_count(q, q_off, q_lengths, s, s_off, radius, grid=None) -> Tuple[torch.Tensor, int]:
    """Uncapped neighbour counts (int32 per query) and their max (host int, one sync)."""
    _dev(q, q_off, s, s_off)
    q, s = _c(q, torch.float32), _c(s, torch.float32)
    counts = torch.empty(q.shape[0], dtype=torch.int32, device=q.device)
    mx = torch.empty(1, dtype=torch.int32, device=q.device)
    max_q = max(q_lengths) if len(q_lengths) else 0
    if grid is not None and grid.serves(s, radius):
        _lib.check(_lib.load().fgr_radius_search_grid(
            _ptr(q), _ptr(q_off), len(q_lengths), q.shape[0], max_q, _ptr(s), _ptr(s_off),
            s.shape[0], _ptr(grid.ws), grid.nbytes, float(radius), NB_INDEX, 0, None, _ptr(counts),
            _ptr(mx), _stream()), 'fgr_radius_search_grid')
        return counts, int(mx.item())
    _lib.check(_lib.load().fgr_radius_count(_ptr(q), _ptr(q_off), _ptr(s), _ptr(s_off),
                                            len(q_lengths), q.shape[0], max_q, float(radius), _ptr(counts),
                                            _ptr(mx), _stream()), 'fgr_radius_count')
    return counts, int(mx.item())


def radius_search(q: torch.Tensor, q_off: torch.Tensor, q_lengths: Sequence[int], s: torch.Tensor,
                  s_off: torch.Tensor, s_lengths: Sequence[int], radius: float, limit: int,
                  mode: int = NB_INDEX, grid: 'RadiusGrid' = None) -> torch.Tensor:
    """Radius neighbours, (Nq, width) int64 padded with the shadow index Ns_total.

    mode NB_INDEX: ball_query semantics, width = limit (no host sync).
    mode NB_DIST:  nanoflann semantics, width = min(max count, limit) (one host sync).
    ``grid``: a RadiusGrid over these supports (radius_grid()), used when it serves this
    radius and width <= 256; otherwise the brute-force scan.
    """
    _dev(q, q_off, s, s_off)
    q, s = _c(q, torch.float32), _c(s, torch.float32)
    assert q.dim() == 2 and q.shape[1] == 3 and s.dim() == 2 and s.shape[1] == 3
    nc = len(q_lengths)
    assert len(s_lengths) == nc and q_off.numel() == nc + 1 and s_off.numel() == nc + 1
    assert sum(q_lengths) == q.shape[0] and sum(s_lengths) == s.shape[0]
    L = _lib.load()
    st = _stream()
    max_q = max(q_lengths) if nc else 0
    r = float(radius)
    if mode == NB_INDEX:
        if limit <= 0:
            raise _lib.FgrError('ball_query semantics need a positive neighbour limit')
        width = int(limit)
    else:
        _, m = radius_count(q, q_off, q_lengths, s, s_off, r, grid)
        width = m if limit <= 0 else min(m, int(limit))
    out = torch.empty((q.shape[0], width), dtype=torch.int64, device=q.device)
    if grid is not None and grid.serves(s, r) and width <= GRID_MAX_WIDTH:
        t0 = _begin('radius_search')
        _lib.check(L.fgr_radius_search_grid(
            _ptr(q), _ptr(q_off), nc, q.shape[0], max_q, _ptr(s), _ptr(s_off), s.shape[0],
            _ptr(grid.ws), grid.nbytes, r, int(mode), width, _ptr(out), None, None, st),
            'fgr_radius_search_grid')
        _end('radius_search', t0, 12 * q.shape[0] + 8 * q.shape[0] * width)
        return out
    t0 = _begin('radius_search')
    _lib.check(L.fgr_radius_search(_ptr(q), _ptr(q_off), _ptr(s), _ptr(s_off), nc, q.shape[0],
                                   s.shape[0], max_q, r, int(mode), width, _ptr(out), st),
               'fgr_radius_search')
    # D4: 12 (Nq + Ns) + idx_bytes * Nq * K
    _end('radius_search', t0, 12 * (q.shape[0] + s.shape[0]) + 8 * q.shape[0] * width)
    return out


# ------------------------------------------------------------------------------------------
# KPConv
# ------------------------------------------------------------------------------------------
def kpconv_gather(q, s, idx, x, kernel_points, extent) -> Tuple[torch.Tensor, torch.Tensor]:
    """-> (wf (Nq, K, Cin), nnorm (Nq,) f32) of the KPConv gather-weight stage."""
    _dev(q, s, idx, x, kernel_points)
    q, s, x = _c(q, torch.float32), _c(s, torch.float32), _c(x, torch.float32)
    idx = _c(idx, torch.int64)
    kp = _c(kernel_points, torch.float32)
    nq, ns = q.shape[0], s.shape[0]
    assert idx.dim() == 2 and idx.shape[0] == nq and x.dim() == 2 and x.shape[0] == ns
    assert kp.dim() == 2 and kp.shape[1] == 3
    K, cin = kp.shape[0], x.shape[1]
    wf = torch.empty((nq, K, cin), dtype=torch.float32, device=q.device)
    nnorm = torch.empty((nq,), dtype=torch.float32, device=q.device)
    L = _lib.load()
    nb = _lib._sz(0)
    _lib.check(L.fgr_kpconv_gather_workspace(ns, cin, nb), 'fgr_kpconv_gather_workspace')
    ws = _workspace(q.device, nb.value) if nb.value else None
    t0 = _begin('kpconv_gather', (nq, idx.shape[1], cin, K))
    _lib.check(L.fgr_kpconv_gather(_ptr(q), _ptr(s), nq, ns, _ptr(idx), idx.shape[1], _ptr(x), cin,
                                   _ptr(kp), K, float(extent), _ptr(wf), _ptr(nnorm), _ptr(ws),
                                   nb.value, _stream()), 'fgr_kpconv_gather')
    _end('kpconv_gather', t0, lambda: gather_bytes(idx, ns, cin, K))
    return wf, nnorm


def gather_bytes(idx, ns, cin, n_kp):
    """Algorithmic HBM bytes of one fgr_kpconv_gather launch:
    sum_q [8*H (idx row) + 12 (q) + v_q*(12 + 4*cin) (valid xyz + feature rows)
           + 4*K*cin (wf row) + 4 (nnorm)]."""
    nq, H = idx.shape
    v = int((idx < ns).sum().item())
    return nq * (8 * H + 12 + 4 * n_kp * cin + 4) + v * (12 + 4 * cin)


def max_pool(x, idx) -> torch.Tensor:
    _dev(x, idx)
    x, idx = _c(x, torch.float32), _c(idx, torch.int64)
    out = torch.empty((idx.shape[0], x.shape[1]), dtype=torch.float32, device=x.device)
    t0 = _begin('max_pool')
    _lib.check(_lib.load().fgr_max_pool(_ptr(x), x.shape[0], x.shape[1], _ptr(idx), idx.shape[0],
                                        idx.shape[1], _ptr(out), _stream()), 'fgr_max_pool')
    _end('max_pool', t0, lambda: max_pool_bytes(idx, x.shape[0], x.shape[1]))
    return out


def max_pool_bytes(idx, ns, c):
    """Algorithmic HBM bytes of one fgr_max_pool launch (finegrained_kpconv_blocks.py:125-141):
    sum_q [8 H (idx row) + 4 C (output row)] + 4 C per DISTINCT support row named by the table
    (each is needed from HBM once; its repeats across queries are cache traffic)."""
    nq, H = idx.shape
    u = int(torch.unique(idx[idx < ns]).numel())
    return nq * (8 * H + 4 * c) + u * 4 * c


# ------------------------------------------------------------------------------------------
# normalisation / embedding
# ------------------------------------------------------------------------------------------
def instnorm(x, seg_off, lengths, row_div=None, act=ACT_NONE, residual=None, post_act=ACT_NONE,
             eps=1e-5, out=None) -> torch.Tensor:
    """Per-segment InstanceNorm1d with fused row division / activation / residual.
    ``lengths`` are the host-side segment lengths (their count and max size the launch)."""
    _dev(x, seg_off, row_div, residual)
    x = _c(x, torch.float32)
    n, c = x.shape
    n_seg = len(lengths)
    max_len = max(lengths) if n_seg else 0
    if residual is not None:
        residual = _c(residual, torch.float32)
        assert residual.shape == x.shape
    if row_div is not None:
        row_div = _c(row_div, torch.float32)
        assert row_div.shape == (n,)
    assert seg_off.numel() == n_seg + 1 and sum(lengths) == n
    if out is None:
        out = torch.empty_like(x)
    L = _lib.load()
    nb = _lib._sz(0)
    _lib.check(L.fgr_instnorm_workspace(max_len, c, n_seg, nb), 'fgr_instnorm_workspace')
    ws = torch.empty(nb.value, dtype=torch.uint8, device=x.device) if nb.value else None
    t0 = _begin('instnorm')
    _lib.check(L.fgr_instnorm(_ptr(x), n, c, _ptr(seg_off), n_seg, max_len, _ptr(row_div),
                              float(eps), act, _ptr(residual), post_act, _ptr(out), _ptr(ws),
                              nb.value, _stream()), 'fgr_instnorm')
    # D4: 8 N C (read + write) + 4 N C per residual + 4 N for the row divisor
    _end('instnorm', t0, n * c * (8 + (4 if residual is not None else 0))
         + (4 * n if row_div is not None else 0))
    return out


def layernorm(x, weight, bias, eps=1e-5, add=None, pre_bias=None, out=None) -> torch.Tensor:
    """LN(x) * weight + bias (+ add). ``pre_bias``: x += pre_bias IN PLACE first."""
    _dev(x, weight, bias, add, pre_bias)
    assert x.dtype == torch.float32 and x.is_contiguous()
    n, d = x.shape
    if add is not None:
        add = _c(add, torch.float32)
        assert add.shape == x.shape
    if pre_bias is not None:
        pre_bias = _c(pre_bias, torch.float32)
        assert pre_bias.shape == (d,)
    if out is None:
        out = torch.empty_like(x)
    assert out.is_contiguous() and out.shape == x.shape
    t0 = _begin('layernorm')
    _lib.check(_lib.load().fgr_layernorm(_ptr(x), n, d, _ptr(weight.contiguous()),
                                         _ptr(bias.contiguous()), float(eps), _ptr(add),
                                         _ptr(pre_bias), _ptr(out), _stream()), 'fgr_layernorm')
    _end('layernorm', t0, n * d * (8 + (4 if add is not None else 0)
                                   + (4 if pre_bias is not None else 0)))
    return out


def layernorm_dual(x, norm_a, norm_b, add_b=None, out_a=None, out_b=None):
    """(LN_a(x), LN_b(x) (+ add_b)) in one pass (fgr_layernorm_dual): two nn.LayerNorm modules
    of the same width and eps over the same rows."""
    _dev(x, norm_a.weight, norm_b.weight, add_b)
    assert x.dtype == torch.float32 and x.is_contiguous() and norm_a.eps == norm_b.eps
    n, d = x.shape
    if add_b is not None:
        add_b = _c(add_b, torch.float32)
        assert add_b.shape == x.shape
    out_a = torch.empty_like(x) if out_a is None else out_a
    out_b = torch.empty_like(x) if out_b is None else out_b
    assert out_a.is_contiguous() and out_b.is_contiguous()
    t0 = _begin('layernorm')
    _lib.check(_lib.load().fgr_layernorm_dual(
        _ptr(x), n, d, _ptr(norm_a.weight.contiguous()), _ptr(norm_a.bias.contiguous()), None,
        _ptr(out_a), _ptr(norm_b.weight.contiguous()), _ptr(norm_b.bias.contiguous()),
        _ptr(add_b), _ptr(out_b), float(norm_a.eps), _stream()), 'fgr_layernorm_dual')
    _end('layernorm', t0, n * d * (12 + (4 if add_b is not None else 0)))
    return out_a, out_b


def add(a, b, out=None) -> torch.Tensor:
    """a + b (same shape, fp32) on fgr_add: the post-norm layer's with_pos_embed."""
    _dev(a, b)
    a, b = _c(a, torch.float32), _c(b, torch.float32)
    assert a.shape == b.shape
    if out is None:
        out = torch.empty_like(a)
    assert out.is_contiguous() and out.shape == a.shape
    _lib.check(_lib.load().fgr_add(_ptr(a), _ptr(b), a.numel(), _ptr(out), _stream()), 'fgr_add')
    return out


def sine_pos_embed(xyz, d_model, temperature=10000.0, scale=1.0) -> torch.Tensor:
    _dev(xyz)
    xyz = _c(xyz, torch.float32)
    assert xyz.dim() == 2 and xyz.shape[1] == 3
    out = torch.empty((xyz.shape[0], d_model), dtype=torch.float32, device=xyz.device)
    _lib.check(_lib.load().fgr_sine_pos_embed(_ptr(xyz), xyz.shape[0], d_model, float(temperature),
                                              float(scale * 2 * math.pi), _ptr(out), _stream()),
               'fgr_sine_pos_embed')
    return out


# ------------------------------------------------------------------------------------------
# Res2Net hierarchy
# ------------------------------------------------------------------------------------------
def res2net_fragments3(weights: torch.Tensor) -> torch.Tensor:
    """(nums, w, w) Linear weights (out, in) -> the bf16x6 image of fgr_res2net_chain6:
    K zero-padded to a multiple of 32, each value split exactly into three bf16 terms
    (h = bf16(x), m = bf16(x - h), l = bf16(x - h - m)), laid out in 16x16x32 B-fragment
    order [i][jt][ks][term][g][c][8] with value W_i[16 jt + c][32 ks + 8 g + e]."""
    nums, w, _ = weights.shape
    ks = (w + 31) // 32
    wp = torch.zeros((nums, w, ks * 32), dtype=torch.float32, device=weights.device)
    wp[..., :w] = weights
    hi = wp.to(torch.bfloat16)
    r = wp - hi.float()
    mid = r.to(torch.bfloat16)
    lo = (r - mid.float()).to(torch.bfloat16)
    t = torch.stack([hi, mid, lo], 0).reshape(3, nums, w // 16, 16, ks, 4, 8)
    return t.permute(1, 2, 4, 0, 5, 3, 6).contiguous()     # [i, jt, ks, t, g, c, e]


def res2net_fragments_h3(weights: torch.Tensor):
    """(nums, w, w) Linear weights (out, in) -> (image, inverse scales) of
    fgr_res2net_chain_h3: each output row (i, n) scaled by 2^e so its max |w| lies in
    [2^14, 2^15) (wsc[i, n] = 2^-e), rows zero-padded to Wp = 16 ceil(w / 16) (one 16-column
    tile per wave) and K to a multiple of 32, split into two fp16 terms (h = f16(x),
    m = f16(x - h), round to nearest), in 16x16x32 fragment order
    [i][jt][ks][term][g][c][8] with value W_i[16 jt + c][32 ks + 8 g + e] * 2^e."""
    nums, w, _ = weights.shape
    wp_rows = (w + 15) // 16 * 16
    ks = (wp_rows + 31) // 32
    mx = weights.abs().amax(dim=2)                                     # (nums, w)
    e = torch.where(mx > 0, 15 - torch.frexp(mx).exponent, torch.zeros_like(mx, dtype=torch.int32))
    e = e.clamp(max=127)
    sc = torch.ldexp(torch.ones_like(mx), e.float())
    wp = torch.zeros((nums, wp_rows, ks * 32), dtype=torch.float32, device=weights.device)
    wp[:, :w, :w] = weights * sc[..., None]
    hi = wp.to(torch.float16)
    lo = (wp - hi.float()).to(torch.float16)
    t = torch.stack([hi, lo], 0).reshape(2, nums, wp_rows // 16, 16, ks, 4, 8)
    img = t.permute(1, 2, 4, 0, 5, 3, 6).contiguous()                 # [i, jt, ks, t, g, c, e]
    return img, (1.0 / sc).contiguous()


def res2net_chain_supported(w, h3=False):
    """bf16x6 chain (fgr_res2net_chain6): w = 112, 224; the f16x3 chain: any w % 4 == 0 up to
    224 whose 16-column tile count has a kernel instance (28, 56, 112, 224: every reference
    width)."""
    if h3:
        return w % 4 == 0 and (w + 15) // 16 in (2, 4, 7, 14)
    return w in (112, 224)


def res2net_chain(h, w, scale, w_frag, bias, x, cat, w_scale=None):
    """cat[:, :] = [sp_0..sp_{scale-2} | h_{scale-1} | x] by fgr_res2net_chain_h3 (scaled split
    fp16, (w_frag, w_scale) = res2net_fragments_h3) or, when w_scale is None,
    fgr_res2net_chain6 (exact three-term split bf16, w_frag = res2net_fragments3)."""
    _dev(h, w_frag, w_scale, bias, x, cat)
    h = _c(h, torch.float32)
    n = h.shape[0]
    assert h.shape[1] == scale * w and cat.shape[0] == n and cat.stride(1) == 1
    cin = 0 if x is None else x.shape[1]
    if x is not None:
        x = _c(x, torch.float32)
    L = _lib.load()
    # MFMA work: (scale - 1) chained w x w Linears over n rows, 3 (f16x3) or 6 (bf16x6) fp16 /
    # bf16 matrix-core products per product (res2net.py:126-159)
    t0 = _begin('res2net', 'h3' if w_scale is not None else 'x6')
    work = 2 * n * w * w * (scale - 1) * (3 if w_scale is not None else 6)
    if w_scale is not None:
        _lib.check(L.fgr_res2net_chain_h3(
            _ptr(h), n, w, scale, _ptr(w_frag), _ptr(w_scale), _ptr(bias), _ptr(x), cin,
            _ptr(cat), cat.stride(0), _stream()), 'fgr_res2net_chain_h3')
    else:
        _lib.check(L.fgr_res2net_chain6(_ptr(h), n, w, scale, _ptr(w_frag), _ptr(bias), _ptr(x),
                                        cin, _ptr(cat), cat.stride(0), _stream()),
                   'fgr_res2net_chain6')
    _end('res2net', t0, work)
    return cat


# ------------------------------------------------------------------------------------------
# attention
# ------------------------------------------------------------------------------------------
# head_dim 32 / 64 (every reference config): fgr_attention_f16x3 (fp32-accurate scaled
# split-fp16 MFMA, default) or, in the 'bf16' mode (the BASELINE configs[4] compute mode, set
# together with linear.MODE by set_precision), fgr_attention_bf16 -- one bf16 product per fp32
# product. Any other head_dim (4, 8, 16, 128, 256) or unaligned operand: fgr_attention (fp32
# MFMA). FGREG_ATTN = f16x3 | bf16 overrides the attention mode alone (profiling A/B switch).
ATTN_MODE = os.environ.get('FGREG_ATTN', 'f16x3')
assert ATTN_MODE in ('f16x3', 'bf16'), ATTN_MODE


def attention(q, k, v, q_off, kv_off, kv_seg, max_q_len, n_head, out=None,
              max_kv_len=None, dropout=None, lse=None) -> torch.Tensor:
    """Packed-segment MHA core: rows of query segment i attend to key segment kv_seg[i].

    q, k, v: (rows, n_head * dh) views with unit column stride (may be column slices of
    one fused QKV tensor). Returns o (Nq, n_head * dh). ``max_kv_len`` defaults to
    ``max_q_len`` (self / cross attention over one segmentation). ``dropout`` = (seed, p):
    the training forward's attention-weight dropout (fgr_attention_f16x3_drop, in either
    precision mode; head dim 32 / 64). ``lse`` (rows, n_head) fp32: the training forward
    (fgr_attention_f16x3_train) also writes each row's log2-sum-exp there for the backward
    (only for shapes ``attention_lse_ok`` accepts).
    """
    _dev(q, k, v, q_off, kv_off, kv_seg)
    for t in (q, k, v):
        assert t.dtype == torch.float32 and t.dim() == 2 and t.stride(1) == 1
    d = q.shape[1]
    assert k.shape[1] == d and v.shape[1] == d and d % n_head == 0 and k.shape[0] == v.shape[0]
    dh = d // n_head
    if out is None:
        out = torch.empty((q.shape[0], d), dtype=torch.float32, device=q.device)
    n_seg = q_off.numel() - 1
    n_kv_seg = kv_off.numel() - 1
    assert kv_seg.dtype == torch.int32 and kv_seg.numel() == n_seg
    max_kv_len = max_q_len if max_kv_len is None else max_kv_len
    L = _lib.load()
    split = (dh in (32, 64)
             and all(t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0 for t in (q, k, v, out)))
    t0 = _begin('attention')
    if lse is not None:
        assert split and ATTN_MODE == 'f16x3' and lse.is_contiguous() and lse.shape == (q.shape[0], n_head)
        seed, p = (int(dropout[0]), float(dropout[1])) if dropout is not None else (0, 0.0)
        nb = _lib.ws_size('fgr_attention_f16x3_workspace', k.shape[0], n_kv_seg, n_head)
        ws = _workspace(q.device, nb)
        _lib.check(L.fgr_attention_f16x3_train(
            _ptr(q), q.stride(0), _ptr(k), k.stride(0), _ptr(v), v.stride(0), _ptr(out),
            out.stride(0), _ptr(q_off), _ptr(kv_off), _ptr(kv_seg), n_seg, n_kv_seg, k.shape[0],
            int(max_q_len), int(max_kv_len), n_head, dh, float(math.sqrt(1.0 / float(dh))),
            _ptr(ws), ws.numel(), seed & 0xFFFFFFFF, p, _ptr(lse), _stream()),
            'fgr_attention_f16x3_train')
    elif dropout is not None and float(dropout[1]) > 0.0:
        # training with dropout: the f16x3 kernel in either precision mode (the bf16 mode's
        # training attention with dropout is fp32-accurate; its backward, fgr_attention_bwd_drop,
        # is fp32 in both modes and draws the same mask)
        if not split:
            raise NotImplementedError('attention dropout needs head dim 32 / 64 and 16-B aligned '
                                      'rows')
        nb = _lib._sz(0)
        _lib.check(L.fgr_attention_f16x3_workspace(k.shape[0], n_kv_seg, n_head, nb),
                   'fgr_attention_f16x3_workspace')
        ws = _workspace(q.device, nb.value)
        _lib.check(L.fgr_attention_f16x3_drop(
            _ptr(q), q.stride(0), _ptr(k), k.stride(0), _ptr(v), v.stride(0), _ptr(out),
            out.stride(0), _ptr(q_off), _ptr(kv_off), _ptr(kv_seg), n_seg, n_kv_seg, k.shape[0],
            int(max_q_len), int(max_kv_len), n_head, dh, float(math.sqrt(1.0 / float(dh))),
            _ptr(ws), ws.numel(), int(dropout[0]) & 0xFFFFFFFF, float(dropout[1]), _stream()),
            'fgr_attention_f16x3_drop')
    elif split:
        name = 'fgr_attention_' + ATTN_MODE
        nb = _lib._sz(0)
        _lib.check(getattr(L, name + '_workspace')(k.shape[0], n_kv_seg, n_head, nb),
                   name + '_workspace')
        ws = _workspace(q.device, nb.value)
        _lib.check(getattr(L, name)(
            _ptr(q), q.stride(0), _ptr(k), k.stride(0), _ptr(v), v.stride(0), _ptr(out),
            out.stride(0), _ptr(q_off), _ptr(kv_off), _ptr(kv_seg), n_seg, n_kv_seg, k.shape[0],
            int(max_q_len), int(max_kv_len), n_head, dh, float(math.sqrt(1.0 / float(dh))),
            _ptr(ws), ws.numel(), _stream()), name)
    else:
        _lib.check(L.fgr_attention(_ptr(q), q.stride(0), _ptr(k), k.stride(0), _ptr(v),
                                   v.stride(0), _ptr(out), out.stride(0), _ptr(q_off),
                                   _ptr(kv_off), _ptr(kv_seg), n_seg, int(max_q_len), n_head,
                                   dh, float(math.sqrt(1.0 / float(dh))), _stream()),
                   'fgr_attention')
    _end('attention', t0, lambda: attention_flops(q_off, kv_off, kv_seg, d))
    return out


def attention_lse_ok(q, k, v, n_head) -> bool:
    """True if ops.attention can hand the backward its log-sum-exp (``lse``)."""
    dh = q.shape[1] // n_head
    return (ATTN_MODE == 'f16x3' and dh in (32, 64)
            and all(t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0 for t in (q, k, v)))


def copy_batch(srcs, dsts):
    """dst.copy_(src) for every pair (same shape / dtype, contiguous, device tensors) in one
    fgr_copy_batch launch per 32 pairs."""
    n = len(srcs)
    if n == 0:
        return
    for a, b in zip(srcs, dsts):
        assert a.shape == b.shape and a.dtype == b.dtype and a.is_contiguous() and b.is_contiguous()
    _dev(*srcs, *dsts)
    arr = ctypes.c_void_p * n
    src = arr(*[t.data_ptr() for t in srcs])
    dst = arr(*[t.data_ptr() for t in dsts])
    nb = (ctypes.c_int64 * n)(*[t.numel() * t.element_size() for t in srcs])
    _lib.check(_lib.load().fgr_copy_batch(n, src, dst, nb, _stream()), 'fgr_copy_batch')


_WS = {}
_WS_RETIRED = []
_WS_SCOPE = None      # a PrivateWorkspace while one is entered (HIP-graph warm-up / capture)


class PrivateWorkspace:
    """Scratch buffers owned by one client (a captured HIP graph, fgreg/regtr.py _CoreGraph):
    while entered (``with ws:``), every ``_workspace`` request is served from this object
    instead of the shared per-(device, stream) buffers, so the graph bakes in scratch memory
    no other graph and no eager launch ever touches, whatever stream it is replayed on.
    Outgrown buffers stay referenced (a capture may point at them)."""

    def __init__(self):
        self.bufs, self.retired, self._prev = {}, [], []

    def get(self, device, nbytes):
        buf = self.bufs.get(device)
        if buf is None or buf.numel() < nbytes:
            if buf is not None:
                self.retired.append(buf)
            buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
            self.bufs[device] = buf
        return buf

    def __enter__(self):
        global _WS_SCOPE
        self._prev.append(_WS_SCOPE)
        _WS_SCOPE = self
        return self

    def __exit__(self, *exc):
        global _WS_SCOPE
        _WS_SCOPE = self._prev.pop()
        return False


def _workspace(device, nbytes):
    """Grow-only scratch buffer per device, reused by consecutive launches on the current
    stream (stream order serialises the reuse). Outgrown buffers are kept alive: a captured
    HIP graph may still point at them. Inside a ``PrivateWorkspace`` scope the buffer is that
    scope's own (each captured graph has one)."""
    if _WS_SCOPE is not None:
        return _WS_SCOPE.get(device, nbytes)
    key = (device, _raw_stream(device.index) if _raw_stream is not None and device.index is not None
           else torch.cuda.current_stream(device).cuda_stream)
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        if buf is not None:
            _WS_RETIRED.append(buf)
        buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
        _WS[key] = buf
    return buf


def attention_flops(q_off, kv_off, kv_seg, d):
    """Algorithmic flops of one fgr_attention launch: 4 * Nq * Nk * d per segment
    (QK^T + AV over all heads)."""
    qo, ko, ks = q_off.tolist(), kv_off.tolist(), kv_seg.tolist()
    return sum(4 * (qo[i + 1] - qo[i]) * (ko[ks[i] + 1] - ko[ks[i]]) * d for i in range(len(ks)))


def ln_qkv_supported(m, d, n_head) -> bool:
    return bool(_lib.load().fgr_gemm_f16x3_ln_qkv_supported(int(m), int(d), int(n_head)))


def ln_qkv_attention(x, norm, w_img, bias, pos, q_off, kv_seg, max_len, n_head, side=None):
    """The pre-norm attention sub-layer's in_proj + attention core in two launches:
    fgr_gemm_f16x3_ln_qkv (LayerNorm(x) + pos -> q fp32 and the K / V images of every global
    64-row tile, transformers.py:193-196 / :213-221) then fgr_attention_f16x3_img (head dim 32).
    ``side`` = (norm2, out2): out2 = norm2(x) from the same statistics. -> o (N, d)."""
    _dev(x, bias, pos, q_off, kv_seg)
    n, d = x.shape
    x, pos = x.contiguous(), pos.contiguous()
    gamma, beta = norm.weight.contiguous(), norm.bias.contiguous()
    L = _lib.load()
    nb = _lib._sz(0)
    _lib.check(L.fgr_kv_image_bytes(n, n_head, d // n_head, nb), 'fgr_kv_image_bytes')
    img = _workspace(x.device, nb.value)
    q = torch.empty((n, d), dtype=torch.float32, device=x.device)
    g2 = b2 = out2 = None
    if side is not None:
        g2, b2, out2 = side[0].weight.contiguous(), side[0].bias.contiguous(), side[1]
        assert out2.shape == x.shape and out2.stride(1) == 1
    t0 = _begin('gemm', (n, 3 * d, d))
    _lib.check(L.fgr_gemm_f16x3_ln_qkv(
        _ptr(x), x.stride(0), _ptr(gamma), _ptr(beta), float(norm.eps), _ptr(pos), pos.stride(0),
        _ptr(w_img.img), _ptr(q), q.stride(0), _ptr(bias), n, d, n_head, _ptr(img), _ptr(g2),
        _ptr(b2), _ptr(out2), out2.stride(0) if out2 is not None else 0, _stream()),
        'fgr_gemm_f16x3_ln_qkv')
    _end('gemm', t0, 2 * n * 3 * d * d)
    o = torch.empty((n, d), dtype=torch.float32, device=x.device)
    t0 = _begin('attention')
    _lib.check(L.fgr_attention_f16x3_img(
        _ptr(q), q.stride(0), _ptr(img), n, _ptr(o), o.stride(0), _ptr(q_off), _ptr(q_off),
        _ptr(kv_seg), q_off.numel() - 1, int(max_len), n_head, d // n_head,
        float(math.sqrt(1.0 / float(d // n_head))), _stream()), 'fgr_attention_f16x3_img')
    _end('attention', t0, lambda: attention_flops(q_off, q_off, kv_seg, d))
    return o


def qkv_supported(m, d, n_head) -> bool:
    return bool(_lib.load().fgr_gemm_f16x3_qkv_supported(int(m), int(d), int(n_head)))


def qkv_bf16_supported(m, d, n_head) -> bool:
    return bool(_lib.load().fgr_gemm_bf16_qkv_supported(int(m), int(d), int(n_head)))


def qkv_attention(h, w_img, bias, q_off, kv_seg, max_len, n_head, mode='f16x3'):
    """The attention sub-layer's in_proj + attention core in two launches, head dim 64:
    fgr_gemm_f16x3_qkv (h W^T + b -> q fp32 and the K / V images of every global 64-row tile)
    then fgr_attention_f16x3_img; mode 'bf16': fgr_gemm_bf16_qkv (bf16 images) then
    fgr_attention_bf16_img. -> o (N, d)."""
    _dev(h, bias, q_off, kv_seg)
    n, d = h.shape
    h = h.contiguous()
    L = _lib.load()
    nb = _lib._sz(0)
    bytes_fn = 'fgr_kv_image_bytes' if mode == 'f16x3' else 'fgr_kv_image_bf16_bytes'
    _lib.check(getattr(L, bytes_fn)(n, n_head, d // n_head, nb), bytes_fn)
    img = _workspace(h.device, nb.value)
    q = torch.empty((n, d), dtype=torch.float32, device=h.device)
    t0 = _begin('gemm', (n, 3 * d, d))
    gemm_fn = 'fgr_gemm_f16x3_qkv' if mode == 'f16x3' else 'fgr_gemm_bf16_qkv'
    _lib.check(getattr(L, gemm_fn)(_ptr(h), h.stride(0), _ptr(w_img.img), _ptr(q), q.stride(0),
                                   _ptr(bias), n, d, n_head, _ptr(img), _stream()), gemm_fn)
    _end('gemm', t0, 2 * n * 3 * d * d)
    o = torch.empty((n, d), dtype=torch.float32, device=h.device)
    t0 = _begin('attention')
    attn_fn = 'fgr_attention_f16x3_img' if mode == 'f16x3' else 'fgr_attention_bf16_img'
    _lib.check(getattr(L, attn_fn)(
        _ptr(q), q.stride(0), _ptr(img), n, _ptr(o), o.stride(0), _ptr(q_off), _ptr(q_off),
        _ptr(kv_seg), q_off.numel() - 1, int(max_len), n_head, d // n_head,
        float(math.sqrt(1.0 / float(d // n_head))), _stream()), attn_fn)
    _end('attention', t0, lambda: attention_flops(q_off, q_off, kv_seg, d))
    return o


FFN_FUSE = os.environ.get('FGREG_FFN_FUSE', '1') != '0'


def ffn_supported(m, d, f) -> bool:
    """True if the pre-norm feed-forward sub-layer of an (m, d) input with hidden width f runs
    as one launch (fgr_ffn_f16x3: d = 256, the ModelNet transformer; FGREG_FFN_FUSE=0 off)."""
    return FFN_FUSE and bool(_lib.load().fgr_ffn_f16x3_supported(m, d, f))


def ffn(x, norm, w1_img, b1, w2_img, b2, bound, out=None) -> torch.Tensor:
    """x + linear2(ReLU(linear1(norm(x)))) in one launch (transformers.py:231-238):
    w1_img = linear.weight_image(linear1.weight, mode='f16x3'), w2_img =
    linear.weight_image(linear2.weight, mode='ffn2'), bound (2,) = {max_j ||W1_j||, max |b1|}
    on the device."""
    _dev(x, b1, b2, bound)
    m, d = x.shape
    f = b1.numel()
    assert x.dtype == torch.float32 and x.stride(1) == 1 and b2.numel() == d
    x = x if (x.stride(0) % 4 == 0 and x.data_ptr() % 16 == 0) else x.contiguous()
    g, b = norm.weight.contiguous(), norm.bias.contiguous()
    b1, b2, bound = b1.contiguous(), b2.contiguous(), bound.contiguous()
    if out is None:
        out = torch.empty((m, d), dtype=torch.float32, device=x.device)
    t0 = _begin('gemm', ('ffn', m, d, f))
    _lib.check(_lib.load().fgr_ffn_f16x3(
        _ptr(x), x.stride(0), _ptr(g), _ptr(b), float(norm.eps), _ptr(w1_img.img), _ptr(b1),
        _ptr(w2_img.img), _ptr(b2), _ptr(bound), _ptr(out), out.stride(0), m, d, f, _stream()),
        'fgr_ffn_f16x3')
    _end('gemm', t0, 4 * m * d * f)
    return out


def corr_head_supported(m, d) -> bool:
    return bool(_lib.load().fgr_corr_head_supported(int(m), int(d)))


def corr_head(f, img0c, b0c, img2, b2, w4, b4):
    """CorrespondenceRegressor (finegrained_regtr.py:411-455) on f (m, d) in two launches
    (fgr_corr_head_f16x3): -> corr (m, 3), logits (m, 1). img0c: the f16x3 image of the stacked
    [W0; Wc; 0] (d + 16, d) with bias b0c; img2: coor_mlp[2]'s image; w4 / b4: coor_mlp[4]."""
    _dev(f, b0c, b2, w4, b4)
    m, d = f.shape
    assert f.stride(1) == 1 and f.stride(0) % 4 == 0 and f.data_ptr() % 16 == 0
    w4, b4 = _c(w4, torch.float32), _c(b4, torch.float32)
    assert w4.shape == (3, d) and b0c.numel() == d + 16 and b2.numel() == d
    hidden = _workspace(f.device, 4 * m * d)
    corr = torch.empty((m, 3), dtype=torch.float32, device=f.device)
    logits = torch.empty((m, 1), dtype=torch.float32, device=f.device)
    t0 = _begin('gemm', (m, 2 * d + 16, d))
    _lib.check(_lib.load().fgr_corr_head_f16x3(
        _ptr(f), f.stride(0), m, d, _ptr(img0c.img), _ptr(_c(b0c, torch.float32)), _ptr(img2.img),
        _ptr(_c(b2, torch.float32)), _ptr(w4), _ptr(b4), _ptr(hidden), _ptr(corr), _ptr(logits),
        _stream()), 'fgr_corr_head_f16x3')
    _end('gemm', t0, 2 * m * (d + 16) * d + 2 * m * d * d + 6 * m * d)
    return corr, logits


def corr_attention(q, k, xyz, q_off, kv_off, kv_seg, v_off, max_q_len, scale) -> torch.Tensor:
    """CorrespondenceDecoder.simple_attention over packed (layer, cloud) segments
    (fgr_corr_attention): -> (rows, 3) softmax-weighted partner coordinates."""
    _dev(q, k, xyz, q_off, kv_off, kv_seg, v_off)
    for t in (q, k):
        assert t.dtype == torch.float32 and t.dim() == 2 and t.stride(1) == 1
    xyz = _c(xyz, torch.float32)
    d = q.shape[1]
    assert k.shape[1] == d and xyz.dim() == 2 and xyz.shape[1] == 3
    assert kv_seg.dtype == torch.int32 and kv_seg.numel() == q_off.numel() - 1
    out = torch.empty((q.shape[0], 3), dtype=torch.float32, device=q.device)
    t0 = _begin('attention')
    _lib.check(_lib.load().fgr_corr_attention(
        _ptr(q), q.stride(0), _ptr(k), k.stride(0), _ptr(xyz), _ptr(out), _ptr(q_off),
        _ptr(kv_off), _ptr(kv_seg), _ptr(v_off), q_off.numel() - 1, int(max_q_len), d,
        float(scale), _stream()), 'fgr_corr_attention')
    _end('attention', t0, lambda: attention_flops(q_off, kv_off, kv_seg, d) // 2)
    return out


def corr_topk_mask(corr, q, k, q_off, kv_off, kv_seg, n_clouds, max_q_len, max_kv_len, scale,
                   n_top) -> torch.Tensor:
    """num_neighbors > 0 of CorrespondenceDecoder.simple_attention (finegrained_regtr.py:
    353-357) on fgr_corr_topk_mask: rows of ``corr`` (the fgr_corr_attention output, same
    segments) outside their direction's top-k index union become NaN, in place. Returns the
    (2, max_kv_len) uint8 union flags (src direction first)."""
    _dev(corr, q, k, q_off, kv_off, kv_seg)
    for t in (q, k):
        assert t.dtype == torch.float32 and t.dim() == 2 and t.stride(1) == 1
    assert corr.dtype == torch.float32 and corr.is_contiguous() and corr.shape == (q.shape[0], 3)
    d = q.shape[1]
    flags = torch.empty((2, max_kv_len), dtype=torch.uint8, device=q.device)
    L = _lib.load()
    nb = _lib._sz(0)
    _lib.check(L.fgr_corr_topk_workspace(q.shape[0], max_kv_len, nb), 'fgr_corr_topk_workspace')
    ws = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=q.device)
    _lib.check(L.fgr_corr_topk_mask(
        _ptr(q), q.stride(0), _ptr(k), k.stride(0), _ptr(corr), _ptr(q_off), _ptr(kv_off),
        _ptr(kv_seg), q_off.numel() - 1, n_clouds, q.shape[0], int(max_q_len), int(max_kv_len), d,
        float(scale), int(n_top), _ptr(flags), _ptr(ws), nb.value, _stream()), 'fgr_corr_topk_mask')
    return flags


# ------------------------------------------------------------------------------------------
# pose
# ------------------------------------------------------------------------------------------
def procrustes(a, b, w, threshold=0.85) -> torch.Tensor:
    """(…, N, 3), (…, N, 3), (…, N) -> (…, 3, 4); threshold None = unthresholded."""
    _dev(a, b, w)
    lead = a.shape[:-2]
    n = a.shape[-2]
    a2 = _c(a, torch.float32).reshape(-1, n, 3)
    b2 = _c(b, torch.float32).reshape(-1, n, 3)
    w2 = _c(w, torch.float32).reshape(-1, n)
    out = torch.empty((a2.shape[0], 3, 4), dtype=torch.float32, device=a.device)
    thr = -1.0 if threshold is None else float(threshold)
    _lib.check(_lib.load().fgr_procrustes(_ptr(a2), _ptr(b2), _ptr(w2), a2.shape[0], n, thr,
                                          _ptr(out), _stream()), 'fgr_procrustes')
    return out.reshape(*lead, 3, 4)


def pair_pose(xyz, corr, logits, seg_off, n_pairs, threshold=0.85) -> torch.Tensor:
    """Pose stage of the forward from packed tensors -> (L, B, 3, 4)."""
    _dev(xyz, corr, logits, seg_off)
    xyz, corr, logits = (_c(t, torch.float32) for t in (xyz, corr, logits))
    n_layers, n_tot = corr.shape[0], corr.shape[1]
    assert xyz.shape == (n_tot, 3) and logits.shape == (n_layers, n_tot)
    assert seg_off.numel() == 2 * n_pairs + 1
    out = torch.empty((n_layers, n_pairs, 3, 4), dtype=torch.float32, device=xyz.device)
    t0 = _begin('pose')
    _lib.check(_lib.load().fgr_pair_pose(_ptr(xyz), _ptr(corr), _ptr(logits), n_tot,
                                         _ptr(seg_off), n_pairs, n_layers, float(threshold),
                                         _ptr(out), _stream()), 'fgr_pair_pose')
    # D4: per (layer, point) xyz 12 + corr 12 + logit 4 = 28 B, + 48 B per pose
    _end('pose', t0, n_layers * (28 * n_tot + 48 * n_pairs))
    return out
