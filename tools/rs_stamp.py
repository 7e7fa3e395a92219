"""Phase timing of the row-stationary GEMM from in-kernel clock stamps (diagnostic build
ablib/libfgreg_stamp.so from tools/build_stamp.sh; GPU box):
    FGREG_LIB_PATH=ablib/libfgreg_stamp.so python tools/rs_stamp.py
Per shape: the launch's span (s_memrealtime, 100 MHz), the block start skew, and per block
(s_memtime cycles): prologue (rows loaded + split), wait for panel 0, the panel loop per panel,
the tail (last panel + epilogue)."""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
import fgreg  # noqa: E402
from fgreg import _lib, ops  # noqa: E402
from fgreg import linear as lin  # noqa: E402

SHAPES = [(9544, 768, 256, 'plain'), (9544, 768, 256, 'ln'), (9544, 1024, 256, 'ln_relu'),
          (9544, 256, 256, 'res'), (57264, 256, 256, 'relu'), (9544, 1792, 256, 'plain'),
          (11472, 896, 128, 'plain'), (40000, 224, 32, 'plain')]


def stamps(L, n=1 << 14):
    buf = (ctypes.c_uint64 * (n * 8))()
    assert L.fgr_debug_rs_stamps(ctypes.cast(buf, ctypes.c_void_p), n) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 8).astype(np.int64)
    a = a[a[:, 6] > 0]
    t = a[:, 0].max()
    return a[a[:, 0] > t - 100000]          # the last launch (1 ms window)


def main():
    torch.manual_seed(0)
    dev = torch.device('cuda')
    L = _lib.load()
    L.fgr_debug_rs_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    for m, n, k, kind in SHAPES:
        x = torch.randn(m, k, device=dev)
        w = torch.randn(n, k, device=dev) / k ** 0.5
        b = torch.randn(n, device=dev)
        r = torch.randn(m, n, device=dev) if kind == 'res' else None
        norm = torch.nn.LayerNorm(k).to(dev)
        pos = torch.randn(m, k, device=dev)

        def run():
            if kind.startswith('ln'):
                return lin.linear_ln(x, norm, w, b, act=ops.ACT_RELU if kind == 'ln_relu' else ops.ACT_NONE,
                                     add=pos)
            return lin.linear(x, w, b, act=ops.ACT_RELU if kind == 'relu' else ops.ACT_NONE, residual=r)
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(20):
            run()
        ev1.record()
        torch.cuda.synchronize()
        us = ev0.elapsed_time(ev1) / 20 * 1e3
        a = stamps(L)
        span = (a[:, 6].max() - a[:, 0].min()) * 0.01           # us
        skew = (a[:, 0] - a[:, 0].min()) * 0.01
        cyc = a[:, 5] - a[:, 1]
        clk = np.median(cyc / np.maximum((a[:, 6] - a[:, 0]) * 0.01, 1e-3)) / 1e3   # GHz
        pro = (a[:, 2] - a[:, 1]) / clk / 1e3
        w0 = (a[:, 3] - a[:, 2]) / clk / 1e3
        np_ = a[:, 7]
        loop = (a[:, 4] - a[:, 3]) / np.maximum(np_ - 1, 1) / clk / 1e3
        tail = (a[:, 5] - a[:, 4]) / clk / 1e3
        tot = cyc / clk / 1e3
        q = lambda v: f'{np.percentile(v, 10):6.2f}/{np.median(v):6.2f}/{np.percentile(v, 90):6.2f}'
        print(f'{m:6d}x{n:5d}x{k:4d} {kind:8s} launch {us:6.1f}us span {span:6.1f}us blocks {len(a):5d} '
              f'panels {int(np.median(np_)):2d} clk {clk:.2f}GHz | p10/med/p90 us: start skew {q(skew)} '
              f'block {q(tot)} prologue {q(pro)} wait0 {q(w0)} per-panel {q(loop)} tail {q(tail)}', flush=True)


if __name__ == '__main__':
    main()
