"""Fused feed-forward sub-layer (ops.ffn, csrc/ffn.hip) at the ModelNet transformer's shape vs
the two-launch path (linear_ln -> linear), graph-free event timing of back-to-back launches
(development tool, GPU box). With FGREG_LIB_PATH pointing at a -DFGR_FFN_STAMP build it also
prints the loop's phase split from the in-kernel clock stamps.
    python tools/ffn_bench.py [rows] [iters]"""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
from fgreg import _lib, ops  # noqa: E402
from fgreg import linear as lin  # noqa: E402


def timeit(fn, iters):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 9544
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    d, f = 256, 1024
    dev = torch.device('cuda')
    torch.manual_seed(0)
    x = 3 + 2 * torch.randn(m, d, device=dev)
    norm = torch.nn.LayerNorm(d).to(dev)
    w1 = torch.randn(f, d, device=dev) / d ** 0.5
    b1 = torch.randn(f, device=dev) * 0.5
    w2 = torch.randn(d, f, device=dev) / f ** 0.5
    b2 = torch.randn(d, device=dev)
    bound = torch.stack([w1.norm(dim=1).max(), b1.abs().max()]).contiguous()
    i1, i2 = lin.weight_image(w1, mode='f16x3'), lin.weight_image(w2, mode='ffn2')
    fused = lambda: ops.ffn(x, norm, i1, b1, i2, b2, bound)                              # noqa: E731
    two = lambda: lin.linear(lin.linear_ln(x, norm, w1, b1, act=ops.ACT_RELU), w2, b2, residual=x)  # noqa: E731
    tf, tt = timeit(fused, iters), timeit(two, iters)
    fl = 4.0 * m * d * f
    print(f'rows {m}: fused {tf:.1f} us ({fl / tf / 1e6:.1f} TF fp32-eq, {fl / tf / 1e6 / 833.3:.3f} of '
          f'the f16x3 pipe), two launches {tt:.1f} us')
    L = _lib.load()
    if hasattr(L, 'fgr_debug_ffn_stamps'):
        L.fgr_debug_ffn_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        fused()
        torch.cuda.synchronize()
        nb = (m + 63) // 64
        buf = (ctypes.c_uint64 * (nb * 32))()
        assert L.fgr_debug_ffn_stamps(ctypes.cast(buf, ctypes.c_void_p), nb) == 0
        a = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 4, 8).astype(np.float64)
        med = np.median(a.reshape(-1, 8), axis=0)
        names = ['prologue', 'dma wait', 'barrier', 'issue', 'mfma', 'read wait', 'epilogue', 'total']
        units = 4 * f // 32
        print('median cycles per wave: ' + ', '.join(f'{n} {v:.0f}' for n, v in zip(names, med)))
        print('per unit: ' + ', '.join(f'{n} {v / units:.0f}' for n, v in zip(names[1:6], med[1:6])))


if __name__ == '__main__':
    main()
