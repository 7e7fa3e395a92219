"""GEMM probe for PMC passes (development tool): times one dense-layer shape of the
forward with the selected split mode, `iters` launches after a warmup.
usage: python tools/gemm_probe.py M N K [iters] [mode]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
import fgreg.linear as lin  # noqa: E402

M, N, K = (int(a) for a in sys.argv[1:4])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
lin.set_mode(sys.argv[5] if len(sys.argv) > 5 else 'f16x3')
dev = torch.device('cuda:0')
x = torch.randn(M, K, device=dev)
w = torch.randn(N, K, device=dev)
for _ in range(3):
    lin.linear(x, w)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(iters):
    lin.linear(x, w)
b.record()
torch.cuda.synchronize()
us = a.elapsed_time(b) / iters * 1e3
print(f'M={M} N={N} K={K} {lin.MODE}: {us:.1f} us {2 * M * N * K / us / 1e6:.1f} TF', flush=True)
