"""Library fp16 GEMM throughput on the forward's shapes (development tool, GPU): what hipBLASLt
reaches on the same skinny shapes, as a ceiling estimate for the hand-written kernels.
usage: python tools/blas_ceiling.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_tiles import SHAPES, timeit  # noqa: E402


def main():
    dev = torch.device('cuda:0')
    for (M, N, K) in SHAPES:
        line = f'M={M:6d} N={N:5d} K={K:5d}'
        for dt in (torch.float16, torch.bfloat16, torch.float32):
            a = torch.randn(M, K, device=dev).to(dt)
            b = torch.randn(N, K, device=dev).to(dt)
            o = torch.empty(M, N, device=dev, dtype=dt)
            us = timeit(lambda: torch.mm(a, b.t(), out=o))
            line += f' | {str(dt)[6:]} {us:6.1f}us {2 * M * N * K / us / 1e6:6.0f}TF'
        print(line, flush=True)


if __name__ == '__main__':
    main()
