"""Attention block-count quantisation probe (development tool, GPU): ops.attention at head dim
64 (d 512, 8 heads) on two segments of L queries / keys for L around the 256-block boundary
(16 pairs x ceil(L / 64) blocks), graph-timed.
usage: python tools/attn_quant.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_tiles import timeit  # noqa: E402


def main():
    from fgreg import ops
    dev = torch.device('cuda:0')
    g = torch.Generator(device=dev).manual_seed(0)
    for d, nh in ((512, 8), (256, 8)):
        for L in (960, 1000, 1024, 1025, 1060, 1088, 1100, 1152):
            lens = [L, L]
            n = sum(lens)
            qkv = torch.randn(n, 3 * d, device=dev, generator=g)
            q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
            off = ops.offsets(lens, dev)
            seg = torch.tensor([1, 0], dtype=torch.int32, device=dev)
            out = torch.empty(n, d, device=dev)
            us = timeit(lambda: ops.attention(q, k, v, off, off, seg, L, nh, out=out))
            blocks = 2 * nh * ((L + 63) // 64)
            print(f'd={d} dh={d // nh} L={L:5d} blocks={blocks:4d}: {us:6.1f} us  '
                  f'{us / (L * L):.2e} us/key^2', flush=True)


if __name__ == '__main__':
    main()
