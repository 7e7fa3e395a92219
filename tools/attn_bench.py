"""Attention microbenchmark (development tool, GPU): ops.attention on the forward's packed
segment shapes, device time from HIP-graph replays, error vs an fp64 reference.
usage: python tools/attn_bench.py [bf16]      (bf16: ops.ATTN_MODE = 'bf16' instead of f16x3)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_tiles import timeit  # noqa: E402

CASES = [('modelnet self', [596] * 16, 256, 8), ('3dmatch self', [1060, 1060], 512, 8),
         ('3dmatch dh32', [1060, 1060], 256, 8), ('3dlomatch', [935, 936], 512, 8)]


def run_case(ops, dev, g, name, lens, d, nh):
    n = sum(lens)
    qkv = torch.randn(n, 3 * d, device=dev, generator=g)
    q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
    off = ops.offsets(lens, dev)
    seg = torch.arange(len(lens), dtype=torch.int32, device=dev)
    out = torch.empty(n, d, device=dev)
    ops.attention(q, k, v, off, off, seg, max(lens), nh, out=out)
    us = timeit(lambda: ops.attention(q, k, v, off, off, seg, max(lens), nh, out=out))
    # fp64 reference on the first segment
    L0, dh = lens[0], d // nh
    qd, kd, vd = (t[:L0].double().view(L0, nh, dh).transpose(0, 1) for t in (q, k, v))
    ref = torch.softmax(qd @ kd.transpose(1, 2) / dh ** 0.5, -1) @ vd
    ref = ref.transpose(0, 1).reshape(L0, d)
    err = float((out[:L0].double() - ref).abs().max() / ref.abs().max())
    flop = 4 * sum(l * l for l in lens) * d
    print(f'{name:14s} {ops.ATTN_MODE} n={n:6d} d={d} heads={nh}: '
          f'{us:7.1f} us  {flop / us / 1e6:6.1f} TF(fp32-eq)  err {err:.1e}', flush=True)


def main():
    from fgreg import ops
    if 'bf16' in sys.argv[1:]:
        ops.ATTN_MODE = 'bf16'
    dev = torch.device('cuda:0')
    g = torch.Generator(device=dev).manual_seed(0)
    for name, lens, d, nh in CASES:
        run_case(ops, dev, g, name, lens, d, nh)


if __name__ == '__main__':
    main()
