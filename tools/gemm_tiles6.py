"""Pre-split f16x3 GEMM sweep (development tool, GPU): the A operand split once by
fgr_split_rows_h3 (timed separately), fgr_gemm_h3_presplit per FGR_GEMM_G6_TILE config,
checked against fp64. usage: python tools/gemm_tiles6.py [configs]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
import fgreg.linear as lin  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_tiles import SHAPES, timeit  # noqa: E402


def main():
    cfgs = sys.argv[1] if len(sys.argv) > 1 else 'abcdefgh'
    # upper-case configs: one scale per row (FGR_SPLIT_RS=1 split); do not mix with lower case
    if cfgs.isupper():
        os.environ['FGR_SPLIT_RS'] = '1'
    dev = torch.device('cuda:0')
    lin.set_mode('f16x3')
    g = torch.Generator(device=dev).manual_seed(0)
    for (M, N, K) in SHAPES:
        x = torch.randn(M, K, device=dev, generator=g)
        w = torch.randn(N, K, device=dev, generator=g) * 0.05
        ref = x.double() @ w.double().t()
        out = torch.empty(M, N, device=dev)
        a = lin.split_rows(x)
        us_split = timeit(lambda: lin.split_rows(x, a))
        line = f'M={M:6d} N={N:5d} K={K:5d} | split {us_split:5.1f}us'
        for t in cfgs:
            os.environ['FGR_GEMM_G6_TILE'] = t
            y = lin.linear_presplit(a, w, out=out)
            err = float((y.double() - ref).abs().max() / ref.abs().max())
            us = timeit(lambda: lin.linear_presplit(a, w, out=out))
            tf = 2 * M * N * K / us / 1e6
            line += f' | {t} {us:6.1f}us {tf:5.0f}TF{"" if err < 2e-6 else " ERR%.1e" % err}'
        os.environ['FGR_GEMM_G6_TILE'] = ''
        us0 = timeit(lambda: lin.linear(x, w, out=out))
        print(line + f' || current {us0:6.1f}us', flush=True)


if __name__ == '__main__':
    main()
