"""Row-stationary GEMM sweep (development tool, GPU): times fgr_gemm_f16x3 on the forward's
K <= 256 shapes for the k-looped default (FGR_GEMM_RS=0 behaviour via FGR_GEMM16_TILE of the
old choice) and the rs kernel at row tiles RT in {1, 2} and panels per block NC, each variant
checked against an fp64 product.
usage: python tools/rs_sweep.py > gpurun_out/rs_sweep.txt"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import fgreg.linear as lin  # noqa: E402
from gemm_tiles import timeit  # noqa: E402

SHAPES = [(9544, 768, 256), (9544, 256, 256), (9544, 1024, 256), (9544, 1792, 256),
          (57264, 256, 256), (11472, 896, 128), (9544, 896, 128), (11472, 512, 256),
          (11472, 128, 256), (57264, 3, 256), (57264, 1, 256), (40000, 128, 256),
          (2120, 896, 128), (2120, 1792, 256), (26778, 256, 128), (40000, 224, 32),
          (26778, 448, 64), (26778, 64, 256)]
# the k-looped kernel the dispatcher picked before the rs kernel (gemm16.hip h3_tile_kloop)
OLD = {(9544, 768, 256): 'y', (9544, 256, 256): 'X', (9544, 1024, 256): 'y',
       (9544, 1792, 256): 'y', (57264, 256, 256): 'X', (11472, 896, 128): 'y',
       (9544, 896, 128): 'y', (11472, 512, 256): 'y', (11472, 128, 256): 'X',
       (57264, 3, 256): 'X', (57264, 1, 256): 'X', (40000, 128, 256): 'X',
       (2120, 896, 128): 'X', (2120, 1792, 256): 'Y', (26778, 256, 128): 'X',
       (40000, 224, 32): 'X', (26778, 448, 64): 'X', (26778, 64, 256): 'X'}
VARIANTS = [('2', ''), ('1', ''), ('2', '0'), ('2', '4'), ('2', '8'), ('2', '16')]


def main():
    dev = torch.device('cuda:0')
    lin.set_mode('f16x3')
    g = torch.Generator(device=dev).manual_seed(0)
    for (M, N, K) in SHAPES:
        x = torch.randn(M, K, device=dev, generator=g)
        w = torch.randn(N, K, device=dev, generator=g) * 0.05
        b = torch.randn(N, device=dev, generator=g)
        ref = x.double() @ w.double().t() + b.double()
        out = torch.empty(M, N, device=dev)
        os.environ['FGR_GEMM16_TILE'] = OLD[(M, N, K)]
        us_old = timeit(lambda: lin.linear(x, w, b, out=out))
        line = f'M={M:6d} N={N:5d} K={K:4d} | old {OLD[(M, N, K)]} {us_old:6.1f}us'
        os.environ['FGR_GEMM16_TILE'] = 'z'
        best = None
        for rt, nc in VARIANTS:
            os.environ['FGR_RS_RT'], os.environ['FGR_RS_NC'] = rt, nc
            y = lin.linear(x, w, b, out=out)
            err = float((y.double() - ref).abs().max() / ref.abs().max())
            us = timeit(lambda: lin.linear(x, w, b, out=out))
            line += f' | rt{rt}/nc{nc or "auto"} {us:6.1f}us{"" if err < 2e-6 else " ERR%.1e" % err}'
            if best is None or us < best[1]:
                best = (f'rt{rt}/nc{nc or "auto"}', us)
        os.environ['FGR_RS_RT'], os.environ['FGR_RS_NC'] = '', ''
        os.environ['FGR_GEMM16_TILE'] = ''
        print(line + f' || best {best[0]} {us_old / best[1]:.2f}x', flush=True)


if __name__ == '__main__':
    main()
