"""Row-stationary GEMM at K = 384..512 (development tool, GPU): the default dispatch vs the rs
kernel (FGR_GEMM16_TILE=z) at panels per block NC (auto / 4 / 8 / 16) and with the deferred
epilogue (FGR_RS_DEFER), graph-timed, each checked against fp64.
usage: python tools/rs512_sweep.py > gpurun_out/rs512_sweep.txt"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import fgreg.linear as lin  # noqa: E402
from gemm_tiles import timeit  # noqa: E402

SHAPES = [(2120, 1536, 512), (2120, 512, 512), (2120, 1024, 512), (2120, 256, 512),
          (12720, 512, 512), (10967, 256, 512), (26778, 256, 512), (10967, 128, 512),
          (11226, 512, 512), (1871, 1536, 512), (8568, 256, 512), (2120, 896, 384)]
VARIANTS = [('', '0'), ('', '1'), ('4', '0'), ('8', '0'), ('16', '0'), ('8', '1')]


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
        us_def = timeit(lambda: lin.linear(x, w, b, out=out))
        line = f'M={M:6d} N={N:5d} K={K:4d} | default {us_def:6.1f}us'
        os.environ['FGR_GEMM16_TILE'] = 'z'
        best = None
        for nc, d in VARIANTS:
            os.environ['FGR_RS_NC'], os.environ['FGR_RS_DEFER'] = nc, d
            y = lin.linear(x, w, b, out=out)
            err = float((y.double() - ref).abs().max() / ref.abs().max())
            us = timeit(lambda: lin.linear(x, w, b, out=out))
            tag = f'nc{nc or "auto"}/d{d}'
            line += f' | {tag} {us:6.1f}us{"" if err < 2e-6 else " ERR%.1e" % err}'
            if best is None or us < best[1]:
                best = (tag, us)
        for e in ('FGR_GEMM16_TILE', 'FGR_RS_NC', 'FGR_RS_DEFER'):
            os.environ[e] = ''
        print(line + f' || best {best[0]} {us_def / best[1]:.2f}x', flush=True)


if __name__ == '__main__':
    main()
