"""Tile sweep of the forward's long-contraction GEMMs only (development tool, GPU): every
FGR_GEMM16_TILE variant on 9544x1024x2048, 11472x512x1024, 9544x256x3840, 9544x256x1024,
graph-timed, each checked against fp64.
usage: python tools/gemm_longk.py > gpurun_out/gemm_longk.txt"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import fgreg.linear as lin  # noqa: E402
from gemm_tiles import timeit  # noqa: E402

SHAPES = [(9544, 1024, 2048), (11472, 512, 1024), (9544, 256, 3840), (9544, 256, 1024)]
CFGS = 'abcdefghijklmnopqrstuvwxy' + 'ABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789'


def main():
    dev = torch.device('cuda:0')
    lin.set_mode('f16x3')
    g = torch.Generator(device=dev).manual_seed(0)
    for (M, N, K) in SHAPES:
        x = torch.randn(M, K, device=dev, generator=g)
        w = torch.randn(N, K, device=dev, generator=g) * 0.05
        ref = x.double() @ w.double().t()
        out = torch.empty(M, N, device=dev)
        os.environ['FGR_GEMM16_TILE'] = ''
        us0 = timeit(lambda: lin.linear(x, w, out=out))
        res = []
        for t in CFGS:
            os.environ['FGR_GEMM16_TILE'] = t
            try:
                y = lin.linear(x, w, out=out)
            except RuntimeError:
                continue
            err = float((y.double() - ref).abs().max() / ref.abs().max())
            if err > 1e-5:
                res.append((1e9, t + '!ERR'))
                continue
            res.append((timeit(lambda: lin.linear(x, w, out=out)), t))
        os.environ['FGR_GEMM16_TILE'] = ''
        res.sort()
        print(f'M={M} N={N} K={K}: default {us0:.1f} us | best ' +
              ' '.join(f'{t}:{u:.1f}' for u, t in res[:6]), flush=True)


if __name__ == '__main__':
    main()
