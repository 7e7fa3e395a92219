"""A/B of the row-stationary GEMM's panel loop (development tool, GPU): FGR_RS_DEFER=0 (epilogue
right after each panel's MFMAs) vs 1 (the previous panel's epilogue after this panel's MFMAs),
graph-timed on the forward's rs shapes (plain, + residual, + LayerNorm prologue), each checked
against fp64. usage: python tools/rs_defer_ab.py > gpurun_out/rs_defer_ab.txt"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import fgreg.linear as lin  # noqa: E402
from fgreg import ops  # noqa: E402
from gemm_tiles import timeit  # noqa: E402

# (M, N, K, kind): kind '' plain, 'r' residual, 'ln' LayerNorm prologue + pos add, 'relu'
SHAPES = [(9544, 768, 256, 'ln'), (9544, 1024, 256, 'ln'), (9544, 1792, 256, ''),
          (57264, 256, 256, 'relu'), (11472, 896, 128, ''), (9544, 896, 128, ''),
          (40000, 224, 32, ''), (26778, 448, 64, ''), (9544, 256, 256, 'r'), (9544, 768, 256, ''),
          (2120, 896, 128, ''), (26778, 256, 128, '')]


def main():
    dev = torch.device('cuda:0')
    lin.set_mode('f16x3')
    g = torch.Generator(device=dev).manual_seed(0)
    os.environ['FGR_GEMM16_TILE'] = 'z'
    for (M, N, K, kind) in SHAPES:
        x = torch.randn(M, K, device=dev, generator=g)
        w = torch.randn(N, K, device=dev, generator=g) * 0.05
        b = torch.randn(N, device=dev, generator=g)
        r = torch.randn(M, N, device=dev, generator=g) if kind == 'r' else None
        pos = torch.randn(M, K, device=dev, generator=g)
        norm = torch.nn.LayerNorm(K).to(dev)
        out = torch.empty(M, N, device=dev)
        act = ops.ACT_RELU if kind == 'relu' else ops.ACT_NONE
        if kind == 'ln':
            xin = torch.nn.functional.layer_norm(x.double(), (K,)) + pos.double()
            f = lambda: lin.linear_ln(x, norm, w, b, add=pos, out=out)
        else:
            xin = x.double()
            f = lambda: lin.linear(x, w, b, act=act, residual=r, out=out)
        ref = xin @ w.double().t() + b.double()
        if r is not None:
            ref = ref + r.double()
        if act == ops.ACT_RELU:
            ref = ref.clamp_min(0)
        line = f'M={M:6d} N={N:5d} K={K:4d} {kind or "plain":5s}'
        res = {}
        for d in ('0', '1'):
            os.environ['FGR_RS_DEFER'] = d
            y = f()
            err = float((y.double() - ref).abs().max() / ref.abs().max())
            res[d] = timeit(f)
            line += f' | defer{d} {res[d]:6.1f}us{"" if err < 2e-6 else " ERR%.1e" % err}'
        os.environ['FGR_RS_DEFER'] = '0'
        print(line + f' || {res["0"] / res["1"]:.3f}x', flush=True)


if __name__ == '__main__':
    main()
