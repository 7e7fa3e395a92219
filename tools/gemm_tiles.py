"""GEMM tile sweep (development tool, GPU): times fgr_gemm_f16x3 per tile configuration
(FGR_GEMM16_TILE) on the forward's shapes and checks every variant against an fp64 product.
usage: python tools/gemm_tiles.py [configs] [bf16] [3d] [ks] > gpurun_out/gemm_tiles.txt
(bf16: fgr_gemm_bf16 with FGR_GEMM_BF16_TILE, checked against bf16-rounded operands)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
import fgreg.linear as lin  # noqa: E402

SHAPES = [(9544, 768, 256), (9544, 1024, 2048), (9544, 256, 1024), (9544, 256, 3840),
          (9544, 256, 256), (9544, 1024, 256), (11472, 512, 1024), (11472, 128, 1920),
          (9544, 1792, 256), (57264, 256, 256), (11472, 896, 128), (2120, 1536, 512),
          (2120, 512, 1024), (2120, 512, 512), (26778, 256, 512), (40000, 128, 256),
          (9543, 130, 1000), (333, 896, 128)]
# the 3DMatch / 3DLoMatch transformer and head shapes (2 x 1060 tokens) and its decoder
SHAPES_3D = [(2120, 1536, 512), (2120, 512, 1024), (2120, 512, 512), (2120, 1024, 512),
             (2120, 1024, 2048), (2120, 256, 3840), (2120, 128, 1920), (2120, 256, 1024),
             (2120, 256, 512), (2120, 896, 128), (2120, 1792, 256), (10967, 128, 1920),
             (10967, 512, 1024), (12720, 512, 512), (10967, 256, 512), (10967, 64, 960)]


def timeit(fn, iters=20):
    """Device time per call: `iters` calls captured in one HIP graph (the forward replays its
    GEMMs from a graph too), so host launch overhead does not enter small shapes."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(iters):
            fn()
    graph.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        graph.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (3 * iters) * 1e3


# split-K factors swept per tile ('' = the dispatcher's own choice): `ks` in argv sweeps 1/2/4/8
KSPLITS = ['']


def main():
    global KSPLITS
    cfgs = sys.argv[1] if len(sys.argv) > 1 else 'btukABCDEFGHIJ'
    if 'ks' in sys.argv[2:]:
        KSPLITS = ['1', '2', '4', '8']
    bf = 'bf16' in sys.argv[2:]
    shapes = SHAPES_3D if '3d' in sys.argv[2:] else SHAPES
    if os.environ.get('GEMM_SHAPES'):          # "M,N,K;M,N,K": these shapes only
        shapes = [tuple(int(v) for v in t.split(',')) for t in os.environ['GEMM_SHAPES'].split(';')]
    env = 'FGR_GEMM_BF16_TILE' if bf else 'FGR_GEMM16_TILE'
    dev = torch.device('cuda:0')
    lin.set_mode('bf16' if bf else 'f16x3')
    g = torch.Generator(device=dev).manual_seed(0)
    for (M, N, K) in shapes:
        x = torch.randn(M, K, device=dev, generator=g)
        w = torch.randn(N, K, device=dev, generator=g) * 0.05
        if bf:
            ref = x.bfloat16().double() @ w.bfloat16().double().t()
        else:
            ref = (x.double() @ w.double().t())
        line = f'M={M:6d} N={N:5d} K={K:5d}'
        best = None
        variants = [(t, ks) for t in cfgs for ks in KSPLITS]
        for t, ks in variants:
            os.environ[env] = t
            os.environ['FGR_GEMM_KSPLIT'] = ks
            out = torch.empty(M, N, device=dev)
            y = lin.linear(x, w, out=out)
            err = float((y.double() - ref).abs().max() / ref.abs().max())
            us = timeit(lambda: lin.linear(x, w, out=out))
            tf = 2 * M * N * K / us / 1e6
            tag = t + (f'/{ks}' if ks else '')
            line += f' | {tag} {us:6.1f}us {tf:5.0f}TF{"" if err < 1e-5 else " ERR%.1e" % err}'
            if best is None or us < best[1]:
                best = (tag, us)
        os.environ[env] = ''
        os.environ['FGR_GEMM_KSPLIT'] = ''
        us0 = timeit(lambda: lin.linear(x, w, out=out))
        print(line + f' || default {us0:6.1f}us best {best[0]}', flush=True)


if __name__ == '__main__':
    main()
