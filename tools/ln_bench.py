"""LayerNorm microbenchmark (development tool, GPU): ops.layernorm at the transformer's
shapes, with the pending bias and the added residual, device time from HIP-graph replays
(FGR_LN_LPR selects the lanes per row). usage: python tools/ln_bench.py"""
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
    for n, d in [(9544, 256), (2120, 512), (2120, 256)]:
        x = torch.randn(n, d, device=dev)
        add = torch.randn(n, d, device=dev)
        pb = torch.randn(d, device=dev)
        g, b = torch.randn(d, device=dev), torch.randn(d, device=dev)
        out = torch.empty(n, d, device=dev)
        for lpr in ('', '32', '64'):
            os.environ['FGR_LN_LPR'] = lpr
            us = timeit(lambda: ops.layernorm(x, g, b, 1e-5, add=add, out=out))
            us2 = timeit(lambda: ops.layernorm(x, g, b, 1e-5, pre_bias=pb, add=add, out=out))
            print(f'n={n} d={d} lpr={lpr or "default"}: {us:6.2f} us ({3 * n * d * 4 / us / 1e3:5.0f} GB/s), '
                  f'with pre-bias {us2:6.2f} us ({4 * n * d * 4 / us2 / 1e3:5.0f} GB/s)', flush=True)


if __name__ == '__main__':
    main()
