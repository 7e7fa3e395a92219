"""Times the row-resident f16x3 GEMM (fgr_gemm_rows_f16x3, LayerNorm fused) against the
LayerNorm launch + tiled f16x3 GEMM it replaces, at the transformer / head shapes of the
bench workload (development tool, GPU)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
import fgreg.linear as lin  # noqa: E402
import fgreg.ops as ops  # noqa: E402
from microbench import timeit  # noqa: E402


def main():
    dev = torch.device('cuda:0')
    lin.set_mode('f16x3')
    shapes = [(9493, 768, 256, True), (9493, 1024, 256, True), (9493, 256, 256, False),
              (56958, 256, 256, False), (11472, 896, 128, False), (56958, 3, 256, False),
              (56958, 1, 256, False)]
    for (M, N, K, with_ln) in shapes:
        x = torch.randn(M, K, device=dev)
        pos = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) / K ** 0.5
        b = torch.randn(N, device=dev)
        ln = torch.nn.LayerNorm(K).to(dev) if with_ln else None
        add = pos if with_ln else None

        def unfused():
            lin.ROWS = '0'
            return lin.linear(x, w, b, ln=ln, add=add)

        def fused():
            lin.ROWS = '2'
            return lin.linear(x, w, b, ln=ln, add=add)
        ref, got = unfused(), fused()
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        tu, tf = timeit(unfused, 20), timeit(fused, 20)
        print(f'M={M:6d} N={N:5d} K={K:4d} ln={int(with_ln)}: tiled(+LN) {tu:7.1f} us  '
              f'rows {tf:7.1f} us  rel {err:.1e}', flush=True)
    lin.ROWS = '1'


if __name__ == '__main__':
    main()
