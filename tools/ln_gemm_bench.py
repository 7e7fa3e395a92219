"""LayerNorm + Linear: fused (fgr_gemm_f16x3_ln) vs ops.layernorm then linear() on the ModelNet
transformer shapes (development tool, GPU; device time from HIP-graph replays).
usage: python tools/ln_gemm_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_tiles import timeit  # noqa: E402


def main():
    from fgreg import linear as fl
    from fgreg import ops
    dev = torch.device('cuda:0')
    torch.manual_seed(0)
    for m, n, k, pos, act in ((9544, 768, 256, True, 0), (9544, 1024, 256, False, 2),
                              (20000, 768, 256, True, 0)):
        x = torch.randn(m, k, device=dev) + 1
        p = torch.randn(m, k, device=dev) if pos else None
        norm = torch.nn.LayerNorm(k).to(dev)
        w = torch.randn(n, k, device=dev) / 16
        b = torch.randn(n, device=dev)
        out = torch.empty(m, n, device=dev)
        fused = fl.ln_fusable(m, n, k)
        t_f = timeit(lambda: fl.linear_ln(x, norm, w, b, act=act, add=p, out=out))
        fl.LN_FUSE = False
        h = torch.empty(m, k, device=dev)
        t_ln = timeit(lambda: ops.layernorm(x, norm.weight, norm.bias, norm.eps, add=p, out=h))
        t_g = timeit(lambda: fl.linear(h, w, b, act=act, out=out))
        fl.LN_FUSE = True
        print(f'{m}x{n}x{k} pos={pos} act={act} fused={fused}: fused {t_f:6.1f} us | '
              f'layernorm {t_ln:5.1f} + gemm {t_g:5.1f} = {t_ln + t_g:6.1f} us', flush=True)
        if 'sweep' in sys.argv[1:]:          # W panels per block of the fused launch
            res = []
            for nc in (4, 6, 8, 12, 16, 24, 48):
                os.environ['FGR_RS_NC'] = str(nc)
                res.append(f'nc{nc} {timeit(lambda: fl.linear_ln(x, norm, w, b, act=act, add=p, out=out)):5.1f}')
            os.environ.pop('FGR_RS_NC')
            print('   fused by nc: ' + ' | '.join(res), flush=True)


if __name__ == '__main__':
    main()
