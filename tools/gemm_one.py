"""Runs one fgr_gemm_f16x3 / fgr_gemm_bf16 shape with one tile config N times (development
tool for rocprofv3 --pmc passes). usage: python tools/gemm_one.py M N K cfg [bf16|ln] [iters]
(cfg 'ln': the LayerNorm-fused launch fgr_gemm_f16x3_ln with a positional add)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
import fgreg.linear as lin  # noqa: E402


def main():
    M, N, K = (int(v) for v in sys.argv[1:4])
    cfg = sys.argv[4]
    bf = len(sys.argv) > 5 and sys.argv[5] == 'bf16'
    ln = len(sys.argv) > 5 and sys.argv[5] == 'ln'
    iters = int(sys.argv[6]) if len(sys.argv) > 6 else 50
    if not ln:
        os.environ['FGR_GEMM_BF16_TILE' if bf else 'FGR_GEMM16_TILE'] = cfg
    lin.set_mode('bf16' if bf else 'f16x3')
    dev = torch.device('cuda:0')
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, K, device=dev, generator=g)
    w = torch.randn(N, K, device=dev, generator=g) * 0.05
    out = torch.empty(M, N, device=dev)
    if ln:
        norm = torch.nn.LayerNorm(K).to(dev)
        pos = torch.randn(M, K, device=dev, generator=g)
        assert lin.ln_fusable(M, N, K)
        for _ in range(iters):
            lin.linear_ln(x, norm, w, add=pos, out=out)
        torch.cuda.synchronize()
        print('done', M, N, K, 'ln')
        return
    for _ in range(iters):
        lin.linear(x, w, out=out)
    torch.cuda.synchronize()
    print('done', M, N, K, cfg, 'bf16' if bf else 'f16x3')


if __name__ == '__main__':
    main()
