"""Fused KPConv microbenchmark (development tool, GPU): records every KPConv call of one
forward of the bench workload (real neighbour tables and feature widths), then times
fgr_kpconv_fused against the unfused gather + weight GEMM on each call (device time from
HIP-graph replays) and prints the error of each against the other.
usage: python tools/kpf_bench.py [modelnet|3dmatch|3dlomatch] [variants, e.g. 1236]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_tiles import timeit  # noqa: E402


def main():
    import fgreg
    from fgreg import backbone, ops
    from fgreg import linear as lin
    from fgreg.synthetic import make_batch
    wl = sys.argv[1] if len(sys.argv) > 1 else 'modelnet'
    if wl == '3dlomatch':
        fgreg.set_precision('bf16')
    dev = torch.device('cuda:0')
    torch.manual_seed(0)
    np.random.seed(0)
    cfg = fgreg.config.get(wl)
    model = fgreg.RegTR(cfg).eval().to(dev)
    B = 8 if wl == 'modelnet' else 1
    src, tgt, _ = make_batch(wl, B)
    calls = []
    orig = backbone.KPConv.forward_unnormalized

    def rec(self, q, s, idx, x):
        calls.append((self, q, s, idx, x))
        return orig(self, q, s, idx, x)
    backbone.KPConv.forward_unnormalized = rec
    with torch.no_grad():
        model({'src_xyz': [torch.from_numpy(a).to(dev) for a in src],
               'tgt_xyz': [torch.from_numpy(a).to(dev) for a in tgt]})
    backbone.KPConv.forward_unnormalized = orig
    tot_u = 0.0
    tot_f = {}
    variants = sys.argv[2] if len(sys.argv) > 2 else '1'
    with torch.no_grad():
        for conv, q, s, idx, x in calls:
            cin, cout = x.shape[1], conv.out_channels
            mode = backbone._kpf_mode(cin, conv.K)
            if mode is None:
                continue

            def unfused():
                wf, nn_ = ops.kpconv_gather(q, s, idx, x, conv.kernel_points, conv.KP_extent)
                return lin.linear(wf.view(wf.shape[0], -1), conv.weights, transpose=True), nn_

            def fused():
                return ops.kpconv_fused(q, s, idx, x, conv.kernel_points, conv.KP_extent,
                                        conv.weights, mode)
            a, na = unfused()
            tu = timeit(unfused)
            tot_u += tu
            v = float((idx < s.shape[0]).float().sum(1).mean())
            msg = []
            for var in variants:
                os.environ['FGR_KPF_TILE'] = var
                b, nb = fused()
                err = float((a - b).abs().max() / a.abs().max().clamp_min(1e-30))
                tf = timeit(fused)
                tot_f[var] = tot_f.get(var, 0.0) + tf
                msg.append(f'{var}: {tf:6.1f} ({tf / tu:.2f}x, {err:.0e}'
                           f'{"" if torch.equal(na, nb) else " NNORM DIFF"})')
            print(f'nq {q.shape[0]:6d} ns {s.shape[0]:6d} H {idx.shape[1]:3d} v {v:5.1f} '
                  f'cin {cin:4d} cout {cout:4d}: unfused {tu:6.1f} us | ' + '  '.join(msg),
                  flush=True)
    print(f'total: unfused {tot_u:.1f} us | ' + '  '.join(
        f'{k}: {t:.1f} ({t / max(tot_u, 1e-9):.2f}x)' for k, t in tot_f.items()))


if __name__ == '__main__':
    main()
