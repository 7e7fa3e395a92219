"""Replays the KPConv gather launches of one ModelNet B=8 forward back to back and prints
per-launch device time (HIP events around 50 replays) and algorithmic GB/s.
usage (GPU box): python tools/gather_probe.py"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
import fgreg  # noqa: E402
from fgreg import ops  # noqa: E402
from fgreg.synthetic import make_batch  # noqa: E402


def main():
    dev = torch.device('cuda:0')
    torch.manual_seed(0)
    model = fgreg.RegTR(fgreg.config.get('modelnet')).to(dev).eval()
    src, tgt, _ = make_batch('modelnet', 8)
    b = {'src_xyz': [torch.from_numpy(s).to(dev) for s in src],
         'tgt_xyz': [torch.from_numpy(t).to(dev) for t in tgt]}
    calls = []
    orig = ops.kpconv_gather

    def rec(*a):
        calls.append(a)
        return orig(*a)
    ops.kpconv_gather = rec
    import fgreg.backbone as bb
    if hasattr(bb, 'ops'):
        bb.ops.kpconv_gather = rec
    with torch.no_grad():
        model(b)
    torch.cuda.synchronize()
    tot_b, tot_t = 0.0, 0.0
    for a in calls:
        q, s, idx, x, kp, ext = a
        nb = ops.gather_bytes(idx, s.shape[0], x.shape[1], kp.shape[0])
        for _ in range(5):
            orig(*a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            orig(*a)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 50
        tot_b += nb
        tot_t += us
        print(f'nq {q.shape[0]:6d} ns {s.shape[0]:6d} width {idx.shape[1]:3d} cin {x.shape[1]:4d} '
              f'valid {(idx < s.shape[0]).float().mean().item() * idx.shape[1]:5.1f}  '
              f'{nb / 1e6:7.1f} MB  {us:7.1f} us  {nb / us / 1e3:6.0f} GB/s')
    print(f'all {len(calls)} launches: {tot_b / 1e6:.1f} MB in {tot_t:.1f} us = '
          f'{tot_b / tot_t / 1e3:.0f} GB/s ({tot_b / tot_t / 1e3 / 8000:.1%} of 8 TB/s)')


if __name__ == '__main__':
    main()
