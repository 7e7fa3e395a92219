"""Per-shape device time of fgreg.autograd.wgrad (fgr_gemm_f16x3_wgrad, dW = dY^T X with the
bias gradient) on the ModelNet B=8 training step's weight-gradient shapes: 20 calls in one HIP
graph, replayed 10 times; rate in fp32-equivalent flops (2 rows m n) and against the f16x3 pipe.
usage: [FGR_WGRAD_WGS=...] python tools/wgrad_bench.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))

# (rows, m = cout, n = cin) of the ModelNet B=8 training step (profiles/r05_train_wgrad_table.json):
# transformer in_proj / out_proj / FFN, Res2Net conv1 / splits / conv3, KPConv (m = 15 cin),
# the InfoNCE logits (m = padded positives), the head
SHAPES = [(9544, 768, 256), (9544, 1024, 1792), (9544, 1024, 256), (9544, 256, 1024),
          (9544, 224, 224), (9544, 256, 256), (9544, 3840, 256), (11472, 112, 112),
          (11472, 512, 896), (4753, 4800, 256), (57264, 256, 256), (9544, 1792, 256),
          (11472, 1920, 128)]
PEAK_TF = 2500.0 / 3           # f16x3: three fp16 products per fp32 product


def per_call_us(fn, reps=20, replays=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(replays):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * replays)


def main():
    from fgreg import autograd as ag
    from fgreg import ops
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    print(f"{'rows':>6} {'m':>5} {'n':>5} {'us':>8} {'TF':>7} {'frac':>6} {'MB in':>7}", flush=True)
    tot = 0.0
    for rows, m, n in SHAPES:
        a = torch.randn(rows, m, device=dev)
        b = torch.randn(rows, n, device=dev)
        with ops.PrivateWorkspace():
            us = per_call_us(lambda: ag.wgrad(a, b, bias_grad=True))
        tf = 2.0 * rows * m * n / us / 1e6
        tot += us
        print(f"{rows:>6} {m:>5} {n:>5} {us:8.1f} {tf:7.1f} {tf / PEAK_TF:6.3f} {4 * rows * (m + n) / 1e6:7.1f}",
              flush=True)
    print(f"sum {tot:.1f} us")


if __name__ == '__main__':
    main()
