"""Per-call device time of ops.instnorm on 3DMatch-size segment shapes (two clouds per call,
LeakyReLU, with and without the residual): 20 calls captured in one HIP graph, replayed 10
times, time per call from events around the replays; beside it the HBM floor of the call's
algorithmic bytes (8 N C, + 4 N C with the residual).
usage: [FGREG_LIB_PATH=...] python tools/in_bench.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))

SHAPES = [(20000, 64), (20000, 128), (13389, 128), (13389, 256), (5484, 256), (5484, 512),
          (1060, 512), (1060, 1024)]


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
    import fgreg.ops as ops
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    print(f"{'rows x 2, C':>16} {'res':>4} {'us/call':>9} {'HBM floor us':>13}")
    for n, c in SHAPES:
        lens = [n, n - 1]
        x = torch.randn(sum(lens), c, device=dev) * 2 + 1
        r = torch.randn_like(x)
        off = ops.offsets(lens, dev)
        for res in (None, r):
            us = per_call_us(lambda: ops.instnorm(x, off, lens, residual=res, act=ops.ACT_LEAKY))
            floor = x.numel() * 4 * (2 + (res is not None)) / 8e12 * 1e6
            print(f"{n:>8} x 2, {c:<5} {'y' if res is not None else 'n':>4} {us:9.2f} "
                  f"{floor:13.2f}", flush=True)


if __name__ == '__main__':
    main()
