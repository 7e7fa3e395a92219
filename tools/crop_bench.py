"""Input-side timing: the ModelNet crop test pipeline for a batch of B
raw 2048-point clouds, host (fgreg.transforms, NumPy, one core) vs GPU-resident
(fgreg.transforms_gpu: host draws + csrc/crop.hip), and the two kernels alone (HIP events).

  python tools/crop_bench.py [B] [reps]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
from fgreg import _lib, transforms as T, transforms_gpu as TG  # noqa: E402
from fgreg.synthetic import _box_surface  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    raws = [_box_surface(np.random.default_rng(i), 2048).astype(np.float32) for i in range(B)]
    idx = list(range(B))
    raw_d = [torch.from_numpy(r).cuda() for r in raws]
    TG.modelnet_crop_test_gpu(raw_d, idx)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        [T.modelnet_crop_test(r, i) for r, i in zip(raws, idx)]
    host = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        TG.modelnet_crop_test_gpu(raw_d, idx)
    torch.cuda.synchronize()
    gpu = (time.perf_counter() - t0) / reps
    # kernel time: both entry points timed by the library's own events
    L = _lib.load()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    st = torch.cuda.current_stream()
    ms = []
    orig_mask, orig_asm = L.fgr_crop_pairs_mask, L.fgr_crop_pairs_assemble

    def timed(fn):
        def call(*a):
            ev[0].record(st)
            rc = fn(*a)
            ev[1].record(st)
            ev[1].synchronize()
            ms.append(ev[0].elapsed_time(ev[1]))
            return rc
        return call
    L.fgr_crop_pairs_mask, L.fgr_crop_pairs_assemble = timed(orig_mask), timed(orig_asm)
    try:
        for _ in range(reps):
            TG.modelnet_crop_test_gpu(raw_d, idx)
    finally:
        L.fgr_crop_pairs_mask, L.fgr_crop_pairs_assemble = orig_mask, orig_asm
    k_mask = float(np.median(ms[0::2])) * 1e3
    k_asm = float(np.median(ms[1::2])) * 1e3
    print(f'B={B}: host pipeline {host * 1e3:.2f} ms/batch ({host / B * 1e3:.3f} ms/pair), '
          f'GPU-resident {gpu * 1e3:.2f} ms/batch ({gpu / B * 1e3:.3f} ms/pair, '
          f'{host / gpu:.1f}x); kernels: mask {k_mask:.1f} us, assemble {k_asm:.1f} us')


if __name__ == '__main__':
    main()
