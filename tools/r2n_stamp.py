"""Phase split of the f16x3 Res2Net chain (res2net_chain_h3_kernel) from in-kernel clock stamps
(development tool, GPU box; FGREG_LIB_PATH = a -DFGR_R2N_STAMP build): ModelNet's w = 112
bottleneck (128 -> 512, 11472 rows) in eval, median cycles per phase and step over blocks and
waves: build (loads, a = sp + h, row max atomics), barrier 1, split + barrier 2, MFMA +
epilogue, barrier 3.
    FGREG_LIB_PATH=abtest/libfgreg_r2nstamp.so python tools/r2n_stamp.py [rows] [cin cout]"""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
from fgreg import _lib  # noqa: E402
from fgreg.backbone import my_Bottle2neck, my_res2Net  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 11472
    cin, cout = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (128, 512)
    dev = torch.device('cuda')
    torch.manual_seed(0)
    m = my_res2Net(my_Bottle2neck, cin, cout, baseWidth=14, scale=8).to(dev).eval()
    x = torch.randn(n, cin, device=dev)
    with torch.no_grad():
        for _ in range(5):
            m(x)
    torch.cuda.synchronize()
    L = _lib.load()
    L.fgr_debug_r2n_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    nb = min(1024, (n + 31) // 32)
    buf = (ctypes.c_uint64 * (nb * 14 * 36))()
    assert L.fgr_debug_r2n_stamps(ctypes.cast(buf, ctypes.c_void_p), nb) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 14, 36).astype(np.float64)
    w = m.layer1[0].width
    nw = (w + 15) // 16
    a = a[:, :nw]
    print(f'width {w}, {nw} waves, {nb} blocks; total per wave (median): {np.median(a[:, :, 35] - a[:, :, 0]):.0f} cycles')
    names = ['build', 'barrier1', 'split+barrier2', 'mfma+epilogue', 'barrier3']
    for i in range(7):
        t = [a[:, :, 5 * i + k] for k in range(6)]
        t[0] = a[:, :, 0] if i == 0 else a[:, :, 5 * i]
        d = [np.median(t[k + 1] - t[k]) for k in range(5)]
        print(f'  step {i}: ' + '  '.join(f'{nm} {v:6.0f}' for nm, v in zip(names, d)))
    print(f'  tail (copies): {np.median(a[:, :, 35] - a[:, :, 35 - 1 - 0]):.0f}')


if __name__ == '__main__':
    main()
