"""The weight-split GEMM (csrc/gemm_ws.hip) on the ModelNet transformer's K = 256 shapes against
the row-stationary / k-looped dispatch (FGR_GEMM_WS=0 in a child process), event timing of
back-to-back launches (development tool, GPU box). With FGREG_LIB_PATH pointing at a
-DFGR_WS_STAMP build it prints the phase split of the in-kernel clock stamps.
    python tools/ws_bench.py [iters]"""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))
from fgreg import _lib, ops  # noqa: E402
from fgreg import linear as lin  # noqa: E402


def timeit(fn, iters):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device('cuda')
    torch.manual_seed(0)
    m, d, nh = 9544, 256, 8
    x = torch.randn(m, d, device=dev)
    pos = torch.randn(m, d, device=dev)
    norm = torch.nn.LayerNorm(d).to(dev)
    w3 = torch.randn(3 * d, d, device=dev) / d ** 0.5
    b3 = torch.randn(3 * d, device=dev)
    w1 = torch.randn(d, d, device=dev) / d ** 0.5
    b1 = torch.randn(d, device=dev)
    off = ops.offsets([m // 2, m - m // 2], dev)
    seg = torch.tensor([0, 1], dtype=torch.int32, device=dev)
    i3 = lin.weight_image(w3, mode='f16x3')
    L = _lib.load()
    nb = _lib._sz(0)
    L.fgr_kv_image_bytes(m, nh, d // nh, nb)
    img = torch.empty(nb.value, dtype=torch.uint8, device=dev)
    q = torch.empty(m, d, device=dev)

    def qkv():
        _lib.check(L.fgr_gemm_f16x3_ln_qkv(
            x.data_ptr(), d, norm.weight.data_ptr(), norm.bias.data_ptr(), 1e-5, pos.data_ptr(), d,
            i3.img.data_ptr(), q.data_ptr(), d, b3.data_ptr(), m, d, nh, img.data_ptr(), None, None,
            None, 0, ops._stream()), 'qkv')
    out2 = torch.empty(m, d, device=dev)

    def qkv2():
        _lib.check(L.fgr_gemm_f16x3_ln_qkv(
            x.data_ptr(), d, norm.weight.data_ptr(), norm.bias.data_ptr(), 1e-5, pos.data_ptr(), d,
            i3.img.data_ptr(), q.data_ptr(), d, b3.data_ptr(), m, d, nh, img.data_ptr(),
            norm.weight.data_ptr(), norm.bias.data_ptr(), out2.data_ptr(), d, ops._stream()), 'qkv2')
    cases = {'in_proj LN+pos+KV 9544x768x256': qkv,
             'in_proj LN+pos+KV+out2 9544x768x256': qkv2,
             'out_proj +res 9544x256x256': lambda: lin.linear(x, w1, b1, residual=pos),
             'plain 9544x768x256': lambda: lin.linear(x, w3, b3)}
    # blocks per launch (stamps of blocks a launch did not run are stale): the split in_proj
    # runs three 64-row blocks per row tile, the others one 48-row block
    nblocks = {'in_proj LN+pos+KV 9544x768x256': 3 * ((m + 63) // 64),
               'in_proj LN+pos+KV+out2 9544x768x256': 3 * ((m + 63) // 64),
               'out_proj +res 9544x256x256': (m + 47) // 48,
               'plain 9544x768x256': (m + 47) // 48}
    for name, fn in cases.items():
        print(f'{name}: {timeit(fn, iters):.1f} us')
    if hasattr(L, 'fgr_debug_ws_stamps'):
        L.fgr_debug_ws_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        for name, fn in cases.items():
            fn()
            torch.cuda.synchronize()
            nbk = min(nblocks[name], 2048)
            buf = (ctypes.c_uint64 * (nbk * 32))()
            assert L.fgr_debug_ws_stamps(ctypes.cast(buf, ctypes.c_void_p), nbk) == 0
            a = np.frombuffer(buf, dtype=np.uint64).reshape(nbk, 4, 8).astype(np.float64)
            t0 = a[:, :, 0].min()
            rel = a - a[:, :, :1]
            print(f'  {name}: block start spread {np.median(a[:, 0, 0] - t0):.0f} (median) / '
                  f'{np.max(a[:, 0, 0] - t0):.0f} (max) cycles, last block end {np.max(a[:, :, 3]) - t0:.0f}; '
                  f'median per wave: prologue '
                  f'{np.median(rel[:, :, 1]):.0f}, ' + ', '.join(
                      f'pass{p} mfma {np.median(rel[:, :, 2 + 2 * p] - rel[:, :, 1 + 2 * p if p else 1]):.0f} '
                      f'epi {np.median(rel[:, :, 3 + 2 * p] - rel[:, :, 2 + 2 * p]):.0f}'
                      for p in range(3) if np.median(a[:, :, 3 + 2 * p]) > 0) +
                  (f', stores {np.median(rel[:, :, 7] - rel[:, :, 3]):.0f} (p90 '
                   f'{np.percentile(rel[:, :, 7] - rel[:, :, 3], 90):.0f}), wave total '
                   f'{np.median(rel[:, :, 7]):.0f} (p90 {np.percentile(rel[:, :, 7], 90):.0f})'
                   if np.median(a[:, :, 7]) > 0 else ''))


if __name__ == '__main__':
    main()
