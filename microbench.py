"""Per-op micro-benchmark on the GPU (development tool): times the attention core in both
precision modes at the bench workload's shapes (16 clouds x ~600 superpoints, d 256,
8 heads) with HIP events, and prints fp32-equivalent TFLOP/s."""
import sys
import time

import torch

sys.path.insert(0, 'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd')
import fgreg.ops as ops  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def attention(lens=(600,) * 16, d=256, nh=8):
    dev = torch.device('cuda:0')
    n = sum(lens)
    qkv = torch.randn(n, 3 * d, device=dev)
    off = ops.offsets(list(lens), dev)
    B = len(lens) // 2
    cross = torch.tensor([(c + B) % len(lens) for c in range(len(lens))], dtype=torch.int32, device=dev)
    flops = sum(4 * l * lens[(i + B) % len(lens)] * d for i, l in enumerate(lens))
    for mode in ('fp32', 'bf16x6', 'f16x3'):
        ops.ATTN_MODE = mode
        us = timeit(lambda: ops.attention(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], off, off,
                                          cross, max(lens), nh))
        print(f'attention {mode:7s} lens={lens[0]}x{len(lens)} d={d}: {us:8.1f} us  '
              f'{flops / us / 1e6:7.1f} TFLOP/s fp32-equivalent', flush=True)


def gemm_shapes():
    """Records every linear() call of one bench forward (B = 8 ModelNet pairs) and times each
    shape in both GEMM modes."""
    import collections
    import numpy as np
    import fgreg
    import fgreg.linear as lin
    from fgreg.synthetic import make_batch
    dev = torch.device('cuda:0')
    cfg = fgreg.config.get('modelnet')
    torch.manual_seed(0)
    model = fgreg.RegTR(cfg).to(dev).eval()
    src, tgt, _ = make_batch('modelnet', 8)
    batch = {'src_xyz': [torch.from_numpy(a).to(dev) for a in src],
             'tgt_xyz': [torch.from_numpy(a).to(dev) for a in tgt]}
    calls = []
    orig = lin.linear

    def rec(x, w, bias=None, act=0, residual=None, transpose=False, tag=None, out=None):
        n = w.shape[-1] if transpose else w.shape[0]
        calls.append((x.shape[0], n, x.shape[1], transpose, residual is not None))
        return orig(x, w, bias, act, residual, transpose, tag, out)
    import fgreg.backbone as bb, fgreg.transformer as tr, fgreg.regtr as rr
    for m in (lin, bb, tr, rr):
        if hasattr(m, 'linear'):
            m.linear = rec
    with torch.no_grad():
        model(batch)
    for m in (lin, bb, tr, rr):
        if hasattr(m, 'linear'):
            m.linear = orig
    shapes = collections.Counter(calls)
    modes = ('fp32', 'bf16x6', 'f16x3')
    tot = {m: 0.0 for m in modes}
    flops = 0
    for (M, N, K, tp, res), cnt in sorted(shapes.items(), key=lambda kv: -kv[0][0] * kv[0][1] * kv[0][2] * kv[1]):
        x = torch.randn(M, K, device=dev)
        w = torch.randn(K, N, device=dev) if tp else torch.randn(N, K, device=dev)
        r = torch.randn(M, N, device=dev) if res else None
        line = f'M={M:6d} N={N:5d} K={K:5d} x{cnt:2d} '
        for mode in modes:
            lin.set_mode(mode)
            us = timeit(lambda: orig(x, w, None, 0, r, tp), iters=20)
            tot[mode] += us * cnt
            line += f' {mode} {us:7.1f} us ({2 * M * N * K / us / 1e6:6.1f} TF)'
        flops += 2 * M * N * K * cnt
        print(line, flush=True)
    lin.set_mode('fp32')
    print(f'total per forward: {flops / 1e9:.1f} GFLOP; ' +
          ', '.join(f'{k} {v / 1e3:.3f} ms' for k, v in tot.items()), flush=True)


def gemm_tiles(mode='bf16x6'):
    """Split GEMM per tile configuration (bf16x6: FGR_GEMM6_TILE a=128x128, b=128x64,
    c=64x64, d=64x128; f16x3: FGR_GEMM16_TILE a=128x128, b=64x128, c=64x64, d=128x64)."""
    import os
    import fgreg.linear as lin
    dev = torch.device('cuda:0')
    lin.set_mode(mode)
    var = 'FGR_GEMM6_TILE' if mode == 'bf16x6' else 'FGR_GEMM16_TILE'
    print(f'tiles {mode}', flush=True)
    shapes = [(9493, 1024, 2048), (9493, 768, 256), (9493, 256, 3840), (9493, 1024, 256),
              (9493, 256, 1024), (11472, 512, 1024), (9493, 1792, 256), (9493, 256, 256),
              (56958, 256, 256), (11472, 128, 1920), (9493, 512, 1024), (9493, 1024, 512),
              (11472, 896, 128), (11472, 512, 256), (11472, 128, 512), (9493, 256, 512)]
    for (M, N, K) in shapes:
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev)
        line = f'M={M:6d} N={N:5d} K={K:5d}'
        for t in ('abcd' if mode == 'bf16x6' else 'abcdefghijklm'):
            os.environ[var] = t
            us = timeit(lambda: lin.linear(x, w), iters=20)
            line += f'  {t}: {us:7.1f} us ({2 * M * N * K / us / 1e6:6.1f} TF)'
        print(line, flush=True)
    os.environ[var] = ''


if __name__ == '__main__':
    import os
    which = sys.argv[1:] or ['attention']
    if 'attention' in which:
        attention()
        attention(lens=(2000,) * 2)
    if 'gemm' in which:
        gemm_shapes()
    if 'tiles' in which:
        gemm_tiles()
    if 'tiles16' in which:
        gemm_tiles('f16x3')
    if 'gemm1' in which:
        import fgreg.linear as lin
        lin.set_mode('bf16x6')
        dev = torch.device('cuda:0')
        for (M, N, K) in [(9493, 256, 1024), (9493, 1024, 2048)]:
            x = torch.randn(M, K, device=dev)
            w = torch.randn(N, K, device=dev)
            us = timeit(lambda: lin.linear(x, w), iters=20)
            print(f'M={M} N={N} K={K}: {us:.1f} us', flush=True)
