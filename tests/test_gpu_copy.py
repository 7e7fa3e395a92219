"""fgr_copy_batch (csrc/copy.hip): the batched device-to-device copies of the HIP-graph
replay (static kpconv_meta inputs in, outputs out, fgreg/regtr.py). Byte-exact for every size
class (empty, sub-16-B tails, 16-B aligned / unaligned ends, multi-chunk), more than one launch
worth of pairs (> 32), and neighbouring bytes untouched."""
import pytest
import torch

from fgreg import ops

pytestmark = pytest.mark.gpu


def test_copy_batch_sizes_and_alignment():
    dev = torch.device('cuda:0')
    g = torch.Generator(device=dev).manual_seed(0)
    sizes = [0, 1, 3, 15, 16, 17, 31, 64, 1000, 16384, 16385, 70001, 1 << 20, 5 * (1 << 20) + 7]
    sizes = sizes * 3                                    # 42 pairs: two launches
    srcs, dsts, guards = [], [], []
    for i, n in enumerate(sizes):
        off = i % 3                                      # 0: 16-B aligned, 1 / 2: unaligned ends
        base = torch.randint(0, 256, (n + off + 32,), generator=g, device=dev, dtype=torch.uint8)
        out = torch.full((n + off + 32,), 0xA5, device=dev, dtype=torch.uint8)
        srcs.append(base[off:off + n])
        dsts.append(out[off:off + n])
        guards.append((out, off, n))
    ops.copy_batch(srcs, dsts)
    torch.cuda.synchronize()
    for s, d, (out, off, n) in zip(srcs, dsts, guards):
        assert torch.equal(s, d)
        assert bool((out[:off] == 0xA5).all()) and bool((out[off + n:] == 0xA5).all())


def test_copy_batch_float_tensors():
    dev = torch.device('cuda:0')
    srcs = [torch.randn(n, 3, device=dev) for n in (1, 717, 9544, 57264)]
    dsts = [torch.zeros_like(s) for s in srcs]
    ops.copy_batch(srcs, dsts)
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(srcs, dsts))
