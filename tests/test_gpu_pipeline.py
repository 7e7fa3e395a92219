"""fgreg.pipeline (preprocessing of later batches on a side stream while earlier cores run,
1-3 cores in flight) yields exactly model(batch) for every batch: same kernels, same order
of operations."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

KEYS = ('src_feat', 'tgt_feat', 'src_kp_warped', 'tgt_kp_warped', 'src_overlap', 'tgt_overlap')


def _batches(kind, dev, sizes):
    from fgreg.synthetic import make_batch
    out = []
    for start, P in sizes:
        src, tgt, _ = make_batch(kind, P, start=start)
        out.append({'src_xyz': [torch.from_numpy(a).to(dev) for a in src],
                    'tgt_xyz': [torch.from_numpy(a).to(dev) for a in tgt]})
    return out


def _same(a, b):
    assert torch.equal(a['pose'], b['pose'])
    for k in KEYS:
        for x, y in zip(a[k], b[k]):
            assert torch.equal(x, y), k


@pytest.mark.parametrize('depth', [1, 2, 3])
@pytest.mark.parametrize('kind', ['modelnet', '3dmatch'])
def test_pipeline_equals_sequential(gpu, kind, depth):
    import fgreg
    torch.manual_seed(0)
    np.random.seed(0)
    model = fgreg.RegTR(fgreg.config.get(kind)).to(gpu).eval()
    P = 2 if kind == 'modelnet' else 1
    # two shape signatures, each seen three times (the graph path captures on the second)
    sizes = [(0, P), (5, P), (0, P), (5, P), (0, P), (5, P)]
    batches = _batches(kind, gpu, sizes)
    with torch.no_grad():
        ref = [model(dict(b)) for b in batches]
    got = list(fgreg.pipeline(model, [dict(b) for b in batches], depth=depth))
    torch.cuda.synchronize()
    assert len(got) == len(ref)
    for a, b in zip(got, ref):
        _same(a, b)


@pytest.mark.parametrize('depth', [1, 2])
def test_pipeline_inputs_produced_on_the_current_stream(gpu, depth):
    """Inputs written by the caller on the current stream right before each draw are read
    by the side-stream preprocessing only after that write (the ready event)."""
    import fgreg
    torch.manual_seed(1)
    model = fgreg.RegTR(fgreg.config.get('modelnet')).to(gpu).eval()
    base = _batches('modelnet', gpu, [(0, 2)])[0]
    with torch.no_grad():
        ref = model(dict(base))

    def gen():
        for _ in range(4):
            b = {k: [torch.empty_like(t) for t in v] for k, v in base.items()}
            torch.cuda._sleep(200000)                    # a slow producer on the stream
            for k in b:
                for d, s in zip(b[k], base[k]):
                    d.copy_(s)
            yield b
    n = 0
    for out in fgreg.pipeline(model, gen(), depth=depth):
        _same(out, ref)
        n += 1
    assert n == 4
