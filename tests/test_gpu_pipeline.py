"""fgreg.pipeline (preprocessing of later batches on a side stream while earlier cores run,
1-3 cores in flight, on 1-3 core streams) yields exactly model(batch) for every batch: same
kernels, same order of operations."""
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


@pytest.mark.parametrize('depth,streams', [(1, 1), (2, 1), (3, 1), (2, 2), (3, 3), (3, 2)])
@pytest.mark.parametrize('kind', ['modelnet', '3dmatch'])
def test_pipeline_equals_sequential(gpu, kind, depth, streams):
    import fgreg
    torch.manual_seed(0)
    np.random.seed(0)
    model = fgreg.RegTR(fgreg.config.get(kind)).to(gpu).eval()
    P = 2 if kind == 'modelnet' else 1
    # two shape signatures, each seen six times (the graph path captures on the second
    # sighting per stream slot)
    sizes = [(0, P), (5, P)] * 6
    batches = _batches(kind, gpu, sizes)
    with torch.no_grad():
        ref = [model(dict(b)) for b in batches]
    got = list(fgreg.pipeline(model, [dict(b) for b in batches], depth=depth, streams=streams))
    torch.cuda.synchronize()
    assert len(got) == len(ref)
    for a, b in zip(got, ref):
        _same(a, b)


@pytest.mark.parametrize('depth,streams', [(1, 1), (2, 1), (2, 2)])
def test_pipeline_inputs_produced_on_the_current_stream(gpu, depth, streams):
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
    for out in fgreg.pipeline(model, gen(), depth=depth, streams=streams):
        _same(out, ref)
        n += 1
    assert n == 4


def test_pipeline_outputs_usable_on_the_current_stream(gpu):
    """Cores on the second stream: their outputs are complete for work the caller enqueues on
    the current stream right after the yield, and stay valid while later cores run."""
    import fgreg
    torch.manual_seed(2)
    model = fgreg.RegTR(fgreg.config.get('modelnet')).to(gpu).eval()
    batches = _batches('modelnet', gpu, [(0, 2), (3, 2)] * 4)
    with torch.no_grad():
        ref = [model(dict(b)) for b in batches]
    sums, kept = [], []
    for out in fgreg.pipeline(model, [dict(b) for b in batches], depth=3, streams=2):
        sums.append(out['pose'].sum())              # enqueued on the current stream at once
        kept.append(out)
    torch.cuda.synchronize()
    for s, out, r in zip(sums, kept, ref):
        assert torch.equal(s, r['pose'].sum())
        _same(out, r)


@pytest.mark.parametrize('kind', ['modelnet', '3dmatch'])
def test_pipeline_on_a_cold_model(gpu, kind):
    """A freshly built model whose weight images / BN-folded weights do not exist yet: the first
    cores build them on their own core streams, and the later cores (on the other stream) are
    ordered after that (ops.note_state / STATE_EPOCH). Outputs equal model(batch) run
    afterwards, bit for bit."""
    import fgreg
    from fgreg import ops
    torch.manual_seed(3)
    np.random.seed(3)
    model = fgreg.RegTR(fgreg.config.get(kind)).to(gpu).eval()
    P = 2 if kind == 'modelnet' else 1
    batches = _batches(kind, gpu, [(0, P), (4, P)] * 3)
    got = list(fgreg.pipeline(model, [dict(b) for b in batches], depth=2, streams=2))
    torch.cuda.synchronize()
    assert not ops.STATE_READERS                      # unregistered when the pipeline ends
    with torch.no_grad():
        ref = [model(dict(b)) for b in batches]
    for a, b in zip(got, ref):
        _same(a, b)


def test_pipeline_then_weight_update(gpu):
    """An in-place weight update between two pipelines (the training -> evaluation pattern):
    the stale images are re-split (in place, after the core streams' forwards) and the second
    pipeline equals model(batch) with the new weights."""
    import fgreg
    torch.manual_seed(4)
    model = fgreg.RegTR(fgreg.config.get('modelnet')).to(gpu).eval()
    batches = _batches('modelnet', gpu, [(0, 2), (3, 2)] * 2)
    list(fgreg.pipeline(model, [dict(b) for b in batches], depth=2, streams=2))
    with torch.no_grad():
        for p in model.parameters():
            p.mul_(1.01)
    got = list(fgreg.pipeline(model, [dict(b) for b in batches], depth=2, streams=2))
    torch.cuda.synchronize()
    with torch.no_grad():
        ref = [model(dict(b)) for b in batches]
    for a, b in zip(got, ref):
        _same(a, b)
