"""Pipelined inference over a stream of batches (serving / benchmark loops).

``pipeline(model, batches)`` yields ``model(batch)`` for every batch, in order, with the same
outputs, but runs the preprocessing of batch i + 1 (grid subsampling and radius search: the
eager part of the forward, with one host sync per pyramid level) on a side stream while
batch i's post-preprocessing forward (the HIP-graph replay) still runs on the current
stream. Without it every forward's preprocessing waits, at its first voxel-count readback,
for the previous forward's whole core to drain, and the GPU then idles while the host
enqueues the rest of the preprocessing.

Ordering contract (no extra synchronisation needed by the caller):
  * batch i + 1 is drawn from the iterator BEFORE batch i's core is enqueued, and the side
    stream waits for an event recorded on the current stream at that moment -- so any work
    the caller enqueued to produce batch i + 1 (an H2D copy, a crop kernel) is complete
    before its preprocessing reads it, while batch i's core (enqueued after) is not waited
    for;
  * batch i's core waits for its preprocessing's completion event; every kpconv_meta tensor
    is marked as used by the current stream (record_stream), so the caching allocator does not
    hand its memory to the side stream while the current stream may still read it;
  * outputs are produced on the current stream, as with ``model(batch)``.
"""
import torch

from .regtr import RegTR


def _meta_tensors(meta):
    for k in ('points', 'neighbors', 'pools', 'upsamples', 'stack_lengths'):
        for t in meta[k]:
            if torch.is_tensor(t):
                yield t
    for t in meta['_host']['offsets']:
        yield t


def _prepare(model, batch, side, ready):
    main = torch.cuda.current_stream()
    with torch.cuda.stream(side):
        side.wait_event(ready)
        meta = model._prepare(batch)
        done = torch.cuda.Event()
        done.record(side)
    for t in _meta_tensors(meta):
        t.record_stream(main)
    for t in list(batch['src_xyz']) + list(batch['tgt_xyz']):
        t.record_stream(side)
    return meta, done


def pipeline(model: RegTR, batches):
    """Yields model(batch) for each batch of ``batches`` (an iterable of forward() batch
    dicts on one device), preprocessing batch i + 1 while batch i's core runs."""
    if model.training and torch.is_grad_enabled():
        raise NotImplementedError('fgreg.pipeline is inference only (eval() / no_grad)')
    it = iter(batches)
    cur = next(it, None)
    if cur is None:
        return
    dev = cur['src_xyz'][0].device
    if dev.type != 'cuda':
        raise RuntimeError('fgreg.pipeline needs GPU batches')
    with torch.no_grad(), torch.cuda.device(dev):
        side = torch.cuda.Stream(dev)
        ready = torch.cuda.Event()
        ready.record()
        meta, done = _prepare(model, cur, side, ready)
        while cur is not None:
            nxt = next(it, None)
            if nxt is not None:
                ready = torch.cuda.Event()
                ready.record()                      # before cur's core is enqueued
            torch.cuda.current_stream().wait_event(done)
            out = model._forward(cur, meta)
            if nxt is not None:
                meta, done = _prepare(model, nxt, side, ready)
            yield out
            cur = nxt
