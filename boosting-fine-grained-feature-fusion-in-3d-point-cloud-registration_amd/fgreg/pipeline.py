"""Pipelined inference over a stream of batches (serving / benchmark loops).

``pipeline(model, batches)`` yields ``model(batch)`` for every batch, in order, with the same
outputs, but runs the preprocessing of batch i + 1 (grid subsampling and radius search: the
eager part of the forward, with one host sync per pyramid level) on a side stream while
batch i's post-preprocessing forward (the HIP-graph replay) still runs on the current
stream. Without it every forward's preprocessing waits, at its first voxel-count readback,
for the previous forward's whole core to drain, and the GPU then idles while the host
enqueues the rest of the preprocessing.

``depth`` cores are kept enqueued ahead of the output being yielded (default 2): the
preprocessing of batch i + 2 runs (with its host readbacks) while the cores of batches i and
i + 1 are both queued, so the GPU does not idle when a preprocessing takes longer than one
core (the 20k-point workloads). depth = 1 is the one-ahead pipeline.
Graph replays clone their outputs (fgreg.regtr._CoreGraph.run), so an output stays valid
while the next core runs.

``streams`` core streams (default 2, FGREG_PIPE_STREAMS): core i runs on core stream
i mod streams (dedicated streams; streams = 1: the current stream), each replaying its own instance of
the shape signature's HIP graph (RegTR._forward(slot=...)), so consecutive cores overlap on
the GPU: the drain / ramp of every one of a core's ~300 dependent launches (a few us each)
is filled by the other core's kernels. Each core is still one whole forward of its batch;
its outputs are made visible to the current stream (an event wait) before they are yielded.

Ordering contract (no extra synchronisation needed by the caller):
  * batch i + 1 is drawn from the iterator BEFORE batch i's core is enqueued, and the side
    stream waits for an event recorded on the current stream at that moment -- so any work
    the caller enqueued to produce batch i + 1 (an H2D copy, a crop kernel) is complete
    before its preprocessing reads it, while batch i's core (enqueued after) is not waited
    for;
  * batch i's core waits for its preprocessing's completion event; every kpconv_meta tensor
    is marked as used by the current stream (record_stream), so the caching allocator does not
    hand its memory to the side stream while the current stream may still read it;
  * outputs are produced on the current stream, as with ``model(batch)``;
  * lazily built model state (weight images, BN-folded weights: ops.note_state) is built by
    the first forward that needs it, on that forward's core stream: a core whose enqueue
    built state (ops.STATE_EPOCH moved) is waited for by the next core (every later core is
    then ordered after it), and the new tensors are marked as used by every core stream. A
    cold model therefore runs its first core(s) one after the other; once the state exists
    the cores overlap. The core streams are registered in ops.STATE_READERS while the
    pipeline runs, so an in-place weight-image refresh waits for their forwards.
"""
import os
from collections import deque

import torch

from . import ops
from .regtr import RegTR

DEPTH = int(os.environ.get('FGREG_PIPE_DEPTH', '2'))
STREAMS = int(os.environ.get('FGREG_PIPE_STREAMS', '2'))


def _meta_tensors(meta):
    for k in ('points', 'neighbors', 'pools', 'upsamples', 'stack_lengths'):
        for t in meta[k]:
            if torch.is_tensor(t):
                yield t
    for t in meta['_host']['offsets']:
        yield t


def _prepare(model, batch, side, ready, users):
    with torch.cuda.stream(side):
        side.wait_event(ready)
        meta = model._prepare(batch)
        done = torch.cuda.Event()
        done.record(side)
    for t in _meta_tensors(meta):
        for st in users:
            t.record_stream(st)
    for t in list(batch['src_xyz']) + list(batch['tgt_xyz']):
        t.record_stream(side)
    return meta, done


def _out_tensors(out):
    for v in out.values():
        if torch.is_tensor(v):
            yield v
        elif isinstance(v, (list, tuple)):
            for t in v:
                if torch.is_tensor(t):
                    yield t


def pipeline(model: RegTR, batches, depth=None, streams=None):
    """Yields model(batch) for each batch of ``batches`` (an iterable of forward() batch
    dicts on one device), preprocessing later batches while earlier cores run (``depth``
    cores in flight ahead of the yielded output; default DEPTH = FGREG_PIPE_DEPTH or 2) on
    ``streams`` core streams (default STREAMS = FGREG_PIPE_STREAMS or 2)."""
    if model.training and torch.is_grad_enabled():
        raise NotImplementedError('fgreg.pipeline is inference only (eval() / no_grad)')
    depth = max(1, int(DEPTH if depth is None else depth))
    n_streams = max(1, int(STREAMS if streams is None else streams))
    it = iter(batches)
    first = next(it, None)
    if first is None:
        return
    dev = first['src_xyz'][0].device
    if dev.type != 'cuda':
        raise RuntimeError('fgreg.pipeline needs GPU batches')
    with torch.no_grad(), torch.cuda.device(dev):
        side = torch.cuda.Stream(dev)
        main = torch.cuda.current_stream()
        # several core streams: all of them dedicated (a core on the current stream would queue
        # behind the waits that make earlier outputs visible to the caller, serialising it
        # with the core before it)
        cores = [main] if n_streams == 1 else [torch.cuda.Stream(dev) for _ in range(n_streams)]

        def draw():
            """the next batch and an event recorded now, before any later core is enqueued"""
            b = next(it, None)
            if b is None:
                return None
            ready = torch.cuda.Event()
            ready.record()
            return b, ready

        def finish(out, st):
            """the core's outputs, visible to (and owned by) the current stream"""
            if st is not main:
                ev = torch.cuda.Event()
                ev.record(st)
                main.wait_event(ev)
                for t in _out_tensors(out):
                    t.record_stream(main)
            return out

        ready = torch.cuda.Event()
        ready.record()
        prepared = deque([(first,) + _prepare(model, first, side, ready, cores)])
        outs = deque()
        i = 0
        built = None            # event after the last core whose enqueue built model state
        ops.take_new_state()    # state built before the pipeline: ordered by the current stream
        for st in cores:
            if st is not main:
                ops.STATE_READERS[st] = None
        try:
            while prepared:
                while prepared and len(outs) < depth:
                    b, meta, done = prepared.popleft()
                    item = draw()                       # before b's core is enqueued
                    st = cores[i % n_streams]
                    st.wait_event(done)
                    if built is not None:
                        st.wait_event(built)
                        built = None
                    epoch = ops.STATE_EPOCH
                    with torch.cuda.stream(st):
                        out = model._forward(b, meta, slot=i % n_streams)
                    end = torch.cuda.Event()
                    end.record(st)
                    if st is not main:
                        ops.STATE_READERS[st] = end
                    if ops.STATE_EPOCH != epoch:
                        # this core built state the next ones read: order them after it and
                        # keep the allocator from reusing it under another core stream
                        built = end
                        for t in ops.take_new_state():
                            for s2 in cores:
                                t.record_stream(s2)
                    outs.append((out, st))
                    i += 1
                    if item is not None:
                        prepared.append((item[0],) + _prepare(model, item[0], side, item[1], cores))
                yield finish(*outs.popleft())
            while outs:
                yield finish(*outs.popleft())
        finally:
            for st in cores:
                ops.STATE_READERS.pop(st, None)
