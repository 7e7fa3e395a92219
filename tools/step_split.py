"""Where the wall time of one forward goes (development tool, GPU): the eager preprocessing
alone (with its host syncs), the rest of the forward (HIP-graph replay of the core) and the
full forward, each timed over `iters` back-to-back calls.
usage: python tools/step_split.py [workload]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))


def main():
    import fgreg
    from fgreg.synthetic import make_batch
    wl = sys.argv[1] if len(sys.argv) > 1 else 'modelnet'
    cfgname, P, kind = {'modelnet': ('modelnet', 8, 'modelnet'), '3dmatch': ('3dmatch', 1, '3dmatch')}[wl]
    dev = torch.device('cuda:0')
    torch.manual_seed(0)
    model = fgreg.RegTR(fgreg.config.get(cfgname)).to(dev).eval()
    src, tgt, _ = make_batch(kind, P)
    bs = [torch.from_numpy(s).to(dev) for s in src]
    bt = [torch.from_numpy(t).to(dev) for t in tgt]
    iters = 20

    def timeit(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / iters * 1e3

    with torch.no_grad():
        full = timeit(lambda: model({'src_xyz': bs, 'tgt_xyz': bt}))
        prep = timeit(lambda: model.preprocessor(bs + bt))
        # host time of the preprocessing: wall minus what the GPU needed
        t0 = time.perf_counter()
        for _ in range(iters):
            model.preprocessor(bs + bt)
        host = (time.perf_counter() - t0) / iters * 1e3
        torch.cuda.synchronize()
        from fgreg import regtr
        g = next(iter(regtr._GRAPHS[model]['graphs'].values()))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.graph.replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        replay_host, replay_wall = (t1 - t0) * 1e3, (t2 - t0) * 1e3
        rep = timeit(lambda: g.graph.replay())
    print(f'{wl}: graph.replay() host call {replay_host:.3f} ms, wall {replay_wall:.3f} ms, '
          f'back-to-back replays {rep:.3f} ms', flush=True)
    print(f'{wl}: full forward {full:.3f} ms, preprocessing alone {prep:.3f} ms '
          f'(host-side enqueue {host:.3f} ms), core ~{full - prep:.3f} ms', flush=True)


if __name__ == '__main__':
    main()
