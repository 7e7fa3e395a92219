"""Shapes of the host-side op calls of one forward (development tool, GPU): wraps the
fgreg.ops entry points, runs one eager forward and prints (op, shapes, count).
usage: python tools/op_shapes.py [workload] [op-substring]"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd'))


def main():
    import numpy as np
    import fgreg
    from fgreg import ops, regtr
    from fgreg.synthetic import make_batch
    wl = sys.argv[1] if len(sys.argv) > 1 else 'modelnet'
    filt = sys.argv[2] if len(sys.argv) > 2 else ''
    cfgname, P = {'modelnet': ('modelnet', 8), '3dmatch': ('3dmatch', 1)}[wl]
    regtr.GRAPHS = False
    dev = torch.device('cuda:0')
    torch.manual_seed(0)
    np.random.seed(0)
    model = fgreg.RegTR(fgreg.config.get(cfgname)).to(dev).eval()
    src, tgt, _ = make_batch(wl, P)
    seen = collections.Counter()
    for name in dir(ops):
        fn = getattr(ops, name)
        if not callable(fn) or name.startswith('_') or filt not in name or isinstance(fn, type):
            continue

        def wrap(f, n):
            def g(*a, **k):
                shp = tuple(tuple(x.shape) for x in a if torch.is_tensor(x))
                seen[(n, shp)] += 1
                return f(*a, **k)
            return g
        setattr(ops, name, wrap(fn, name))
    with torch.no_grad():
        model({'src_xyz': [torch.from_numpy(s).to(dev) for s in src],
               'tgt_xyz': [torch.from_numpy(t).to(dev) for t in tgt]})
    torch.cuda.synchronize()
    for (n, shp), c in sorted(seen.items()):
        print(f'{n:24s} x{c:3d} {shp}', flush=True)


if __name__ == '__main__':
    main()
