"""torch.profiler over two timed training steps (GPU box): which aten ops launch the torch
elementwise kernels of the step (counts per step, self CPU time), to find what the autograd
graph adds between the libfgreg kernels. usage: python tools/train_torch_prof.py [out.txt]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    import bench
    steps = {}

    def hook(step_fn):
        steps['fn'] = step_fn
    bench._TRAIN_STEP_HOOK = hook
    sys.argv = ['bench.py', '--train', '--steps', '2', '--warmup', '3']
    bench.main()
    fn = steps['fn']
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
    text = prof.key_averages().table(sort_by='count', row_limit=60)
    if out:
        with open(out, 'w') as f:
            f.write(text)
    else:
        print(text)


if __name__ == '__main__':
    main()
