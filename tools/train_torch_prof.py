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
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
    text = prof.key_averages().table(sort_by='count', row_limit=60)
    # where the elementwise ops come from (top Python frames of each call site)
    keep = ('aten::add', 'aten::add_', 'aten::mul', 'aten::copy_', 'aten::cat', 'aten::fill_',
            'aten::zero_', 'aten::div', 'aten::sub')
    rows = [e for e in prof.key_averages(group_by_stack_n=6) if e.key in keep]
    rows.sort(key=lambda e: -e.count)
    lines = []
    for e in rows[:40]:
        lines.append(f'{e.count:6d}  {e.key}')
        for fr in e.stack[:6]:
            lines.append(f'          {fr}')
    text += '\n\n' + '\n'.join(lines)
    if out:
        with open(out, 'w') as f:
            f.write(text)
    else:
        print(text)


if __name__ == '__main__':
    main()
