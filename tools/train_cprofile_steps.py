"""Host-side profile of the training step's TIMED steps only (GPU box): bench.py --train hands
its step function over (_TRAIN_STEP_HOOK), cProfile runs 10 steps of it; own time per function.
usage: python tools/train_cprofile_steps.py [out.txt]"""
import cProfile
import io
import os
import pstats
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    import bench
    steps = {}
    bench._TRAIN_STEP_HOOK = lambda fn: steps.setdefault('fn', fn)
    sys.argv = ['bench.py', '--train', '--steps', '2', '--warmup', '3']
    bench.main()
    fn = steps['fn']
    prof = cProfile.Profile()
    prof.enable()
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    prof.disable()
    s = io.StringIO()
    st = pstats.Stats(prof, stream=s)
    st.sort_stats('tottime').print_stats(50)
    text = s.getvalue()
    if out:
        with open(out, 'w') as f:
            f.write(text)
    print(text[:6000])


if __name__ == '__main__':
    main()
