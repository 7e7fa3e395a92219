"""Host-side profile of the training step (GPU box): cProfile over bench.py --train's timed
steps, the functions with the most own time and the most cumulative time.
usage: python tools/train_cprofile.py [out.txt]"""
import cProfile
import io
import os
import pstats
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    import bench
    sys.argv = ['bench.py', '--train', '--steps', '10', '--warmup', '3']
    prof = cProfile.Profile()
    prof.enable()
    bench.main()
    prof.disable()
    s = io.StringIO()
    st = pstats.Stats(prof, stream=s)
    st.sort_stats('tottime').print_stats(45)
    st.sort_stats('cumulative').print_stats(60)
    text = s.getvalue()
    if out:
        with open(out, 'w') as f:
            f.write(text)
    else:
        print(text)


if __name__ == '__main__':
    main()
