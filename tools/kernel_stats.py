"""Per-step kernel summary of a rocprofv3 --stats run of `bench.py --profile`.

usage: python tools/kernel_stats.py <kernel_stats.csv> <forwards> [<ms_per_step>] [top]

<forwards> = warmup + timed steps of the profiled run: every forward launches the same
kernels, so a kernel's per-step time is its total / forwards. Kernels with fewer calls than
forwards ran only once (weight splitting on the first forward) and are listed apart, not in
the per-step sum. With <ms_per_step> (from the same run's JSON line) the script states the
host / launch gap = ms_per_step - sum of per-step kernel time.
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    fwd = float(sys.argv[2])
    step_ms = float(sys.argv[3]) if len(sys.argv) > 3 else None
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
    per, once = [], []
    for r in rows:
        (per if int(r['Calls']) >= fwd else once).append(r)
    tot = sum(float(r['TotalDurationNs']) for r in per) / 1e6 / fwd
    for r in sorted(per, key=lambda r: -float(r['TotalDurationNs']))[:top]:
        ms = float(r['TotalDurationNs']) / 1e6 / fwd
        print(f"{ms:8.3f} ms/step {100 * ms / tot:6.2f}% n/step={int(r['Calls']) / fwd:6.1f} "
              f"avg={float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:110]}")
    print(f'sum of per-step kernel time: {tot:.3f} ms/step over {len(per)} kernels '
          f'({fwd:.0f} forwards)')
    if step_ms is not None:
        print(f'ms_per_step (same run, bench JSON): {step_ms:.3f} -> host/launch gap '
              f'{step_ms - tot:.3f} ms/step ({100 * (step_ms - tot) / step_ms:.1f} %)')
    if once:
        print('one-time kernels (first forward only, not in the sum):')
        for r in sorted(once, key=lambda r: -float(r['TotalDurationNs'])):
            print(f"  {float(r['TotalDurationNs']) / 1e6:8.3f} ms total, {r['Calls']} calls  "
                  f"{r['Name'][:100]}")


if __name__ == '__main__':
    main()
