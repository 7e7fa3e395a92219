"""Per-step kernel summary of the TIMED steps of a `rocprofv3 --kernel-trace` run of
`bench.py --profile`.

usage: python tools/kernel_stats.py <kernel_trace.csv> <timed steps> [<ms_per_step>] [top]

bench.py --profile launches torch's spin kernel (torch.cuda._sleep) right before and right
after its timed region; only the dispatches between the last two such markers are summed,
so warmup forwards and one-time work (weight splitting) are excluded by construction and
the per-step kernel sum is comparable with the same run's ms_per_step. Also reports the
GPU-busy time (union of dispatch intervals) per step.
"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = float(sys.argv[2])
    step_ms = float(sys.argv[3]) if len(sys.argv) > 3 else None
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    marks = [i for i, r in enumerate(rows) if 'sleep' in r['Kernel_Name'].lower()
             or 'spin' in r['Kernel_Name'].lower()]
    assert len(marks) >= 2, 'no marker kernels in the trace'
    a, b = marks[-2], marks[-1]
    sel = rows[a + 1:b]
    tot_ns, calls = defaultdict(float), defaultdict(int)
    for r in sel:
        d = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
        tot_ns[r['Kernel_Name']] += d
        calls[r['Kernel_Name']] += 1
    tot = sum(tot_ns.values()) / 1e6 / steps
    busy, cur_s, cur_e = 0, None, None
    for r in sel:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    span = (int(rows[b]['Start_Timestamp']) - int(rows[a]['End_Timestamp'])) / 1e6 / steps
    for name in sorted(tot_ns, key=lambda n: -tot_ns[n])[:top]:
        ms = tot_ns[name] / 1e6 / steps
        print(f"{ms:8.3f} ms/step {100 * ms / tot:6.2f}% n/step={calls[name] / steps:6.1f} "
              f"avg={tot_ns[name] / calls[name] / 1e3:8.1f}us  {name[:110]}")
    print(f'timed region: {len(sel)} dispatches over {steps:.0f} steps; sum of kernel time '
          f'{tot:.3f} ms/step; GPU busy (union) {busy / 1e6 / steps:.3f} ms/step; '
          f'marker-to-marker span {span:.3f} ms/step')
    if step_ms is not None:
        print(f'ms_per_step (same run, bench JSON): {step_ms:.3f} -> host/launch gap '
              f'{step_ms - busy / 1e6 / steps:.3f} ms/step')


if __name__ == '__main__':
    main()
