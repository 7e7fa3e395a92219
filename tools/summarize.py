"""Prints the key numbers of one or more bench JSON lines (gpurun_out/*.json)."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, f"{d['value']:.1f} pairs/s  {d['ms_per_step']:.3f} ms/step")
    for k in ('roofline', 'roofline_attention', 'roofline_gemm'):
        if k in d:
            v = d[k]
            print(f"   {k:20s} achieved {v['achieved']:9.1f} {v['unit']:28s} frac {v['frac']:.3f} "
                  f"share {v.get('share_of_step', 0):.3f}")
    for k, v in d.get('rooflines_other', {}).items():
        print(f"   {k:20s} achieved {v['achieved']:9.1f} GB/s frac {v['frac']:.3f} "
              f"{v['us_per_step']:8.1f} us/step")
    if d.get('cpu_baseline'):
        print('   cpu', {k: v for k, v in d['cpu_baseline'].items() if k != 'sample'})
