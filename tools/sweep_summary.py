"""Prints each shape's variants of a tools/gemm_tiles.py output sorted by time (! = error
above the check's bound). usage: python tools/sweep_summary.py <sweep.txt> ..."""
import re
import sys

for f in sys.argv[1:]:
    print(f)
    for line in open(f).read().splitlines():
        if not line.startswith('M='):
            continue
        head, *parts = line.strip().split(' | ')
        last = parts[-1].split(' || ')
        parts[-1] = last[0]
        tail = last[1] if len(last) > 1 else ''
        res = []
        for p in parts:
            m = re.match(r'(\S+)\s+([\d.]+)us', p)
            if m:
                res.append((float(m.group(2)), m.group(1), 'ERR' in p))
        res.sort()
        print(head, '|', tail, '|', ' '.join(f'{t}={u:.1f}{"!" if e else ""}' for u, t, e in res))
