"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin): one line per kernel
with VGPRs, AGPRs, spills, LDS bytes and occupancy. usage: hipcc ... 2>&1 | python tools/kres.py [filter]"""
import re
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ''
cur, rows = None, []
for line in sys.stdin:
    m = re.search(r'remark:\s+(.*?):\s+(\S+)\s+\[-Rpass', line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2)
    if k == 'Function Name':
        cur = {'name': v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if flt in r['name']:
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('AGPRs', '?'):>3} agpr spill {r.get('VGPRs Spill', '?'):>3} "
              f"lds {r.get('LDS Size [bytes/block]', '?'):>6} occ {r.get('Occupancy [waves/SIMD]', '?')}  {r['name'][:110]}")
