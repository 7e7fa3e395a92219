"""Per-launch HBM traffic of one op from two rocprofv3 PMC passes of `bench.py --profile`.

usage: python tools/pmc_traffic.py <op> <kernel-regex> <fetch counter_collection.csv>
                                   <write counter_collection.csv> > profiles/pmc_kpconv.json

Every dispatch of a kernel matching <kernel-regex> is one launch of <op> (e.g.
fgr_kpconv_gather = kpconv_gather_wide / _narrow / _c1). Corrections per
MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of wide coalesced reads on gfx950
-> x2; WRITE_SIZE is exact for 16-B-per-lane stores. FETCH_SIZE / WRITE_SIZE are in KB.
"""
import csv
import json
import re
import sys


def total(path, counter, rx):
    tot, ids = 0.0, set()
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] == counter and rx.search(r['Kernel_Name']):
            tot += float(r['Counter_Value'])
            ids.add(r['Dispatch_Id'])
    return tot, len(ids)


def main():
    op, rx, fetch_csv, write_csv = sys.argv[1], re.compile(sys.argv[2]), sys.argv[3], sys.argv[4]
    f_kb, nf = total(fetch_csv, 'FETCH_SIZE', rx)
    w_kb, nw = total(write_csv, 'WRITE_SIZE', rx)
    assert nf == nw and nf > 0, (nf, nw)
    fetch = 2.0 * f_kb * 1024 / nf
    write = w_kb * 1024 / nw
    print(json.dumps({
        'op': op, 'kernel_regex': sys.argv[2], 'launches': nf,
        'fetch_size_kb_total_raw': f_kb, 'write_size_kb_total': w_kb,
        'hbm_read_bytes_per_launch': fetch, 'hbm_write_bytes_per_launch': write,
        'hbm_bytes_per_launch': fetch + write,
        'corrections': 'FETCH_SIZE x2 (gfx950 tallies 128-B requests at 64 B), WRITE_SIZE as is',
        'sources': [fetch_csv, write_csv]}, indent=1))


if __name__ == '__main__':
    main()
