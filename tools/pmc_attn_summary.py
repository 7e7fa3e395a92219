"""Summarise tools/pmc_attn.sh output per (mode, attention kernel instance): the counters of
the last launches and the derived fractions (development tool).
usage: python tools/pmc_attn_summary.py gpurun_out/pmca_<tag> [out.json]"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    root = sys.argv[1]
    res = {}
    for mode_dir in sorted(glob.glob(os.path.join(root, '*'))):
        mode = os.path.basename(mode_dir)
        vals = collections.defaultdict(lambda: collections.defaultdict(list))
        for f in glob.glob(os.path.join(mode_dir, '**', '*counter_collection.csv'), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r['Kernel_Name']
                k = k[k.find('attn_'):].split('(')[0]
                vals[k][r['Counter_Name']].append(float(r['Counter_Value']))
        for kern, cv in vals.items():
            avg = {c: sum(v[-10:]) / len(v[-10:]) for c, v in cv.items() if v}
            wc = avg.get('SQ_WAVE_CYCLES', 0)
            gui = avg.get('GRBM_GUI_ACTIVE', 0)
            d = {'counters': avg}
            if wc:
                d['wait_any_frac'] = avg.get('SQ_WAIT_ANY', 0) / wc
                d['wait_inst_frac'] = avg.get('SQ_WAIT_INST_ANY', 0) / wc
                d['valu_insts_per_mfma'] = avg.get('SQ_INSTS_VALU', 0) / max(avg.get('SQ_INSTS_MFMA', 1), 1)
                d['lds_insts_per_mfma'] = avg.get('SQ_INSTS_LDS', 0) / max(avg.get('SQ_INSTS_MFMA', 1), 1)
            if gui:
                # SQ_VALU_MFMA_BUSY_CYCLES summed over 256 CUs x 4 SIMDs; GRBM_GUI_ACTIVE summed
                # over 8 XCDs (MI355X_MICROARCH.md)
                d['mfma_busy_frac'] = avg.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (gui / 8) / 1024
            res[f'{mode}:{kern}'] = d
            print(f'{mode:6s} {kern:40s} ' + ' '.join(
                f'{k}={v:.3f}' for k, v in d.items() if k != 'counters'))
    if len(sys.argv) > 2:
        with open(sys.argv[2], 'w') as f:
            json.dump(res, f, indent=1)


if __name__ == '__main__':
    main()
