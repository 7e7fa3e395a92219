"""Summarise tools/pmc_gemm.sh output: per config, the last launches' counters (development
tool). usage: python tools/pmc_summary.py gpurun_out/pmcg"""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    for d in sorted(glob.glob(os.path.join(root, '*_*_*_*'))):
        vals = collections.defaultdict(list)
        for f in glob.glob(os.path.join(d, '*', '*', '*counter_collection.csv')) + \
                glob.glob(os.path.join(d, '*', '*counter_collection.csv')):
            for r in csv.DictReader(open(f)):
                if 'gemm' not in r['Kernel_Name'] and 'g5' not in r['Kernel_Name']:
                    continue
                vals[r['Counter_Name']].append(float(r['Counter_Value']))
        avg = {k: sum(v[-10:]) / len(v[-10:]) for k, v in vals.items() if v}
        line = os.path.basename(d) + ': ' + ' '.join(f'{k}={v:.3g}' for k, v in sorted(avg.items()))
        print(line)
        wc = avg.get('SQ_WAVE_CYCLES')
        if wc:
            print('   wait_any %.2f wait_inst %.2f  valu_insts/mfma %.1f lds/mfma %.2f  mfma_busy/gui %.3f  L2 hit %.2f' % (
                avg.get('SQ_WAIT_ANY', 0) / wc, avg.get('SQ_WAIT_INST_ANY', 0) / wc,
                avg.get('SQ_INSTS_VALU', 0) / max(avg.get('SQ_INSTS_MFMA', 1), 1),
                avg.get('SQ_INSTS_LDS', 0) / max(avg.get('SQ_INSTS_MFMA', 1), 1),
                avg.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / max(avg.get('GRBM_GUI_ACTIVE', 1), 1) / 256 / 4,
                avg.get('TCC_HIT_sum', 0) / max(avg.get('TCC_HIT_sum', 0) + avg.get('TCC_MISS_sum', 0), 1)))


if __name__ == '__main__':
    main()
