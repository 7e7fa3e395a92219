#!/bin/bash
# Two PMC passes (issue / wait / MFMA-busy / LDS counters) over one kernel of a command
# (development tool, GPU box). usage: bash tools/pmc_kernel.sh <tag> <kernel regex> <python args...>
set -o pipefail
tag=$1; rx=$2; shift 2
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
d=$R/gpurun_out/pmck_$tag
mkdir -p $d
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-include-regex "$rx" -d $d/p1 -o p1 --output-format csv -- python3 "$@" > $d/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex "$rx" -d $d/p2 -o p2 --output-format csv -- python3 "$@" > $d/p2.log 2>&1 || exit 1
python3 - $d <<'PY'
import collections, csv, glob, os, sys
d = sys.argv[1]
vals = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
        vals[r['Counter_Name']].append(float(r['Counter_Value']))
avg = {k: sum(v[-5:]) / len(v[-5:]) for k, v in vals.items() if v}
print(' '.join(f'{k}={v:.4g}' for k, v in sorted(avg.items())))
wc = avg.get('SQ_WAVE_CYCLES', 0)
if wc:
    print('wait_any %.2f wait_inst %.2f (lds %.2f) active %.2f | valu/mfma %.2f lds/mfma %.2f | mfma_busy/gui %.3f | bank_conflict/lds_active %.3f' % (
        avg.get('SQ_WAIT_ANY', 0) / wc, avg.get('SQ_WAIT_INST_ANY', 0) / wc, avg.get('SQ_WAIT_INST_LDS', 0) / wc,
        avg.get('SQ_ACTIVE_INST_ANY', 0) / wc,
        avg.get('SQ_INSTS_VALU', 0) / max(avg.get('SQ_INSTS_MFMA', 1), 1),
        avg.get('SQ_INSTS_LDS', 0) / max(avg.get('SQ_INSTS_MFMA', 1), 1),
        avg.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / max(avg.get('GRBM_GUI_ACTIVE', 1), 1) / 256 / 4,
        avg.get('SQ_LDS_BANK_CONFLICT', 0) / max(avg.get('SQ_ACTIVE_INST_LDS', 1), 1)))
PY
