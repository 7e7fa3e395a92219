#!/bin/bash
# Per-launch event timing of the bench's roofline replay vs the kernel trace (GPU box):
# the same workload with --lead-cycles 0 (the default) and a 250k-cycle spin lead, then a rocprofv3 kernel trace
# of a default run, whose per-kernel average durations the event averages should match.
# usage: bash tools/timing_check.sh <tag> [workload]
set -o pipefail
tag=$1; wl=${2:-modelnet}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --lead-cycles 0 \
    --gemm-table gpurun_out/tc_${tag}_lead0_gemm.json > gpurun_out/tc_${tag}_lead0.json 2> gpurun_out/tc_${tag}_lead0.err || exit 1
timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --lead-cycles 250000 \
    --gemm-table gpurun_out/tc_${tag}_lead_gemm.json > gpurun_out/tc_${tag}_lead.json 2> gpurun_out/tc_${tag}_lead.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tc_${tag}_prof -- \
    python3 bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/tc_${tag}_prof.json 2> gpurun_out/tc_${tag}_prof.err || exit 1
for f in lead0 lead; do
  python3 - gpurun_out/tc_${tag}_$f.json $f <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d['roofline']; g = d['roofline_gemm']; a = d['roofline_attention']
print(f"{sys.argv[2]:6s} step {d['ms_per_step']:.3f} ms | gather {r['frac']:.3f} {r['avg_launch_us']:.1f}us | gemm {g['frac']:.3f} {g['avg_launch_us']:.1f}us | attn {a['frac']:.3f} {a['avg_launch_us']:.1f}us")
PY
done
echo DONE
