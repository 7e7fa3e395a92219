#!/bin/bash
# Same-box A/B of environment switches on one bench workload (GPU box). usage:
#   bash tools/ab_env.sh <tag> <workload> "NAME=V NAME2=V" "NAME=V ..." ...
# one bench line (+ per-shape GEMM table) per configuration, in order, each under its own limit
set -o pipefail
tag=$1; wl=$2; shift 2
mkdir -p gpurun_out
i=0
for cfg in "$@"; do
  i=$((i + 1))
  env $cfg timeout -k 10 300 python bench.py --workload $wl --steps 30 --warmup 10 --no-cpu-baseline \
      --gemm-table gpurun_out/ab_${tag}_${i}_gemm.json > gpurun_out/ab_${tag}_${i}.json 2> gpurun_out/ab_${tag}_${i}.err || { echo "config $i failed"; tail -5 gpurun_out/ab_${tag}_${i}.err; exit 1; }
  python3 - "$cfg" gpurun_out/ab_${tag}_${i}.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print(f"{sys.argv[1]:60s} {d['value']:8.1f} pairs/s {d['ms_per_step']:.3f} ms  gemm {d['roofline_gemm']['frac']:.3f} x{d['roofline_gemm']['launches_per_step']:.0f} {d['roofline_gemm']['avg_launch_us']:.1f}us  attn {d['roofline_attention']['frac']:.3f} {d['roofline_attention']['avg_launch_us']:.1f}us")
PY
done
