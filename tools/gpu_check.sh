#!/bin/bash
# Quick GPU check (on the box, from the repo root): the GPU test suite, then short bench lines
# for the given workloads with their headline roofline fractions.
# usage: bash tools/gpu_check.sh <tag> [workload ...]      (default workloads: modelnet 3dmatch)
set -o pipefail
tag=${1:-chk}; shift
wls=${@:-modelnet 3dmatch}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/tests_$tag.log 2>&1 || { tail -40 gpurun_out/tests_$tag.log; exit 1; }
tail -2 gpurun_out/tests_$tag.log
for wl in $wls; do
  timeout -k 10 300 python bench.py --workload $wl --steps 30 --warmup 5 --no-cpu-baseline \
      > gpurun_out/bench_${wl}_$tag.json 2> gpurun_out/bench_${wl}_$tag.err || { tail -20 gpurun_out/bench_${wl}_$tag.err; exit 1; }
  python3 - gpurun_out/bench_${wl}_$tag.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d['config']['workload'], 'value', round(d['value'], 1), 'ms/step', round(d['ms_per_step'], 3),
      'gather', round(d['roofline']['frac'], 3), 'gemm', round(d['roofline_gemm']['frac'], 3),
      'gemm share', round(d['roofline_gemm']['share_of_step'], 3),
      'attn', round(d['roofline_attention']['frac'], 3))
PY
done
