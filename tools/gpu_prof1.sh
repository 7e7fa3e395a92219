#!/bin/bash
# One workload: bench line with the per-shape GEMM table, then a kernel-trace profile of the
# timed steps (--no-pipeline) summarised per step. usage: bash tools/gpu_prof1.sh <tag> <workload>
set -o pipefail
tag=$1; wl=${2:-modelnet}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload $wl --steps 30 --warmup 5 --no-cpu-baseline --gemm-table gpurun_out/gemm_${wl}_$tag.json > gpurun_out/bench_${wl}_$tag.json 2> gpurun_out/bench_${wl}_$tag.err || exit 1
timeout -k 10 300 python bench.py --workload $wl --no-pipeline --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/benchnp_${wl}_$tag.json 2> gpurun_out/benchnp_${wl}_$tag.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${wl}_$tag -- python3 bench.py --profile --no-pipeline --workload $wl --steps 20 --warmup 2 > gpurun_out/prof_${wl}_$tag.json 2> gpurun_out/prof_${wl}_$tag.err || exit 1
ms=$(python3 -c "import json;print(json.loads(open('gpurun_out/benchnp_${wl}_$tag.json').read().strip().splitlines()[-1])['ms_per_step'])")
python3 tools/kernel_stats.py gpurun_out/prof_${wl}_$tag/*/*_kernel_trace.csv 20 $ms > gpurun_out/kstats_${wl}_$tag.txt || exit 1
head -30 gpurun_out/kstats_${wl}_$tag.txt
