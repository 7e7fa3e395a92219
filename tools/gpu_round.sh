#!/bin/bash
# One GPU session: parity tests, bench, kernel-trace profile, PMC traffic passes of the gather.
# usage (on the GPU box, from the repo root): bash tools/gpu_round.sh <tag>
# The profiled bench runs 3 warmup + 1 counting + 10 timed + 10 GEMM-instrumented forwards:
# per-step kernel stats = python tools/kernel_stats.py <kernel_stats.csv> 24
set -o pipefail
tag=${1:-run}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/tests_$tag.log 2>&1; echo "EXIT $?" >> gpurun_out/tests_$tag.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'kpconv_gather|row_positive' --output-format csv -d gpurun_out/pmcf_$tag -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcf_$tag.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'kpconv_gather|row_positive' --output-format csv -d gpurun_out/pmcw_$tag -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcw_$tag.log 2>&1 || exit 1
echo DONE
