#!/bin/bash
# Copies one gpu_round.sh run's summaries from gpurun_out/ into profiles/ under <tag>:
# bench lines (pipelined and --no-pipeline), per-shape GEMM tables, rocprofv3 --stats
# summaries and the per-step kernel table of the timed region (the traced run is
# --no-pipeline, so its GPU-busy union is checked against the no-pipeline ms_per_step).
# usage: bash tools/collect_round.sh <tag>
set -e
tag=$1
for wl in modelnet 3dmatch 3dlomatch; do
  cp gpurun_out/bench_${wl}_$tag.json profiles/${tag}_${wl}_bench.json
  cp gpurun_out/benchnp_${wl}_$tag.json profiles/${tag}_${wl}_bench_nopipe.json
  cp gpurun_out/gemm_${wl}_$tag.json profiles/${tag}_${wl}_gemm_table.json
  cp gpurun_out/prof_${wl}_$tag/*/*_kernel_stats.csv profiles/${tag}_${wl}_kernel_stats.csv
  # the traced process's own timed steps (bench.py --profile --no-pipeline under rocprofv3) --
  # the same run as the trace; the separate --no-pipeline bench line is printed beside it
  ms=$(python3 -c "import json;print(json.loads(open('gpurun_out/prof_${wl}_$tag.json').read().strip().splitlines()[-1])['ms_per_step'])")
  msb=$(python3 -c "import json;print(json.loads(open('gpurun_out/benchnp_${wl}_$tag.json').read().strip().splitlines()[-1])['ms_per_step'])")
  { python3 tools/kernel_stats.py gpurun_out/prof_${wl}_$tag/*/*_kernel_trace.csv 20 $ms
    echo "no-pipeline bench line of the same build (separate process, 50 steps): $msb ms/step"; } > profiles/${tag}_${wl}_kernel_stats_per_step.txt
done
for wl in modelnet 3dmatch 3dlomatch; do
  [ -f gpurun_out/pmc_kpconv_${wl}_$tag.json ] && cp gpurun_out/pmc_kpconv_${wl}_$tag.json profiles/pmc_kpconv_$wl.json
done
