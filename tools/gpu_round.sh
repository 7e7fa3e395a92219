#!/bin/bash
# One GPU session: parity tests, bench lines, kernel-trace profiles of the timed steps only,
# PMC traffic passes of the KPConv gather. Every GPU step has its own time limit and the
# steps are chained: the first failure (fault, abort, timeout) ends the script.
# usage (on the GPU box, from the repo root): bash tools/gpu_round.sh <tag> [skip-tests]
set -o pipefail
tag=${1:-run}
export TMPDIR=/tmp
mkdir -p gpurun_out
W=2; K=20          # profiled runs: python tools/kernel_stats.py <kernel_trace.csv> $K <ms_per_step>
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      -p no:cacheprovider > gpurun_out/tests_$tag.log 2>&1 || { echo "TESTS FAILED $?"; tail -30 gpurun_out/tests_$tag.log; exit 1; }
  tail -3 gpurun_out/tests_$tag.log
fi
# PMC passes first (their summaries feed the bench lines' roofline.traffic): FETCH_SIZE and
# WRITE_SIZE in separate runs, gather kernels only, per workload
for wl in modelnet 3dmatch 3dlomatch; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'kpconv_gather' --output-format csv -d gpurun_out/pmcf_${wl}_$tag -- python3 bench.py --profile --workload $wl --steps 3 --warmup 1 > gpurun_out/pmcf_${wl}_$tag.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'kpconv_gather' --output-format csv -d gpurun_out/pmcw_${wl}_$tag -- python3 bench.py --profile --workload $wl --steps 3 --warmup 1 > gpurun_out/pmcw_${wl}_$tag.log 2>&1 || exit 1
  op=fgr_kpconv_gather; rx=kpconv_gather
  # the bench lines below read profiles/pmc_kpconv_<wl>.json on this box; the copy under
  # gpurun_out/ travels back (tools/collect_round.sh commits it)
  python3 tools/pmc_traffic.py $op $rx $(ls gpurun_out/pmcf_${wl}_$tag/*/*counter_collection.csv) $(ls gpurun_out/pmcw_${wl}_$tag/*/*counter_collection.csv) > profiles/pmc_kpconv_$wl.json || exit 1
  cp profiles/pmc_kpconv_$wl.json gpurun_out/pmc_kpconv_${wl}_$tag.json
done
# bench lines (pipelined = the driver's default) and the same workloads with --no-pipeline:
# the kernel traces below run --no-pipeline (the tracer serialises the side stream), so their
# GPU-busy union is compared with the no-pipeline ms_per_step (tools/kernel_stats.py)
for wl in modelnet 3dmatch 3dlomatch; do
  timeout -k 10 400 python bench.py --workload $wl --steps 50 --warmup 10 --gemm-table gpurun_out/gemm_${wl}_$tag.json > gpurun_out/bench_${wl}_$tag.json 2> gpurun_out/bench_${wl}_$tag.err || exit 1
  timeout -k 10 400 python bench.py --workload $wl --no-pipeline --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/benchnp_${wl}_$tag.json 2> gpurun_out/benchnp_${wl}_$tag.err || exit 1
done
for wl in modelnet 3dmatch 3dlomatch; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${wl}_$tag -- python3 bench.py --profile --no-pipeline --workload $wl --steps $K --warmup $W > gpurun_out/prof_${wl}_$tag.json 2> gpurun_out/prof_${wl}_$tag.err || exit 1
done
echo DONE
