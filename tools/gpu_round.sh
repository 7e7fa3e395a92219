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
for wl in modelnet 3dmatch; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'kpconv_gather|kpconv_fused_kernel' --output-format csv -d gpurun_out/pmcf_${wl}_$tag -- python3 bench.py --profile --workload $wl --steps 3 --warmup 1 > gpurun_out/pmcf_${wl}_$tag.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'kpconv_gather|kpconv_fused_kernel' --output-format csv -d gpurun_out/pmcw_${wl}_$tag -- python3 bench.py --profile --workload $wl --steps 3 --warmup 1 > gpurun_out/pmcw_${wl}_$tag.log 2>&1 || exit 1
  # the KPConv stage's op: the fused kernel when it ran (FGREG_KPF), else the gather
  if grep -q kpconv_fused gpurun_out/pmcf_${wl}_$tag/*/*counter_collection.csv; then op=fgr_kpconv_fused; rx=kpconv_fused_kernel; else op=fgr_kpconv_gather; rx=kpconv_gather; fi
  # the bench lines below read profiles/pmc_kpconv_<wl>.json on this box; the copy under
  # gpurun_out/ travels back (tools/collect_round.sh commits it)
  python3 tools/pmc_traffic.py $op $rx $(ls gpurun_out/pmcf_${wl}_$tag/*/*counter_collection.csv) $(ls gpurun_out/pmcw_${wl}_$tag/*/*counter_collection.csv) > profiles/pmc_kpconv_$wl.json || exit 1
  cp profiles/pmc_kpconv_$wl.json gpurun_out/pmc_kpconv_${wl}_$tag.json
done
timeout -k 10 400 python bench.py --steps 50 --warmup 10 --gemm-table gpurun_out/gemm_$tag.json > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit 1
timeout -k 10 400 python bench.py --workload 3dmatch --steps 50 --warmup 10 --gemm-table gpurun_out/gemm3d_$tag.json > gpurun_out/bench3d_$tag.json 2> gpurun_out/bench3d_$tag.err || exit 1
timeout -k 10 400 python bench.py --workload 3dlomatch --steps 50 --warmup 10 --gemm-table gpurun_out/gemmlo_$tag.json > gpurun_out/benchlo_$tag.json 2> gpurun_out/benchlo_$tag.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -- python3 bench.py --profile --steps $K --warmup $W > gpurun_out/prof_$tag.json 2> gpurun_out/prof_$tag.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3d_$tag -- python3 bench.py --profile --workload 3dmatch --steps $K --warmup $W > gpurun_out/prof3d_$tag.json 2> gpurun_out/prof3d_$tag.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/proflo_$tag -- python3 bench.py --profile --workload 3dlomatch --steps $K --warmup $W > gpurun_out/proflo_$tag.json 2> gpurun_out/proflo_$tag.err || exit 1
echo DONE
