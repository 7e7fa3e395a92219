#!/bin/bash
# round-4 working check (GPU box): new kernels' tests first (a fault ends the script there),
# then the training / multi-rank / bf16 suites, the rs A/B, the train and ModelNet bench lines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04}
timeout -k 10 400 python -u -m pytest "tests/test_gpu_kernels.py::test_corr_head_fused_vs_fp64" tests/test_gpu_gemm_ln.py tests/test_gpu_forward.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_${tag}_a.log 2>&1 || { echo "TESTS A FAILED"; tail -30 gpurun_out/tests_${tag}_a.log; exit 1; }
tail -2 gpurun_out/tests_${tag}_a.log
timeout -k 10 240 python -u tools/rs_defer_ab.py > gpurun_out/rs_defer_ab_${tag}.txt 2>&1 || { echo "AB FAILED"; tail -20 gpurun_out/rs_defer_ab_${tag}.txt; exit 1; }
cat gpurun_out/rs_defer_ab_${tag}.txt | grep -v amdgpu.ids
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_dist.py "tests/test_gpu_bf16.py::test_bf16_forward_3dlomatch_vs_oracle" -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_${tag}_b.log 2>&1
rc=$?
tail -4 gpurun_out/tests_${tag}_b.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 200 python bench.py --train --steps 10 --warmup 3 > gpurun_out/bench_train_${tag}.json 2> gpurun_out/bench_train_${tag}.err || exit 1
cat gpurun_out/bench_train_${tag}.json
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_modelnet_${tag}.json 2> gpurun_out/bench_modelnet_${tag}.err || exit 1
head -c 400 gpurun_out/bench_modelnet_${tag}.json
