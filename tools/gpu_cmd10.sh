set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/ln_gemm_bench.py sweep > gpurun_out/ln_bench10.txt 2>&1 || { tail -20 gpurun_out/ln_bench10.txt; exit 1; }
cat gpurun_out/ln_bench10.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_s10.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/tests_s10.log; exit 1; }
tail -1 gpurun_out/tests_s10.log
