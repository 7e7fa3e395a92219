set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "gemm" > gpurun_out/t_gemm.log 2>&1 || { tail -30 gpurun_out/t_gemm.log; exit 1; }
tail -1 gpurun_out/t_gemm.log
timeout -k 10 300 python -u tools/rs_probe.py > gpurun_out/rs_probe.txt 2>&1 || { tail -20 gpurun_out/rs_probe.txt; exit 1; }
cat gpurun_out/rs_probe.txt
timeout -k 10 300 python -u tools/rs_sweep.py > gpurun_out/rs_sweep.txt 2>&1 || { tail -20 gpurun_out/rs_sweep.txt; exit 1; }
cat gpurun_out/rs_sweep.txt
