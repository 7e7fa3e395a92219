set -o pipefail
cd $GRAFT_REPO_ROOT
FGR_GEMM_WSP=1 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "split_vs_fp64 or ws_dynamic" tests/test_gpu_gemm_ln.py > gpurun_out/wsp_t1.log 2>&1 || { tail -30 gpurun_out/wsp_t1.log; exit 1; }
tail -3 gpurun_out/wsp_t1.log
FGR_GEMM_WSP=1 timeout -k 10 120 python3 -u tools/ws_bench.py 50 > gpurun_out/wsp_b1.log 2>&1 && FGR_GEMM_WSP=0 timeout -k 10 120 python3 -u tools/ws_bench.py 50 > gpurun_out/wsp_b0.log 2>&1 && FGR_GEMM_WSP=1 FGR_WSP_NPW=4 timeout -k 10 120 python3 -u tools/ws_bench.py 50 > gpurun_out/wsp_b4.log 2>&1
echo "== wsp"; cat gpurun_out/wsp_b1.log; echo "== one-round"; cat gpurun_out/wsp_b0.log; echo "== npw4"; cat gpurun_out/wsp_b4.log
