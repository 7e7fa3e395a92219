set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "attention" > gpurun_out/t_attn.log 2>&1 || { tail -30 gpurun_out/t_attn.log; exit 1; }
tail -1 gpurun_out/t_attn.log
timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/attn_swz.txt 2>&1 || { tail -20 gpurun_out/attn_swz.txt; exit 1; }
timeout -k 10 300 python -u tools/attn_bench.py bf16 >> gpurun_out/attn_swz.txt 2>&1 || { tail -20 gpurun_out/attn_swz.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/attn_swz.txt
