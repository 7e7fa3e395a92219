# split-K sweep of the few-row shapes (3DMatch / 3DLoMatch transformer + KPConv), f16x3 and bf16
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_splitk.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/splitk_tests.log 2>&1; tail -3 gpurun_out/splitk_tests.log
timeout -k 10 400 python tools/gemm_tiles.py IWSBXT 3d ks > gpurun_out/splitk_h3.txt 2>&1 || exit 1
timeout -k 10 400 python tools/gemm_tiles.py IWSBXT bf16 3d ks > gpurun_out/splitk_bf16.txt 2>&1 || exit 1
cat gpurun_out/splitk_h3.txt gpurun_out/splitk_bf16.txt | sed 's/ | /\n   /g' | awk '{print}' > /dev/null
