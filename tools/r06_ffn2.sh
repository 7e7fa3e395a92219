set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_ffn.py > gpurun_out/t_r06d_ffn.log 2>&1 || { echo FFN TESTS FAILED; tail -40 gpurun_out/t_r06d_ffn.log; exit 1; }
tail -2 gpurun_out/t_r06d_ffn.log
timeout -k 10 120 python tools/ffn_bench.py 9544 50 || exit 1
FGR_FFN_V=1 timeout -k 10 120 python tools/ffn_bench.py 9544 50 || exit 1
