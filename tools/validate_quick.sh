# quick validation on the GPU box: the full -m gpu suite, the long-K GEMM sweep and a ModelNet bench line
# usage: bash tools/validate_quick.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_s24.log 2>&1 || { tail -30 gpurun_out/tests_s24.log; exit 1; }
tail -1 gpurun_out/tests_s24.log
timeout -k 10 300 python -u tools/gemm_longk.py > gpurun_out/gemm_longk2.txt 2>&1 || exit 1
grep "^M=" gpurun_out/gemm_longk2.txt
timeout -k 10 300 python bench.py --workload modelnet --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_mn24.json 2> gpurun_out/bench_mn24.err || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_mn24.json').read().strip().splitlines()[-1]); print('modelnet', round(d['value'],1), round(d['ms_per_step'],3), round(d['roofline_gemm']['frac'],3))"
