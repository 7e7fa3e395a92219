set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_s8.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/tests_s8.log; exit 1; }
tail -1 gpurun_out/tests_s8.log
for wl in modelnet 3dmatch 3dlomatch; do
  timeout -k 10 300 python bench.py --workload $wl --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_${wl}_s8.json 2> gpurun_out/bench_${wl}_s8.err || { tail -20 gpurun_out/bench_${wl}_s8.err; exit 1; }
  python3 - gpurun_out/bench_${wl}_s8.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d['config']['workload'][:12], 'value', round(d['value'], 1), 'ms/step', round(d['ms_per_step'], 3),
      'gemm', round(d['roofline_gemm']['frac'], 3), 'gemm ms/step', round(d['roofline_gemm']['share_of_step'] * d['ms_per_step'], 3))
PY
done
