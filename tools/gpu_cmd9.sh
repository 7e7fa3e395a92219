set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_ln.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_ln9.log 2>&1 || { echo LN TESTS FAILED; tail -40 gpurun_out/tests_ln9.log; exit 1; }
tail -1 gpurun_out/tests_ln9.log
timeout -k 10 180 python -u tools/ln_gemm_bench.py > gpurun_out/ln_bench9.txt 2>&1 || { tail -20 gpurun_out/ln_bench9.txt; exit 1; }
cat gpurun_out/ln_bench9.txt
timeout -k 10 300 python -u tools/rs_sweep.py > gpurun_out/rs_sweep9.txt 2>&1 || { tail -20 gpurun_out/rs_sweep9.txt; exit 1; }
for fz in 1 0; do
  FGR_LN_FUSE=$fz timeout -k 10 300 python bench.py --workload modelnet --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_modelnet_ln${fz}_9.json 2> gpurun_out/bench_modelnet_ln${fz}_9.err || { tail -20 gpurun_out/bench_modelnet_ln${fz}_9.err; exit 1; }
  python3 - gpurun_out/bench_modelnet_ln${fz}_9.json $fz <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('LN_FUSE', sys.argv[2], 'value', round(d['value'], 1), 'ms/step', round(d['ms_per_step'], 3),
      'gemm', round(d['roofline_gemm']['frac'], 3), 'gemm ms/step', round(d['roofline_gemm']['share_of_step'] * d['ms_per_step'], 3))
PY
done
