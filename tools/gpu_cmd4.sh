set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "attention or instnorm" > gpurun_out/t_k.log 2>&1 || { tail -30 gpurun_out/t_k.log; exit 1; }
tail -1 gpurun_out/t_k.log
timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/attn_swz.txt 2>&1 || { tail -20 gpurun_out/attn_swz.txt; exit 1; }
timeout -k 10 300 python -u tools/attn_bench.py bf16 >> gpurun_out/attn_swz.txt 2>&1 || { tail -20 gpurun_out/attn_swz.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/attn_swz.txt
for wl in modelnet 3dmatch 3dlomatch; do
  timeout -k 10 300 python bench.py --workload $wl --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${wl}_s4.json 2> gpurun_out/bench_${wl}_s4.err || { tail -20 gpurun_out/bench_${wl}_s4.err; exit 1; }
  python3 - gpurun_out/bench_${wl}_s4.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
o = d['rooflines_other']
print(d['config']['workload'][:12], 'value', round(d['value'], 1), 'ms/step', round(d['ms_per_step'], 3),
      'gemm', round(d['roofline_gemm']['frac'], 3), 'attn', round(d['roofline_attention']['frac'], 3),
      'attn us/step', round(d['roofline_attention']['share_of_step'] * d['ms_per_step'] * 1000, 1),
      'instnorm us/step', round(o['instnorm']['us_per_step'], 1))
PY
done
