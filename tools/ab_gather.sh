#!/bin/bash
# tests, then bench lines with gather tables for three libraries on modelnet + 3dmatch
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_forward.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_r05ac.log 2>&1 || { tail -20 gpurun_out/t_r05ac.log; exit 1; }
tail -1 gpurun_out/t_r05ac.log
for wl in modelnet 3dmatch; do
  i=0
  for lib in "" ablib/libfgreg_u4.so ablib/libfgreg_base.so "" ablib/libfgreg_u4.so ablib/libfgreg_base.so; do
    i=$((i+1))
    FGREG_LIB_PATH=$lib timeout -k 10 300 python bench.py --workload $wl --steps 30 --warmup 10 --no-cpu-baseline --gather-table gpurun_out/gt_r05ac_${wl}_$i.json > gpurun_out/b_r05ac_${wl}_$i.json 2> gpurun_out/b_r05ac_${wl}_$i.err || { tail -5 gpurun_out/b_r05ac_${wl}_$i.err; exit 1; }
    python3 - "$lib" gpurun_out/b_r05ac_${wl}_$i.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
ro = d['rooflines_other']
print(f"{sys.argv[1] or 'new':28s} {d['value']:8.1f} pairs/s {d['ms_per_step']:.3f} ms gather {d['roofline']['frac']:.3f} {d['roofline']['avg_launch_us']:.1f}us r2n {d['roofline_res2net']['us_per_step']:.1f}us ln {ro['layernorm']['us_per_step']:.1f}us")
PY
  done
done
