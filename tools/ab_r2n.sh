#!/bin/bash
# Res2Net chain A/B (GPU box): parity tests, then bench lines per configuration
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_forward.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "res2net or forward" > gpurun_out/t_r05ad.log 2>&1 || { tail -20 gpurun_out/t_r05ad.log; exit 1; }
tail -1 gpurun_out/t_r05ad.log
for wl in modelnet 3dmatch; do
  bash tools/ab_env.sh r05ad_$wl $wl "FGREG_X=new" "FGREG_R2N224=h3" "FGREG_LIB_PATH=ablib/libfgreg_head.so" "FGREG_X=new" "FGREG_R2N224=h3" "FGREG_LIB_PATH=ablib/libfgreg_head.so" || exit 1
  for i in 1 2 3 4 5 6; do python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r05ad_${wl}_$i.json')); print('   r2n', round(d['roofline_res2net']['us_per_step'],1), 'us/step', round(d['roofline_res2net']['frac'],3))"; done
done
