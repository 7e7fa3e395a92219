#!/bin/bash
# Res2Net chain A/B (GPU box): parity tests, then bench lines per configuration
# (w = 224 chain: bf16x6 vs f16x3 with 48-row blocks vs f16x3 with 32-row blocks)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_forward.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "res2net or forward" > gpurun_out/t_r05ai.log 2>&1 || { tail -20 gpurun_out/t_r05ai.log; exit 1; }
tail -1 gpurun_out/t_r05ai.log
for wl in modelnet 3dmatch; do
  bash tools/ab_env.sh r05ai_$wl $wl "FGREG_R2N224=x6" "FGREG_R2N224=h3" "FGREG_R2N224=h3 FGR_R2N_ROWS=32" "FGREG_R2N224=x6" "FGREG_R2N224=h3" || exit 1
  for i in 1 2 3 4 5; do python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r05ai_${wl}_$i.json')); print('   r2n', round(d['roofline_res2net']['us_per_step'],1), 'us/step', round(d['roofline_res2net']['frac'],3))"; done
done
