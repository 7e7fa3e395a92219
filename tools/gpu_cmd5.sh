set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_s5.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/tests_s5.log; exit 1; }
tail -1 gpurun_out/tests_s5.log
timeout -k 10 400 bash tools/pmc_attn.sh s5 > gpurun_out/pmc_attn_s5.log 2>&1 || { tail -20 gpurun_out/pmc_attn_s5.log; exit 1; }
python3 tools/pmc_attn_summary.py gpurun_out/pmca_s5 gpurun_out/pmc_attn_s5.json || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_attn_s5.json'))
for k,v in d.items(): print(k, {x: v['counters'].get(x) for x in ('SQ_LDS_BANK_CONFLICT','SQ_INSTS_LDS','SQ_WAIT_ANY','SQ_WAVE_CYCLES')}, round(v['mfma_busy_frac'],3))"
