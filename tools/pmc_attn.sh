# PMC passes for the attention kernel of the ModelNet forward (development tool, GPU box)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmca
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-include-regex 'attn_f16x3' -d $R/gpurun_out/pmca/p1 -o p1 --output-format csv -- python3 $R/bench.py --profile --steps 3 --warmup 2 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex 'attn_f16x3' -d $R/gpurun_out/pmca/p2 -o p2 --output-format csv -- python3 $R/bench.py --profile --steps 3 --warmup 2 || exit 1
