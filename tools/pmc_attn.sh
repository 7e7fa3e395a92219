# PMC passes over the attention kernel (development tool, GPU box): tools/attn_bench.py's
# shapes, issue / wait / MFMA counters and the LDS / VALU mix. usage: bash tools/pmc_attn.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
d=$R/gpurun_out/pmca
mkdir -p $d
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-include-regex 'attn_f16x3' -d $d/p1 -o p1 --output-format csv -- python3 $R/tools/attn_bench.py || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-include-regex 'attn_f16x3' -d $d/p2 -o p2 --output-format csv -- python3 $R/tools/attn_bench.py || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_BRANCH --kernel-include-regex 'attn_f16x3' -d $d/p3 -o p3 --output-format csv -- python3 $R/tools/attn_bench.py || exit 1
