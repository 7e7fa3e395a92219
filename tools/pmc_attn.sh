# PMC passes over the attention kernels (development tool, GPU box): tools/attn_bench.py's
# shapes in the f16x3 and bf16 modes, issue / wait / MFMA counters and the LDS / VALU mix, in
# separate passes (one counter group each). usage: bash tools/pmc_attn.sh [tag]
#   -> gpurun_out/pmca_<tag>/<mode>/p{1,2,3}; summary: python tools/pmc_attn_summary.py gpurun_out/pmca_<tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tag=${1:-run}
for mode in ${MODES:-f16x3 bf16}; do
d=$R/gpurun_out/pmca_$tag/$mode
mkdir -p $d
export FGREG_ATTN=$mode
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-include-regex 'attn_f16x3_|attn_bf16_' -d $d/p1 -o p1 --output-format csv -- python3 $R/tools/attn_bench.py || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-include-regex 'attn_f16x3_|attn_bf16_' -d $d/p2 -o p2 --output-format csv -- python3 $R/tools/attn_bench.py || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_MFMA --kernel-include-regex 'attn_f16x3_|attn_bf16_' -d $d/p3 -o p3 --output-format csv -- python3 $R/tools/attn_bench.py || exit 1
done
