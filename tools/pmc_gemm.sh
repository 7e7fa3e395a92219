set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcg
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/pmcg/list.txt 2>&1 || true
for cfg in b I; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA -d $R/gpurun_out/pmcg/p1_$cfg -o p1 --output-format csv -- python3 $R/tools/gemm_one.py 9544 1024 2048 $cfg f16x3 20 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $R/gpurun_out/pmcg/p2_$cfg -o p2 --output-format csv -- python3 $R/tools/gemm_one.py 9544 1024 2048 $cfg f16x3 20 || exit 1
done
