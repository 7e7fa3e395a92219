# PMC passes (development tool, GPU box) over one GEMM shape in one mode: issue / wait /
# MFMA-busy counters per tile config. usage: bash tools/pmc_gemm2.sh M N K "cfgs" f16x3|bf16 tag
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
M=$1; N=$2; K=$3; CFGS=$4; MODE=${5:-f16x3}; TAG=${6:-x}
mkdir -p $R/gpurun_out/pmcg_$TAG
for cfg in $CFGS; do
d=$R/gpurun_out/pmcg_$TAG/${M}_${N}_${K}_${MODE}_$cfg
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA -d $d/p1 -o p1 --output-format csv -- python3 $R/tools/gemm_one.py $M $N $K $cfg $MODE 20 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $d/p2 -o p2 --output-format csv -- python3 $R/tools/gemm_one.py $M $N $K $cfg $MODE 20 || exit 1
done
