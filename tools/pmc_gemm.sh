# PMC passes over one GEMM shape (development tool, GPU box): issue / wait / MFMA-busy
# counters and L2 hit rate per tile config. usage: bash tools/pmc_gemm.sh M N K "cfgs"
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
M=${1:-9544}; N=${2:-1024}; K=${3:-2048}; CFGS=${4:-"b I"}
mkdir -p $R/gpurun_out/pmcg
for cfg in $CFGS; do
d=$R/gpurun_out/pmcg/${M}_${N}_${K}_$cfg
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA -d $d/p1 -o p1 --output-format csv -- python3 $R/tools/gemm_one.py $M $N $K $cfg f16x3 20 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $d/p2 -o p2 --output-format csv -- python3 $R/tools/gemm_one.py $M $N $K $cfg f16x3 20 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $d/p3 -o p3 --output-format csv -- python3 $R/tools/gemm_one.py $M $N $K $cfg f16x3 20 || exit 1
done
