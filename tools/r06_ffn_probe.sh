set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/ffn_bench.py 9544 50 > gpurun_out/ffnb_prod.txt 2>&1 || exit 1
FGREG_LIB_PATH=abtest/libfgreg_stamp.so timeout -k 10 120 python tools/ffn_bench.py 9544 50 > gpurun_out/ffnb_stamp.txt 2>&1 || exit 1
cat gpurun_out/ffnb_prod.txt gpurun_out/ffnb_stamp.txt
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-include-regex ffn_f16x3 -d $GRAFT_REPO_ROOT/gpurun_out/pmc_ffn/p1 -o p1 --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ffn_bench.py 9544 10 > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex ffn_f16x3 -d $GRAFT_REPO_ROOT/gpurun_out/pmc_ffn/p2 -o p2 --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ffn_bench.py 9544 10 > /dev/null 2>&1 || exit 1
echo PMC DONE
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_metrics.py tests/test_gpu_train.py -k "metrics or dropout" > gpurun_out/t_r06c_new.log 2>&1 || { echo NEW TESTS FAILED; tail -40 gpurun_out/t_r06c_new.log; exit 1; }
tail -3 gpurun_out/t_r06c_new.log
