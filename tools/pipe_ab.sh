set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pipe_tests.log 2>&1 || { tail -30 gpurun_out/pipe_tests.log; exit 1; }
tail -2 gpurun_out/pipe_tests.log
for wl in modelnet 3dmatch 3dlomatch; do
  timeout -k 10 200 python bench.py --workload $wl --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/pipe_$wl.json 2>gpurun_out/pipe_$wl.err || exit 1
  timeout -k 10 200 python bench.py --workload $wl --steps 30 --warmup 5 --no-cpu-baseline --no-pipeline > gpurun_out/nopipe_$wl.json 2>gpurun_out/nopipe_$wl.err || exit 1
  python tools/summarize.py gpurun_out/pipe_$wl.json gpurun_out/nopipe_$wl.json | grep pairs
done
