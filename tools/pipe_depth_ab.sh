# fgreg.pipeline depth A/B (run on the GPU box from the repo root): bench lines per workload
# at FGREG_PIPE_DEPTH 1 / 2 / 3, same box, summary to stdout
set -o pipefail
mkdir -p gpurun_out
for wl in modelnet 3dmatch 3dlomatch; do for dp in 1 2 3; do
  FGREG_PIPE_DEPTH=$dp timeout -k 10 300 python bench.py --workload $wl --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_${wl}_pd$dp.json 2> gpurun_out/bench_${wl}_pd$dp.err || { tail -20 gpurun_out/bench_${wl}_pd$dp.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/bench_${wl}_pd$dp.json').read().strip().splitlines()[-1]); print('$wl depth $dp', round(d['value'],1), 'pairs/s', round(d['ms_per_step'],3), 'ms/step')"
done; done
