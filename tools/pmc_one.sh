# PMC traffic passes of the KPConv gather for one workload (as tools/gpu_round.sh does for all) and a bench line reading them
# usage (on the GPU box): bash tools/pmc_one.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
wl=3dlomatch; tag=r03f
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'kpconv_gather' --output-format csv -d gpurun_out/pmcf_${wl}_$tag -- python3 bench.py --profile --workload $wl --steps 3 --warmup 1 > gpurun_out/pmcf_${wl}_$tag.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'kpconv_gather' --output-format csv -d gpurun_out/pmcw_${wl}_$tag -- python3 bench.py --profile --workload $wl --steps 3 --warmup 1 > gpurun_out/pmcw_${wl}_$tag.log 2>&1 || exit 1
python3 tools/pmc_traffic.py fgr_kpconv_gather kpconv_gather $(ls gpurun_out/pmcf_${wl}_$tag/*/*counter_collection.csv) $(ls gpurun_out/pmcw_${wl}_$tag/*/*counter_collection.csv) > profiles/pmc_kpconv_$wl.json || exit 1
cp profiles/pmc_kpconv_$wl.json gpurun_out/pmc_kpconv_${wl}_$tag.json
timeout -k 10 300 python bench.py --workload $wl --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_${wl}_pmc.json 2> gpurun_out/bench_${wl}_pmc.err || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_${wl}_pmc.json').read().strip().splitlines()[-1]); print(d['roofline'])"
