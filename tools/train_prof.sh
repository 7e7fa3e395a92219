#!/bin/bash
# rocprofv3 kernel trace of bench.py --train --profile (GPU box): per-step kernel table of the
# timed training steps. usage: bash tools/train_prof.sh <tag>
set -o pipefail
tag=${1:-run}
export TMPDIR=/tmp
mkdir -p gpurun_out
K=5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trainprof_$tag -- python3 bench.py --train --profile --steps $K --warmup 2 > gpurun_out/trainprof_$tag.json 2> gpurun_out/trainprof_$tag.err || { tail -20 gpurun_out/trainprof_$tag.err; exit 1; }
ms=$(python3 -c "import json;print(json.load(open('gpurun_out/trainprof_$tag.json'))['value'])")
python3 tools/kernel_stats.py $(ls gpurun_out/trainprof_$tag/*/*kernel_trace.csv) $K $ms 45 > gpurun_out/trainprof_${tag}_per_step.txt
head -45 gpurun_out/trainprof_${tag}_per_step.txt
tail -3 gpurun_out/trainprof_${tag}_per_step.txt
