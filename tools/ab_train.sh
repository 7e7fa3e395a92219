#!/bin/bash
# Training A/B (GPU box): the backward tests, then bench.py --train per environment setting.
# usage: [ABK="pytest -k expr"] bash tools/ab_train.sh <tag> "NAME=V ..." "NAME=V ..." ...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "${ABK:-wgrad or linear_backward or kpconv_backward or deterministic or train_step_vs or segnorm or batchnorm or image_bits}" > gpurun_out/t_train_$tag.log 2>&1 || { tail -30 gpurun_out/t_train_$tag.log; exit 1; }
tail -1 gpurun_out/t_train_$tag.log
i=0
for cfg in "$@"; do
  i=$((i + 1))
  env $cfg timeout -k 10 300 python bench.py --train --steps 10 --warmup 3 > gpurun_out/train_${tag}_$i.json 2> gpurun_out/train_${tag}_$i.err || { echo "config $i failed"; tail -5 gpurun_out/train_${tag}_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/train_${tag}_$i.json')); print(f\"{sys.argv[1]:40s} {d['value']:7.2f} ms/step  split {d.get('split_ms')}\")" "$cfg"
done
