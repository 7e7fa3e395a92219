#!/bin/bash
# Round-6 GPU session: new-kernel tests first (isolated), then the full GPU suite, then same-box
# bench A/B lines. Every GPU step under its own limit; the first failure ends the script.
# usage (GPU box, repo root): bash tools/r06_check.sh <tag> [ab "ENV=V ..." "ENV=V ..."]
set -o pipefail
tag=${1:-r06}
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
if [ -n "$NEWTESTS" ]; then
  timeout -k 10 300 $T $NEWTESTS > gpurun_out/t_${tag}_new.log 2>&1 || { echo "NEW TESTS FAILED"; tail -40 gpurun_out/t_${tag}_new.log; exit 1; }
  tail -2 gpurun_out/t_${tag}_new.log
fi
if [ -z "$SKIPFULL" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_${tag}_all.log 2>&1 || { echo "FULL SUITE FAILED"; tail -40 gpurun_out/t_${tag}_all.log; exit 1; }
  tail -2 gpurun_out/t_${tag}_all.log
fi
if [ "$2" = "ab" ]; then
  shift 2
  bash tools/ab_env.sh $tag ${WL:-modelnet} "$@" || exit 1
fi
echo DONE
