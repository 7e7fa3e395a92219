#!/bin/bash
# Runs "name|command" steps on the GPU box, each under its own time limit; a step that
# fails with pytest's "tests failed" (1) lets the next run, anything else (fault, abort,
# timeout) ends the call. usage: bash tools/gpu_steps.sh <secs> "name|cmd" ...
export TMPDIR=/tmp
mkdir -p gpurun_out
lim=$1; shift
for st in "$@"; do
    name=${st%%|*}; cmd=${st#*|}
    echo "== $name: $cmd"
    timeout -k 10 "$lim" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "== $name exit $rc"; tail -3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
