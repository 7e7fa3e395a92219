# same-box A/B of two builds: FGREG_LIB_PATH=<alt .so> vs the in-tree libfgreg.so
# usage: bash tools/lib_ab.sh <alt.so> <workload> [<workload> ...]
alt=$1; shift
for wl in "$@"; do
  for r in 1 2; do
    timeout -k 10 200 python bench.py --workload $wl --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_new_$wl.json 2>/dev/null || exit 1
    FGREG_LIB_PATH=$alt timeout -k 10 200 python bench.py --workload $wl --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_base_$wl.json 2>/dev/null || exit 1
    python tools/summarize.py gpurun_out/ab_new_$wl.json gpurun_out/ab_base_$wl.json | grep pairs
  done
done
