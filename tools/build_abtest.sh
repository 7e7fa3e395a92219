#!/bin/bash
# A/B or diagnostic build (CPU side) of libfgreg into abtest/libfgreg_<name>.so (abtest/ is
# git-ignored but travels to the GPU box, unlike ablib/), from a scratch copy of csrc/ with
# extra hipcc flags. usage: bash tools/build_abtest.sh <name> "<extra hipcc flags>"
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
pkg=$root/boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd
name=$1; extra=$2
tmp=/tmp/fgr_abtest_build_$name
rm -rf $tmp && mkdir -p $tmp/pkg/csrc $tmp/pkg/fgreg $tmp/include $root/abtest
cp $pkg/csrc/*.hip $pkg/csrc/*.h $pkg/csrc/*.cpp $pkg/csrc/Makefile $tmp/pkg/csrc/
cp $pkg/csrc/*.o $tmp/pkg/csrc/ 2>/dev/null || true
cp $root/include/*.h $tmp/include/
for f in ${TOUCH:-ffn.hip gemm_ws.hip}; do touch $tmp/pkg/csrc/$f; done
make -C $tmp/pkg/csrc -j8 \
    "COMMON=-O3 -std=c++17 -fPIC --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function -mllvm -amdgpu-mfma-vgpr-form=1 $extra" > $tmp/build.log 2>&1 \
  || { tail -30 $tmp/build.log; exit 1; }
cp $tmp/pkg/fgreg/libfgreg.so $root/abtest/libfgreg_$name.so
echo built $root/abtest/libfgreg_$name.so
