#!/bin/bash
# Diagnostic build (CPU side): libfgreg with the rs kernel's clock stamps (-DFGR_RS_STAMP)
# into ablib/libfgreg_<name>.so (default name: stamp), from a scratch copy of csrc/ (the
# product objects untouched). usage: bash tools/build_stamp.sh [name] [extra hipcc flags]
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
pkg=$root/boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd
name=${1:-stamp}; extra=$2
tmp=/tmp/fgr_stamp_build_$name
rm -rf $tmp && mkdir -p $tmp/pkg/csrc $tmp/include $root/ablib
cp $pkg/csrc/*.hip $pkg/csrc/*.h $pkg/csrc/*.cpp $pkg/csrc/Makefile $tmp/pkg/csrc/
cp $root/include/*.h $tmp/include/
mkdir -p $tmp/pkg/fgreg
make -C $tmp/pkg/csrc -j8 COMMON_EXTRA=1 \
    "COMMON=-O3 -std=c++17 -fPIC --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function -mllvm -amdgpu-mfma-vgpr-form=1 -DFGR_RS_STAMP $extra" > $tmp/build.log 2>&1
cp $tmp/pkg/fgreg/libfgreg.so $root/ablib/libfgreg_$name.so
echo built $root/ablib/libfgreg_$name.so
