#!/bin/bash
# A/B build (CPU side): libfgreg from a scratch copy of csrc/ into ablib/libfgreg_<name>.so,
# with extra hipcc flags (e.g. -DFGR_RS_NB=4) and optionally the sources of a git ref instead
# of the working tree. The product objects stay untouched.
# usage: bash tools/build_variant.sh <name> "<extra hipcc flags>" [git-ref]
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
rel=boosting-fine-grained-feature-fusion-in-3d-point-cloud-registration_amd
name=$1; extra=$2; ref=$3
tmp=/tmp/fgr_variant_build_$name
rm -rf $tmp && mkdir -p $tmp/pkg/csrc $tmp/pkg/fgreg $tmp/include $root/ablib
if [ -n "$ref" ]; then
  git -C $root archive $ref $rel/csrc include | tar -x -C $tmp
  mv $tmp/$rel/csrc/* $tmp/pkg/csrc/
else
  cp $root/$rel/csrc/*.hip $root/$rel/csrc/*.h $root/$rel/csrc/*.cpp $root/$rel/csrc/Makefile $tmp/pkg/csrc/
  cp $root/include/*.h $tmp/include/
fi
make -C $tmp/pkg/csrc -j8 \
    "COMMON=-O3 -std=c++17 -fPIC --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function -mllvm -amdgpu-mfma-vgpr-form=1 $extra" > $tmp/build.log 2>&1 \
  || { tail -30 $tmp/build.log; exit 1; }
cp $tmp/pkg/fgreg/libfgreg.so $root/ablib/libfgreg_$name.so
echo built $root/ablib/libfgreg_$name.so
