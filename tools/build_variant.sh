#!/bin/bash
# Build libsift_hip.so variants with extra compile flags into build_ab/<name>.so (shipped to the GPU box, git-ignored)
# usage: tools/build_variant.sh <name> "<-D flags>"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
PKG=$R/sift-scale-space-extrema-detection_amd
OUT=$R/build_ab/$1.tmp
mkdir -p $OUT $R/build_ab
for f in sift_gauss sift_extrema sift_refine sift_image sift_api; do
  X=""
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result $X $2 -c -o $OUT/$f.o $PKG/csrc/$f.hip &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/build_ab/$1.so $OUT/*.o
rm -rf $OUT
