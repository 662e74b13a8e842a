#!/bin/bash
# Build libsift_hip.so variants with extra compile flags into build_ab/<name>.so (shipped to the GPU box, git-ignored)
# usage: tools/build_variant.sh <name> "<-D flags>"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
PKG=$R/sift-scale-space-extrema-detection_amd
OUT=$R/build_ab/$1.tmp
mkdir -p $OUT $R/build_ab
pids=()
for f in sift_gauss sift_extrema sift_refine sift_image sift_api; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result $2 -c -o $OUT/$f.o $PKG/csrc/$f.hip &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "variant $1: compile failed"; rm -rf $OUT; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/build_ab/$1.so $OUT/*.o
rm -rf $OUT
