#!/bin/bash
# Build an A/B variant of libfhecore with extra compiler defines into tools/variants/<name>.so
# usage: tools/build_variant.sh name "-DFOO=1 -DBAR=2"
set -e
name=$1; defs=$2
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/tools/variants/$name; mkdir -p $out
for f in context.cpp capi.cpp prof.cpp ntt.hip ntt_ks.hip elementwise.hip rns.hip galois.hip serialize.cpp pipeline.hip keygen.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $defs -c $root/gpu-fhe_amd/csrc/$f -o $out/$f.o &
done
wait || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $root/tools/variants/$name.so $out/*.o
rm -rf $out
echo built tools/variants/$name.so
