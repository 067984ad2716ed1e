#!/bin/bash
# Build an A/B variant of libfhecore with extra compiler defines into tools/variants/<name>.so
# (for experiments: the shipped sources have no A/B switches left -- the measured alternatives are
# recorded in DESIGN.md §8 -- so a variant means editing a copy of the sources or adding a define)
# usage: tools/build_variant.sh name "-DFOO=1 -DBAR=2"   (REV=<git rev>: build that commit's sources,
# e.g. REV=HEAD for the committed build against an edited working tree; COMPAT=1 adds
# tools/variant_compat.cpp, the entry points a commit before round 5 lacks)
set -e
name=$1; defs=$2
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/tools/variants/$name; mkdir -p $out
src=$root/gpu-fhe_amd/csrc
if [ -n "$REV" ]; then
  tmp=$(mktemp -d /tmp/fhe_rev_XXXX)
  git -C "$root" archive "$REV" gpu-fhe_amd/csrc include | tar -x -C "$tmp"
  src=$tmp/gpu-fhe_amd/csrc
fi
pids=()
for f in host_tables.cpp context.cpp capi.cpp prof.cpp ntt.hip ntt_ks.hip elementwise.hip rns.hip galois.hip wire.cpp serialize.cpp pipeline.hip keygen.hip dist.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $defs -c $src/$f -o $out/$f.o &
  pids+=($!)
done
if [ -n "$COMPAT" ]; then
  /opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -c $root/tools/variant_compat.cpp -o $out/variant_compat.o &
  pids+=($!)
fi
for p in "${pids[@]}"; do wait "$p" || exit 1; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $root/tools/variants/$name.so $out/*.o -L/opt/rocm/lib -lrccl
rm -rf $out
echo built tools/variants/$name.so
