#!/bin/bash
# A/B timing on the GPU box: GPU parity tests of the in-tree build, then tools/time_ntt.py for each
# named variant in tools/variants/.  usage: tools/gpu_ab.sh <outdir> variant...
out=$1; shift
mkdir -p "$out"
timeout -k 10 400 python -m pytest tests -m gpu -x -q > "$out/gputests.log" 2>&1 || exit 1
for v in "$@"; do
  FHECORE_LIB=$PWD/tools/variants/$v.so timeout -k 10 120 python tools/time_ntt.py 16 64 >> "$out/times.txt" 2>/dev/null || exit 2
done
