#!/bin/bash
# PMC A/B of tools/variants/<name>.so builds on tools/time_ntt.py (run ON the GPU box via gpurun).
# usage: tools/pmc_ab.sh outdir "counters" variant...
set -o pipefail
out=$1; ctr=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$out"
for v in "$@"; do
  FHECORE_LIB=$PWD/tools/variants/$v.so timeout -k 10 300 rocprofv3 --pmc $ctr -d "$out/$v" -o run --output-format csv -- python3 tools/time_ntt.py 16 64 > "$out/$v.log" 2>&1 || exit $?
done
echo done
