#!/bin/bash
# HBM traffic passes (FETCH_SIZE / WRITE_SIZE / EA request sizes, each in its own pass) for the
# base and memory-pattern-only (abl1) builds on tools/time_ntt.py.  Run ON the GPU box via gpurun.
set -o pipefail
out=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$out"
i=0
for v in base abl1; do
  for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ" "TCC_EA0_WRREQ TCC_EA0_WRREQ_64B GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    FHECORE_LIB=$PWD/tools/variants/$v.so timeout -k 10 300 rocprofv3 --pmc $ctr -d "$out/$v/p$i" -o run --output-format csv -- python3 tools/time_ntt.py 16 64 > "$out/$v.p$i.log" 2>&1 || exit $?
  done
done
echo done
