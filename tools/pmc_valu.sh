#!/bin/bash
# VALUBusy / VALUUtilization for the NTT kernels and the register-only butterfly microbenchmark.
set -o pipefail
out=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$out"
timeout -k 10 300 rocprofv3 --pmc VALUBusy VALUUtilization -d "$out/ntt" -o run --output-format csv -- python3 tools/time_ntt.py 16 64 > "$out/ntt.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc VALUBusy VALUUtilization -d "$out/bfly" -o run --output-format csv -- ./tools/microbench/bfly_rate > "$out/bfly.log" 2>&1 || exit $?
echo done
