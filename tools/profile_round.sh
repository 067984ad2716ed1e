#!/bin/bash
# Round profile bundle for the default bench command (run ON the GPU box via gpurun):
#   bench.json         the bench line
#   stats/             rocprofv3 --kernel-trace --stats of the same command
#   fetch/, write/     PMC passes (FETCH_SIZE, WRITE_SIZE), one counter group per pass
set -o pipefail
out=${1:-gpurun_out/round}
shift || true
args="$@"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$out"
timeout -k 10 300 python3 bench.py $args > "$out/bench.json" 2> "$out/bench.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/stats" -o run --output-format csv -- python3 bench.py $args --no-cpu-baseline --no-pmc --no-dist-check > "$out/stats.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o run --output-format csv -- python3 bench.py $args --no-cpu-baseline --no-pmc --no-dist-check > "$out/fetch.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$out/write" -o run --output-format csv -- python3 bench.py $args --no-cpu-baseline --no-pmc --no-dist-check > "$out/write.log" 2>&1 || exit $?
echo "profile bundle: $out"
