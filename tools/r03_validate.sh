#!/bin/bash
# Round-3 validation on the GPU box: GPU tests, then the default bench line (driver's arguments)
# and the other workloads' lines with their CPU baselines.  usage: tools/r03_validate.sh <out>
set -o pipefail
out=${1:-gpurun_out/r03v}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/gputests.log" 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 > "$out/bench_w5.json" 2> "$out/bench_w5.err" || exit $?
for w in vec mulrelin rotate keyswitch; do
  timeout -k 10 300 python3 bench.py --workload $w --cpu-seconds 4 > "$out/bench_$w.json" 2> "$out/bench_$w.err" || exit $?
done
echo validate done
