#!/bin/bash
# GPU-box session step: GPU tests of the in-tree build, then a same-box A/B of bench lines against
# tools/variants/<name>.so, then a rocprofv3 kernel trace of one workload (idle gaps:
# tools/trace_gaps.py).  usage: tools/ab_run.sh <out> <reps> "<bench args>" "<trace args>" variant...
set -o pipefail
out=$1; reps=$2; args=$3; targs=$4; shift 4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gputests.log" 2>&1 || exit $?
tail -2 "$out/gputests.log"
bash tools/ab_bench.sh "$out/ab.txt" "$reps" "$args" default "$@" || exit $?
cat "$out/ab.txt"
if [ -n "$targs" ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$out/kt" -o kt -- python3 bench.py --no-cpu-baseline --no-pmc $targs > "$out/trace_line.json" 2> "$out/trace.err" || exit $?
  f=$(find "$out/kt" -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_gaps.py "$f" --last 600 > "$out/gaps.txt" && cat "$out/gaps.txt"
fi
echo ab_run done
