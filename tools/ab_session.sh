#!/bin/bash
# One GPU-box A/B session (run ON the box via gpurun): the GPU suite on the in-tree build, then
# same-box alternating bench lines of the in-tree build ("default") against tools/variants/<v>.so
# builds (tools/build_variant.sh; REV=<git rev> builds a committed revision as the baseline).
# usage: tools/ab_session.sh <out> <reps> "<bench args>" <variant...>
set -o pipefail
out=$1; reps=$2; args=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$out"
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gputests.log" 2>&1 || exit $?
tail -n1 "$out/gputests.log"
timeout -k 10 700 bash tools/ab_bench.sh "$out/ab.txt" "$reps" "$args" default "$@" || exit $?
echo "ab session done"
