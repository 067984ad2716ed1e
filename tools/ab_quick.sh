#!/bin/bash
# Same-box A/B without the GPU suite (run ON the box via gpurun): alternating bench lines of the
# in-tree build ("default") and tools/variants/<v>.so.  usage: tools/ab_quick.sh <out> <reps> "<bench args>" <variant...>
set -o pipefail
out=$1; reps=$2; args=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$(dirname "$out")"
timeout -k 10 900 bash tools/ab_bench.sh "$out" "$reps" "$args" default "$@" || exit $?
cat "$out"
echo "ab done"
