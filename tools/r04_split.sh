#!/bin/bash
# Round-4 session: the GPU suite on the in-tree build, then same-box A/B of the default line
# against tools/variants/<name>.so.  usage: tools/r04_split.sh <out> <variants...>
set -o pipefail
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$out"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gputests.log" 2>&1 || exit $?
tail -n1 "$out/gputests.log"
timeout -k 10 600 bash tools/ab_bench.sh "$out/ab_hm.txt" 4 "--no-keyswitch-leg --no-dist-check" default "$@" || exit $?
echo split done
