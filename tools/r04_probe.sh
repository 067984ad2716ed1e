#!/bin/bash
# One GPU-box session of round-4 measurements: the GPU suite on the candidate build, same-box A/B
# lines against the in-tree build, the key-switch stream-split probe and the rank-shape model.
# usage: tools/r04_probe.sh <out> <candidate variant> <other variants...>
set -o pipefail
out=$1; cand=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$out"
FHECORE_LIB=$PWD/tools/variants/$cand.so timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gputests.log" 2>&1 || exit $?
tail -1 "$out/gputests.log"
timeout -k 10 400 bash tools/ab_bench.sh "$out/ab_hm.txt" 3 "--no-keyswitch-leg" default "$cand" || exit $?
timeout -k 10 400 bash tools/ab_bench.sh "$out/ab_ks.txt" 3 "--workload keyswitch" default "$cand" "$@" || exit $?
timeout -k 10 300 python3 -u tools/ks_stream_probe.py > "$out/ks_streams.json" 2> "$out/ks_streams.err" || exit $?
timeout -k 10 500 python3 -u tools/shard_shape.py > "$out/shard_shape.json" 2> "$out/shard_shape.err" || exit $?
echo probe done
