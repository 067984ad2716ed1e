#!/bin/bash
# Every bench line of a round (with its cpu_baseline) plus the rocprofv3 / PMC bundle of the
# headline and key-switch commands (run ON the GPU box via gpurun).  usage: tools/round_bundle.sh <out>
set -o pipefail
out=${1:-gpurun_out/bundle}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$out"
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gputests.log" 2>&1 || exit $?
bash tools/profile_round.sh "$out/hm" || exit $?
for w in "keyswitch" "ntt" "vec" "mulrelin" "ntt-batch --steps 5 --warmup 2" "hommult --bits 62" "hommult --bits 63"; do
  tag=$(echo $w | cut -d' ' -f1-3 | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python3 bench.py --workload $w > "$out/bench_$tag.json" 2> "$out/bench_$tag.err" || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/ks/stats" -o run --output-format csv -- python3 bench.py --workload keyswitch --no-cpu-baseline > "$out/ks.json" 2> "$out/ks.err" || exit $?
echo bundle done
