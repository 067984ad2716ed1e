#!/bin/bash
# Round-3 evidence bundle (run ON the GPU box): the default bench line with the driver's arguments
# and with the defaults, rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes of the default
# command, and the key-switch VALU counters (tools/valu_roofline.py input).  usage: <out>
set -o pipefail
out=${1:-gpurun_out/r03b}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$out"
timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 > "$out/bench_w5.json" 2> "$out/bench_w5.err" || exit $?
bash tools/profile_round.sh "$out/hm" || exit $?
PMC_CMD="bench.py --workload keyswitch --steps 20 --warmup 5 --no-cpu-baseline" bash tools/pmc_stall.sh "$out/kspmc" || exit $?
for w in keyswitch ntt "ntt-batch --steps 5 --warmup 2"; do
  tag=$(echo $w | cut -d' ' -f1 | tr -d '-')
  timeout -k 10 300 python3 bench.py --workload $w > "$out/bench_$tag.json" 2> "$out/bench_$tag.err" || exit $?
done
echo bundle done
