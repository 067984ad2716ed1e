#!/bin/bash
# A round's evidence on the GPU box, in two sessions that each fit one gpurun call:
#   A: the GPU suite, the default line at the driver's arguments (--warmup 5 --steps 20), and the
#      rocprofv3 bundle of the default command (tools/profile_round.sh: line, kernel-trace stats,
#      FETCH_SIZE and WRITE_SIZE passes);
#   B: every other workload's line (with its cpu_baseline), the key-switch kernel-trace stats and
#      its SQ_INSTS_VALU passes (tools/kspmc.sh; summarise with tools/valu_roofline.py);
#   R: the 2-rank rehearsal of the driver's multi-GPU launch on the box's one GPU (gloo: RCCL
#      refuses two ranks on one device), with its dist_check.
# usage: tools/round_bundle.sh <out> A|B|R
set -o pipefail
out=${1:-gpurun_out/bundle}; part=${2:-A}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$out"
if [ "$part" = A ]; then
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gputests.log" 2>&1 || exit $?
  tail -n1 "$out/gputests.log"
  timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 > "$out/bench_w5.json" 2> "$out/bench_w5.err" || exit $?
  bash tools/profile_round.sh "$out/hm" || exit $?
elif [ "$part" = R ]; then
  FHE_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --warmup 5 --steps 20 \
    > "$out/rehearsal_2rank.json" 2> "$out/rehearsal_2rank.err" || exit $?
else
  for w in "keyswitch" "ntt" "vec" "mulrelin" "rotate" "ntt-batch --steps 5 --warmup 2"; do
    tag=$(echo $w | cut -d' ' -f1 | tr -d '-')
    timeout -k 10 300 python3 bench.py --workload $w > "$out/bench_$tag.json" 2> "$out/bench_$tag.err" || exit $?
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/ks/stats" -o run --output-format csv -- python3 bench.py --workload keyswitch --no-cpu-baseline --no-dist-check --no-pmc > "$out/ks.json" 2> "$out/ks.err" || exit $?
  bash tools/kspmc.sh "$out/k" || exit $?
fi
echo "bundle $part done"
