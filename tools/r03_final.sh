#!/bin/bash
# Round-3 closing runs on the GPU box: the key-switch line (its roofline_valu reads the committed
# profiles/r03_keyswitch_pmc.json at the same batch) and a 2-rank gloo rehearsal of the default line
# on the one GPU.  usage: tools/r03_final.sh <out>
set -o pipefail
out=${1:-gpurun_out/r03f}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$out"
timeout -k 10 300 python3 bench.py --workload keyswitch > "$out/bench_keyswitch.json" 2> "$out/bench_keyswitch.err" || exit $?
FHE_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 \
  > "$out/rehearsal_2rank.json" 2> "$out/rehearsal_2rank.err" || exit $?
echo final done
