#!/bin/bash
# Key-switch VALU counters of the in-tree build (tools/valu_roofline.py input), then the key-switch
# bench line that reads them.  usage: tools/kspmc.sh <out>
set -o pipefail
out=${1:-gpurun_out/kspmc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$out"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1 || exit $?
tail -1 "$out/tests.log"
PMC_CMD="bench.py --workload keyswitch --steps 20 --warmup 5 --no-cpu-baseline --no-dist-check --no-pmc" bash tools/pmc_stall.sh "$out/kspmc" || exit $?
echo kspmc done
