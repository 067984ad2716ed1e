set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5g
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5g/gputests.log 2>&1 || { tail -30 gpurun_out/r5g/gputests.log; exit 1; }
tail -1 gpurun_out/r5g/gputests.log
timeout -k 10 900 bash tools/ab_bench.sh gpurun_out/r5g/ab.txt 3 "--workload keyswitch --warmup 20 --steps 100" default base || exit $?
cat gpurun_out/r5g/ab.txt
