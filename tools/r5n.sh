set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5n
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5n/gputests.log 2>&1; rc=$?; tail -3 gpurun_out/r5n/gputests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 900 bash tools/ab_bench.sh gpurun_out/r5n/ab.txt 3 "--workload keyswitch --warmup 20 --steps 100" default base || exit $?
cat gpurun_out/r5n/ab.txt
timeout -k 10 600 bash tools/ab_bench.sh gpurun_out/r5n/ab_mr.txt 2 "--workload mulrelin --warmup 10 --steps 50" default base || exit $?
cat gpurun_out/r5n/ab_mr.txt
