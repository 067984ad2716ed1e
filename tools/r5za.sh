set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5za
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_keyswitch_batch.py -q --timeout 120 --timeout-method thread > gpurun_out/r5za/gputests.log 2>&1; rc=$?; tail -1 gpurun_out/r5za/gputests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 900 bash tools/ab_bench.sh gpurun_out/r5za/ab.txt 3 "--workload mulrelin" default base || exit $?
echo done
