set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5q
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_galois.py tests/test_gpu_pipeline.py tests/test_gpu_keyswitch_batch.py tests/test_gpu_dist.py tests/test_gpu_wide.py -q --timeout 120 --timeout-method thread > gpurun_out/r5q/gputests.log 2>&1; rc=$?; tail -2 gpurun_out/r5q/gputests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 900 bash tools/ab_bench.sh gpurun_out/r5q/ab.txt 3 "--workload keyswitch --warmup 20 --steps 100" default base || exit $?
cat gpurun_out/r5q/ab.txt
timeout -k 10 600 bash tools/ab_bench.sh gpurun_out/r5q/ab_mulrelin.txt 2 "--workload mulrelin" default base || exit $?
