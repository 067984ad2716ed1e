set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5o
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_galois.py tests/test_gpu_pipeline.py tests/test_gpu_keyswitch_batch.py tests/test_gpu_dist.py tests/test_gpu_wide.py -q --timeout 120 --timeout-method thread > gpurun_out/r5o/gputests.log 2>&1; rc=$?; tail -2 gpurun_out/r5o/gputests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 900 bash tools/ab_bench.sh gpurun_out/r5o/ab.txt 3 "--workload keyswitch --warmup 20 --steps 100" default base || exit $?
cat gpurun_out/r5o/ab.txt
