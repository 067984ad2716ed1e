set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5d
FHECORE_LIB=$GRAFT_REPO_ROOT/tools/variants/ksrot1.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_keyswitch_batch.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5d/parity_ksrot1.log 2>&1 || exit $?
tail -1 gpurun_out/r5d/parity_ksrot1.log
bash tools/ab_quick.sh gpurun_out/r5d/ab.txt 3 "--warmup 100 --steps 200" rot1 ksrot ksrot1
