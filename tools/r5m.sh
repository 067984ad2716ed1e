set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5m
for i in 1 2; do
  FHECORE_LIB=$GRAFT_REPO_ROOT/tools/variants/base.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_galois.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5m/galois_base_$i.log 2>&1; echo "base run $i rc=$?"; tail -1 gpurun_out/r5m/galois_base_$i.log
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_galois.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5m/galois_new.log 2>&1; echo "new galois rc=$?"; tail -1 gpurun_out/r5m/galois_new.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5m/gputests_new.log 2>&1; echo "new suite rc=$?"; tail -3 gpurun_out/r5m/gputests_new.log
