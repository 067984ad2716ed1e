set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5i
for v in default tg2; do
  if [ $v = default ]; then unset FHECORE_LIB; else export FHECORE_LIB=$GRAFT_REPO_ROOT/tools/variants/$v.so; fi
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py tests/test_gpu_dist.py -k "keyswitch or chain or dist" -x -q --timeout 120 --timeout-method thread > gpurun_out/r5i/parity_$v.log 2>&1 || { tail -20 gpurun_out/r5i/parity_$v.log; exit 1; }
  tail -1 gpurun_out/r5i/parity_$v.log
done
unset FHECORE_LIB
timeout -k 10 900 bash tools/ab_bench.sh gpurun_out/r5i/ab.txt 3 "--workload keyswitch --warmup 20 --steps 100" default base tg2 || exit $?
cat gpurun_out/r5i/ab.txt
