set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5j
export FHECORE_LIB=$GRAFT_REPO_ROOT/tools/variants/pfirst.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py tests/test_gpu_dist.py -k "keyswitch or chain or dist" -x -q --timeout 120 --timeout-method thread > gpurun_out/r5j/parity_pfirst.log 2>&1 || { tail -20 gpurun_out/r5j/parity_pfirst.log; exit 1; }
tail -1 gpurun_out/r5j/parity_pfirst.log
unset FHECORE_LIB
timeout -k 10 900 bash tools/ab_bench.sh gpurun_out/r5j/ab.txt 4 "--workload keyswitch --warmup 20 --steps 100" default pfirst || exit $?
cat gpurun_out/r5j/ab.txt
