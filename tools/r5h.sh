set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5h
FHECORE_LIB=$GRAFT_REPO_ROOT/tools/variants/mdpre.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "keyswitch" -x -q --timeout 120 --timeout-method thread > gpurun_out/r5h/parity_mdpre.log 2>&1 || { tail -20 gpurun_out/r5h/parity_mdpre.log; exit 1; }
tail -1 gpurun_out/r5h/parity_mdpre.log
timeout -k 10 900 bash tools/ab_bench.sh gpurun_out/r5h/ab.txt 3 "--workload keyswitch --warmup 20 --steps 100" default mdpre || exit $?
cat gpurun_out/r5h/ab.txt
