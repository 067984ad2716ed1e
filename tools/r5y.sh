set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5y
timeout -k 10 900 bash tools/ab_bench.sh gpurun_out/r5y/ab.txt 2 "--workload ntt-batch --steps 5 --warmup 2" default st15 st9 st6 st8 || exit $?
echo done
