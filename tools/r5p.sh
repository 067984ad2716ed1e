set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5p
bash tools/ab_bench.sh gpurun_out/r5p/ab.txt 3 "--warmup 5 --steps 20" default r4 || exit $?
bash tools/ab_bench.sh gpurun_out/r5p/ab_mulrelin.txt 2 "--workload mulrelin" default r4 || exit $?
echo done
