set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5x
timeout -k 10 900 bash tools/ab_bench.sh gpurun_out/r5x/ab.txt 3 "--warmup 5 --steps 20" default hmnts ksnts || exit $?
echo done
