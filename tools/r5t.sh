set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5t
timeout -k 10 900 bash tools/ab_bench.sh gpurun_out/r5t/ab.txt 3 "--workload vec" default ntl t512 t128 ntl512 || exit $?
echo done
