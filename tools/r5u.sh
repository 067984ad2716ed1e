set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5u
timeout -k 10 900 bash tools/ab_bench.sh gpurun_out/r5u/ab.txt 3 "--workload vec" default ntl512 ntl1024 nt512s ntl128 || exit $?
echo done
