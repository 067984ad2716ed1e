set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5v
timeout -k 10 900 bash tools/ab_bench.sh gpurun_out/r5v/ab.txt 3 "--workload vec" default nt512s nt256s nt128s nts512 || exit $?
echo done
