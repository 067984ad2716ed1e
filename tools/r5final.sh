set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5f3
bash tools/round_bundle.sh gpurun_out/r5f3 A || exit $?
bash tools/round_bundle.sh gpurun_out/r5f3 B || exit $?
echo final bundle done
