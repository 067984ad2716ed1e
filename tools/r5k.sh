set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5k
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5k/gputests.log 2>&1 || { tail -30 gpurun_out/r5k/gputests.log; exit 1; }
tail -1 gpurun_out/r5k/gputests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5k/smoke.log 2>&1 || { tail -20 gpurun_out/r5k/smoke.log; exit 1; }
tail -1 gpurun_out/r5k/smoke.log
bash tools/round_bundle.sh gpurun_out/r5k R || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/r5k/rehearsal_2rank.json').read().strip().splitlines()[-1]); print(d['value'], d['dist_check'])"
