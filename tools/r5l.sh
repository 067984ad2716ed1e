set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5l
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5l/gputests.log 2>&1 || { tail -30 gpurun_out/r5l/gputests.log; exit 1; }
tail -1 gpurun_out/r5l/gputests.log
timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 > gpurun_out/r5l/bench_w5.json 2> gpurun_out/r5l/bench_w5.err || { tail -20 gpurun_out/r5l/bench_w5.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r5l/bench_w5.json').read().strip().splitlines()[-1]); print(d['value'], d.get('roofline_valu'))"
