set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5zd
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5zd/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r5zd/smoke.log
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5zd/gputests.log 2>&1 || exit $?
tail -1 gpurun_out/r5zd/gputests.log
timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 > gpurun_out/r5zd/bench_w5.json 2> gpurun_out/r5zd/bench_w5.err || exit $?
echo done
