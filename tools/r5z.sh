set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5z
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5z/gputests.log 2>&1 || exit $?
tail -1 gpurun_out/r5z/gputests.log
timeout -k 10 300 python3 bench.py --workload ntt-batch --steps 5 --warmup 2 > gpurun_out/r5z/bench_nttbatch.json 2> gpurun_out/r5z/bench_nttbatch.err || exit $?
timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 > gpurun_out/r5z/bench_w5.json 2> gpurun_out/r5z/bench_w5.err || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5z/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r5z/smoke.log
echo done
