set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5a
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5a/gputests.log 2>&1 || exit $?
tail -n1 gpurun_out/r5a/gputests.log
timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 --no-pmc > gpurun_out/r5a/bench_w5.json 2> gpurun_out/r5a/bench_w5.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5a/ks -o run --output-format csv -- python3 bench.py --workload keyswitch --no-cpu-baseline --no-dist-check --no-pmc > gpurun_out/r5a/ks.json 2> gpurun_out/r5a/ks.err || exit $?
echo done
