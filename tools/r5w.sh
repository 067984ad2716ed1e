set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5w
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5w/gputests.log 2>&1 || exit $?
tail -1 gpurun_out/r5w/gputests.log
timeout -k 10 300 python3 bench.py --workload vec > gpurun_out/r5w/bench_vec.json 2> gpurun_out/r5w/bench_vec.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5w/vec_stats -o run --output-format csv -- python3 bench.py --workload vec --no-cpu-baseline --no-pmc > gpurun_out/r5w/vec_prof.json 2> gpurun_out/r5w/vec_prof.err || exit $?
echo done
