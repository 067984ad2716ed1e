#!/bin/bash
# One gpurun session as a list of named steps, run ON the GPU box in order; each step has its own
# time limit and the session stops at the first failing step (no retries).  Replaces the per-call
# one-off scripts of earlier rounds: the exact step list goes into the profiles/*.txt header of
# whatever a session produced.
# usage: tools/gpu_session.sh <out-dir> <step>...
#   smoke                        __graft_entry__.smoke()                   -> <out>/smoke.log
#   tests                        the whole GPU suite                       -> <out>/gputests.log
#   tests=<path or -k expr>      a test file (path ending in .py) or a -k selection of the suite
#   line:<tag>[=<bench args>]    one bench.py line                         -> <out>/bench_<tag>.json
#   ab:<tag>=<reps>|<bench args>|<variant> ...   same-box A/B (tools/ab_bench.sh) -> <out>/ab_<tag>.txt
#   bundle=A|B|R                 tools/round_bundle.sh part                -> <out>/
#   prof:<tag>[=<bench args>]    tools/profile_round.sh of a bench command -> <out>/<tag>/
#   py:<tag>=<script and args>   any python3 tool (e.g. tools/shard_shape.py --hybrid) -> <out>/<tag>.out
#   gloo:<tag>=<ranks>|<bench args>  bench.py with <ranks> gloo ranks on this one GPU (the rehearsal
#                                of the driver's multi-GPU launch)            -> <out>/gloo_<tag>.json
# example: tools/gpu_session.sh gpurun_out/s1 smoke tests "line:w5=--warmup 5 --steps 20"
set -o pipefail
out=${1:?out dir}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$out"
for step in "$@"; do
  name=${step%%=*}; arg=""; [ "$name" != "$step" ] && arg=${step#*=}
  echo "== $step"
  case $name in
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > "$out/smoke.log" 2>&1 || exit $?
      tail -n1 "$out/smoke.log" ;;
    tests)
      if [ -z "$arg" ]; then sel=(tests -m gpu); log=gputests
      elif [[ $arg == *.py* ]]; then sel=($arg); log=tests_$(basename "${arg%%.py*}")
      else sel=(tests -m gpu -k "$arg"); log=tests_k; fi
      timeout -k 10 600 python3 -u -m pytest "${sel[@]}" -x -q --timeout 120 --timeout-method thread \
        > "$out/$log.log" 2>&1 || { tail -n30 "$out/$log.log"; exit 1; }
      tail -n1 "$out/$log.log" ;;
    line:*)
      tag=${name#line:}
      timeout -k 10 400 python3 bench.py $arg > "$out/bench_$tag.json" 2> "$out/bench_$tag.err" \
        || { tail -n20 "$out/bench_$tag.err"; exit 1; }
      cut -c1-400 "$out/bench_$tag.json" ;;
    ab:*)
      tag=${name#ab:}; IFS='|' read -r reps args variants <<< "$arg"
      timeout -k 10 1000 bash tools/ab_bench.sh "$out/ab_$tag.txt" "$reps" "$args" default $variants \
        || exit $?
      cat "$out/ab_$tag.txt" ;;
    bundle)
      bash tools/round_bundle.sh "$out" "$arg" || exit $? ;;
    py:*)
      tag=${name#py:}
      timeout -k 10 600 python3 $arg > "$out/$tag.out" 2> "$out/$tag.err" || { tail -n20 "$out/$tag.err"; exit 1; }
      tail -n5 "$out/$tag.out" ;;
    gloo:*)
      tag=${name#gloo:}; IFS='|' read -r nr bargs <<< "$arg"
      FHE_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 \
        --nproc-per-node "$nr" --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus "$nr" \
        $bargs > "$out/gloo_$tag.json" 2> "$out/gloo_$tag.err" || { tail -n20 "$out/gloo_$tag.err"; exit 1; }
      cut -c1-400 "$out/gloo_$tag.json" ;;
    prof:*)
      bash tools/profile_round.sh "$out/${name#prof:}" $arg || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session done"
