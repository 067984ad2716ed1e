#!/bin/bash
# Same-box A/B of bench.py lines: alternate the in-tree build ("default") with variants in
# tools/variants/<name>.so (+ tools/variants/peak_<name>.so for the ALU ceiling, when present).
# usage: tools/ab_bench.sh outfile reps "bench args" name...
out=$1; reps=$2; args=$3; shift 3
for r in $(seq $reps); do
  for v in "$@"; do
    if [ "$v" = default ]; then unset FHECORE_LIB FHE_PEAK_LIB; else
      export FHECORE_LIB=$PWD/tools/variants/$v.so
      if [ -f tools/variants/peak_$v.so ]; then export FHE_PEAK_LIB=$PWD/tools/variants/peak_$v.so; else unset FHE_PEAK_LIB; fi
    fi
    line=$(timeout -k 10 150 python3 bench.py --no-cpu-baseline --no-pmc $args 2>/dev/null) || exit 1
    echo "$v $(echo "$line" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); a=d.get("roofline_alu") or {}; k=d.get("keyswitch_leg") or {}; print(d["value"], d.get("ntt_per_sec"), k.get("value"), d.get("kernel_ms"), d.get("ntt_kernel_ms"), k.get("kernel_ms"), a.get("peak_source","")[-40:])')" >> $out
  done
done
