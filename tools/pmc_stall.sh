#!/bin/bash
# Where the NTT kernels' wave-cycles go (run ON the GPU box via gpurun): per library build given
# as arguments (default: the in-tree one), one pass of SQ wave-state counters + GRBM cycles and one
# pass of instruction-mix / LDS counters over tools/time_ntt.py.  Summarise with
# tools/pmc_summary.py <out>/<tag>.
# usage: tools/pmc_stall.sh <out> [lib.so ...]   (PMC_CMD overrides the profiled command, e.g.
#        PMC_CMD="bench.py --workload keyswitch --steps 20 --warmup 5 --no-cpu-baseline --no-pmc";
#        a profiled bench.py must get --no-pmc: its own live PMC passes would nest a rocprofv3)
set -o pipefail
cmd=${PMC_CMD:-tools/time_ntt.py 16 64}
out=$1; shift
libs=("$@"); [ ${#libs[@]} -eq 0 ] && libs=("gpu-fhe_amd/lib/libfhecore.so")
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$out"
for lib in "${libs[@]}"; do
  tag=$(basename "$lib" .so)
  export FHECORE_LIB=$GRAFT_REPO_ROOT/$lib
  timeout -k 10 120 python3 $cmd >> "$out/times.txt" 2>/dev/null || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/$tag/trace" -o run --output-format csv -- python3 $cmd > "$out/$tag.trace.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d "$out/$tag/pmc1" -o run --output-format csv -- python3 $cmd > "$out/$tag.pmc1.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS -d "$out/$tag/pmc2" -o run --output-format csv -- python3 $cmd > "$out/$tag.pmc2.log" 2>&1 || exit $?
done
echo done
