#!/bin/bash
# Collect kernel-trace stats + PMC counter passes for a command (run ON the GPU box via gpurun).
# usage: tools/pmc.sh <outdir> <python args...>   e.g. tools/pmc.sh gpurun_out/pmc bench.py --steps 3
set -o pipefail
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- python3 "$@" > "$out/trace.log" 2>&1 || exit $?
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_THREAD_CYCLES_VALU SQ_LDS_UNALIGNED_STALL"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass -d "$out/pmc$i" -o run --output-format csv -- python3 "$@" > "$out/pmc$i.log" 2>&1 || exit $?
done
echo "pmc done: $out"
