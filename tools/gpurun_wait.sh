#!/bin/bash
# Submits one gpurun call, resubmitting only while the pool has no box for it (gpurun's transient
# "no free box" / infrastructure answers, where nothing ran and nothing was charged).  A call that
# ran -- whatever its exit status -- is never resubmitted.  usage: tools/gpurun_wait.sh <log> <timeout> <command>
log=$1; to=$2; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|backing off\|stopped responding while being prepared\|taken away by the GPU service" "$log" && ! grep -q "status=ok\|status=fail" "$log"; then
    sleep 90; continue
  fi
  exit $rc
done
exit 3
