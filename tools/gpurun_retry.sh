#!/bin/bash
# Submits one gpurun call; re-submits only while gpurun reports that NOTHING ran (no free box /
# slot, a push that never reached a box: "status=transient", nothing charged), up to 8 tries.
# A call that ran -- whatever its exit status -- is never repeated.
# usage: bash tools/gpurun_retry.sh <log> <timeout> <command>
LOG=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" && grep -Eq "charged=(0.0s|Nones)" "$LOG"; then sleep 150; continue; fi
  exit $rc
done
exit 3
