#!/bin/bash
# Runs one GPU step under its own time limit; stops the whole call on a fault,
# abort, segfault or timeout (exit >= 124), but lets ordinary test failures
# (exit 1/2) through so later measurement steps still run.
#   tools/gpu_step.sh <seconds> <log> <cmd...>
secs=$1; log=$2; shift 2
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc: $*" >> "$log"
tail -n 5 "$log"
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
  echo "[gpu_step] fatal rc=$rc, stopping" ; exit $rc
fi
exit 0
