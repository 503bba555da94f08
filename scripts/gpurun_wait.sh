#!/bin/bash
# gpurun, re-queued only while the pool has no free box (exit 3: nothing ran,
# nothing charged); any other outcome is returned as is.
# usage: scripts/gpurun_wait.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && ! grep -q "backing off" "$LOG" && exit $rc
  sleep 150
done
exit $rc
