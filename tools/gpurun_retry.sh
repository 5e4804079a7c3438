#!/bin/bash
# gpurun, asked again only while the pool has no box or slot free (exit 3:
# nothing ran, nothing charged).  Any other exit -- success, a failing
# command, a refusal -- ends it.  usage: tools/gpurun_retry.sh <log> <timeout> <command>
LOG=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep 120
done
echo "rc=$rc" >> "$LOG"
