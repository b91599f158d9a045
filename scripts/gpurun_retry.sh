#!/bin/bash
# Re-submit a gpurun call ONLY when no box could be acquired (exit 3: nothing ran, nothing
# charged).  Any other outcome -- including a failing command -- is returned as is.
# usage: scripts/gpurun_retry.sh <log> <timeout_s> '<command>'
log=$1; t=$2; shift 2
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then echo "exit $rc" >> "$log"; exit $rc; fi
  echo "[retry $i: no box]" >> "$log.retries"
  sleep 60
done
echo "exit 3" >> "$log"
