#!/bin/bash
# Submit one gpurun call, resubmitting only while gpurun answers 3 (no box or
# slot free: nothing ran, nothing charged), at most 12 times, 3 minutes apart.
# Any other exit status (the command ran, or was refused) ends the loop.
#   tools/gpurun_wait.sh <log> <gpurun args...>
LOG=$1
shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun "$@" > "$LOG" 2>&1
  rc=$?
  echo "exit $rc (try $i)" >> "$LOG"
  [ $rc -ne 3 ] && exit $rc
  sleep 180
done
exit 3
