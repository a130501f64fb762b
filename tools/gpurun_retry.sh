#!/bin/bash
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status
# Client-side wrapper (dev tool): run one gpurun call, and call again only when gpurun
# reports that no box was taken (exit 3: no free box, or an infrastructure failure before
# the command ran; nothing ran and nothing was charged).  Any other exit status, including
# a failed or killed command on the box, is returned as is.
#   tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for attempt in 1 2 3 4 5 6 7 8 9 10 11 12; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  echo "attempt $attempt rc=$rc" >> "$LOG.attempts"
  [ $rc -eq 3 ] || exit $rc
  sleep 120
done
exit 3
