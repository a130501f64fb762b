#!/bin/bash
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status
# One GPU session from a list of steps (dev tool): tools/session.sh TAG 'cmd1' 'cmd2' ...
# Each step runs under its own time limit (prefix it with `timeout -k 10 N`), its stdout and
# stderr go to gpurun_out/TAG_<i>.log.  Exit status 1 (a failed assertion, a non-zero
# script result) lets the session go on; anything else (a time limit 124/137, an abort 134,
# a segfault 139, a fault) ends it there, so no further GPU work runs after trouble.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 1
TAG=$1; shift
i=0
for step in "$@"; do
  i=$((i + 1))
  echo "== [$i] $step $(date +%T)"
  bash -c "$step" > "$O/${TAG}_$i.log" 2>&1
  rc=$?
  echo "== [$i] rc=$rc $(date +%T)"
  tail -3 "$O/${TAG}_$i.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 127 ]; then exit $rc; fi
done
