#!/bin/bash
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status
# Library switches read at render time, on the share probe (dev tool):
#   tools/env_grid.sh OUT "scene width spp" "VAR=val[,VAR2=val2]" ...   ("-": no switch)
# e.g. "RT_TAIL_FRAC=4,RT_TAIL_K=2" or "RT_SPLIT_MIN=2".  One JSON line per share
# (tools/share_probe.py), tagged with the combination.
OUT=$1; CFG=$2; shift 2
for combo in "$@"; do
  ( if [ "$combo" != "-" ]; then
      IFS=',' read -r -a kv <<< "$combo"
      for a in "${kv[@]}"; do export "${a?}"; done
    fi
    timeout -k 10 300 python3 tools/share_probe.py $CFG ) | grep '^{' | sed "s/^{/{\"combo\": \"$combo\", /" || exit $?
done > "$OUT" 2>&1
