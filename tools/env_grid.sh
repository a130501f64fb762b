#!/bin/bash
# Tail-phase parameter grid on the share probe (dev tool):
#   tools/tail_grid.sh OUT "scene width spp" "tf,tk[,need]" ...
# tf/tk = RT_TAIL_FRAC / RT_TAIL_K ("-" leaves the default), need = RT_CHUNK_NEED.
# One JSON line per share (tools/share_probe.py), tagged with the combination.
OUT=$1; CFG=$2; shift 2
for combo in "$@"; do
  IFS=',' read -r tf tk need <<< "$combo"
  ( [ "$tf" != "-" ] && export RT_TAIL_FRAC=$tf
    [ "$tk" != "-" ] && [ -n "$tk" ] && export RT_TAIL_K=$tk
    [ -n "$need" ] && export RT_CHUNK_NEED=$need
    timeout -k 10 300 python3 tools/share_probe.py $CFG ) | grep '^{' | sed "s/^{/{\"combo\": \"$combo\", /" || exit $?
done > "$OUT" 2>&1
