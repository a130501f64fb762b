#!/bin/bash
# Timing probe over the demo scenes (dev tool): tools/probe_all.sh OUTLOG [mode]
OUT=$1; MODE=${2:-fused}
for a in "cornell 800 256" "cornell_smoke 600 64" "book1 600 64" "book2 400 256" "book3 600 64" "model:512x64 400 64"; do
  timeout -k 10 180 python3 tools/gpu_probe.py $a $MODE || exit $?
done > "$OUT" 2>&1
