#!/bin/bash
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status
# BASELINE.json configs C2-C5 at full size on one GPU (dev tool): tools/probe_configs.sh OUTLOG
OUT=$1
for a in "cornell 800 1024" "book1 1200 512" "book2 800 4096" "model 1920 1024"; do
  timeout -k 10 300 python3 tools/gpu_probe.py $a fused || exit $?
done > "$OUT" 2>&1
