#!/bin/bash
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status
# A/B the in-tree library against go_raytracer_amd/build_prev on the full-size
# configs, alternating, in one box (dev tool): tools/ab_configs.sh OUTLOG
OUT=$1
PREV=$PWD/go_raytracer_amd/build_prev/librt_amd.so
for a in "book1 1200 512" "book2 800 2048" "model 1920 512" "cornell 800 1024"; do
  for rep in 1 2; do
    RT_AMD_LIB=$PREV timeout -k 10 300 python3 tools/gpu_probe.py $a fused | sed 's/^{/{"lib": "prev", /' || exit $?
    timeout -k 10 300 python3 tools/gpu_probe.py $a fused | sed 's/^{/{"lib": "cur", /' || exit $?
  done
done > "$OUT" 2>&1
