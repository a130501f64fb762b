#!/bin/bash
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status
# Alternate several libraries on one config (dev tool):
#   tools/ab_libs3.sh OUTLOG REPS "scene width spp" name=path/librt_amd.so ...
# ("cur" = the in-tree library).  One gpu_probe.py run per (rep, lib), appended as JSON lines.
OUT=$1; REPS=$2; CFG=$3; shift 3
for rep in $(seq "$REPS"); do
  for spec in "$@"; do
    name=${spec%%=*}; lib=${spec#*=}
    if [ "$lib" = cur ]; then
      timeout -k 10 300 python3 tools/gpu_probe.py $CFG fused > /tmp/ab_one.json || exit $?
    else
      RT_AMD_LIB=$PWD/$lib timeout -k 10 300 python3 tools/gpu_probe.py $CFG fused > /tmp/ab_one.json || exit $?
    fi
    sed "s/^{/{\"lib\": \"$name\", /" /tmp/ab_one.json >> "$OUT"
  done
done
