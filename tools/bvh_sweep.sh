#!/bin/bash
# SAH parameter sweep (dev tool): tools/bvh_sweep.sh OUTLOG "scene width spp" ["scene width spp" ...]
OUT=$1; shift
for sc in "$@"; do
  for cfg in "4 1 1" "2 1 1" "1 1 1" "4 1.5 1" "2 1.5 1" "4 2 1" "8 1 1" "4 1 2"; do
    read L CT CI <<< "$cfg"
    RT_BVH_LEAF=$L RT_BVH_CT=$CT RT_BVH_CI=$CI timeout -k 10 300 python3 tools/gpu_probe.py $sc fused \
      | sed "s/^{/{\"leaf\": $L, \"ct\": $CT, \"ci\": $CI, /" || exit $?
  done
done > "$OUT" 2>&1
