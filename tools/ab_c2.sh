#!/bin/bash
# C2 timing A/B over library variants, alternating (dev tool): tools/ab_c2.sh OUT
OUT=$1
B=$PWD/go_raytracer_amd
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/gpu_probe.py cornell 800 1024 fused | sed 's/^{/{"lib": "cur", /' || exit $?
  RT_AMD_LIB=$B/build_prev/librt_amd.so timeout -k 10 120 python3 tools/gpu_probe.py cornell 800 1024 fused | sed 's/^{/{"lib": "prev", /' || exit $?
  for v in $B/build_abl/*/librt_amd.so; do
    n=$(basename $(dirname $v))
    RT_AMD_LIB=$v timeout -k 10 120 python3 tools/gpu_probe.py cornell 800 1024 fused | sed "s/^{/{\"lib\": \"$n\", /" || exit $?
  done
done > "$OUT" 2>&1
