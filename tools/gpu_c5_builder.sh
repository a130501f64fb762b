#!/bin/bash
# C5 (model 1920x1080x1024) with the host SAH tree and device PLOC trees of every
# library variant (dev tool): tools/gpu_c5_builder.sh OUT.jsonl
OUT=$1
B=$PWD/go_raytracer_amd
for rep in 1 2; do
  RT_TIMING=1 RT_BVH_BUILDER=host timeout -k 10 300 python3 tools/gpu_probe.py model 1920 1024 fused 2>&1 | sed 's/^{/{"lib": "cur", "builder": "host", /' || exit $?
  for so in "" $B/build_abl/*/librt_amd.so; do
    n=cur; [ -z "$so" ] || n=$(basename "$(dirname "$so")")
    RT_AMD_LIB=$so RT_TIMING=1 RT_BVH_BUILDER=device timeout -k 10 300 python3 tools/gpu_probe.py model 1920 1024 fused 2>&1 | sed "s/^{/{\"lib\": \"$n\", \"builder\": \"device\", /" || exit $?
  done
done > "$OUT" 2>&1
