#!/bin/bash
# A/B: register budget (waves/SIMD) and fast div/sqrt build on a few configs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for lib in "" "$R/go_raytracer_amd/build_fast/librt_amd_fast.so"; do
for w in 2 3; do
  for cfg in "cornell 800 256" "book2 800 16" "book1 1200 36" "model:512x64 960 16"; do
    RT_AMD_LIB=$lib RT_FUSED_WAVES=$w timeout -k 10 200 python3 tools/gpu_probe.py $cfg fused | sed "s/^/lib=${lib:+fast} waves=$w /" || exit 1
  done
done
done
