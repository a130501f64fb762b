#!/bin/bash
# C4/C5 ablation timings (dev tool): tools/ablate_c4.sh OUT
OUT=$1
for rep in 1 2; do
  for so in go_raytracer_amd/build_abl/*/librt_amd.so; do
    n=$(basename $(dirname $so))
    for a in "book2 800 1024" "model 1920 256"; do
      RT_AMD_LIB=$PWD/$so timeout -k 10 300 python3 tools/gpu_probe.py $a fused | sed "s/^{/{\"lib\": \"$n\", /" | cut -c1-120 || exit $?
    done
  done
done > "$OUT" 2>&1
