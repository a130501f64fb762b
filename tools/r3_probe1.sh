#!/bin/bash
# round-3 probe: BVH8 vs BVH4 phase profiles (model, book2) and C4 weight-stack pushes
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for v in 0 1; do
  for s in "model 960 256" "book2 400 1024"; do
    RT_BVH8=$v RT_AMD_LIB=$L/phases/librt_amd.so timeout -k 10 200 python3 tools/phase_probe.py $s | sed "s/^{/{\"bvh8\": $v, /" || exit 1
  done
done > $O/phases_bvh8.jsonl
for lib in pushes hbmpushes; do
  RT_AMD_LIB=$L/$lib/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py book2 400 1024 fused | sed "s/^{/{\"lib\": \"$lib\", /" || exit 1
done > $O/pushes_c4.jsonl
