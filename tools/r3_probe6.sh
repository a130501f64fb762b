#!/bin/bash
# round-3 probe: traversal-stack culling (entry distances on the stack) -- in-tree
# (mesh sets, 8 LDS entries) vs build_abl/{nocull, cull12, cullall}, alternated
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2; do
  for s in "model 1920 512" "book1 1200 512" "book2 800 1024"; do
    timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "cur", /' || exit 1
    for v in nocull cull12 cullall; do
      RT_AMD_LIB=$L/$v/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed "s/^{/{\"lib\": \"$v\", /" || exit 1
    done
  done
done > $O/ab_cull.jsonl
