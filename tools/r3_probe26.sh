#!/bin/bash
# round-3 probe: the mesh kernel's (C5) traversal short stack with the spare LDS of its
# 4-wave budget (TRI_SHORT x TRI_WLDS: 16 x 4 now; 20 x 4, 22 x 4, 28 x 2)
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2 3; do
  for s in "model 960 512"; do
    timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "cur", /' || exit 1
    for v in t20w4 t22w4 t28w2; do
      RT_AMD_LIB=$L/$v/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed "s/^{/{\"lib\": \"$v\", /" || exit 1
    done
  done
done > $O/ab_tri_stack.jsonl
