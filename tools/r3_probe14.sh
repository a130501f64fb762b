#!/bin/bash
# round-3 probe: C3 kernel at 2 / 3 waves per SIMD (build_abl/mesh{2,3}: the BVH4 nodes
# then fit the LDS scene cache) vs in-tree (4 waves, tree through L1/L2)
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2 3; do
  timeout -k 10 200 python3 tools/gpu_probe.py book1 1200 512 fused | sed 's/^{/{"lib": "cur", /' || exit 1
  for v in mesh2 mesh3; do
    RT_AMD_LIB=$L/$v/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py book1 1200 512 fused | sed "s/^{/{\"lib\": \"$v\", /" || exit 1
  done
done > $O/ab_c3_lds.jsonl
