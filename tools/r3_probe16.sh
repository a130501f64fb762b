#!/bin/bash
# round-3 probe: 2-prim leaves with a paired record fetch (RT_LEAF_PAIR) on C4 (host SAH,
# RT_BVH_LEAF=2) against the single-prim default; timing only (images are identical in
# distribution, not bitwise: the tree differs)
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2; do
  timeout -k 10 200 python3 tools/gpu_probe.py model 960 512 fused | sed 's/^{/{"lib": "cur_leaf1", /' || exit 1
  RT_BVH_LEAF=2 timeout -k 10 200 python3 tools/gpu_probe.py model 960 512 fused | sed 's/^{/{"lib": "cur_leaf2", /' || exit 1
  RT_BVH_LEAF=2 RT_AMD_LIB=$L/leafpair/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py model 960 512 fused | sed 's/^{/{"lib": "pair_leaf2", /' || exit 1
  RT_AMD_LIB=$L/leafpair/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py model 960 512 fused | sed 's/^{/{"lib": "pair_leaf1", /' || exit 1
done > $O/ab_c4_leafpair.jsonl
