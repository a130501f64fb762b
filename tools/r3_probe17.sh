#!/bin/bash
# round-3 probe: 2-prim leaves with the paired record fetch (RT_LEAF_PAIR build):
#   C5 (model, PLOC): RT_PLOC_PAIR=1 merges sibling leaves into one BVH4 leaf
#   C4 (book2, host SAH): RT_BVH_LEAF=2
# against the default single-prim trees; timing only (the trees differ)
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2; do
  timeout -k 10 200 python3 tools/gpu_probe.py model 960 512 fused | sed 's/^{/{"lib": "cur", /' || exit 1
  RT_AMD_LIB=$L/pair2/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py model 960 512 fused | sed 's/^{/{"lib": "pair2", /' || exit 1
  RT_PLOC_PAIR=1 RT_AMD_LIB=$L/pair2/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py model 960 512 fused | sed 's/^{/{"lib": "pair2_ploc", /' || exit 1
  timeout -k 10 200 python3 tools/gpu_probe.py book2 400 1024 fused | sed 's/^{/{"lib": "cur", /' || exit 1
  RT_BVH_LEAF=2 RT_AMD_LIB=$L/pair2/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py book2 400 1024 fused | sed 's/^{/{"lib": "pair2_leaf2", /' || exit 1
done > $O/ab_pair.jsonl
