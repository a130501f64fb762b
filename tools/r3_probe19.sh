#!/bin/bash
# round-3 probe: the BVH4 node step's last three loads in a block of their own
# (RT_NODE_LOADS_APART; pair2 = RT_LEAF_PAIR, measured -0.9/-1.3 % on C5 with single-prim
# leaves) against the current build; C3, C4, C5 alternated
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2 3; do
  for s in "book1 600 512" "book2 400 1024" "model 960 512"; do
    timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "cur", /' || exit 1
    for v in apart pair2; do
      RT_AMD_LIB=$L/$v/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed "s/^{/{\"lib\": \"$v\", /" || exit 1
    done
  done
done > $O/ab_apart.jsonl
