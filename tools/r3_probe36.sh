#!/bin/bash
# round-3 probe: branchless pushes of a BVH4 node step's far children (RT_PUSH_NOBRANCH:
# three LDS writes, the stack pointer advanced past the valid ones) against the
# exec-branch pushes; C3-C5 alternated, then bitwise images
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2 3; do
  for s in "book1 1200 484 fused 1.5" "book2 400 1024 fused" "model 960 512 fused"; do
    timeout -k 10 200 python3 tools/gpu_probe.py $s | sed 's/^{/{"lib": "cur", /' || exit 1
    RT_AMD_LIB=$L/pushnb/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py $s | sed 's/^{/{"lib": "pushnb", /' || exit 1
  done
done > $O/ab_pushnb.jsonl
timeout -k 10 300 python3 tools/ab_bitwise.py $L/pushnb/librt_amd.so > $O/ab_pushnb_bitwise.txt 2>&1
