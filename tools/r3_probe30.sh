#!/bin/bash
# round-3 probe: the wave batch in SGPRs (RT_BATCH_SGPR: v_readlane of the leader's atomic
# result, readfirstlane bounds; C2's kernel 4 -> 0 spilled VGPRs) against the in-tree build;
# C2-C5 alternated, then bitwise images
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2 3; do
  for s in "cornell 800 1024" "book1 1200 512" "book2 400 1024" "model 960 512"; do
    timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "cur", /' || exit 1
    RT_AMD_LIB=$L/sgb/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "sgb", /' || exit 1
  done
done > $O/ab_sgb.jsonl
timeout -k 10 300 python3 tools/ab_bitwise.py $L/sgb/librt_amd.so > $O/ab_sgb_bitwise.txt 2>&1
