#!/bin/bash
# round-3 probe: the C3/C5 kernels compiled in their own translation unit with the
# iterative-ILP scheduler (in-tree build) against HEAD's single-TU build (build_prev);
# C2-C5 alternated at full size, then bitwise images
set -o pipefail
O=gpurun_out; mkdir -p $O
P=$PWD/go_raytracer_amd/build_prev/librt_amd.so
for rep in 1 2 3; do
  for s in "cornell 800 1024 fused" "book1 1200 484 fused 1.5" "book2 400 1024 fused" "model 1920 1024 fused"; do
    RT_AMD_LIB=$P timeout -k 10 200 python3 tools/gpu_probe.py $s | sed 's/^{/{"lib": "prev", /' || exit 1
    timeout -k 10 200 python3 tools/gpu_probe.py $s | sed 's/^{/{"lib": "split", /' || exit 1
  done
done > $O/ab_split_ilp.jsonl
timeout -k 10 300 python3 tools/ab_bitwise.py $P > $O/ab_split_ilp_bitwise.txt 2>&1
