#!/bin/bash
# round-3 probe: C2 occupancy variants (build_abl/{w7l4, w6l4, brute5}) vs in-tree
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2 3; do
  timeout -k 10 200 python3 tools/gpu_probe.py cornell 800 1024 fused | sed 's/^{/{"lib": "cur", /' || exit 1
  for v in w7l4 w6l4 brute5; do
    RT_AMD_LIB=$L/$v/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py cornell 800 1024 fused | sed "s/^{/{\"lib\": \"$v\", /" || exit 1
  done
done > $O/ab_c2_occ.jsonl
