#!/bin/bash
# round-3 probe: cascaded weight merge (build_abl/cascade) vs in-tree, alternated; HBM
# weight-stack pushes of both (build_abl/{hbmpushes, cascade_pushes}) on book2
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2; do
  for s in "book2 800 1024" "cornell 800 1024" "book1 1200 512" "model 1920 512"; do
    timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "cur", /' || exit 1
    RT_AMD_LIB=$L/cascade/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "cascade", /' || exit 1
  done
done > $O/ab_cascade.jsonl
for v in hbmpushes cascade_pushes; do
  RT_AMD_LIB=$L/$v/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py book2 400 1024 fused | sed "s/^{/{\"lib\": \"$v\", /" || exit 1
done > $O/pushes_cascade.jsonl
