#!/bin/bash
# round-3 probe: Philox round keys recomputed per call (build_abl/rngkeys) vs in-tree
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2 3; do
  for s in "cornell 800 1024" "book1 1200 512" "book2 800 1024"; do
    timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "cur", /' || exit 1
    RT_AMD_LIB=$L/rngkeys/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "rngkeys", /' || exit 1
  done
done > $O/ab_rngkeys.jsonl
