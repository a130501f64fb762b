#!/bin/bash
# round-3 probe: Philox rounds fully unrolled (RT_RNG_UNROLL; the compiler kept a loop of
# three rounds) against the in-tree build; C2-C5 alternated, then bitwise images
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2 3; do
  for s in "cornell 800 1024 fused" "book1 1200 484 fused 1.5" "book2 400 1024 fused" "model 960 512 fused"; do
    timeout -k 10 200 python3 tools/gpu_probe.py $s | sed 's/^{/{"lib": "cur", /' || exit 1
    RT_AMD_LIB=$L/rngunroll/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py $s | sed 's/^{/{"lib": "rngunroll", /' || exit 1
  done
done > $O/ab_rng_unroll.jsonl
timeout -k 10 300 python3 tools/ab_bitwise.py $L/rngunroll/librt_amd.so > $O/ab_rng_unroll_bitwise.txt 2>&1
