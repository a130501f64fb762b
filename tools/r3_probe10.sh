#!/bin/bash
# round-3 probe: medium boundary roots skipped when the free flight is past the closest
# hit (build_abl/mediaskip): bitwise check against the in-tree library, then timings
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
timeout -k 10 300 python3 tools/ab_bitwise.py $L/nomediaskip/librt_amd.so > $O/bitwise_mediaskip.jsonl 2>&1 || exit 1
for rep in 1 2 3; do
  for s in "book2 800 1024" "cornell_smoke 600 1024"; do
    timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "cur", /' || exit 1
    RT_AMD_LIB=$L/nomediaskip/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "nomediaskip", /' || exit 1
  done
done > $O/ab_mediaskip.jsonl
