#!/bin/bash
# round-3 probe: in-tree vs go_raytracer_amd/build_prev on C2-C5, alternated (3 reps)
set -o pipefail
O=gpurun_out; mkdir -p $O
P=$PWD/go_raytracer_amd/build_prev/librt_amd.so
for rep in 1 2 3; do
  for s in "cornell 800 1024" "book1 1200 512" "book2 800 1024" "model 1920 512"; do
    timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "cur", /' || exit 1
    RT_AMD_LIB=$P timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "prev", /' || exit 1
  done
done > $O/ab_${1:-cur}.jsonl
