#!/bin/bash
# round-3 probe: LLVM AMDGPU scheduler strategies for the whole library (-mllvm
# -amdgpu-sched-strategy=...), per config, against the default; alternated
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2; do
  for s in "cornell 800 1024" "book1 1200 512" "book2 400 1024" "model 960 512"; do
    timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "cur", /' || exit 1
    for v in ilp memcl itilp itmin; do
      RT_AMD_LIB=$L/$v/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed "s/^{/{\"lib\": \"$v\", /" || exit 1
    done
  done
done > $O/ab_sched_strategy.jsonl
