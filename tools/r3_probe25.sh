#!/bin/bash
# round-3 probe: book2 kernel LDS split, full-size C4 (800 x 800 x 4096) and 400 x 400
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2; do
  for s in "book2 800 4096" "book2 400 1024"; do
    timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "cur", /' || exit 1
    for v in s13w4 s18w2 s21w1; do
      RT_AMD_LIB=$L/$v/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed "s/^{/{\"lib\": \"$v\", /" || exit 1
    done
  done
done > $O/ab_tex_stack2.jsonl
