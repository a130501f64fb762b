#!/bin/bash
# round-3 probe: the book2 kernel's LDS split between the traversal short stack and the
# weight stack (TEX_SHORT x TEX_WLDS: 12 x 4 now; 16 x 3, 18 x 2, 13 x 4), C4 at 400 x 400
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2 3; do
  timeout -k 10 200 python3 tools/gpu_probe.py book2 400 1024 fused | sed 's/^{/{"lib": "cur", /' || exit 1
  for v in s16w3 s18w2 s13w4; do
    RT_AMD_LIB=$L/$v/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py book2 400 1024 fused | sed "s/^{/{\"lib\": \"$v\", /" || exit 1
  done
done > $O/ab_tex_stack.jsonl
