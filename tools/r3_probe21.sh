#!/bin/bash
# round-3 probe: camera constants from the kernel-argument segment in every kernel
# (RT_CAM_KERNARG_ALL) against g_cam in LDS for the book2 and mesh kernels (C4, C5)
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2 3; do
  for s in "book2 400 1024" "model 960 512"; do
    timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "cur", /' || exit 1
    RT_AMD_LIB=$L/camkall/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "camkall", /' || exit 1
  done
done > $O/ab_camkall.jsonl
