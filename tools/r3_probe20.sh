#!/bin/bash
# round-3 probe: camera constants re-read from the kernel-argument segment at the ray start
# (RT_CAM_KERNARG: C2 SGPR spills 78 -> 34, C3 101 -> 32) against SGPR-resident constants;
# C2 and C3 alternated, then the bitwise check of the images
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2 3; do
  for s in "cornell 800 1024" "book1 1200 512"; do
    timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "cur", /' || exit 1
    RT_AMD_LIB=$L/camk/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "camk", /' || exit 1
  done
done > $O/ab_camk.jsonl
timeout -k 10 300 python3 tools/ab_bitwise.py $L/camk/librt_amd.so > $O/ab_camk_bitwise.txt 2>&1
