#!/bin/bash
# round-3 probe: the adopted kernarg camera reads (in-tree build) against the SGPR-resident
# camera (camsgpr = -DRT_CAM_SGPR, the previous behaviour) on C2-C5, plus the grab / shading
# parameters re-read at their phase (kpg, kpgs) on C2
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2 3; do
  for v in cur camsgpr kpg kpgs; do
    if [ $v = cur ]; then unset RT_AMD_LIB; else export RT_AMD_LIB=$L/$v/librt_amd.so; fi
    timeout -k 10 200 python3 tools/gpu_probe.py cornell 800 1024 fused | sed "s/^{/{\"lib\": \"$v\", /" || exit 1
  done
  unset RT_AMD_LIB
  for s in "book1 1200 512" "book2 400 1024" "model 960 512"; do
    timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "cur", /' || exit 1
    RT_AMD_LIB=$L/camsgpr/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "camsgpr", /' || exit 1
  done
done > $O/ab_cam_final.jsonl
