#!/bin/bash
# round-3 probe: (1) dominated clamp weights merged vs pushed (build_abl/nomerge), C2-C5
# timings alternated + HBM pushes (build_abl/hbmpushes); (2) sphere precision split
# RT_SPHERE_FP64_R 0 / 16 / 256: C3/C4 timings alternated, then full-size parity at 16
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2; do
  for s in "book2 800 1024" "model 1920 512" "book1 1200 512" "cornell 800 1024"; do
    timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "cur", /' || exit 1
    RT_AMD_LIB=$L/nomerge/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "nomerge", /' || exit 1
  done
done > $O/ab_merge.jsonl
RT_AMD_LIB=$L/hbmpushes/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py book2 400 1024 fused > $O/hbmpushes_merge.jsonl || exit 1
for rep in 1 2; do
  for v in 0 16 256; do
    for s in "book1 1200 512" "book2 800 1024"; do
      RT_SPHERE_FP64_R=$v timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed "s/^{/{\"fp64_r\": $v, /" || exit 1
    done
  done
done > $O/ab_sphere.jsonl
RT_SPHERE_FP64_R=16 PARITY_LOG=$O/parity_sphere_16.jsonl timeout -k 10 300 python3 -u -m pytest \
  tests/test_render_gpu.py -q --timeout 240 --timeout-method thread \
  -k "full_size_parity and (book1 or book2)" > $O/sphere_tests_16.log 2>&1
exit 0
