#!/bin/bash
# round-3 probe: per-sphere precision (RT_SPHERE_FP64_R: 0 = every sphere in fp64, as in
# round 2; 256 = the default split) -- full-size C3/C4 parity, then alternated timings
set -o pipefail
O=gpurun_out; mkdir -p $O
for v in 0 256; do
  RT_SPHERE_FP64_R=$v PARITY_LOG=$O/parity_sphere_$v.jsonl timeout -k 10 300 python3 -u -m pytest \
    tests/test_render_gpu.py -x -q --timeout 240 --timeout-method thread \
    -k "full_size_parity and (book1 or book2)" > $O/sphere_tests_$v.log 2>&1 || exit 1
done
for rep in 1 2; do
  for v in 0 256; do
    for s in "book1 1200 512" "book2 800 1024"; do
      RT_SPHERE_FP64_R=$v timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed "s/^{/{\"fp64_r\": $v, /" || exit 1
    done
  done
done > $O/ab_sphere.jsonl
