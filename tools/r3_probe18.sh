#!/bin/bash
# round-3 probe: the termination fold loading only the lane's live LDS weight entries
# (RT_FOLD_NST) against loading all of them; C2 plus the media and mesh kernels
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2 3; do
  for s in "cornell 800 1024" "book2 400 1024" "model 960 512"; do
    timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "cur", /' || exit 1
    RT_AMD_LIB=$L/foldnst/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py $s fused | sed 's/^{/{"lib": "foldnst", /' || exit 1
  done
done > $O/ab_foldnst.jsonl
