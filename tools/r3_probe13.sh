#!/bin/bash
# round-3 probe: C2 weight-only ablations (timing only; images differ) and phase profile
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2; do
  timeout -k 10 200 python3 tools/gpu_probe.py cornell 800 1024 fused | sed 's/^{/{"lib": "cur", /' || exit 1
  for v in nofold nolpdf; do
    RT_AMD_LIB=$L/$v/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py cornell 800 1024 fused | sed "s/^{/{\"lib\": \"$v\", /" || exit 1
  done
done > $O/ab_c2_ablate.jsonl
for s in "cornell 800 256" "model 960 256" "book2 400 1024" "book1 600 512"; do
  RT_AMD_LIB=$L/phases/librt_amd.so timeout -k 10 200 python3 tools/phase_probe.py $s || exit 1
done > $O/phases_r3.jsonl
