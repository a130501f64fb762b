#!/bin/bash
# round-3 probe: C2 in-tree vs go_raytracer_amd/build_prev (tools/build_prev.sh), alternated
set -o pipefail
O=gpurun_out; mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/gpu_probe.py cornell 800 1024 fused | sed 's/^{/{"lib": "cur", /' || exit 1
  RT_AMD_LIB=$PWD/go_raytracer_amd/build_prev/librt_amd.so timeout -k 10 120 python3 tools/gpu_probe.py cornell 800 1024 fused | sed 's/^{/{"lib": "prev", /' || exit 1
done > $O/ab_c2_qshade.jsonl
