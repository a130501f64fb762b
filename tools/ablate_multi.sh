#!/bin/bash
# Time every ablation build on several configs (dev tool): tools/ablate_multi.sh OUTLOG "scene w spp" ...
OUT=$1; shift
for cfg in "$@"; do
  for so in go_raytracer_amd/build_abl/*/librt_amd.so; do
    n=$(basename $(dirname $so))
    RT_AMD_LIB=$PWD/$so timeout -k 10 300 python3 tools/gpu_probe.py $cfg fused | sed "s/^{/{\"lib\": \"$n\", /" || exit $?
  done
done > "$OUT" 2>&1
