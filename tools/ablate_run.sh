#!/bin/bash
# Time every ablation build on one config (dev tool): tools/ablate_run.sh OUTLOG scene width spp
OUT=$1; shift
for rep in 1 2; do
  for so in go_raytracer_amd/build_abl/*/librt_amd.so; do
    n=$(basename $(dirname $so))
    RT_AMD_LIB=$PWD/$so timeout -k 10 300 python3 tools/gpu_probe.py "$@" fused | sed "s/^{/{\"lib\": \"$n\", /" || exit $?
  done
done > "$OUT" 2>&1
