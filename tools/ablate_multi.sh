#!/bin/bash
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status
# Time library builds on several configs, alternating (dev tool):
#   tools/ablate_multi.sh OUTLOG REPS "scene width spp" ...
# Libraries: the in-tree one ("cur"), go_raytracer_amd/build_prev ("prev", if built by
# tools/build_prev.sh) and every go_raytracer_amd/build_abl/<name>/librt_amd.so
# (tools/build_variant.sh).  One JSON line per render (tools/gpu_probe.py).
OUT=$1; REPS=$2; shift 2
B=$PWD/go_raytracer_amd
for rep in $(seq "$REPS"); do
  for cfg in "$@"; do
    for so in "" $B/build_prev/librt_amd.so $B/build_abl/*/librt_amd.so; do
      [ -z "$so" ] || [ -f "$so" ] || continue
      n=cur; [ -z "$so" ] || n=$(basename "$(dirname "$so")")
      RT_AMD_LIB=$so timeout -k 10 300 python3 tools/gpu_probe.py $cfg fused | sed "s/^{/{\"lib\": \"$n\", /" || exit $?
    done
  done
done > "$OUT" 2>&1
