#!/bin/bash
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status
# Time named library builds on several configs, alternating (dev tool):
#   tools/ab_libs.sh OUTLOG REPS "name=path.so,name2=path2.so,..." "scene width spp" ...
# "cur" (or an empty path) is the in-tree library.  One JSON line per render
# (tools/gpu_probe.py), tagged with the library's name.
OUT=$1; REPS=$2; LIBS=$3; shift 3
IFS=',' read -r -a PAIRS <<< "$LIBS"
for rep in $(seq "$REPS"); do
  for cfg in "$@"; do
    for pair in "${PAIRS[@]}"; do
      n=${pair%%=*}; so=${pair#*=}; [ "$so" = "$pair" ] && so=""
      RT_AMD_LIB=$so timeout -k 10 300 python3 tools/gpu_probe.py $cfg fused | sed "s/^{/{\"lib\": \"$n\", /" || exit $?
    done
  done
done > "$OUT" 2>&1
