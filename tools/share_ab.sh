#!/bin/bash
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status
# Share-probe A/B (dev tool): alternate library builds / knob settings on
# tools/share_probe.py, one labelled JSON line per (variant, N):
#   tools/share_ab.sh OUTLOG REPS name=lib|cur|ENV=VAL ...   (e.g. cur xw5=path/librt_amd.so grab8=RT_GRAB_MIN=8)
# SP_ARGS="scene width spp" picks the scene (default: cornell 800 1024)
OUT=$1; REPS=$2; shift 2
for rep in $(seq "$REPS"); do
  for spec in "$@"; do
    name=${spec%%=*}; arg=${spec#*=}
    if [ "$arg" = cur ] || [ "$spec" = cur ]; then
      timeout -k 10 120 python3 tools/share_probe.py $SP_ARGS > /tmp/sp.json || exit $?
    elif [[ $arg == *.so ]]; then
      RT_AMD_LIB=$PWD/$arg timeout -k 10 120 python3 tools/share_probe.py $SP_ARGS > /tmp/sp.json || exit $?
    else
      env "$arg" timeout -k 10 120 python3 tools/share_probe.py $SP_ARGS > /tmp/sp.json || exit $?
    fi
    sed "s/^{/{\"lib\": \"$name\", /" /tmp/sp.json >> "$OUT"
  done
done
