#!/bin/bash
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status
# share-probe A/B: alternate variants, label lines
OUT=${1:-gpurun_out/share_ab.jsonl}
for rep in 1 2; do
  for v in cur gss6 gss7 grab8 grab16; do
    case $v in
      cur) timeout -k 10 120 python3 tools/share_probe.py > /tmp/sp.json || exit $? ;;
      gss6|gss7) RT_AMD_LIB=$PWD/go_raytracer_amd/build_abl/$v/librt_amd.so timeout -k 10 120 python3 tools/share_probe.py > /tmp/sp.json || exit $? ;;
      grab8) RT_GRAB_MIN=8 timeout -k 10 120 python3 tools/share_probe.py > /tmp/sp.json || exit $? ;;
      grab16) RT_GRAB_MIN=16 timeout -k 10 120 python3 tools/share_probe.py > /tmp/sp.json || exit $? ;;
    esac
    sed "s/^{/{\"lib\": \"$v\", /" /tmp/sp.json >> $OUT
  done
done
