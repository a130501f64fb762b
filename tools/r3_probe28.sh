#!/bin/bash
# round-3 probe: waves stop refilling once the chunk range is used up ("done") against
# refilling with invalid ids until they drain ("nodone", -DRT_GRAB_AFTER_END); row shares
# of 1/2/4/8 ranks (tools/share_probe.py), alternated
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2; do
  for v in nodone done; do
    for s in "cornell 800 1024" "model 1920 1024" "book1 1200 484"; do
      RT_AMD_LIB=$L/$v/librt_amd.so timeout -k 10 300 python3 tools/share_probe.py $s | sed "s/^{/{\"lib\": \"$v\", /" || exit 1
    done
  done
done > $O/ab_grab_done.jsonl
