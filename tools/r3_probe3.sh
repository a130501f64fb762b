#!/bin/bash
# round-3 probe: C2 share timings (tools/share_probe.py), in-tree library vs the
# prefetched-refill build (RT_GRAB_PREFETCH), default and smaller batches, alternated
set -o pipefail
O=gpurun_out; mkdir -p $O
L=$PWD/go_raytracer_amd/build_abl
for rep in 1 2; do
  timeout -k 10 200 python3 tools/share_probe.py cornell 800 1024 | sed 's/^{/{"lib": "cur", /' || exit 1
  RT_AMD_LIB=$L/prefetch/librt_amd.so timeout -k 10 200 python3 tools/share_probe.py cornell 800 1024 | sed 's/^{/{"lib": "prefetch", /' || exit 1
  RT_GRAB_MIN=64 RT_AMD_LIB=$L/prefetch/librt_amd.so timeout -k 10 200 python3 tools/share_probe.py cornell 800 1024 | sed 's/^{/{"lib": "prefetch64", /' || exit 1
  RT_GRAB_MIN=128 RT_AMD_LIB=$L/prefetch/librt_amd.so timeout -k 10 200 python3 tools/share_probe.py cornell 800 1024 | sed 's/^{/{"lib": "prefetch128", /' || exit 1
done > $O/share_prefetch.jsonl
