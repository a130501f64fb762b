#!/bin/bash
# round-3 probe: the chunk range split into 8 partitions, one per XCD group, each drawn
# first by its own waves (RT_PARTS=8) against one global counter (RT_PARTS=1); bitwise
# images at small size, then alternated full-size timings per config
set -o pipefail
O=gpurun_out; mkdir -p $O
export RT_AMD_LIB=$PWD/go_raytracer_amd/build_abl/parts/librt_amd.so
rm -f $O/ab_parts.jsonl
timeout -k 10 300 python3 tools/env_ab.py RT_PARTS=1,8 $O/ab_parts.jsonl model:1920:1024 cornell:800:1024 book2:800:1024 || exit 1
timeout -k 10 200 python3 tools/env_ab.py RT_PARTS=1,8 $O/ab_parts.jsonl cornell:800:1024 || exit 1
timeout -k 10 200 python3 tools/env_ab.py RT_PARTS=1,8 $O/ab_parts.jsonl book1:1200:484 || exit 1
timeout -k 10 300 python3 tools/env_ab.py RT_PARTS=1,8 $O/ab_parts.jsonl book2:800:4096 || exit 1
