#!/bin/bash
# round-3 probe: C5's tree from the host SAH builder against the device PLOC build (the
# default above 65,536 prims), render time only; images differ (another tree)
set -o pipefail
O=gpurun_out; mkdir -p $O
rm -f $O/ab_c5_builder.jsonl
timeout -k 10 600 python3 tools/env_ab.py RT_BVH_BUILDER=device,host $O/ab_c5_builder.jsonl model:1920:1024 || exit 1
