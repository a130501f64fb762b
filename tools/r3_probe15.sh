#!/bin/bash
# round-3 probe: re-tune the fused loop's scheduling rounds after this round's traversal
# changes (tools/sched_sweep.py: step budget x shade_min)
set -o pipefail
O=gpurun_out; mkdir -p $O
{
  timeout -k 10 300 python3 tools/sched_sweep.py model 1920 512 6,8,12,16 1,16,32 || exit 1
  timeout -k 10 300 python3 tools/sched_sweep.py book2 800 1024 6,8,12,16 1,16,32 || exit 1
  timeout -k 10 300 python3 tools/sched_sweep.py book1 1200 512 8,12,16,24 1,8,16 || exit 1
} > $O/sched_r3.jsonl
