#!/bin/bash
# round-3 probe: chunk size K above 32 on the whole-image configs (fewer chunk flushes, i.e.
# fewer pixel atomics and grabs; images do not depend on K)
set -o pipefail
O=gpurun_out; mkdir -p $O
{
  KS=16,32,64,128 timeout -k 10 300 python3 tools/chunk_probe.py book2 800 4096 || exit 1
  KS=16,32,64,128 timeout -k 10 300 python3 tools/chunk_probe.py model 1920 1024 || exit 1
  KS=16,32,64,128 timeout -k 10 300 python3 tools/chunk_probe.py cornell 800 1024 || exit 1
  KS=16,32,64,128 timeout -k 10 300 python3 tools/chunk_probe.py book1 1200 484 || exit 1
} > $O/chunk_big_r3.jsonl
