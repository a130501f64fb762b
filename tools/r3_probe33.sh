#!/bin/bash
# round-3 probe: C2's record loop reading the quad records with scalar loads
# (RT_BRUTE_SMEM=1) against the LDS copy (=0), after this round's SGPR changes
set -o pipefail
O=gpurun_out; mkdir -p $O
rm -f $O/ab_brute_smem.jsonl
timeout -k 10 300 python3 tools/env_ab.py RT_BRUTE_SMEM=0,1 $O/ab_brute_smem.jsonl cornell:800:1024 quads:400:1024 || exit 1
timeout -k 10 300 python3 tools/env_ab.py RT_BRUTE_SMEM=0,1 $O/ab_brute_smem.jsonl cornell:800:1024 || exit 1
