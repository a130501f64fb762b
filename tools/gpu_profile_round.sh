#!/bin/bash
# Bench + rocprof kernel stats + PMC traffic for the bench kernel + share probe (one GPU call).
# usage: tools/gpu_profile_round.sh TAG
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R" || exit 1
bash tools/gpu_bench_prof.sh "$TAG" || exit $?
cat "$O/bench_$TAG.json"
timeout -k 10 400 python3 tools/pmc_traffic.py "$O/pmc_$TAG.json" --steps 1 --warmup 1 > "$O/pmc_$TAG.log" 2>&1 || { tail -20 "$O/pmc_$TAG.log"; exit 1; }
timeout -k 10 200 python3 tools/share_probe.py > "$O/share_$TAG.jsonl" 2>&1 || exit 1
grep '^{' "$O/share_$TAG.jsonl"
bash tools/probe_configs.sh "$O/configs_$TAG.jsonl" && cut -c1-160 "$O/configs_$TAG.jsonl"
