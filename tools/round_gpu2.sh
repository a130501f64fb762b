#!/bin/bash
# GPU call: gpu tests, output-path bench, PMC traffic for the bench kernel, C2-C5 probes.
# usage: tools/round_gpu2.sh TAG
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$O/pytest_$TAG.log" 2>&1 || { tail -40 "$O/pytest_$TAG.log"; exit 1; }
tail -2 "$O/pytest_$TAG.log"
timeout -k 10 120 python3 tools/output_bench.py "$O/output_bench_$TAG.jsonl" || exit $?
timeout -k 10 400 python3 tools/pmc_traffic.py "$O/pmc_$TAG.json" --steps 1 --warmup 1 > "$O/pmc_$TAG.log" 2>&1 || { tail -20 "$O/pmc_$TAG.log"; exit 1; }
bash tools/probe_configs.sh "$O/configs_$TAG.jsonl" || exit $?
cat "$O/configs_$TAG.jsonl" | cut -c1-200
