#!/bin/bash
# GPU call: gpu tests (obj_mixed deselected), obj bisection, output bench, PMC, C2-C5 probes.
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "not obj_mixed" > "$O/pytest_$TAG.log" 2>&1 || { tail -40 "$O/pytest_$TAG.log"; exit 1; }
tail -2 "$O/pytest_$TAG.log"
timeout -k 10 300 python3 -u tools/bisect_obj.py > "$O/bisect_obj_$TAG.jsonl" 2>&1 || { tail -20 "$O/bisect_obj_$TAG.jsonl"; exit 1; }
cut -c1-300 "$O/bisect_obj_$TAG.jsonl"
timeout -k 10 120 python3 tools/output_bench.py "$O/output_bench_$TAG.jsonl" || exit $?
timeout -k 10 400 python3 tools/pmc_traffic.py "$O/pmc_$TAG.json" --steps 1 --warmup 1 > "$O/pmc_$TAG.log" 2>&1 || { tail -20 "$O/pmc_$TAG.log"; exit 1; }
bash tools/probe_configs.sh "$O/configs_$TAG.jsonl" || exit $?
cut -c1-200 "$O/configs_$TAG.jsonl"
