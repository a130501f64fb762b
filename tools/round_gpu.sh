#!/bin/bash
# One GPU call: gpu tests, then bench + rocprof kernel stats (tools/gpu_bench_prof.sh).
# usage: tools/round_gpu.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd "$R" && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$R/gpurun_out/pytest_$TAG.log" 2>&1 || { tail -30 "$R/gpurun_out/pytest_$TAG.log"; exit 1; }
tail -3 "$R/gpurun_out/pytest_$TAG.log"
bash "$R/tools/gpu_bench_prof.sh" "$TAG" "$@" || exit $?
cat "$R/gpurun_out/bench_$TAG.json"
