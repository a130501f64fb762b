#!/bin/bash
# Run bench.py once, then the same command under rocprofv3 kernel-trace stats.
# usage: tools/gpu_bench_prof.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
cd "$R" && timeout -k 10 600 python3 bench.py "$@" > "$R/gpurun_out/bench_$TAG.json" 2> "$R/gpurun_out/bench_$TAG.err" || exit $?
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --no-cpu-baseline "$@" > "$R/gpurun_out/prof_$TAG.log" 2>&1
