#!/bin/bash
# One GPU session on the box (dev tool): tools/gpu_session.sh TAG STEP [STEP ...]
#   tests    pytest -m gpu (PARITY_LOG -> gpurun_out/parity_TAG.jsonl)
#   ab       tools/ab_configs.sh: build_prev vs in-tree library, alternating, C2-C5
#   configs  tools/probe_configs.sh: C2-C5 at full size, one render each
#   bench    bench.py (default flags; the pmc step's traffic.json when it ran first) -> gpurun_out/bench_TAG.json
#   prof     rocprofv3 --kernel-trace --stats of bench.py -> gpurun_out/prof_TAG/
#   share    tools/share_probe.py for cornell, book2, model
#   pmc      tools/pmc_traffic.py TAG C2 C3 C4 C5 -> profiles/traffic.json + profiles/TAG_pmc_*.json
# Every step has its own time limit; the first failing step ends the session.
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 1
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    tests) PARITY_LOG=$O/parity_$TAG.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q \
             --timeout 300 --timeout-method thread > "$O/tests_$TAG.log" 2>&1 ;;
    ab) timeout -k 10 900 bash tools/ab_configs.sh "$O/ab_$TAG.jsonl" ;;
    configs) timeout -k 10 600 bash tools/probe_configs.sh "$O/configs_$TAG.jsonl" ;;
    bench) T=$O/profiles_$TAG/traffic.json; BA=(); [ -f "$T" ] && BA=(--traffic "$T")
           timeout -k 10 600 python3 bench.py "${BA[@]}" > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err" ;;
    prof) (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof_$TAG" \
             -o run -- python3 "$R/bench.py" --no-cpu-baseline --steps 5 > "$O/prof_$TAG.log" 2>&1) ;;
    share) for s in "cornell 800 1024" "book2 800 4096" "model 1920 1024"; do
             timeout -k 10 600 python3 tools/share_probe.py $s || exit $?
           done > "$O/share_$TAG.jsonl" 2>&1 ;;
    pmc) timeout -k 10 1100 python3 tools/pmc_traffic.py "$TAG" C2 C3 C4 C5 > "$O/pmc_$TAG.log" 2>&1 ;;
    *) echo "unknown step $step"; false ;;
  esac
  rc=$?
  echo "== $step rc=$rc $(date +%T)"
  [ $rc -eq 0 ] || exit $rc
done
