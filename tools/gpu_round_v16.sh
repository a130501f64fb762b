set -o pipefail
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_v16.log 2>&1 || { tail -30 $O/pytest_v16.log; exit 1; }
tail -1 $O/pytest_v16.log
timeout -k 10 200 python3 tools/share_probe.py > $O/share_v16.jsonl 2>&1 || { tail -5 $O/share_v16.jsonl; exit 1; }
grep '^{' $O/share_v16.jsonl
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench_v16.json 2>$O/bench_v16.err || { tail -5 $O/bench_v16.err; exit 1; }
cut -c1-300 $O/bench_v16.json
bash tools/ab_configs.sh $O/ab_configs_v16.jsonl && cut -c1-110 $O/ab_configs_v16.jsonl
