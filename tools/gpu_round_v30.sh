set -o pipefail
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_v30.log 2>&1 || { tail -30 $O/pytest_v30.log; exit 1; }
tail -1 $O/pytest_v30.log
bash tools/ab_configs.sh $O/ab_configs_v30.jsonl && cut -c1-110 $O/ab_configs_v30.jsonl
