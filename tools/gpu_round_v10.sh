set -o pipefail
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_v10.log 2>&1 || { tail -30 $O/pytest_v10.log; exit 1; }
tail -2 $O/pytest_v10.log
timeout -k 10 300 python3 tools/ab_bitwise.py go_raytracer_amd/build_prev/librt_amd.so > $O/ab_bitwise_v10.jsonl 2>&1 || { tail -5 $O/ab_bitwise_v10.jsonl; exit 1; }
grep -c '"bitwise_equal": true' $O/ab_bitwise_v10.jsonl; grep '"bitwise_equal": false' $O/ab_bitwise_v10.jsonl | head -5
bash tools/ab_c2.sh $O/ab_c2_v10.jsonl && cut -c1-110 $O/ab_c2_v10.jsonl
bash tools/ab_configs.sh $O/ab_configs_v10.jsonl && cut -c1-110 $O/ab_configs_v10.jsonl
