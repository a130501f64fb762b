set -o pipefail
O=gpurun_out
B=$PWD/go_raytracer_amd
timeout -k 10 120 python3 tools/share_probe.py > $O/share_v12.jsonl 2>&1 || { tail -5 $O/share_v12.jsonl; exit 1; }
cat $O/share_v12.jsonl
for rep in 1 2; do
  for v in prev tex3 tex4; do
    L=$B/build_abl/$v/librt_amd.so; [ $v = prev ] && L=$B/build_prev/librt_amd.so
    RT_AMD_LIB=$L timeout -k 10 300 python3 tools/gpu_probe.py book2 800 2048 fused | sed "s/^{/{\"lib\": \"$v\", /" | cut -c1-140 || exit 1
    RT_AMD_LIB=$L timeout -k 10 300 python3 tools/gpu_probe.py book1 1200 512 fused | sed "s/^{/{\"lib\": \"$v\", /" | cut -c1-140 || exit 1
  done
done
