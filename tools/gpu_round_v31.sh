B=$PWD/go_raytracer_amd
for rep in 1 2; do
  for sb in 4 8 16; do
    RT_STEP_BUDGET=$sb timeout -k 10 200 python3 tools/gpu_probe.py model 1920 256 fused | sed "s/^{/{\"lib\": \"cur_sb$sb\", /" | cut -c1-120 || exit 1
  done
  RT_AMD_LIB=$B/build_abl/mesh5/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py model 1920 256 fused | sed "s/^{/{\"lib\": \"mesh5\", /" | cut -c1-120 || exit 1
  RT_AMD_LIB=$B/build_abl/mesh5/librt_amd.so timeout -k 10 200 python3 tools/gpu_probe.py book1 1200 512 fused | sed "s/^{/{\"lib\": \"mesh5\", /" | cut -c1-120 || exit 1
  timeout -k 10 200 python3 tools/gpu_probe.py book1 1200 512 fused | sed "s/^{/{\"lib\": \"cur\", /" | cut -c1-120 || exit 1
done
