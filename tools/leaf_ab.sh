# A/B of the SAH leaf size (dev tool): RT_BVH_LEAF 1 | 2 | 4 on C3/C4 shapes
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status
for rep in 1 2; do
for lf in 1 2 4; do
  export RT_BVH_LEAF=$lf
  timeout -k 10 200 python3 tools/gpu_probe.py book1 1200 256 fused | sed "s/^{/{\"leaf\": $lf, /" || exit 1
  timeout -k 10 200 python3 tools/gpu_probe.py book2 800 512 fused | sed "s/^{/{\"leaf\": $lf, /" || exit 1
done
done
