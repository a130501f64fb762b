# SAH cost sweep (dev tool): RT_BVH_CI (prim test cost, traversal step = 1) on C3/C4 shapes
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status
for ci in 0.5 1 1.5 2 3; do
  for cfg in "book1 1200 256" "book2 800 512"; do
    RT_BVH_CI=$ci timeout -k 10 200 python3 tools/gpu_probe.py $cfg fused | sed "s/^{/{\"ci\": $ci, /" || exit 1
  done
done
