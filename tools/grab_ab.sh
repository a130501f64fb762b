# Chunk-batch size sweep (dev tool): RT_GRAB_MIN on C3-C5 shapes
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status
for g in 64 128 256; do
  for cfg in "book2 800 512" "model 1920 256" "book1 1200 256"; do
    RT_GRAB_MIN=$g timeout -k 10 200 python3 tools/gpu_probe.py $cfg fused | sed "s/^{/{\"grab_min\": $g, /" || exit 1
  done
done
