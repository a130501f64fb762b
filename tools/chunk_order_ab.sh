# A/B of the chunk order (dev tool): RT_CHUNK_ROWS row groups (100000 = whole image) on C2-C5 shapes
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status

for rep in 1 2; do
for cfg in "model 1920 256" "book2 800 512" "book1 1200 256" "cornell 800 256"; do
  for r in 100000 1 4 16; do
    export RT_CHUNK_ROWS=$r
    timeout -k 10 120 python3 tools/gpu_probe.py $cfg fused | sed "s/^{/{\"group_rows\": $r, /" || exit 1
  done
done
done
