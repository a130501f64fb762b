# Fused-loop scheduling sweep (dev tool): RT_STEP_BUDGET x RT_SHADE_MIN on C3-C5 shapes
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status
run() {  # scene width spp budget shade_min
  RT_STEP_BUDGET=$4 RT_SHADE_MIN=$5 timeout -k 10 200 python3 tools/gpu_probe.py $1 $2 $3 fused |
    sed "s/^{/{\"step_budget\": $4, \"shade_min\": $5, /"
}
for sb in 12 16 24 48 1073741824; do run book1 1200 256 $sb 1 || exit 1; done
for sm in 8 16 32 48; do run model 1920 256 8 $sm || exit 1; done
for sm in 8 32; do run book2 800 512 8 $sm || exit 1; done
for sb in 16 24; do run book1 1200 256 $sb 16 || exit 1; done
