#!/bin/bash
set -o pipefail  # a failed GPU step in a pipeline ends the script with its own status
# Scheduling knobs on one GPU's 8-GPU row share (dev tool): tools/share_sweep.sh OUTLOG SCENE WIDTH SPP NRANKS
# (tools/knob_sweep.py with NRANKS: rank 0's rows r % N == 0, kernel time of the fused launch)
OUT=$1; S=$2; W=$3; SPP=$4; N=${5:-8}
for kv in "RT_GRAB_MIN 64,128,256,512" "RT_STEP_BUDGET 4,5,6,7" "RT_SHADE_MIN 8,16,32,48" \
          "RT_CHUNK_NEED 50,100,200,400" "RT_SPLIT_MIN 0,1,4"; do
  set -- $kv
  NRANKS=$N timeout -k 10 300 python3 tools/knob_sweep.py $S $W $SPP $1 $2 3 || exit $?
done > "$OUT" 2>&1
