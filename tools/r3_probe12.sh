#!/bin/bash
# round-3 probe: FETCH_SIZE calibration for per-lane gathers (tools/fetch_calib.hip)
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 120 $O/../tools/fetch_calib > $O/calib_bytes.json || exit 1
i=0
for c in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $c -f csv -d $O/calib_p$i -o run -- $O/../tools/fetch_calib > $O/calib_p$i.log 2>&1 || exit 1
  i=$((i+1))
done
