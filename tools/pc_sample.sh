export TMPDIR=/tmp
R=$PWD
cd /tmp && timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d $R/gpurun_out/pcs -o run -- python3 $R/tools/gpu_probe.py cornell 800 256 fused > $R/gpurun_out/pcs.log 2>&1
echo rc $?
tail -5 $R/gpurun_out/pcs.log
ls -la $R/gpurun_out/pcs/* | head
