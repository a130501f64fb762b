"""Per-kernel register / spill / LDS / occupancy table of rt_render.hip (gfx950).

Compiles the device side with -Rpass-analysis=kernel-resource-usage and prints one
line per kernel.  Extra hipcc flags can be passed on the command line (e.g. -DFOO=1).
"""
import re
import subprocess
import sys
import os

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "go_raytracer_amd", "csrc")


# rt_fused_sets.hip's own flags (Makefile FUSED_SETS_FLAGS)
SETS_FLAGS = ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]


def main(argv):
    srcs = [a for a in argv if a.endswith(".hip")] or ["rt_render.hip", "rt_fused_sets.hip"]
    extra = [a for a in argv if not a.endswith(".hip")]
    out = ""
    for src in srcs:
        cmd = ["/opt/rocm/bin/hipcc", "-DBRUTE_WAVES=6", "-O3", "-std=c++17", "--offload-arch=gfx950",
               "-I../../include", "-I.", "-Wno-unused-result",
               "-fno-hip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize", "--cuda-device-only", "-c", src,
               "-o", "/tmp/_kr.o", "-Rpass-analysis=kernel-resource-usage"] + extra + \
              (SETS_FLAGS if src == "rt_fused_sets.hip" else [])
        out += subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (.*?): (.*?) \[-Rpass", line)
        if not m:
            continue
        key, val = m.group(1).strip(), m.group(2).strip()
        if key == "Function Name":
            cur = {"name": val}
            rows.append(cur)
        elif cur is not None:
            cur[key] = val
    for r in rows:
        name = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
        print(f"{name[:60]:60s} vgpr {r.get('VGPRs','?'):>4s} agpr {r.get('AGPRs','?'):>3s} "
              f"spill {r.get('VGPRs Spill','?'):>3s} sgpr-spill {r.get('SGPRs Spill','?'):>4s} "
              f"lds {r.get('LDS Size [bytes/block]','?'):>6s} occ {r.get('Occupancy [waves/SIMD]','?')}")


if __name__ == "__main__":
    main(sys.argv[1:])
