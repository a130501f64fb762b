#!/usr/bin/env python3
"""PMC counters of the fused kernel for any probe config (dev tool; one --pmc pass
per counter group, kernel-trace only, as MI355X_MICROARCH.md prescribes):
  python3 tools/pmc_probe.py OUT.json "C1 C2,C3 C4" scene width spp"""
import csv, glob, json, os, subprocess, sys

repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out, groups, probe = sys.argv[1], [g.split() for g in sys.argv[2].split(",")], sys.argv[3:]
res = {}
for gi, counters in enumerate(groups):
    d = os.path.join(repo, "gpurun_out", f"pmcp_{gi}")
    cmd = ["timeout", "-k", "10", "600", "rocprofv3", "--kernel-trace", "--pmc", *counters, "-f", "csv",
           "-d", d, "-o", "run", "--", sys.executable, os.path.join(repo, "tools", "gpu_probe.py"),
           *probe, "fused"]
    r = subprocess.run(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True)
    if r.returncode:
        raise SystemExit(f"pass {counters} failed ({r.returncode}):\n{r.stdout[-3000:]}")
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for row in csv.DictReader(open(fn)):
            if "k_fused" not in row.get("Kernel_Name", ""):
                continue
            key = (row["Counter_Name"], row.get("Dispatch_Id", "0"))
            res[key] = res.get(key, 0.0) + float(row["Counter_Value"])
# last dispatch (the timed render) per counter
last = {}
for (c, disp), v in res.items():
    if c not in last or int(disp) > last[c][0]:
        last[c] = (int(disp), v)
final = {c: v for c, (_, v) in last.items()}
json.dump({"probe": probe, "counters": final}, open(out, "w"), indent=1)
print(json.dumps(final, indent=1))
