#!/usr/bin/env python3
"""Collect PMC counters for bench.py's kernels with rocprofv3, one --pmc pass per
counter group (MI355X_MICROARCH.md "HBM" / "rocprofv3 PMC slots"), and write
per-launch HBM traffic + SQ activity to a JSON file.

  FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reads exactly half
  the bytes of a wide coalesced streaming read (the guide's correction: double
  it); for other access widths it is uncalibrated, so both the raw and the
  corrected figure are recorded.  Counters are collected in runs of their own
  (kernel-trace only), never combined with sys/runtime tracing.

usage (on the GPU box, from the repo root):
  python3 tools/pmc_traffic.py OUT.json [bench args ...]
"""
import csv
import glob
import json
import os
import subprocess
import sys

PASSES = [
    ["FETCH_SIZE"],
    ["WRITE_SIZE"],
    ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
     "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"],
    ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
     "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM"],
    ["GRBM_GUI_ACTIVE", "GRBM_COUNT"],
]


def run_pass(repo, tag, counters, bench_args):
    outdir = os.path.join(repo, "gpurun_out", f"pmc_{tag}")
    cmd = ["rocprofv3", "--kernel-trace", "--pmc", *counters, "-f", "csv", "-d", outdir, "-o", "run",
           "--", sys.executable, os.path.join(repo, "bench.py"), "--no-cpu-baseline", *bench_args]
    env = dict(os.environ, TMPDIR="/tmp")
    r = subprocess.run(["timeout", "-k", "10", "600", *cmd], cwd="/tmp", env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise SystemExit(f"rocprofv3 pass {counters} failed ({r.returncode}):\n{r.stdout[-3000:]}")
    files = glob.glob(os.path.join(outdir, "**", "*counter_collection*.csv"), recursive=True)
    vals = {}  # kernel -> counter -> [per dispatch]
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                k = row.get("Kernel_Name", "")
                c = row.get("Counter_Name", "")
                v = float(row.get("Counter_Value", "nan"))
                d = row.get("Dispatch_Id", "0")
                vals.setdefault(k, {}).setdefault(c, {}).setdefault(d, 0.0)
                vals[k][c][d] += v
    return vals


def short(name):
    for key in ("k_fused", "k_extend", "k_shade", "k_resolve", "k_init"):
        if key in name:
            return key
    return None


def main():
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = sys.argv[1]
    bench_args = sys.argv[2:] or ["--steps", "1", "--warmup", "1"]
    merged = {}
    for i, counters in enumerate(PASSES):
        vals = run_pass(repo, f"p{i}", counters, bench_args)
        for k, cs in vals.items():
            s = short(k)
            if not s:
                continue
            for c, per_disp in cs.items():
                xs = list(per_disp.values())
                merged.setdefault(s, {})[c] = {"per_launch_mean": sum(xs) / len(xs), "launches": len(xs)}
    res = {}
    for k, cs in merged.items():
        g = {c: v["per_launch_mean"] for c, v in cs.items()}
        fetch_kb = g.get("FETCH_SIZE")
        write_kb = g.get("WRITE_SIZE")
        entry = {"counters_per_launch": g,
                 "launches": max(v["launches"] for v in cs.values())}
        if fetch_kb is not None and write_kb is not None:
            entry["fetch_bytes_raw"] = fetch_kb * 1024
            entry["write_bytes"] = write_kb * 1024
            # gfx950 correction from MI355X_MICROARCH.md (exact for wide streaming reads)
            entry["hbm_bytes_per_launch"] = (2 * fetch_kb + write_kb) * 1024
            entry["hbm_bytes_per_launch_uncorrected"] = (fetch_kb + write_kb) * 1024
        if "SQ_INSTS_VALU" in g and "SQ_WAVES" in g:
            entry["valu_insts_per_wave"] = g["SQ_INSTS_VALU"] / max(g["SQ_WAVES"], 1)
        if "SQ_ACTIVE_INST_VALU" in g and "SQ_WAVE_CYCLES" in g:
            entry["valu_active_frac_of_wave_cycles"] = g["SQ_ACTIVE_INST_VALU"] / max(g["SQ_WAVE_CYCLES"], 1)
        if "SQ_WAIT_ANY" in g and "SQ_WAVE_CYCLES" in g:
            entry["wait_frac_of_wave_cycles"] = g["SQ_WAIT_ANY"] / max(g["SQ_WAVE_CYCLES"], 1)
        res[k] = entry
    with open(out, "w") as f:
        json.dump({"bench_args": bench_args, "kernels": res}, f, indent=1)
    print(json.dumps(res, indent=1)[:4000])


if __name__ == "__main__":
    main()
