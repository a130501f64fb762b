#!/usr/bin/env python3
"""PMC counters of the fused kernel per BASELINE config with rocprofv3, one --pmc
pass per counter group (MI355X_MICROARCH.md "HBM" / "rocprofv3 PMC slots"), merged
into a copy of profiles/traffic.json (read by bench.py's roofline) plus the raw
per-config counters <tag>_pmc_<config>.json, all written to gpurun_out/profiles_<tag>/
(the box returns only gpurun_out/; copy the files into profiles/ afterwards).

  FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reads exactly half
  the bytes of a wide coalesced streaming read (the guide's correction: double
  it).  Calibrated for the traversal's gathers (tools/fetch_calib.hip,
  profiles/r3_fetch_calib/): per-lane 128-B line gathers also read half (x2),
  per-lane 64-B gathers read exactly (x1, and the HBM moves 64 B: a 64-B gather
  over distinct lines takes half the time of the 128-B one).  A kernel mixing
  both (BVH nodes 128 B, leaf records 64 B) lies between the raw and the
  corrected figure; both are recorded.  Counters are collected in runs of their own
  (kernel-trace only), never combined with sys/runtime tracing.

usage (on the GPU box, from the repo root):
  python3 tools/pmc_traffic.py TAG C2 C3 C4 C5
"""
import csv
import glob
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = {"C2": ("cornell", 800, 1024), "C3": ("book1", 1200, 512),
           "C4": ("book2", 800, 4096), "C5": ("model", 1920, 1024)}
PASSES = [
    ["FETCH_SIZE"],
    ["WRITE_SIZE"],
    ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
     "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"],
    ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
     "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM"],
    ["GRBM_GUI_ACTIVE", "GRBM_COUNT"],
    # the dynamic VALU mix (round 6): per-type instruction counts, for the issue-cost model
    # beside the counter-measured VALU busy
    ["SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32",
     "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT",
     "SQ_INSTS_VALU_FMA_F64"],
    ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64",
     "SQ_INST_CYCLES_SALU", "SQ_INST_CYCLES_SMEM", "SQ_INSTS_LDS", "SQ_ACTIVE_INST_SCA",
     "SQ_ACTIVE_INST_MISC"],
]
# PMC_SET=mem: the vector-memory path (address unit, L1, L2), for reading what binds
# traversal; written to <tag>_pmcmem_<config>.json only (traffic.json is untouched)
PASSES_MEM = [
    ["TA_TA_BUSY_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum"],
    ["TA_DATA_STALLED_BY_TC_CYCLES_sum", "TA_FLAT_READ_WAVEFRONTS_sum"],
    ["TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum", "TCP_TCR_TCP_STALL_CYCLES_sum",
     "TCP_PENDING_STALL_CYCLES_sum"],
    ["TCP_TCC_READ_REQ_LATENCY_sum", "TCP_TCP_TA_DATA_STALL_CYCLES_sum", "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"],
    ["TCC_HIT_sum", "TCC_MISS_sum"],
    ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_DRAM_sum"],
    ["TD_TD_BUSY_sum", "TD_TC_STALL_sum", "GRBM_GUI_ACTIVE", "GRBM_COUNT"],
    ["SQ_INSTS_VMEM", "SQ_INST_LEVEL_VMEM", "SQ_INSTS_FLAT", "SQ_WAIT_INST_LDS", "SQ_INSTS_VALU",
     "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY"],
]
MEM = os.environ.get("PMC_SET") == "mem"
if MEM:
    PASSES = PASSES_MEM


def run_pass(tag, counters, bench_args):
    outdir = os.path.join(REPO, "gpurun_out", f"pmc_{tag}")
    cmd = ["rocprofv3", "--kernel-trace", "--pmc", *counters, "-f", "csv", "-d", outdir, "-o", "run",
           "--", sys.executable, os.path.join(REPO, "bench.py"), "--no-cpu-baseline",
           "--no-extra-configs", *bench_args]
    env = dict(os.environ, TMPDIR="/tmp")
    r = subprocess.run(["timeout", "-k", "10", "300", *cmd], cwd="/tmp", env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise SystemExit(f"rocprofv3 pass {counters} failed ({r.returncode}):\n{r.stdout[-3000:]}")
    vals = {}  # kernel -> counter -> dispatch -> value
    for fn in glob.glob(os.path.join(outdir, "**", "*counter_collection*.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                k, c = row.get("Kernel_Name", ""), row.get("Counter_Name", "")
                d = row.get("Dispatch_Id", "0")
                vals.setdefault(k, {}).setdefault(c, {}).setdefault(d, 0.0)
                vals[k][c][d] += float(row.get("Counter_Value", "nan"))
    return vals


def short(name):
    for key in ("k_fused", "k_extend", "k_shade", "k_resolve", "k_init"):
        if key in name:
            return key
    return None


def collect(tag, cfg):
    scene, width, spp = CONFIGS[cfg]
    bench_args = ["--scene", scene, "--width", str(width), "--spp", str(spp),
                  "--steps", "1", "--warmup", "1"]
    merged = {}
    for i, counters in enumerate(PASSES):
        for k, cs in run_pass(f"{tag}_{cfg}_p{i}", counters, bench_args).items():
            s = short(k)
            if not s:
                continue
            for c, per_disp in cs.items():
                xs = list(per_disp.values())
                merged.setdefault(s, {})[c] = {"per_launch_mean": sum(xs) / len(xs),
                                               "launches": len(xs)}
    res = {}
    for k, cs in merged.items():
        g = {c: v["per_launch_mean"] for c, v in cs.items()}
        e = {"counters_per_launch": g, "launches": max(v["launches"] for v in cs.values())}
        if "FETCH_SIZE" in g and "WRITE_SIZE" in g:
            e["fetch_bytes_raw"] = g["FETCH_SIZE"] * 1024
            e["write_bytes"] = g["WRITE_SIZE"] * 1024
            # gfx950 correction from MI355X_MICROARCH.md (exact for wide streaming reads)
            e["hbm_bytes_per_launch"] = (2 * g["FETCH_SIZE"] + g["WRITE_SIZE"]) * 1024
            e["hbm_bytes_per_launch_uncorrected"] = (g["FETCH_SIZE"] + g["WRITE_SIZE"]) * 1024
        if "SQ_INSTS_VALU" in g:
            e["valu_insts_per_launch"] = g["SQ_INSTS_VALU"]
            e["salu_insts_per_launch"] = g.get("SQ_INSTS_SALU")
        if "SQ_WAIT_ANY" in g and "SQ_WAVE_CYCLES" in g:
            e["wait_frac_of_wave_cycles"] = g["SQ_WAIT_ANY"] / max(g["SQ_WAVE_CYCLES"], 1)
        if "SQ_ACTIVE_INST_VALU" in g and "SQ_WAVE_CYCLES" in g:
            e["valu_active_frac_of_wave_cycles"] = g["SQ_ACTIVE_INST_VALU"] / max(g["SQ_WAVE_CYCLES"], 1)
        if "SQ_ACTIVE_INST_VALU" in g and "GRBM_GUI_ACTIVE" in g:
            # counter-measured SIMD VALU busy (bench.py roofline.valu_busy): SQ_ACTIVE_INST_VALU
            # counts quad-cycles (4 cycles) a wave spends on VALU instructions, summed over
            # waves; the SIMD-32 pipe retires a wave64 instruction every 2 cycles with two or
            # more waves issuing (one wave alone: every 4, MI355X_MICROARCH.md), so busy SIMD
            # cycles = ACTIVE_INST_VALU x 4 / 2, over 1,024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs
            e["valu_active_quads_per_launch"] = g["SQ_ACTIVE_INST_VALU"]
            e["grbm_gui_active_per_launch"] = g["GRBM_GUI_ACTIVE"]
            e["valu_busy_counter"] = (g["SQ_ACTIVE_INST_VALU"] * 2.0) / (1024 * g["GRBM_GUI_ACTIVE"] / 8)
        mix = {k[len("SQ_INSTS_VALU_"):].lower(): v for k, v in g.items()
               if k.startswith("SQ_INSTS_VALU_")}
        if mix and "SQ_INSTS_VALU" in g:
            mix["other"] = g["SQ_INSTS_VALU"] - sum(mix.values())  # moves, logic, compares, ...
            e["valu_mix_per_launch"] = mix
        res[k] = e
    return scene, bench_args, res


def main():
    sys.path.insert(0, REPO)
    import go_raytracer_amd as rt
    rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)
    tag, cfgs = sys.argv[1], sys.argv[2:] or list(CONFIGS)
    try:
        with open(os.path.join(REPO, "profiles", "traffic.json")) as f:
            db = json.load(f)
    except (OSError, ValueError):
        db = {}
    out_dir = os.path.join(REPO, "gpurun_out", f"profiles_{tag}")
    os.makedirs(out_dir, exist_ok=True)
    tpath = os.path.join(out_dir, "traffic.json")
    db["_source"] = ("tools/pmc_traffic.py: 7 separate --pmc passes per config, kernel-trace "
                     "only; FETCH_SIZE doubled (MI355X_MICROARCH.md gfx950 correction); raw "
                     "counters in profiles/<tag>_pmc_<config>.json")
    for cfg in cfgs:
        scene, bench_args, res = collect(tag, cfg)
        _, cam, _, _ = rt.demo_scene(scene)
        cam.Width, cam.SamplesPerPixel = CONFIGS[cfg][1], CONFIGS[cfg][2]
        if scene == "book1":
            cam.AspectRatio = 1.5
        d = cam.derived()
        key = f"{scene}:{d.width}x{d.height}x{d.spp_sqrt ** 2}"
        raw = os.path.join(out_dir, f"{tag}_pmc{'mem' if MEM else ''}_{cfg}.json")
        with open(raw, "w") as f:
            json.dump({"config": cfg, "key": key, "bench_args": bench_args, "kernels": res}, f,
                      indent=1)
        if MEM:
            print(cfg, key, json.dumps(res.get("k_fused", {}).get("counters_per_launch")), flush=True)
            continue
        db[key] = {k: {kk: v for kk, v in e.items() if kk != "counters_per_launch"}
                   for k, e in res.items()}
        for e in db[key].values():
            e["_source"] = f"profiles/{tag}_pmc_{cfg}.json"
        with open(tpath, "w") as f:
            json.dump(db, f, indent=1)
        print(cfg, key, json.dumps(db[key].get("k_fused", {})), flush=True)


if __name__ == "__main__":
    main()
