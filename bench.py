#!/usr/bin/env python3
"""bench.py — Msamples/s of the HIP path tracer on BASELINE.json's configs.

Headline workload (a "step"): one full render of the Cornell box (configs[1] = C2,
main.go:278-320) at 800x800 with 1024 samples per pixel (32x32 strata,
camera.go:211-213), MaxDepth 50 = 655.36 M camera samples, rows interleaved across
ranks (row r -> rank r % N, camera.go:119-122) and gathered to rank 0 with one
RCCL gather over xGMI.  The scene is uploaded to HBM during warmup; the timed region
holds only render + gather.

After the headline, `extra_configs` times BASELINE configs C3 (book1), C4 (book2)
and C5 (model) the same way (row shares on every rank, barrier + max over ranks),
each with its own roofline, so every GPU config has a measured line.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Prints one JSON line (rank 0).  Roofline (DESIGN.md "Roofline"): the fused kernel
keeps path state in registers and LDS, so what binds it is VALU instruction
issue, not HBM.  `roofline` reports the counter-backed VALU-issue fraction
(SQ_INSTS_VALU per launch from a rocprofv3 --pmc pass, profiles/traffic.json,
divided by the live kernel time and the chip's 1228.8 G wave-instructions/s),
next to the counter-backed HBM fraction (FETCH_SIZE x2 + WRITE_SIZE per launch)
and SURVEY.md §8(d)'s wavefront-state model (segments x 164 B ...), which is a
throughput index for a pipeline this kernel does not run.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# VALU issue: 256 CUs x 4 SIMDs x 2.4 GHz, one wave64 VALU instruction per SIMD per
# 2 cycles (SIMD-32, MI355X_MICROARCH.md "Execution model") = 1228.8 G wave-instr/s
PEAK_VALU_GIPS = 256 * 4 * 2.4 / 2
# SURVEY.md §8(d) / BASELINE.md algorithmic bytes: Bytes = 164*S + 48*N + 15*W*H
B_PER_SEG = 164
B_PER_SAMPLE = 48
B_PER_PIXEL = 15
EXTEND_B_PER_SEG = 44        # the extend kernel's share: ray 28 read + hit 16 written
SHADE_B_PER_SEG = 120        # shade's share: hit 16 + ray 28 + key 8 read, ray 28 + key 8 +
#                              weight 12 written, queue 8, fold re-read 12

# BASELINE.json configs timed after the headline (name, scene, width, spp, steps)
EXTRA = [("C3", "book1", 1200, 512, 3),   # main.go:19-91, aspect 1.5 -> 1200x800, 484 spp
         ("C4", "book2", 800, 4096, 1),   # main.go:94-174
         ("C5", "model", 1920, 1024, 2)]  # main.go:371-409, 1M-triangle substitute mesh


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 128 steps of C2: a ~5.4 s timed region (the driver samples GPU activity during it)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--width", type=int, default=800)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--mode", default="auto", choices=["auto", "fused", "wavefront"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra-configs", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline work")
    ap.add_argument("--devices", default=None,
                    help="single-process multi-GPU: comma-separated HIP devices rendered through "
                         "rt_render_multi (rows r on devices[r %% n], peer-gathered to devices[0]); "
                         "the north_star's Go-host path, no torchrun")
    ap.add_argument("--gather", default="peer", choices=["peer", "rccl"],
                    help="--devices mode: collect the shares on devices[0] by peer copies or by "
                         "one RCCL ncclGather (RT_FLAG_GATHER_RCCL; distinct devices)")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "traffic.json"),
                    help="PMC counters per launch (tools/pmc_traffic.py)")
    ap.add_argument("--no-multi-check", action="store_true",
                    help="torchrun jobs: skip rank 0's rt_render_multi check over distinct devices")
    ap.add_argument("--multi-device-check", type=int, default=0, metavar="N",
                    help=argparse.SUPPRESS)  # child-process mode of that check
    return ap.parse_args()


def multi_device_check(ndev):
    """rt_render_multi over DISTINCT devices 0..ndev-1 -- the Go-host path (peer access, peer
    copies into devices[0], one scene upload per device, the RCCL ncclGather option) --
    compared bit for bit with a one-device rt_render of the same image.  A torchrun job on a
    multi-GPU node runs it in a child process of rank 0 after the timed regions, so a
    failure cannot cost the bench line; a one-GPU box has no distinct devices to use."""
    import numpy as np
    import go_raytracer_amd as rt
    res = {"devices": list(range(ndev))}
    t, cam, w, l = rt.demo_scene("cornell")
    cam.Width, cam.SamplesPerPixel = 96, 16
    with rt.Scene(t, w, l) as sc:
        ref, _ = sc.render(cam, seed=5, device=0)
        for name, devs, rccl in (("peer", list(range(ndev)), False),
                                 ("peer_reversed", list(range(ndev))[::-1], False),
                                 ("rccl", list(range(ndev)), True)):
            t0 = time.perf_counter()
            img, _ = sc.render_multi(cam, devs, seed=5, rccl=rccl)
            res[name] = {"bitwise": bool(np.array_equal(ref.view(np.uint32), img.view(np.uint32))),
                         "s": round(time.perf_counter() - t0, 3)}
    return res


def run_multi_device_check(ndev):
    import subprocess
    try:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--multi-device-check",
                            str(ndev)], capture_output=True, text=True, timeout=180)
        out = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode == 0 and out:
            return json.loads(out[-1])
        return {"devices": list(range(ndev)), "error": f"exit {r.returncode}: {r.stderr[-300:]}"}
    except Exception as e:  # timeout or spawn failure
        return {"devices": list(range(ndev)), "error": str(e)[:300]}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(tree, world, lights, cam, target_s):
    """The oracle (C++ fp64 restatement of the Go CPU path, camera.go:112-153) on
    bounded row-interleaved samples of the same image at full spp: with the box's
    CPU share (16 threads: the GPU box's allotment, OMP_NUM_THREADS) and with one
    thread (the reference's -N=1, syncRenderer camera.go:135-153).  The whole
    host's rate is stated as the single-thread rate x nproc (ideal scaling, an
    upper bound for the Go path).  Also times configs[0] (C1, quads 400x400x64,
    -N=1, main.go:220-247) in full."""
    from oracle import pyoracle
    import go_raytracer_amd as rt
    nproc = os.cpu_count() or 1
    threads = min(16, nproc)
    d = cam.derived()
    px_row = d.width * d.spp_sqrt ** 2

    def sample(nthreads, seconds, k):
        # calibrate on k rows spread over the image (row cost varies a lot: the
        # Cornell light), then take every stride-th row for ~`seconds` of work
        _, st = pyoracle.render(tree, world, lights, cam, seed=1, threads=nthreads, rank=0,
                                nranks=max(1, d.height // k), max_rows=k)
        rate = st["samples"] / max(st["seconds"], 1e-6)
        rows_wanted = max(1, int(seconds * rate / px_row))
        stride = max(1, d.height // rows_wanted)
        _, st = pyoracle.render(tree, world, lights, cam, seed=1, threads=nthreads, rank=0,
                                nranks=stride)
        return st, stride, len(range(0, d.height, stride))

    st, stride, rows = sample(threads, target_s, 32)
    st1, stride1, rows1 = sample(1, target_s / 3, 8)
    v16 = st["samples"] / st["seconds"] / 1e6
    v1 = st1["samples"] / st1["seconds"] / 1e6
    # configs[0]: C1 quads 400x400, 64 spp, one thread, the whole image
    tq, camq, wq, lq = rt.demo_scene("quads")
    camq.Width, camq.SamplesPerPixel = 400, 64
    _, stq = pyoracle.render(tq, wq, lq, camq, seed=1, threads=1)
    return {"value": v16, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"every {stride}th row ({rows} rows x {d.width} px) of the same image at "
                      f"full {d.spp_sqrt ** 2} spp, {st['samples']} samples in "
                      f"{st['seconds']:.1f} s, {threads} threads (the GPU box's CPU share)",
            "single_thread": {"value": v1, "unit": "Msamples/s", "cores": 1,
                              "sample": f"every {stride1}th row ({rows1} rows), "
                                        f"{st1['samples']} samples in {st1['seconds']:.1f} s"},
            "host": {"nproc": nproc, "cpu_model": cpu_model(),
                     "extrapolated_all_cores_Msamples_s": round(v1 * nproc, 2),
                     "note": "single-thread rate x nproc: ideal scaling over every host "
                             "thread (not run: the box allots 16)"},
            "c1_plumbing": {"config": "configs[0]: quads 400x400x64, -N=1 (main.go:220-247)",
                            "samples": stq["samples"], "seconds": round(stq["seconds"], 3),
                            "Msamples_s": round(stq["samples"] / stq["seconds"] / 1e6, 3),
                            "segments_per_sample": round(stq["segments"] / stq["samples"], 4)}}


def load_traffic(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def roofline(db, key, kernel, ms, seg, smp, pix, full_smp):
    """Rooflines of one launch of `kernel` (ms = live average launch time).  The PMC
    counts are per launch over the whole image (tools/pmc_traffic.py, one GPU); a launch
    that renders a row share (multi-GPU) is charged its share of them, smp / full_smp."""
    model_bytes = seg * B_PER_SEG + smp * B_PER_SAMPLE + pix * B_PER_PIXEL
    model_gbs = model_bytes / max(ms, 1e-9) / 1e6
    pmc = db.get(key, {}).get(kernel, {})
    share = smp / full_smp if full_smp else 1.0
    valu = pmc.get("valu_insts_per_launch")
    hbm = pmc.get("hbm_bytes_per_launch")
    if valu:
        valu *= share
    if hbm:
        hbm *= share
    r = {"bound": "issue", "kernel": kernel, "achieved": None, "peak": PEAK_VALU_GIPS,
         "unit": "G VALU wave-instr/s", "frac": None, "traffic": hbm}
    if valu:
        a = valu / ms / 1e6
        r.update(achieved=round(a, 2), frac=round(a / PEAK_VALU_GIPS, 4),
                 valu_insts_per_launch=valu)
        # SIMD cycles available per VALU wave-instruction of this launch (`peak` assumes 2)
        r["simd_cycles_per_valu"] = round(4 * 256 * 2.4e6 * ms / valu, 3)
    if pmc.get("valu_busy_counter"):
        # counter-measured VALU busy of the SIMDs (tools/pmc_traffic.py): SQ_ACTIVE_INST_VALU
        # quad-cycles x 4 / 2 cycles per wave64 instruction at the SIMD-32 pipe, over the
        # SIMD cycles of the same launch (1,024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs).  It charges
        # long instructions (transcendentals, fp64) their real occupancy, so 1 - valu_busy
        # is the measured headroom of the VALU pipe; the 2-cycle `frac` prices every
        # instruction alike
        r["valu_busy"] = {"frac": round(pmc["valu_busy_counter"], 4),
                          "source": "SQ_ACTIVE_INST_VALU*4/2 / (1024*GRBM_GUI_ACTIVE/8)"}
    if hbm:
        g = hbm / ms / 1e6
        r["hbm_counter"] = {"achieved": round(g, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                            "frac": round(g / PEAK_HBM_GBS, 4),
                            "bytes_per_launch": hbm, "source": "FETCH_SIZE*2 + WRITE_SIZE"}
        lo = pmc.get("hbm_bytes_per_launch_uncorrected")
        if lo:
            # FETCH_SIZE undercounts 128-B requests by 2 but counts 64-B ones exactly
            # (profiles/r3_fetch_calib: per-lane 128-B node gathers x2, 64-B leaf records
            # x1), so the kernel's bytes lie between the uncorrected and corrected sums
            r["hbm_counter"]["bytes_per_launch_range"] = [round(lo * share), round(hbm)]
    # an index, not a roofline: no peak and no fraction (it can exceed 8 TB/s because
    # these bytes are never moved)
    r["hbm_model"] = {"index_gbs": round(model_gbs, 2), "unit": "GB/s",
                      "bytes_per_launch": model_bytes,
                      "model": "164*segments + 48*samples + 15*pixels (SURVEY §8d wavefront "
                               "state; a throughput index: the fused kernel keeps this state "
                               "in registers/LDS and does not move these bytes)"}
    if pmc.get("_source"):
        r["pmc_source"] = pmc["_source"]
    if share < 0.999:
        r["pmc_share"] = round(share, 6)
    return r


def main():
    args = parse()
    if args.multi_device_check:
        print(json.dumps(multi_device_check(args.multi_device_check)), flush=True)
        return
    import torch
    import torch.distributed as dist

    import go_raytracer_amd as rt

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    devices = [int(x) for x in args.devices.split(",")] if args.devices else None
    if devices:
        if world_size != 1:
            raise SystemExit("--devices is the single-process mode: do not launch it with torchrun")
        if len(devices) != args.gpus:
            raise SystemExit("--devices must list --gpus devices")
        local_rank = devices[0]
    elif world_size != args.gpus and not (world_size == 1 and args.gpus == 1):
        if world_size == 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run "
                             "(or use --devices for one process over N GPUs)")
    torch.cuda.set_device(local_rank)
    nshare = len(devices) if devices else 1  # row shares per launch statistic
    dev = torch.device("cuda", local_rank)
    if world_size > 1:
        dist.init_process_group("nccl", device_id=dev)
    stream = torch.cuda.current_stream(dev)
    db = load_traffic(args.traffic)

    def timed_renders(scene, cam, steps, warmup, buf, gathered, profile=True):
        """warmup + `steps` renders of this rank's share (+ all_gather), barrier and
        synchronize around the timed region; returns (max elapsed, per-step stats)."""
        def step(prof):
            if devices:  # one process: every share on its device, gathered on devices[0]
                return scene.render_multi_device(cam, devices, buf.data_ptr(), seed=args.seed,
                                                 profile=prof, mode=args.mode,
                                                 rccl=args.gather == "rccl")
            st = scene.render_device(cam, buf.data_ptr(), seed=args.seed, device=local_rank,
                                     rank=rank, nranks=world_size, profile=prof,
                                     stream=stream.cuda_stream, mode=args.mode)
            if world_size > 1:  # one RCCL gather of the row tiles to rank 0
                dist.gather(buf, list(gathered.split(buf.shape[0])) if rank == 0 else None, dst=0)
            return st
        t_first = None
        for i in range(warmup):
            t0 = time.perf_counter()
            step(False)
            if i == 0:
                torch.cuda.synchronize()
                t_first = time.perf_counter() - t0
        torch.cuda.synchronize()
        if world_size > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        stats = [step(profile) for _ in range(steps)]
        torch.cuda.synchronize()
        if world_size > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if world_size > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.item(), stats, t_first

    def buffers(d):
        if devices:  # the whole image on devices[0]
            return torch.zeros((d.height, d.width, 3), dtype=torch.float32, device=dev), None
        rows_per = (d.height + world_size - 1) // world_size
        buf = torch.zeros((rows_per, d.width, 3), dtype=torch.float32, device=dev)
        gathered = torch.zeros((world_size * rows_per, d.width, 3), dtype=torch.float32,
                               device=dev)
        return buf, gathered

    # ------------------------------------------------------------ headline (C2)
    t_build0 = time.perf_counter()
    tree, cam, w, l = rt.demo_scene(args.scene)
    cam.Width = args.width
    cam.SamplesPerPixel = args.spp
    if args.scene == "book1":
        cam.AspectRatio = 1.5  # 1200x800 needs aspect 1.5
    d = cam.derived()
    H, W = d.height, d.width
    buf, gathered = buffers(d)
    scene = rt.Scene(tree, w, l)
    t_build = time.perf_counter() - t_build0
    elapsed, stats, t_first = timed_renders(scene, cam, args.steps, args.warmup, buf, gathered)
    samples = torch.tensor([sum(s["samples"] for s in stats)], dtype=torch.float64, device=dev)
    if world_size > 1:
        dist.all_reduce(samples, op=dist.ReduceOp.SUM)
    total_samples = samples.item()
    segments = torch.tensor([sum(s["segments"] for s in stats)], dtype=torch.float64, device=dev)
    if world_size > 1:
        dist.all_reduce(segments, op=dist.ReduceOp.SUM)
    total_segments = segments.item()  # every rank's (rt_render_multi: every share's)
    line = None
    if rank == 0:
        seg = sum(s["segments"] for s in stats)
        smp = sum(s["samples"] for s in stats)
        pix = sum(s["rows"] for s in stats) * W
        mode = {1: "wavefront", 2: "fused"}[stats[0]["mode"]]
        key = f"{args.scene}:{W}x{H}x{d.spp_sqrt ** 2}"
        if mode == "fused":
            ms = sum(s["ms_fused"] for s in stats) / len(stats)
            k = len(stats) * nshare  # per device launch (the slowest share's time)
            roof = roofline(db, key, "k_fused", ms, seg / k, smp / k, pix / k,
                            W * H * d.spp_sqrt ** 2)
            roof["launches"] = len(stats)
            roof["avg_ms"] = round(ms, 4)
        else:  # the wavefront pair: the model's bytes per kernel (cross-check path)
            n_ext = sum(s["n_extend_launches"] for s in stats)
            ms_ext = sum(s["ms_extend"] for s in stats)
            ms_sh = sum(s["ms_shade"] for s in stats)
            roof = {"bound": "hbm", "kernel": "k_extend+k_shade", "unit": "GB/s",
                    "peak": PEAK_HBM_GBS, "traffic": None,
                    "achieved": round((seg * (EXTEND_B_PER_SEG + SHADE_B_PER_SEG) + smp *
                                       B_PER_SAMPLE + pix * B_PER_PIXEL) /
                                      max(ms_ext + ms_sh, 1e-9) / 1e6, 2),
                    "launches": n_ext}
            roof["frac"] = round(roof["achieved"] / PEAK_HBM_GBS, 4)
        from go_raytracer_amd import shard
        torch.cuda.synchronize()
        t_ppm0 = time.perf_counter()
        ppm = rt.format_ppm_device(buf if world_size == 1 else
                                   shard.assemble(gathered, H, world_size))
        n_gpus = len(set(devices)) if devices else world_size
        t_ppm = time.perf_counter() - t_ppm0
        value = total_samples / elapsed / 1e6
        line = {
            "metric": "Msamples/sec (pixels×spp/s) + wall-clock, Cornell Box 800×800×1024spp",
            "value": round(value, 3), "unit": "Msamples/s", "n_gpus": n_gpus,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"{args.scene} {W}x{H} {d.spp_sqrt ** 2}spp maxdepth "
                                   f"{d.max_depth} (BASELINE configs[1], main.go cornellBox)",
                       "scene": args.scene, "width": W, "height": H, "spp": d.spp_sqrt ** 2,
                       "max_depth": d.max_depth,
                       "parallelism": (f"rows%{len(devices)} in one process (rt_render_multi, "
                                       f"devices {devices}, {args.gather} gather)") if devices
                                      else f"rows%{world_size} (RCCL gather to rank 0)"
                                      if world_size > 1 else "rows%1",
                       "mode": mode, "path_slots": stats[0]["path_slots"],
                       "chunk_samples": stats[0]["chunk_samples"],
                       "segments_per_sample": round(seg / max(smp, 1), 4),
                       "Gsegments_per_s": round(total_segments / elapsed / 1e9, 3)},
            "roofline": roof,
            "wall_clock": {"scene_build_s": round(t_build, 3),
                           "first_step_s": None if t_first is None else round(t_first, 3),
                           "render_step_s": round(elapsed / args.steps, 4),
                           "ppm_on_device_s": round(t_ppm, 4), "ppm_bytes": len(ppm)},
        }
    scene.close()

    # ------------------------------------------------------- C3, C4, C5 lines
    extra = {}
    if not args.no_extra_configs:
        import tempfile
        for name, sname, width, spp, steps in EXTRA:
            setup = {}
            asset_dir = None
            if sname == "model":
                # dragon.obj is absent from the reference: its substitute is written to
                # disk first, so the timed setup loads it like the real file
                tg = time.perf_counter()
                tmp = tempfile.TemporaryDirectory()
                with open(os.path.join(tmp.name, "dragon.obj"), "wb") as f:
                    f.write(rt.substitute_mesh_obj())
                asset_dir = tmp.name
                setup["substitute_obj_written_s"] = round(time.perf_counter() - tg, 3)
            tb0 = time.perf_counter()
            t2, cam2, w2, l2 = rt.demo_scene(sname, asset_dir=asset_dir)  # LoadObj for C5
            setup["scene_tree_s"] = round(time.perf_counter() - tb0, 3)
            cam2.Width, cam2.SamplesPerPixel = width, spp
            if sname == "book1":
                cam2.AspectRatio = 1.5
            d2 = cam2.derived()
            b2, g2 = buffers(d2)
            tf = time.perf_counter()
            with rt.Scene(t2, w2, l2) as sc2:
                setup["flatten_bvh_s"] = round(time.perf_counter() - tf, 3)
                setup["bvh_builder"] = ["host SAH", "device PLOC"][sc2.info()["bvh_builder"]]
                spp_keep = cam2.SamplesPerPixel
                cam2.SamplesPerPixel = 1  # warmup: scene upload + state buffers only
                tu = time.perf_counter()
                timed_renders(sc2, cam2, 0, 1, b2, g2, profile=False)
                setup["upload_first_render_s"] = round(time.perf_counter() - tu, 3)
                tbuild = time.perf_counter() - tb0
                cam2.SamplesPerPixel = spp_keep
                el, st2, _ = timed_renders(sc2, cam2, steps, 0, b2, g2)
            tot = torch.tensor([sum(s["samples"] for s in st2)], dtype=torch.float64, device=dev)
            if world_size > 1:
                dist.all_reduce(tot, op=dist.ReduceOp.SUM)
            if rank == 0:
                seg = sum(s["segments"] for s in st2) / steps / nshare
                smp = sum(s["samples"] for s in st2) / steps / nshare
                pix = sum(s["rows"] for s in st2) / steps * d2.width / nshare
                ms = sum(s["ms_fused"] for s in st2) / steps
                key = f"{sname}:{d2.width}x{d2.height}x{d2.spp_sqrt ** 2}"
                roof = roofline(db, key, "k_fused", ms, seg, smp, pix,
                                d2.width * d2.height * d2.spp_sqrt ** 2)
                roof["avg_ms"] = round(ms, 4)
                extra[name] = {
                    "workload": f"{sname} {d2.width}x{d2.height} {d2.spp_sqrt ** 2}spp maxdepth "
                                f"{d2.max_depth}",
                    "value": round(tot.item() / el / 1e6, 3), "unit": "Msamples/s",
                    "ms_per_step": round(el / steps * 1e3, 3), "steps": steps,
                    "segments_per_sample": round(seg / max(smp, 1), 4),
                    "Gsegments_per_s_rank0": round(seg / (ms / 1e3) / 1e9, 3),
                    "tree_width": st2[0]["tree_width"], "lds_scene": st2[0]["lds_scene"],
                    "chunk_samples": st2[0]["chunk_samples"],
                    "scene_setup_s": round(tbuild, 3), "scene_setup": setup, "roofline": roof}
            del b2, g2
    if rank == 0:
        if extra:
            line["extra_configs"] = extra
        cpu = None
        if world_size == 1 and not devices and not args.no_cpu_baseline:
            tree, cam, w, l = rt.demo_scene(args.scene)
            cam.Width, cam.SamplesPerPixel = args.width, args.spp
            if args.scene == "book1":
                cam.AspectRatio = 1.5
            cpu = cpu_baseline(tree, w, l, cam, args.cpu_seconds)
        line["cpu_baseline"] = cpu
        if cpu:
            line["speedup_vs_cpu"] = round(line["value"] / cpu["value"], 1)
            line["speedup_vs_host_extrapolated"] = round(
                line["value"] / cpu["host"]["extrapolated_all_cores_Msamples_s"], 1)
        if world_size > 1 and not args.no_multi_check:
            ndev = torch.cuda.device_count()
            line["checks"] = {"render_multi_distinct_devices":
                              run_multi_device_check(min(ndev, 8)) if ndev >= 2 else
                              {"skipped": f"{ndev} visible device(s)"}}
        print(json.dumps(line), flush=True)
    if world_size > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
