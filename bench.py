#!/usr/bin/env python3
"""bench.py — Msamples/s of the HIP path tracer on BASELINE.json's config C2.

Workload (a "step"): one full render of the Cornell box (main.go:278-320) at
800x800 with 1024 samples per pixel (32x32 strata, camera.go:211-213), MaxDepth
50 = 655.36 M camera samples, rows interleaved across ranks (row r -> rank
r % N) and gathered to every rank with one RCCL all_gather over xGMI.  The scene
is uploaded to HBM during warmup; the timed region holds only render + gather.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Prints one JSON line (rank 0).  See DESIGN.md "Measurement" for the roofline
model (SURVEY.md §8(d) algorithmic bytes) and the CPU baseline definition.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# SURVEY.md §8(d) / BASELINE.md algorithmic bytes: Bytes = 164*S + 48*N + 15*W*H
B_PER_SEG = 164
B_PER_SAMPLE = 48
B_PER_PIXEL = 15
EXTEND_B_PER_SEG = 44        # the extend kernel's share: ray 28 read + hit 16 written
SHADE_B_PER_SEG = 120        # shade's share: hit 16 + ray 28 + key 8 read, ray 28 + key 8 +
#                              weight 12 written, queue 8, fold re-read 12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--width", type=int, default=800)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--mode", default="auto", choices=["auto", "fused", "wavefront"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline work")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per launch (tools/pmc_traffic.py)")
    return ap.parse_args()


def cpu_baseline(tree, world, lights, cam, target_s):
    """The oracle (C++ fp64 restatement of the Go CPU path) on a bounded,
    row-interleaved sample of the same image at full spp."""
    from oracle import pyoracle
    threads = min(16, os.cpu_count() or 1)
    d = cam.derived()
    # calibrate on one row, then pick a row stride that gives ~target_s of work
    _, st = pyoracle.render(tree, world, lights, cam, seed=1, threads=threads, rank=0,
                            nranks=d.height, max_rows=1)
    rate = st["samples"] / max(st["seconds"], 1e-6)
    rows_wanted = max(1, int(target_s * rate / (d.width * d.spp_sqrt ** 2)))
    stride = max(1, d.height // rows_wanted)
    _, st = pyoracle.render(tree, world, lights, cam, seed=1, threads=threads, rank=0,
                            nranks=stride)
    rows = len(range(0, d.height, stride))
    return {"value": st["samples"] / st["seconds"] / 1e6, "unit": "Msamples/s",
            "cores": threads, "kind": "port",
            "sample": f"every {stride}th row ({rows} rows x {d.width} px) of the same image at "
                      f"full {d.spp_sqrt ** 2} spp, {st['samples']} samples in "
                      f"{st['seconds']:.1f} s, {threads} threads"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import go_raytracer_amd as rt

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world_size != args.gpus and not (world_size == 1 and args.gpus == 1):
        if world_size == 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world_size > 1:
        dist.init_process_group("nccl", device_id=dev)

    t_build0 = time.perf_counter()
    tree, cam, w, l = rt.demo_scene(args.scene)
    cam.Width = args.width
    cam.SamplesPerPixel = args.spp
    if args.scene == "book1":
        cam.AspectRatio = 1.5  # 1200x800 needs aspect 1.5
    d = cam.derived()
    H, W = d.height, d.width
    rows_per = (H + world_size - 1) // world_size
    rows_mine = len(range(rank, H, world_size))
    buf = torch.zeros((rows_per, W, 3), dtype=torch.float32, device=dev)
    gathered = torch.zeros((world_size * rows_per, W, 3), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    scene = rt.Scene(tree, w, l)
    t_build = time.perf_counter() - t_build0

    def step(profile):
        st = scene.render_device(cam, buf.data_ptr(), seed=args.seed, device=local_rank,
                                 rank=rank, nranks=world_size, profile=profile,
                                 stream=stream.cuda_stream, mode=args.mode)
        if world_size > 1:
            dist.all_gather_into_tensor(gathered, buf)
        return st

    t_first, t_first0 = None, time.perf_counter()
    for i in range(args.warmup):
        step(False)
        if i == 0:
            torch.cuda.synchronize()
            t_first = time.perf_counter() - t_first0
    torch.cuda.synchronize()
    if world_size > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = [step(True) for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world_size > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    samples = torch.tensor([sum(s["samples"] for s in stats)], dtype=torch.float64, device=dev)
    if world_size > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(samples, op=dist.ReduceOp.SUM)
    elapsed = t.item()
    total_samples = samples.item()

    if rank == 0:
        seg = sum(s["segments"] for s in stats)
        smp = sum(s["samples"] for s in stats)
        pix = sum(s["rows"] for s in stats) * W
        ms_ext = sum(s["ms_extend"] for s in stats)
        ms_sh = sum(s["ms_shade"] for s in stats)
        ms_fu = sum(s["ms_fused"] for s in stats)
        n_ext = sum(s["n_extend_launches"] for s in stats)
        n_sh = sum(s["n_shade_launches"] for s in stats)
        mode = {1: "wavefront", 2: "fused"}[stats[0]["mode"]]
        total_bytes = seg * B_PER_SEG + smp * B_PER_SAMPLE + pix * B_PER_PIXEL
        if mode == "fused":
            # one persistent launch per step does all of the path's work
            kernels = {"k_fused": {"launches": len(stats), "avg_ms": ms_fu / len(stats),
                                   "alg_bytes_per_launch": total_bytes / len(stats),
                                   "achieved_GBs": total_bytes / max(ms_fu, 1e-9) / 1e6}}
        else:
            ext_bytes = seg * EXTEND_B_PER_SEG
            sh_bytes = seg * SHADE_B_PER_SEG + smp * B_PER_SAMPLE + pix * B_PER_PIXEL
            kernels = {
                "k_extend": {"launches": n_ext, "avg_ms": ms_ext / max(n_ext, 1),
                             "alg_bytes_per_launch": ext_bytes / max(n_ext, 1),
                             "achieved_GBs": ext_bytes / max(ms_ext, 1e-9) / 1e6},
                "k_shade": {"launches": n_sh, "avg_ms": ms_sh / max(n_sh, 1),
                            "alg_bytes_per_launch": sh_bytes / max(n_sh, 1),
                            "achieved_GBs": sh_bytes / max(ms_sh, 1e-9) / 1e6},
            }
        dom = max(kernels, key=lambda k: kernels[k]["avg_ms"] * kernels[k]["launches"])
        traffic = None
        if os.path.exists(args.traffic):
            try:
                with open(args.traffic) as f:
                    tr = json.load(f)
                key = f"{args.scene}:{W}x{H}x{d.spp_sqrt ** 2}"
                if key in tr and dom in tr[key]:
                    traffic = tr[key][dom]["hbm_bytes_per_launch"]
            except (OSError, ValueError, KeyError):
                traffic = None
        k = kernels[dom]
        roofline = {"bound": "hbm", "kernel": dom, "achieved": round(k["achieved_GBs"], 2),
                    "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(k["achieved_GBs"] / PEAK_HBM_GBS, 5), "traffic": traffic,
                    "alg_bytes_model": "164*segments + 48*samples + 15*pixels (SURVEY §8d)",
                    "kernels": {n: {kk: round(v, 4) for kk, v in kv.items()}
                                for n, kv in kernels.items()}}
        # end-to-end wall clock around the render (the metric's "+ wall-clock"):
        # scene build on the host (demo scene + flatten + BVH), the first step
        # (scene upload + render), and the P3 text of the image built on the GPU
        from go_raytracer_amd import shard
        torch.cuda.synchronize()
        t_ppm0 = time.perf_counter()
        ppm = rt.format_ppm_device(buf if world_size == 1 else
                                   shard.assemble(gathered, H, world_size))
        t_ppm = time.perf_counter() - t_ppm0
        wall = {"scene_build_s": round(t_build, 3),
                "first_step_s": None if t_first is None else round(t_first, 3),
                "render_step_s": round(elapsed / args.steps, 4),
                "ppm_on_device_s": round(t_ppm, 4), "ppm_bytes": len(ppm)}
        cpu = None
        if world_size == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(tree, w, l, cam, args.cpu_seconds)
        value = total_samples / elapsed / 1e6
        line = {
            "metric": "Msamples/sec (pixels×spp/s) + wall-clock, Cornell Box 800×800×1024spp",
            "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world_size,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"{args.scene} {W}x{H} {d.spp_sqrt ** 2}spp maxdepth {d.max_depth} "
                                   f"(BASELINE configs[1], main.go cornellBox)",
                       "scene": args.scene, "width": W, "height": H, "spp": d.spp_sqrt ** 2,
                       "max_depth": d.max_depth, "parallelism": f"rows%{world_size}",
                       "mode": mode, "path_slots": stats[0]["path_slots"],
                       "segments_per_sample": round(seg / max(smp, 1), 4)},
            "roofline": roofline, "cpu_baseline": cpu, "wall_clock": wall,
        }
        if cpu:
            line["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        print(json.dumps(line), flush=True)
    scene.close()
    if world_size > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
