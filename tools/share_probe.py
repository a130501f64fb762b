#!/usr/bin/env python3
"""Per-rank share timing on one GPU (dev tool): the C2 render of rank 0 of N
(rows r % N == 0) for N = 1, 2, 4, 8, through the bench's device-output path.
Implied strong-scaling efficiency = t(1) / (N * t(N)) ignores the all_gather
(< 1 ms over xGMI for C2).  usage: python3 tools/share_probe.py [scene width spp]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import go_raytracer_amd as rt  # noqa: E402

rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)

scene = sys.argv[1] if len(sys.argv) > 1 else "cornell"
width = int(sys.argv[2]) if len(sys.argv) > 2 else 800
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
t, cam, w, l = rt.demo_scene(scene)
cam.Width, cam.SamplesPerPixel = width, spp
d = cam.derived()
stream = torch.cuda.current_stream()
base = None
with rt.Scene(t, w, l) as sc:
    for n in (1, 2, 4, 8):
        rows = (d.height + n - 1) // n
        buf = torch.zeros((rows, d.width, 3), dtype=torch.float32, device="cuda")
        for _ in range(2):
            sc.render_device(cam, buf.data_ptr(), nranks=n, stream=stream.cuda_stream)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            st = sc.render_device(cam, buf.data_ptr(), nranks=n, stream=stream.cuda_stream,
                                  profile=True)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        tm = sorted(ts)[len(ts) // 2]
        base = base or tm
        print(json.dumps({"scene": scene, "nranks": n, "ms_wall": round(tm * 1e3, 3),
                          "ms_kernel": round(st["ms_fused"], 3), "chunk": st["chunk_samples"],
                          "implied_eff": round(base / (n * tm), 4)}), flush=True)
