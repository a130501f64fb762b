#!/usr/bin/env python3
"""Fixed-cost / tail probe of the fused kernel (dev tool): C2 rank-0 shares under
chunk-size and grab-size knobs, and the kernel time against spp at one rank."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import go_raytracer_amd as rt  # noqa: E402

t, cam, w, l = rt.demo_scene("cornell")
cam.Width = 800
stream = torch.cuda.current_stream()


def run(sc, n, chunk=0, grab=None, spp=1024, reps=5):
    cam.SamplesPerPixel = spp
    d = cam.derived()
    if grab is None:
        os.environ.pop("RT_GRAB_MIN", None)
    else:
        os.environ["RT_GRAB_MIN"] = str(grab)
    buf = torch.zeros(((d.height + n - 1) // n, d.width, 3), dtype=torch.float32, device="cuda")
    sc.render_device(cam, buf.data_ptr(), nranks=n, chunk=chunk, stream=stream.cuda_stream)
    ks = []
    for _ in range(reps):
        st = sc.render_device(cam, buf.data_ptr(), nranks=n, chunk=chunk,
                              stream=stream.cuda_stream, profile=True)
        ks.append(st["ms_fused"])
    k = sorted(ks)[reps // 2]
    print(json.dumps({"nranks": n, "spp": spp, "chunk": st["chunk_samples"], "grab_min": grab,
                      "ms_kernel": round(k, 3), "Gsamples_s": round(st["samples"] / k / 1e6, 3)}),
          flush=True)


with rt.Scene(t, w, l) as sc:
    for spp in (64, 256, 1024):
        run(sc, 1, spp=spp)
    for chunk in (0, 4, 8, 16, 32):
        run(sc, 8, chunk=chunk)
    for grab in (1, 8, 16, 32, 64, 128):
        run(sc, 8, grab=grab)
    for grab in (16, 64):
        run(sc, 1, grab=grab)
