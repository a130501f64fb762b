#!/usr/bin/env python3
"""Grab-size sweep at 1 and 8 ranks for the C2 share (dev tool)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import go_raytracer_amd as rt  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "cur"
grabs = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [32, 64, 128, 256]
t, cam, w, l = rt.demo_scene("cornell")
cam.Width, cam.SamplesPerPixel = 800, 1024
d = cam.derived()
stream = torch.cuda.current_stream()
with rt.Scene(t, w, l) as sc:
    for n in (1, 2, 4, 8):
        buf = torch.zeros(((d.height + n - 1) // n, d.width, 3), dtype=torch.float32, device="cuda")
        for grab in grabs:
            os.environ["RT_GRAB_MIN"] = str(grab)
            sc.render_device(cam, buf.data_ptr(), nranks=n, stream=stream.cuda_stream)
            ks = sorted(sc.render_device(cam, buf.data_ptr(), nranks=n, stream=stream.cuda_stream,
                                         profile=True)["ms_fused"] for _ in range(5))
            print(json.dumps({"lib": tag, "nranks": n, "grab_min": grab, "ms_kernel": round(ks[2], 3)}),
                  flush=True)
