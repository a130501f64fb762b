#!/usr/bin/env python3
"""Chunk size x batch size at 1..8 ranks' C2 shares (dev tool)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import go_raytracer_amd as rt  # noqa: E402

t, cam, w, l = rt.demo_scene("cornell")
cam.Width, cam.SamplesPerPixel = 800, 1024
d = cam.derived()
stream = torch.cuda.current_stream()
with rt.Scene(t, w, l) as sc:
    for n in (1, 2, 8):
        buf = torch.zeros(((d.height + n - 1) // n, d.width, 3), dtype=torch.float32, device="cuda")
        for rep in range(2):
            for k, g in ((0, 0), (8, 256), (8, 512), (16, 128), (16, 256), (32, 128)):
                if g:
                    os.environ["RT_GRAB_MIN"] = str(g)
                else:
                    os.environ.pop("RT_GRAB_MIN", None)
                sc.render_device(cam, buf.data_ptr(), nranks=n, chunk=k, stream=stream.cuda_stream)
                ks = sorted(sc.render_device(cam, buf.data_ptr(), nranks=n, chunk=k,
                                             stream=stream.cuda_stream, profile=True)["ms_fused"]
                            for _ in range(5))
                print(json.dumps({"nranks": n, "chunk": k, "grab_min": g, "ms_kernel": round(ks[2], 3)}),
                      flush=True)
