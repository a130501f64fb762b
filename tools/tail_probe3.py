#!/usr/bin/env python3
"""Tail-phase batch sweep (dev tool): RT_TAIL_WAVES x RT_GRAB_TAIL on C2 shares."""
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
combos = [(0, 64), (16, 64), (32, 64), (64, 64), (128, 64), (32, 32), (64, 32), (64, 128)]
with rt.Scene(t, w, l) as sc:
    for n in (1, 4, 8):
        buf = torch.zeros(((d.height + n - 1) // n, d.width, 3), dtype=torch.float32, device="cuda")
        for rep in range(2):
            for tw, gt in combos:
                os.environ["RT_TAIL_WAVES"], os.environ["RT_GRAB_TAIL"] = str(tw), str(gt)
                sc.render_device(cam, buf.data_ptr(), nranks=n, stream=stream.cuda_stream)
                ks = sorted(sc.render_device(cam, buf.data_ptr(), nranks=n, stream=stream.cuda_stream,
                                             profile=True)["ms_fused"] for _ in range(5))
                print(json.dumps({"nranks": n, "tail_waves": tw, "grab_tail": gt,
                                  "ms_kernel": round(ks[2], 3)}), flush=True)
