#!/usr/bin/env python3
"""Is a multi-GPU share slower per sample than the whole image? (dev tool)
Renders, on one GPU, rank 0 of N's rows (r % N == 0) at full spp and the whole image at spp / N
(the same number of samples, every row), each with the share's chunk size and the default one.
The share's rows are N image rows apart, so its in-flight band spans N times more of the
image: if the whole image at spp / N is faster, the share loses to locality, not to its tail.
usage: python3 tools/locality_probe.py scene width spp [N]  -> JSON lines"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import go_raytracer_amd as rt  # noqa: E402

rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)
scene, width, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
n = int(sys.argv[4]) if len(sys.argv) > 4 else 8
t, cam, w, l = rt.demo_scene(scene)
cam.Width = width


def run(spp_, nranks, **kw):
    cam.SamplesPerPixel = spp_
    ms = []
    for i in range(4):
        _, st = sc.render(cam, seed=1, nranks=nranks, profile=True, **kw)
        if i:
            ms.append(st["ms_fused"])
    return sorted(ms)[1], st


with rt.Scene(t, w, l) as sc:
    share_ms, st = run(spp, n)
    k = st["chunk_samples"]
    rows = [("share", spp, n, {}, share_ms, st)]
    for label, kw in (("whole_default_chunk", {}), ("whole_share_chunk", {"chunk": k})):
        ms, st2 = run(spp // n, 1, **kw)
        rows.append((label, spp // n, 1, kw, ms, st2))
    for label, s_, nr, kw, ms, st_ in rows:
        print(json.dumps({"scene": scene, "width": width, "case": label, "spp": s_, "nranks": nr,
                          "chunk": st_["chunk_samples"], "ms_kernel": round(ms, 3),
                          "segments": st_["segments"],
                          "ns_per_segment": round(ms * 1e6 / st_["segments"], 4)}), flush=True)
