#!/usr/bin/env python3
"""Bitwise A/B of two library builds (dev tool): renders small versions of every demo
scene with the in-tree library and with RT_AMD_LIB=<other> (a child process) and
reports whether the images are identical.  usage: tools/ab_bitwise.py OTHER.so [BASE.so]
(BASE.so, if given, replaces the in-tree library on the first side)"""
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = [("cornell", 64, 64), ("book1", 48, 16), ("book2", 48, 16), ("quads", 32, 16),
          ("cornell_smoke", 48, 16), ("model:96x24", 64, 16), ("simple_light", 48, 16)]


def render_all(out):
    sys.path.insert(0, REPO)
    import go_raytracer_amd as rt
    rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)
    res = {}
    for name, w, spp in SCENES:
        t, cam, wo, li = rt.demo_scene(name)
        cam.Width, cam.SamplesPerPixel = w, spp
        with rt.Scene(t, wo, li) as sc:
            for mode in ("fused", "wavefront"):
                img, st = sc.render(cam, seed=3, mode=mode)
                res[f"{name}/{mode}"] = img
    np.savez(out, **res)


if __name__ == "__main__":
    if sys.argv[1] == "--render":
        render_all(sys.argv[2])
        sys.exit(0)
    other = os.path.abspath(sys.argv[1])
    base_env = dict(os.environ)
    if len(sys.argv) > 2:
        base_env["RT_AMD_LIB"] = os.path.abspath(sys.argv[2])
    subprocess.run([sys.executable, __file__, "--render", "/tmp/ab_cur.npz"], check=True,
                   env=base_env)
    subprocess.run([sys.executable, __file__, "--render", "/tmp/ab_other.npz"], check=True,
                   env=dict(os.environ, RT_AMD_LIB=other))
    a, b = np.load("/tmp/ab_cur.npz"), np.load("/tmp/ab_other.npz")
    for k in a.files:
        same = np.array_equal(a[k], b[k], equal_nan=True)
        diff = float(np.nanmax(np.abs(a[k] - b[k]))) if not same else 0.0
        print(json.dumps({"image": k, "bitwise_equal": bool(same), "max_abs": diff}), flush=True)
