#!/usr/bin/env python3
"""GPU-vs-oracle parity of the obj_mixed feature scene with one component neutralised at a
time (dev tool: find which feature diverges).  usage: python3 tools/bisect_obj.py"""
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import go_raytracer_amd as rt  # noqa: E402
from oracle import pyoracle  # noqa: E402
from tests import scenes  # noqa: E402
from tests.parity import compare  # noqa: E402

FIX = os.path.join(REPO, "tests", "golden", "obj")


def build(mtl_edit=None, rot=150.0, obj_lights=True, room_light=True):
    obj = open(os.path.join(FIX, "mixed.obj"), "rb").read()
    tex = os.path.join(REPO, "assets", "earthmap.ppm")
    mtl = open(os.path.join(FIX, "mixed.mtl")).read().replace("@TEX@", tex)
    if mtl_edit:
        mtl = re.sub(r"newmtl %s\n(?:(?!newmtl).*\n)*" % mtl_edit, "newmtl %s\nKd 0.5 0.5 0.5\n" % mtl_edit,
                     mtl)
    t = rt.Tree(1)
    world, _ = scenes._room(t)
    o = rt.LoadObjOptions(Debug=False, ScaleFactor=1.5, Position=(0.0, 2.5, 0.0))
    model, lights = t.LoadObjWithOptions(None, o, mtl_text=mtl.encode(), obj_text=obj)
    t.add(world, t.rotate_y(model, rot) if rot else model)
    light = t.quad((-2, 9.9, -2), (4, 0, 0), (0, 0, 4), t.light((10, 10, 10)))
    t.add(world, light)
    if not obj_lights:
        lights = t.list()
    if room_light:
        t.add(lights, light)
    return t, scenes._cam(rt, (0, 3, -9), (0, 2.5, 0)), world, lights


def run(tag, **kw):
    t, cam, w, l = build(**kw)
    with rt.Scene(t, w, l) as sc:
        out = {}
        for mode in ("fused", "wavefront"):
            img, st = sc.render(cam, seed=11, mode=mode)
            ref, ost = pyoracle.render(t, w, l, cam, seed=11, threads=8)
            m = compare(img, ref)
            out[mode] = {"frac_close": round(m["frac_close"], 4), "seg_gpu": st["segments"],
                         "seg_ref": ost["segments"], "feat": st["kernel_features"]}
    print(json.dumps({"variant": tag, **out}), flush=True)


if __name__ == "__main__":
    run("full")
    run("norot", rot=0.0)
    run("no_obj_lights", obj_lights=False)
    run("only_obj_lights", room_light=False)
    for m in ["white", "gold", "glass", "lamp", "smoke", "mirror", "shiny", "tex", "ka_tex",
              "metal3", "lamp_tex"]:
        run("neutral_" + m, mtl_edit=m)
