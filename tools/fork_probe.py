"""Dev tool: where do GPU (fp32) and oracle (fp64) paths fork?

python3 tools/fork_probe.py SCENE WIDTH SPP STRIDE [NPIX]

Renders SCENE on the GPU and with the oracle in fp64 and fp32 (rows 0::STRIDE),
prints the parity metrics of GPU vs fp64, fp32-oracle vs fp64 and GPU vs fp32-oracle
(one JSON line each), then traces every sample of up to NPIX mismatching pixels in
both and classifies the first vertex where the paths differ:
  miss/hit   one side hits nothing
  t          same kind of hit, |dt| > 1e-4 * t (a different surface / triangle)
  dir        same hit, the next direction differs by > 1e-3
  len        the paths have different vertex counts only (depth limit / termination)
"""
import json
import sys
from collections import Counter

sys.path.insert(0, ".")
import numpy as np

import go_raytracer_amd as rt

rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)
from oracle import pyoracle
from tests.parity import compare

name, width, spp, stride = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
npix = int(sys.argv[5]) if len(sys.argv) > 5 else 24
t, cam, w, l = rt.demo_scene(name)
cam.Width = width
cam.SamplesPerPixel = spp
if name.startswith("model"):
    cam.AspectRatio = 16 / 9
H = cam.derived().height
W = cam.derived().width
ss = cam.derived().spp_sqrt ** 2
with rt.Scene(t, w, l) as sc:
    img, st = sc.render(cam, seed=1)
    sub = img[0::stride]
    r64, _ = pyoracle.render(t, w, l, cam, seed=1, threads=16, rank=0, nranks=stride)
    r32, _ = pyoracle.render(t, w, l, cam, seed=1, threads=16, rank=0, nranks=stride, precision=32)
    for lab, a, b in (("gpu_vs_64", sub, r64), ("o32_vs_64", r32, r64), ("gpu_vs_o32", sub, r32)):
        m = compare(a, b)
        print(json.dumps({"probe": lab, "scene": name, "width": width, "spp": spp, "stride": stride,
                          **{k: round(float(v), 6) for k, v in m.items()}}), flush=True)
    # forks: one sample per pixel, so a mismatching pixel is a forked sample
    cam.SamplesPerPixel = 1
    img1, _ = sc.render(cam, seed=1)
    ref1, _ = pyoracle.render(t, w, l, cam, seed=1, threads=16, rank=0, nranks=stride)
    d = np.abs(img1[0::stride].astype(np.float64) - ref1).max(axis=2)
    bad = np.argwhere(d > 2.0 ** -10)
    print(json.dumps({"probe": "spp1_forks", "forked_samples": int(len(bad)), "samples": int(d.size)}), flush=True)
    kinds = Counter()
    examples = []
    for (row, col) in bad[:npix]:
        pix = int(row * stride * W + col)
        for s_ in range(1):
            _, s2 = sc.render(cam, seed=1, trace=(pix, s_), rank=0, nranks=1)
            g = s2["trace"]
            o = pyoracle.trace(t, w, l, cam, pix, s_, seed=1)
            kind = None
            for k in range(max(len(g), len(o))):
                if k >= len(g) or k >= len(o):
                    kind = "len"
                    break
                gm, om = g[k][11], o[k][11]
                gbits = np.frombuffer(np.float32(gm).tobytes(), np.uint32)[0]
                ghit = gbits != 0xFFFFFFFF
                ohit = int(om) >= 0
                if ghit != ohit:
                    kind = "miss/hit"
                elif ghit and abs(g[k][8] - o[k][8]) > 1e-4 * max(1.0, abs(o[k][8])):
                    kind = "t"
                elif k + 1 < min(len(g), len(o)) and np.abs(g[k + 1][4:7] / np.linalg.norm(g[k + 1][4:7]) -
                                                          o[k + 1][4:7] / np.linalg.norm(o[k + 1][4:7])).max() > 1e-3:
                    kind = "dir"
                if kind:
                    if len(examples) < 12:
                        examples.append({"pix": pix, "sample": s_, "vertex": k, "kind": kind,
                                         "gpu": [float(x) for x in g[k]], "ref": [float(x) for x in o[k]],
                                         "gpu_ref_bits": f"{gbits:08x}"})
                    break
            if kind:
                kinds[(kind, min(int(k), 3))] += 1
    print(json.dumps({"probe": "fork_kinds", "pixels": int(min(len(bad), npix)), "bad_pixels": int(len(bad)),
                      "kinds": {f"{a}@{b}": c for (a, b), c in sorted(kinds.items())}}), flush=True)
    for e in examples:
        print(json.dumps(e), flush=True)
