"""Dev tool: a census of where GPU (fp32) and oracle (fp64) paths fork, over many samples.

python3 tools/fork_census.py SCENE WIDTH SEEDS [MAXTRACE] [ASPECT]

Renders SCENE at 1 sample per pixel (full image) for seeds 1..SEEDS on the GPU and with the
oracle in fp64; a pixel that differs by more than 2^-10 is a forked sample.  Up to MAXTRACE
of them are traced on both sides (one vertex record per world.Hit) and the first vertex where
the paths differ is classified:
  miss/hit   one side hits nothing
  t          same vertex, different hit distance (|dt| > 1e-4 t): another surface / object
  dir        same hit, the next direction differs (> 1e-3): a different scatter decision
  len        the paths have different vertex counts only
and labelled with the oracle's material kind at that vertex and the hit point, so the
forks can be attributed to objects (tools output: one JSON line per fork, then a summary).
"""
import json
import sys
from collections import Counter

sys.path.insert(0, ".")
import numpy as np

import go_raytracer_amd as rt

rt.tune_from_env()
from oracle import pyoracle

name, width, nseeds = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
maxtrace = int(sys.argv[4]) if len(sys.argv) > 4 else 200
aspect = float(sys.argv[5]) if len(sys.argv) > 5 else None
t, cam, w, l = rt.demo_scene(name)
cam.Width = width
cam.SamplesPerPixel = 1
if aspect:
    cam.AspectRatio = aspect
W = cam.derived().width
MAT = {-1: "miss"}


def first_fork(g, o):
    for k in range(max(len(g), len(o))):
        if k >= len(g) or k >= len(o):
            return k, "len"
        gbits = np.frombuffer(np.float32(g[k][11]).tobytes(), np.uint32)[0]
        ghit = gbits != 0xFFFFFFFF
        ohit = o[k][11] >= 0
        if ghit != ohit:
            return k, "miss/hit"
        if ghit and abs(g[k][8] - o[k][8]) > 1e-4 * max(1.0, abs(o[k][8])):
            return k, "t"
        if k + 1 < min(len(g), len(o)):
            a = g[k + 1][4:7] / np.linalg.norm(g[k + 1][4:7])
            b = o[k + 1][4:7] / np.linalg.norm(o[k + 1][4:7])
            if np.abs(a - b).max() > 1e-3:
                return k, "dir"
    return None, None


kinds, mats, total, forked = Counter(), Counter(), 0, 0
traced = 0
with rt.Scene(t, w, l) as sc:
    for seed in range(1, nseeds + 1):
        img, _ = sc.render(cam, seed=seed)
        ref, _ = pyoracle.render(t, w, l, cam, seed=seed, threads=16)
        d = np.abs(img.astype(np.float64) - ref).max(axis=2)
        bad = np.argwhere(d > 2.0 ** -10)
        total += d.size
        forked += len(bad)
        for (row, col) in bad:
            if traced >= maxtrace:
                break
            traced += 1
            pix = int(row * W + col)
            _, s2 = sc.render(cam, seed=seed, trace=(pix, 0))
            g = s2["trace"]
            o = pyoracle.trace(t, w, l, cam, pix, 0, seed=seed)
            k, kind = first_fork(g, o)
            if k is None:
                kind, k = "none", 0
            ok = o[min(k, len(o) - 1)]
            gk = g[min(k, len(g) - 1)]
            p_ref = (ok[0:3] + ok[4:7] * ok[8]).tolist() if np.isfinite(ok[8]) else None
            p_gpu = (gk[0:3] + gk[4:7] * gk[8]).tolist() if np.isfinite(gk[8]) else None
            gbits = int(np.frombuffer(np.float32(gk[11]).tobytes(), np.uint32)[0])
            rec = {"seed": seed, "pix": pix, "vertex": int(k), "kind": kind,
                   "ref_mat": int(ok[11]), "gpu_prim": (gbits >> 30) if gbits != 0xFFFFFFFF else -1,
                   "gpu_idx": gbits & 0x3FFFFFFF if gbits != 0xFFFFFFFF else -1,
                   "p_ref": p_ref, "p_gpu": p_gpu, "t_ref": float(ok[8]), "t_gpu": float(gk[8]),
                   "o": ok[0:3].tolist(), "d": ok[4:7].tolist(), "dval": float(d[row, col]),
                   "ref_val": float(np.abs(ref[row, col]).max()), "nv_gpu": int(len(g)), "nv_ref": int(len(o)),
                   "selfhit": bool(np.isfinite(gk[8]) and gk[8] < 0.02 and not (ok[8] < 0.02))}
            print(json.dumps(rec), flush=True)
            kinds[(kind, min(int(k), 4))] += 1
            mats[(kind, int(ok[11]))] += 1
print(json.dumps({"summary": name, "width": width, "seeds": nseeds, "samples": total,
                  "forked": forked, "rate": forked / max(1, total), "traced": traced,
                  "kinds": {f"{a}@{b}": c for (a, b), c in sorted(kinds.items())},
                  "by_ref_mat": {f"{a}/{b}": c for (a, b), c in sorted(mats.items())}}), flush=True)
