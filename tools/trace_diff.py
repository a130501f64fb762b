"""Dev tool: find GPU/oracle mismatching samples of a scene and diff their path traces."""
import sys
sys.path.insert(0, ".")
import numpy as np
import go_raytracer_amd as rt
rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)
from oracle import pyoracle
from tests import scenes

np.set_printoptions(linewidth=200, precision=6, suppress=True)
drop = tuple(sys.argv[1:])
t, cam, w, l = scenes.book2_variant(rt, "assets", drop)
cam.SamplesPerPixel = 1
with rt.Scene(t, w, l) as sc:
    img, st = sc.render(cam, seed=7)
ref, ost = pyoracle.render(t, w, l, cam, seed=7, threads=8)
d = np.abs(img.astype(np.float64) - ref).max(axis=2)
bad = np.argwhere(d > 1e-3)
print("mismatching pixels:", len(bad), "of", d.size, "segments", st["segments"], ost["segments"])
W = cam.derived().width
shown = 0
for (row, col) in bad[:12]:
    pix = int(row * W + col)
    with rt.Scene(t, w, l) as sc:
        _, s2 = sc.render(cam, seed=7, trace=(pix, 0))
    g = s2["trace"]
    o = pyoracle.trace(t, w, l, cam, pix, 0, seed=7)
    print(f"--- pixel {pix} gpu {img[row, col]} ref {ref[row, col]}  gpu vertices {len(g)} ref {len(o)}")
    n = max(len(g), len(o))
    for k in range(min(n, 12)):
        gl = g[k] if k < len(g) else None
        ol = o[k] if k < len(o) else None
        if gl is not None:
            ref_bits = np.frombuffer(np.float32(gl[11]).tobytes(), np.uint32)[0]
            print(f"  G k={int(gl[7])} o={gl[0:3]} d={gl[4:7]} t={gl[8]:.6g} ref={ref_bits:08x}")
        if ol is not None:
            print(f"  O k={int(ol[7])} o={ol[0:3]} d={ol[4:7]} t={ol[8]:.6g} mat={int(ol[11])}")
