"""Dev tool: GPU-vs-oracle mismatch of book2 with one component removed at a time."""
import sys
sys.path.insert(0, ".")
import go_raytracer_amd as rt
from oracle import pyoracle
from tests import scenes
from tests.parity import compare

COMPONENTS = ["none", "boxes", "motion", "glass", "metal", "water", "fog", "earth", "marble", "cluster"]
for comp in COMPONENTS:
    drop = () if comp == "none" else (comp,)
    t, cam, w, l = scenes.book2_variant(rt, "assets", drop)
    with rt.Scene(t, w, l) as sc:
        img, st = sc.render(cam, seed=7)
    ref, ost = pyoracle.render(t, w, l, cam, seed=7, threads=8)
    m = compare(img, ref)
    print(f"drop={comp:8s} close={m['frac_close']:.4f} qeq={m['q_equal']:.4f} "
          f"seg gpu={st['segments']} ref={ost['segments']} mean {m['mean_gpu']:.5f} {m['mean_ref']:.5f}",
          flush=True)
