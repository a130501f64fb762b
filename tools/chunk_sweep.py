"""Sweep samples-per-chunk K (dev tool): python3 tools/chunk_sweep.py scene width spp K1,K2,... [nranks]
With nranks, renders rank 0's rows only (one GPU's share of an N-GPU run)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import go_raytracer_amd as rt

scene, width, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
t, cam, w, l = rt.demo_scene(scene)
cam.Width, cam.SamplesPerPixel = width, spp
if scene == "book1":
    cam.AspectRatio = 1.5
nr = int(sys.argv[5]) if len(sys.argv) > 5 else 1
with rt.Scene(t, w, l) as sc:
    sc.render(cam, seed=1, mode="fused", nranks=nr)
    ref = None
    for k in [int(x) for x in sys.argv[4].split(",")]:
        t0 = time.time()
        img, st = sc.render(cam, seed=1, mode="fused", chunk=k, nranks=nr)
        dt = time.time() - t0
        print(json.dumps({"scene": scene, "nranks": nr, "ms": round(dt * 1e3, 2), "chunk": k, "Msamples_s": round(st["samples"] / dt / 1e6, 1),
                          "mean": float(img.mean())}), flush=True)
