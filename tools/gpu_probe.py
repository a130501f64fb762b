"""Quick GPU timing probe: render a config once and print throughput (dev tool).
usage: gpu_probe.py scene width spp [modes] [aspect]   (CHUNK=K: samples per chunk)"""
import sys, time, json
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import go_raytracer_amd as rt
rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)

scene = sys.argv[1] if len(sys.argv) > 1 else "cornell"
width = int(sys.argv[2]) if len(sys.argv) > 2 else 800
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 64
modes = sys.argv[4].split(",") if len(sys.argv) > 4 else ["fused", "wavefront"]
t, cam, w, l = rt.demo_scene(scene)
cam.Width = width
if len(sys.argv) > 5:
    cam.AspectRatio = float(sys.argv[5])
elif scene == "book1":
    cam.AspectRatio = 1.5
with rt.Scene(t, w, l) as sc:
    for mode in modes:
        cam.SamplesPerPixel = 1
        sc.render(cam, seed=1, mode=mode)  # warm: upload + state buffers
        cam.SamplesPerPixel = spp
        t0 = time.time()
        kw = {"chunk": int(__import__("os").environ["CHUNK"])} if __import__("os").environ.get("CHUNK") else {}
        img, st = sc.render(cam, seed=1, profile=True, mode=mode, **kw)
        dt = time.time() - t0
        print(json.dumps({"scene": scene, "mode": mode, "W": width, "spp": spp, "s": round(dt, 4),
                          "Msamples_s": round(st["samples"] / dt / 1e6, 2),
                          "seg_per_sample": round(st["segments"] / st["samples"], 4), **st}), flush=True)
