"""Quick GPU timing probe: render a config once and print throughput (dev tool)."""
import sys, time, json
sys.path.insert(0, ".")
import go_raytracer_amd as rt

scene = sys.argv[1] if len(sys.argv) > 1 else "cornell"
width = int(sys.argv[2]) if len(sys.argv) > 2 else 800
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 64
t, cam, w, l = rt.demo_scene(scene)
cam.Width = width
cam.SamplesPerPixel = spp
if scene == "book1":
    cam.AspectRatio = 1.5
with rt.Scene(t, w, l) as sc:
    img, st = sc.render(cam, seed=1, profile=True)  # warm (upload)
    t0 = time.time()
    img, st = sc.render(cam, seed=1, profile=True)
    dt = time.time() - t0
print(json.dumps({"scene": scene, "W": width, "spp": spp, "s": dt, "Msamples_s": st["samples"] / dt / 1e6,
                  "seg_per_sample": st["segments"] / st["samples"], **st}))
