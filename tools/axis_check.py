import os, sys, json
sys.path.insert(0, os.getcwd())
import numpy as np
import go_raytracer_amd as rt
t, cam, w, l = rt.demo_scene("cornell")
cam.Width, cam.SamplesPerPixel = 200, 256
imgs = []
for flag in ("0", "1"):
    os.environ["RT_BRUTE_AXIS"] = flag
    with rt.Scene(t, w, l) as sc:
        img, st = sc.render(cam, seed=4, chunk=8)
    imgs.append(img)
    print(flag, st["segments"], st["tree_width"], st["ms_total"])
same = float(np.mean(np.all(imgs[0] == imgs[1], axis=-1)))
print(json.dumps({"bitwise_same_frac": same, "max_abs": float(np.max(np.abs(imgs[0] - imgs[1])))}))
