"""Brute-force vs tree crossover (dev tool): Cornell box plus N extra small boxes
(6 quads each), rendered with RT_TREE=2/4 and with the record loop."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import go_raytracer_amd as rt
rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)

for nbox in [int(x) for x in sys.argv[1].split(",")]:
    t, cam, w, l = rt.demo_scene("cornell")
    white = t.lambertian(t.solid(.73, .73, .73))
    lst = t.list()
    for i in range(nbox):
        x, z = 60 + 90 * (i % 5), 60 + 90 * (i // 5)
        t.add(lst, t.box((x, 0, z), (x + 40, 40 + 10 * (i % 3), z + 40), white))
    w = t.list(w, lst)
    cam.Width, cam.SamplesPerPixel = 800, 256
    with rt.Scene(t, w, l) as sc:
        nrefs = sc.info()["n_world_prims"]
        for mode in ("brute", "smem", "2", "4"):
            env = {"brute": {"RT_BRUTE_MAX": "100000", "RT_BRUTE_SMEM": "0"},
                   "smem": {"RT_BRUTE_MAX": "100000", "RT_BRUTE_SMEM": "1"},
                   "2": {"RT_TREE": "2", "RT_BRUTE_MAX": "0", "RT_BRUTE_SMEM": "0"},
                   "4": {"RT_TREE": "4", "RT_BRUTE_MAX": "0", "RT_BRUTE_SMEM": "0"}}[mode]
            rt.untune("RT_TREE")
            for k, v in env.items():
                rt.tune(k, v)
            sc.render(cam, seed=1, mode="fused")
            t0 = time.time()
            img, st = sc.render(cam, seed=1, mode="fused")
            dt = time.time() - t0
            print(json.dumps({"boxes": nbox, "prims": nrefs, "mode": mode, "tree": st["tree_width"],
                              "lds": st["lds_scene"],
                              "Msamples_s": round(st["samples"] / dt / 1e6, 1)}), flush=True)
