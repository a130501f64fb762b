"""Kernel ms per path-slot count (opts.path_slots: resident waves per SIMD) at 1 and 8
row shares (dev tool): usage slots_probe.py scene width spp"""
import json, os, sys
sys.path.insert(0, os.getcwd())
import go_raytracer_amd as rt
rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)
scene, width, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
t, cam, w, l = rt.demo_scene(scene)
cam.Width, cam.SamplesPerPixel = width, spp
with rt.Scene(t, w, l) as sc:
    sc.render(cam, nranks=8)
    for n in (1, 8):
        for waves in (6, 5, 4, 3):
            slots = 256 * 4 * waves * 64  # CUs x SIMDs x waves x lanes
            ms = []
            for _ in range(3):
                _, st = sc.render(cam, nranks=n, path_slots=slots, profile=True)
                ms.append(st["ms_fused"])
            print(json.dumps({"scene": scene, "nranks": n, "waves_per_simd": waves,
                              "path_slots": st["path_slots"], "K": st["chunk_samples"],
                              "ms": round(sorted(ms)[1], 3)}), flush=True)
