set -o pipefail
RT_TIMING=1 timeout -k 10 300 python3 - > gpurun_out/c5_setup_r2l.log 2>&1 <<'PY'
import os, sys, time, tempfile
sys.path.insert(0, ".")
import go_raytracer_amd as rt
tmp = tempfile.mkdtemp()
open(os.path.join(tmp, "dragon.obj"), "wb").write(rt.substitute_mesh_obj())
for rep in range(2):
    t0 = time.time(); t, cam, w, l = rt.demo_scene("model", asset_dir=tmp); t1 = time.time()
    sc = rt.Scene(t, w, l); t2 = time.time()
    cam.Width, cam.SamplesPerPixel = 1920, 1
    img, st = sc.render(cam, seed=1); t3 = time.time()
    print("load %.3f flatten+bvh %.3f first render %.3f total %.3f" % (t1 - t0, t2 - t1, t3 - t2, t3 - t0), flush=True)
    sc.close()
PY
