#!/usr/bin/env python3
"""Time the output path (PrintColor + PPM P3, camera.go:160 / color.go:23-46):
host rt_format_ppm on a host image vs rt_format_ppm_device on the image in HBM
(+ the copy of the text to the host).  Prints one JSON line per image size.

usage (GPU box): python3 tools/output_bench.py [OUT.jsonl]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import go_raytracer_amd as rt  # noqa: E402

rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)


def best(fn, reps=10):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3


def main():
    out = open(sys.argv[1], "w") if len(sys.argv) > 1 else None
    for h, w in [(800, 800), (1080, 1920)]:
        img = np.random.default_rng(1).uniform(0, 1.2, (h, w, 3)).astype(np.float32)
        d = torch.from_numpy(img).cuda()
        n = int(rt.lib().rt_format_ppm_device(d.data_ptr(), w, h, None, 0, 0, None))
        buf = torch.empty(n, dtype=torch.uint8, device="cuda")
        host = best(lambda: rt.format_ppm(img))
        dev_only = best(lambda: rt.lib().rt_format_ppm_device(d.data_ptr(), w, h, buf.data_ptr(),
                                                              n, 0, None))
        dev_copy = best(lambda: rt.format_ppm_device(d))
        d2h_rgb = best(lambda: d.cpu())
        assert rt.format_ppm_device(d) == rt.format_ppm(img)
        rec = {"image": f"{w}x{h}", "ppm_bytes": n,
               "host_format_ms": round(host, 3),
               "host_path_ms": round(host + d2h_rgb, 3),
               "device_format_ms": round(dev_only, 3),
               "device_path_ms": round(dev_copy, 3),
               "rgb_d2h_ms": round(d2h_rgb, 3),
               "note": "host_path = copy fp32 RGB to host + host formatting; device_path = "
                       "size + format on the GPU + copy the text to host (best of 10)"}
        line = json.dumps(rec)
        print(line, flush=True)
        if out:
            out.write(line + "\n")


if __name__ == "__main__":
    main()
