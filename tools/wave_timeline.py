#!/usr/bin/env python3
"""Wave timeline of the fused kernel (dev tool): renders C2 shares (or SCENE=name WIDTH=w
SPP=s) with RT_WAVE_TIMES set and summarises when waves finish relative to the kernel span.
usage: [SCENE=model WIDTH=1920 SPP=1024] python3 tools/wave_timeline.py [nranks ...]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import go_raytracer_amd as rt  # noqa: E402
rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)

SCENE = os.environ.get("SCENE", "cornell")
t, cam, w, l = rt.demo_scene(SCENE)
cam.Width = int(os.environ.get("WIDTH", "800"))
cam.SamplesPerPixel = int(os.environ.get("SPP", "1024"))
path = "/tmp/wave_times.bin"
with rt.Scene(t, w, l) as sc:
    for n in [int(x) for x in sys.argv[1:]] or [1, 8]:
        sc.render(cam, nranks=n)
        rt.tune("RT_WAVE_TIMES", path)
        img, st = sc.render(cam, nranks=n, profile=True)
        rt.untune("RT_WAVE_TIMES")
        a = np.fromfile(path, dtype=np.uint64).reshape(-1, 26).astype(np.int64)
        t0 = a[:, 0].min()
        start = (a[:, 0] - t0) / 100.0  # 100 MHz -> µs
        end = (a[:, 1] - t0) / 100.0
        span = end.max()
        q = lambda x, p: float(np.percentile(x, p))  # noqa: E731
        print(json.dumps({
            "scene": SCENE, "nranks": n, "kernel_ms": round(st["ms_fused"], 3), "waves": len(a),
            "span_us": round(span, 1), "start_p50_us": round(q(start, 50), 1),
            "start_max_us": round(start.max(), 1),
            "end_p1_us": round(q(end, 1), 1), "end_p10_us": round(q(end, 10), 1),
            "end_p50_us": round(q(end, 50), 1), "end_p90_us": round(q(end, 90), 1),
            "idle_frac": round(float(np.sum(span - end) / (span * len(a))), 4),
            "segments_p50": q(a[:, 2], 50), "segments_min": int(a[:, 2].min()),
            "segments_max": int(a[:, 2].max())}), flush=True)
        if a[:, 3].any():  # -DRT_DRAIN_TIMES builds: when each wave's grab came back empty
            dr = (a[:, 3] - t0) / 100.0
            left = end - dr
            print(json.dumps({
                "nranks": n, "drain_p1_us": round(q(dr, 1), 1), "drain_p50_us": round(q(dr, 50), 1),
                "drain_p99_us": round(q(dr, 99), 1), "drain_max_us": round(dr.max(), 1),
                "after_drain_p50_us": round(q(left, 50), 1), "after_drain_p99_us": round(q(left, 99), 1),
                "after_drain_max_us": round(left.max(), 1),
                "drain_p50_by_dispatch_round_us": {
                    int(r): round(float(np.percentile(dr[(np.arange(len(a)) // 4 // 256) % max(len(a) // 4 // 256, 1) == r], 50)), 1)
                    for r in range(max(len(a) // 4 // 256, 1))}}), flush=True)
            rem, act, segs_after = a[:, 4], a[:, 5], a[:, 2] - a[:, 6]
            print(json.dumps({
                "nranks": n, "left_at_drain_p50": q(rem, 50), "left_at_drain_p99": q(rem, 99),
                "busy_lanes_at_drain_p50": q(act, 50),
                "segments_after_drain_p50": q(segs_after, 50), "segments_after_drain_p99": q(segs_after, 99),
                "corr_after_drain_time_vs_left": round(float(np.corrcoef(left, rem)[0, 1]), 3),
                "corr_after_drain_time_vs_segments": round(float(np.corrcoef(left, segs_after)[0, 1]), 3),
                "after_drain_us_by_left_quartile": [round(float(np.median(left[(rem >= lo) & (rem <= hi)])), 1)
                    for lo, hi in zip(np.percentile(rem, [0, 25, 50, 75]), np.percentile(rem, [25, 50, 75, 100]))]}),
                  flush=True)
        # end times by XCD (workgroups are dispatched round-robin: block % 8) and by the
        # wave's slot in its workgroup (one workgroup per CU slot: its 4 waves, one per SIMD)
        blk = np.arange(len(a)) // 4
        xcd = {int(x): round(float(np.percentile(end[blk % 8 == x], 50)), 1) for x in range(8)}
        xcd_max = {int(x): round(float(end[blk % 8 == x].max()), 1) for x in range(8)}
        nblk = len(a) // 4
        resident = nblk // 256  # workgroups per CU
        by_slot = {int(r): round(float(np.percentile(end[(blk // 256) % max(resident, 1) == r], 50)), 1)
                   for r in range(max(resident, 1))}
        seg_slot = {int(r): int(np.median(a[(blk // 256) % max(resident, 1) == r, 2]))
                    for r in range(max(resident, 1))}
        print(json.dumps({"nranks": n, "end_p50_by_xcd_us": xcd, "end_max_by_xcd_us": xcd_max,
                          "end_p50_by_dispatch_round_us": by_slot,
                          "segments_p50_by_dispatch_round": seg_slot}), flush=True)
