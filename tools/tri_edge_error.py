"""Dev tool (CPU): how wrong are fp32 Moller-Trumbore barycentrics on the C5 mesh, and why
did two camera rays see through it?  (rt_kernels.h
hit_tri_rec_m's near-edge band.)

python3 tools/tri_edge_error.py [N_RAYS] > profiles/r6_tri_edge_error.json

1. Builds the "model" scene (the 1M-triangle dragon substitute, RotateY 180 baked into world
   space as the flattener does), aims N rays from around the camera (10, 5, 10) at random
   points in and just outside random triangles, and evaluates Triangle.Hit
   (objects.go:408-461) on the fp32 record data (v0, e0 = v1 - v0, e1 = v2 - v0) in numpy
   fp32 (no fma contraction: a little less accurate than the GPU) and in fp64.  Prints the
   distribution of the barycentric error max(|du|, |dv|, |dw|) and of its ratio to the
   kernel's bound eps * |o - v0|inf * |d|inf * |e|inf / |det| (the band is 16 times that).
2. For every vertex-0 fork of the round-5 census (profiles/r5_census_model_before.jsonl),
   the triangle the fp64 oracle hit, its neighbours across each edge, and whether rays
   perturbed by a few fp32 ulps always hit one of them (a closed surface: a hole in the fp32
   test, not a silhouette graze).
"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import go_raytracer_amd as rt  # noqa: E402


def mesh():
    t, cam, w, l = rt.demo_scene("model")
    v = t.view()
    n = v.n_tris
    dt = np.dtype([('v', '<f8', 9), ('n', '<f8', 9), ('uv', '<f8', 6), ('flags', '<i4'), ('mat', '<i4')])
    T = np.frombuffer((C.c_char * (dt.itemsize * n)).from_address(v.tris), dt).copy()
    return T['v'].reshape(-1, 3, 3)  # object space (the scene's RotateY(180) is applied by callers)


def cross(a, b):
    return np.stack([a[:, 1] * b[:, 2] - a[:, 2] * b[:, 1], a[:, 2] * b[:, 0] - a[:, 0] * b[:, 2],
                     a[:, 0] * b[:, 1] - a[:, 1] * b[:, 0]], 1)


def mt(o, d, v0, e0, e1, dtp):
    o, d, v0, e0, e1 = (x.astype(dtp) for x in (o, d, v0, e0, e1))
    p = cross(d, e1)
    det = (e0 * p).sum(1)
    inv = dtp(1) / det
    tv = o - v0
    u = (tv * p).sum(1) * inv
    q = cross(tv, e0)
    v = (d * q).sum(1) * inv
    t = (e1 * q).sum(1) * inv
    return det, u, v, t


def error_distribution(V, m, rng):
    Vw = V.copy()
    Vw[..., 0] *= -1  # RotateY(180): (x, z) -> (-x, -z), baked as host_flatten.cpp does
    Vw[..., 2] *= -1
    V32 = Vw.astype(np.float32)
    idx = rng.integers(0, len(V), m)
    v0 = V32[idx, 0]
    e0 = (V32[idx, 1] - V32[idx, 0]).astype(np.float32)
    e1 = (V32[idx, 2] - V32[idx, 0]).astype(np.float32)
    bu, bv = rng.uniform(-0.01, 1.01, m), rng.uniform(-0.01, 1.01, m)
    P = Vw[idx, 0] + bu[:, None] * (Vw[idx, 1] - Vw[idx, 0]) + bv[:, None] * (Vw[idx, 2] - Vw[idx, 0])
    O = (np.array([10.0, 5.0, 10.0]) + rng.normal(0, 0.05, (m, 3))).astype(np.float32).astype(np.float64)
    D = (P - O).astype(np.float32).astype(np.float64)
    d64, u64, v64, _ = mt(O, D, v0, e0, e1, np.float64)
    _, u32, v32, _ = mt(O, D, v0, e0, e1, np.float32)
    err = np.maximum.reduce([np.abs(u32 - u64), np.abs(v32 - v64),
                             np.abs((1 - u32 - v32) - (1 - u64 - v64))])
    bound = (np.abs(O - v0).max(1) * np.abs(D).max(1) *
             np.maximum(np.abs(e0).max(1), np.abs(e1).max(1)) / np.abs(d64) * 2.0 ** -24)
    q = [0.5, 0.9, 0.99, 0.999, 0.9999, 1.0]
    return {"rays": m, "quantiles": q,
            "abs_error": np.quantile(err, q).tolist(),
            "error_over_bound": np.quantile(err / bound, q).tolist(),
            "band_over_bound": 16.0}


def census_forks(V):
    path = os.path.join(REPO, "profiles", "r5_census_model_before.jsonl")
    v0, e0, e1 = V[:, 0], V[:, 1] - V[:, 0], V[:, 2] - V[:, 0]
    out = []
    for line in open(path):
        r = json.loads(line)
        if r.get("vertex") != 0:
            continue
        o, d = np.array(r["o"]), np.array(r["d"])
        cs, sn = np.cos(np.pi), np.sin(np.pi)  # the oracle transforms the ray (transformation.go)
        o = np.array([cs * o[0] - sn * o[2], o[1], sn * o[0] + cs * o[2]])
        d = np.array([cs * d[0] - sn * d[2], d[1], sn * d[0] + cs * d[2]])
        det, u, v, t = mt(o[None], d[None], v0, e0, e1, np.float64)
        hit = (np.abs(det) >= 1e-8) & (u >= 0) & (u <= 1) & (v >= 0) & (u + v <= 1) & (t >= 0.001)
        first = int(np.nonzero(hit)[0][np.argmin(t[hit])])
        shared = np.zeros(len(V), int)
        for j in range(3):
            shared += (np.abs(V - V[first][j]).sum(2) < 1e-12).any(1)
        nb = [int(i) for i in np.nonzero(shared >= 2)[0] if i != first]
        cand = np.array([first] + nb)
        rng = np.random.default_rng(0)
        misses = 0
        for _ in range(2000):
            dd = d * (1 + rng.normal(0, 3e-7, 3))
            _, uk, vk, _ = mt(o[None], dd[None], v0[cand], e0[cand], e1[cand], np.float64)
            misses += not ((uk >= 0) & (uk <= 1) & (vk >= 0) & (uk + vk <= 1)).any()
        out.append({"pix": r["pix"], "seed": r["seed"], "t_ref": r["t_ref"], "t_gpu": r["t_gpu"],
                    "oracle_tri": first, "u": float(u[first]), "v": float(v[first]),
                    "w": float(1 - u[first] - v[first]), "neighbours": nb,
                    "perturbed_rays_missing_all": misses, "perturbed_rays": 2000})
    return out


if __name__ == "__main__":
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 400000
    V = mesh()
    res = {"mesh_triangles": len(V), "fp32_barycentric_error": error_distribution(V, m, np.random.default_rng(1)),
           "vertex0_forks_r5": census_forks(V)}
    print(json.dumps(res, indent=1))
