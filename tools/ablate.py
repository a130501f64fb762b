#!/usr/bin/env python3
"""Ablation builds (dev tool): each variant removes or cheapens one part of the
path (results become wrong; only the timing matters) to measure its share of the
fused kernel's time.  Builds go_raytracer_amd/build_abl/<name>.so from the
working tree; run tools/ablate_run.sh on the GPU afterwards."""
import os, shutil, subprocess, sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
V = {
    "base": [],
    "rng_cheap": [("include/rt_rng.h",
        "  return rt_philox4x32_10(pixel, sample, stream, 0u, (uint32_t)seed, (uint32_t)(seed >> 32));",
        "  uint32_t h = pixel * 0x9E3779B1u ^ sample * 0x85EBCA77u ^ stream * 0xC2B2AE3Du ^ (uint32_t)seed;\n"
        "  h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12;\n"
        "  rt_u32x4 o; o.v[0] = h; o.v[1] = h * 0x297A2D39u; o.v[2] = h ^ (h >> 7) * 0x165667B1u; o.v[3] = h * 0x27D4EB2Fu;\n"
        "  return o;")],
    "no_lights": [("go_raytracer_amd/csrc/rt_path.h",
        "          ndir = lights_random<FT>(sc, p, r);",
        "          ndir = onb_transform(b, cosine_direction(rt_unit_f(r.v[3]), rt_unit_f(r.v[2])));"),
        ("go_raytracer_amd/csrc/rt_path.h",
        "        float pdf = 0.5f * lights_pdf<FT>(sc, p, ndir) + 0.5f * bsdf_pdf;",
        "        float pdf = bsdf_pdf + 1e-3f;")],
    "no_fold": [("go_raytracer_amd/csrc/rt_path.h",
        "  if (!(zero && !(s.flags & F_NONFINITE))) {",
        "  if (false) {")],
    "no_flush": [("go_raytracer_amd/csrc/rt_path.h",
        "RT_D void flush_chunk(const Params& P, uint32_t chunk, f3 acc) {",
        "RT_D void flush_chunk(const Params& P, uint32_t chunk, f3 acc) {\n  if (acc.x != -12345.0f) return;")],
    "no_camrng": [("go_raytracer_amd/csrc/rt_path.h",
        "  rt_u32x4 r = rt_rng_draw(P.seed, id.gpix, sample, RT_STREAM_CAMERA);",
        "  rt_u32x4 r = {{sample * 0x9E3779B1u, sample * 0x85EBCA77u, sample * 0xC2B2AE3Du, 0u}};")],
    "dbl_trav": [("go_raytracer_amd/csrc/rt_render.hip",
        "      trav_steps<LDS, FT, W4>(P.sc, lnodes, recs_lds, ts, s.o, s.d, s.time, 0.001f, tr,\n                              P.step_budget);",
        "    { Trav t2 = tr; trav_steps<LDS, FT, W4>(P.sc, lnodes, recs_lds, ts, s.o, s.d, s.time, 0.001f, t2, P.step_budget);\n"
        "      trav_steps<LDS, FT, W4>(P.sc, lnodes, recs_lds, ts, s.o, s.d, s.time, 0.001f, tr, P.step_budget);\n"
        "      tr.best.t = fminf(tr.best.t, t2.best.t + 0.0f * tr.best.t); }")],
    "dbl_media": [("go_raytracer_amd/csrc/rt_render.hip",
        "    trace_media(P, s.o, s.d, s.time, 0.001f, s.gpix, s.s0 + s.j, s.k, best);",
        "  { Hit b2 = best; trace_media(P, s.o, s.d, s.time, 0.001f, s.gpix, s.s0 + s.j, s.k, b2);\n"
        "    trace_media(P, s.o, s.d, s.time, 0.001f, s.gpix, s.s0 + s.j, s.k, best); best.t = fminf(best.t, b2.t + 0.0f * best.t); }")],
    "dbl_lightpdf": [("go_raytracer_amd/csrc/rt_path.h",
        "        float pdf = 0.5f * lights_pdf<FT>(sc, p, ndir) + 0.5f * bsdf_pdf;",
        "        float pdf = 0.25f * (lights_pdf<FT>(sc, p, ndir) + lights_pdf<FT>(sc, p, ndir * 1.0000001f)) + 0.5f * bsdf_pdf;")],
    "dbl_camera": [("go_raytracer_amd/csrc/rt_path.h",
        "  camera_ray(P, id, id.sample0 + j, s.o, s.d, s.time);",
        "  camera_ray(P, id, id.sample0 + j, s.o, s.d, s.time);\n  { f3 o2, d2; float t2; camera_ray(P, id, id.sample0 + j + 7u, o2, d2, t2); s.d = s.d + d2 * 0.0f; }")],
    "dbl_fold": [("go_raytracer_amd/csrc/rt_path.h",
        "    if (s.flags & F_PRE) L = get_pre<SOA>(P, slot, s) * L;",
        "    if (s.flags & F_PRE) L = get_pre<SOA>(P, slot, s) * L;\n"
        "    { f3 L2 = ws.fold(P, slot, s.nst, L * 1.0000001f); L = L + L2 * 0.0f; }")],
    "waves6": [("go_raytracer_amd/csrc/rt_render.hip",
        "constexpr int fused_waves(uint32_t ft) { return ft == 0u ? 5 : ft == FT_MEDIA ? 4 : 3; }",
        "constexpr int fused_waves(uint32_t ft) { return ft == 0u ? 6 : ft == FT_MEDIA ? 4 : 3; }"),
        ("go_raytracer_amd/csrc/rt_path.h", "constexpr int kLdsW = 4;", "constexpr int kLdsW = 3;"),
        ("go_raytracer_amd/csrc/rt_render.hip", "- 28u * 1024u - 512u) / 64u);", "- 24u * 1024u - 512u) / 64u);")],
    "stack8": [("go_raytracer_amd/csrc/rt_path.h", "constexpr int kShortStack = 12;", "constexpr int kShortStack = 8;"),
        ("go_raytracer_amd/csrc/rt_render.hip", "- 28u * 1024u - 512u) / 64u);", "- 24u * 1024u - 512u) / 64u);")],
    "waves7": [("go_raytracer_amd/csrc/rt_render.hip",
        "constexpr int fused_waves(uint32_t ft) { return ft == 0u ? 5 : ft == FT_MEDIA ? 4 : 3; }",
        "constexpr int fused_waves(uint32_t ft) { return ft == 0u ? 7 : ft == FT_MEDIA ? 4 : 3; }"),
        ("go_raytracer_amd/csrc/rt_path.h", "constexpr int kLdsW = 4;", "constexpr int kLdsW = 3;"),
        ("go_raytracer_amd/csrc/rt_path.h", "constexpr int kShortStack = 12;", "constexpr int kShortStack = 8;"),
        ("go_raytracer_amd/csrc/rt_render.hip", "- 28u * 1024u - 512u) / 64u);", "- 20u * 1024u - 512u) / 64u);")],
    "set47w4": [("go_raytracer_amd/csrc/rt_render.hip",
        "constexpr int fused_waves(uint32_t ft) { return ft == 0u ? 6 : ft == FT_MEDIA ? 4 : 3; }",
        "constexpr int fused_waves(uint32_t ft) { return ft == 0u ? 6 : (ft == FT_MEDIA || ft == 47u) ? 4 : 3; }")],
    "allw4": [("go_raytracer_amd/csrc/rt_render.hip",
        "ft == (FT_SPHERE | FT_TRI | FT_METAL | FT_DIEL | FT_CHECKER) ? 4 : 3;",
        "ft == (FT_SPHERE | FT_TRI | FT_METAL | FT_DIEL | FT_CHECKER) ? 4 : 4;")],
    "medw5": [("go_raytracer_amd/csrc/rt_render.hip",
        "return ft == 0u ? 6 : ft == FT_MEDIA ? 4 :",
        "return ft == 0u ? 6 : ft == FT_MEDIA ? 5 :")],
    "dbl_brute": [("go_raytracer_amd/csrc/rt_render.hip",
        "        trav_brute<FT, !LDS>(P.sc, lnodes, s.o, s.d, s.time, 0.001f, tr);",
        "      { Trav t2 = tr; trav_brute<FT, !LDS>(P.sc, lnodes, s.o, s.d * 1.0000001f, s.time, 0.001f, t2);\n"
        "        trav_brute<FT, !LDS>(P.sc, lnodes, s.o, s.d, s.time, 0.001f, tr);\n"
        "        tr.best.t = fminf(tr.best.t, t2.best.t + 0.0f * tr.best.t); }")],
}
V["dbl_trav4"] = [("go_raytracer_amd/csrc/rt_render.hip",
    "        trav_steps<LDS, FT, TREE == 4>(P.sc, lnodes, recs_lds, ts, s.o, s.d, s.time, 0.001f, tr,\n                                       P.step_budget);",
    "      { Trav t2 = tr; trav_steps<LDS, FT, TREE == 4>(P.sc, lnodes, recs_lds, ts, s.o, s.d * 1.0000001f, s.time, 0.001f, t2, P.step_budget);\n"
    "        trav_steps<LDS, FT, TREE == 4>(P.sc, lnodes, recs_lds, ts, s.o, s.d, s.time, 0.001f, tr, P.step_budget);\n"
    "        tr.best.t = fminf(tr.best.t, t2.best.t + 0.0f * tr.best.t); }")]
names = sys.argv[1:] or list(V)
for name in names:
    d = f"/tmp/abl/{name}"
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(d)
    for sub in ("go_raytracer_amd/csrc", "include"):
        shutil.copytree(os.path.join(R, sub), os.path.join(d, sub), ignore=shutil.ignore_patterns("build*"))
    for f, old, new in V[name]:
        p = os.path.join(d, f)
        s = open(p).read()
        assert old in s, (name, old[:60])
        open(p, "w").write(s.replace(old, new))
    out = os.path.join(R, "go_raytracer_amd", "build_abl", name, "librt_amd.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    r = subprocess.run(["make", "-s", "-j8", "-C", f"{d}/go_raytracer_amd/csrc", f"ROOT={d}", f"OUT={out}",
                        f"BUILD={d}/build"], capture_output=True, text=True)
    print(name, "ok" if r.returncode == 0 else r.stderr[-2000:])
