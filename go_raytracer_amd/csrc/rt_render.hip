// rt_render.hip — the MI355X streaming-wavefront path tracer.
//
// Replaces the reference's per-pixel loop (camera.go:90-153) and recursive
// estimator rayColor (camera.go:293-331).  One render = a queue-driven loop of
//   k_extend : persistent closest-hit kernel (BVH top staged in LDS, work pulled
//              64 rays per wave with one atomic) -> SoA hit records
//   k_shade  : emission / Scatter / mixture-pdf light sampling, clamp-vertex
//              bookkeeping, path termination + backward clamp fold, chunk
//              accumulation, regeneration of camera rays, and ballot/prefix
//              compaction of the surviving paths into the next queue
// followed by k_resolve (fixed-point pixel sums -> linear mean RGB).
// Path state lives in HBM as structure-of-arrays indexed by slot.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stddef.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "rt_internal.h"
#include "rt_kernels.h"

namespace rt {

// ---------------------------------------------------------------- params ---
constexpr int kLdsNodes = 512;   // BVH nodes staged in LDS per workgroup (32 KB)
constexpr int kStack = 64;       // traversal stack entries per lane
constexpr int kMaxIt = 1 << 16;  // per-iteration counter slots (no per-iteration memsets)

enum : uint32_t { F_PEND = 1u, F_PRE = 2u, F_NONFINITE = 4u };

struct Counters {
  unsigned long long segments;
  unsigned long long pushes;
  uint32_t chunk_head;
  uint32_t _pad[13];
  uint32_t cnt[kMaxIt];   // queue length entering iteration i
  uint32_t head[kMaxIt];  // extend work head for iteration i
};

struct Params {
  DevScene sc;
  // camera (initialize camera.go:179-253, converted to fp32)
  float p00r[3], du[3], dv[3], cc[3], dku[3], dkv[3];  // p00r = pixel00 - center
  float bg[3];
  float recip_s, maxc;
  int s, defocus, max_depth;
  int width, rank, nranks;
  uint32_t npix;       // pixels of this rank
  uint32_t K;          // samples per chunk
  uint32_t cpp;        // chunks per pixel
  uint32_t n_chunks;
  uint32_t P;          // path slots
  uint32_t ss;         // s*s
  uint64_t seed;
  // wavefront state (SoA, slot-indexed)
  F4* ray_o;   // origin | time
  F4* ray_d;   // direction | 0
  F4* hit;     // t, u, v, prim ref bits
  uint2* path; // chunk, packed(j:12 | vertex:8 | nstack:8 | flags:4)
  F4* pend;    // pending clamp-vertex weight (top of the weight stack)
  F4* pre;     // camera-side product of specular attenuations
  F4* acc;     // chunk accumulator
  F4* stack;   // [vertex][slot] clamp-vertex weights spilled to HBM
  uint32_t* queue[2];
  Counters* ctr;
  unsigned long long* accum;  // 3 planes x npix, fixed point 2^-32
  uint32_t* pflags;           // per pixel NaN (bits 0-2) / Inf (bits 3-5)
  F4* trace;                  // debug path trace (3 F4 per vertex) or null
  uint32_t trace_gpix, trace_sample;
  int trace_cap;
};

RT_D uint32_t pack_path(uint32_t j, uint32_t k, uint32_t nst, uint32_t flags) {
  return (j & 0xFFFu) | ((k & 0xFFu) << 12) | ((nst & 0xFFu) << 20) | ((flags & 0xFu) << 28);
}

RT_D uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
RT_D uint32_t prefix_count(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// chunk c -> (local pixel, global pixel, first sample).  Chunks are pixel-fastest
// so concurrently grabbed chunks touch different accumulators.
struct Ids {
  uint32_t lpix, gpix, row, col, sample0, count;
};
RT_D Ids chunk_ids(const Params& P, uint32_t chunk) {
  Ids r;
  r.lpix = chunk % P.npix;
  uint32_t sub = chunk / P.npix;
  uint32_t row_l = r.lpix / (uint32_t)P.width;
  r.col = r.lpix - row_l * (uint32_t)P.width;
  r.row = row_l * (uint32_t)P.nranks + (uint32_t)P.rank;
  r.gpix = r.row * (uint32_t)P.width + r.col;
  r.sample0 = sub * P.K;
  r.count = min(P.K, P.ss - r.sample0);
  return r;
}

// getRay camera.go:256-270 + sampleSquareStratified :277-282 + defocusDiskSample :285-290
RT_D void camera_ray(const Params& P, const Ids& id, uint32_t sample, F4& ro, F4& rd) {
  rt_u32x4 r = rt_rng_draw(P.seed, id.gpix, sample, RT_STREAM_CAMERA);
  uint32_t si = sample / (uint32_t)P.s, sj = sample - si * (uint32_t)P.s;
  float px = (((float)sj + rt_unit_f(r.v[0])) * P.recip_s) - 0.5f;
  float py = (((float)si + rt_unit_f(r.v[1])) * P.recip_s) - 0.5f;
  float fx = (float)id.col + px, fy = (float)id.row + py;
  // pixelSample - rayOrigin rearranged as (pixel00 - center) + du*fx + dv*fy - disk:
  // the same vector without fp32 cancellation against large camera coordinates
  f3 d = mk3(P.p00r[0] + P.du[0] * fx + P.dv[0] * fy, P.p00r[1] + P.du[1] * fx + P.dv[1] * fy,
             P.p00r[2] + P.du[2] * fx + P.dv[2] * fy);
  f3 o = mk3(P.cc[0], P.cc[1], P.cc[2]);
  if (P.defocus) {
    rt_u32x4 q = rt_rng_draw(P.seed, id.gpix, sample, RT_STREAM_CAMERA | 1u);
    f3 dk = uniform_disk(rt_unit_f(q.v[0]), rt_unit_f(q.v[1]));
    f3 off = mk3(P.dku[0], P.dku[1], P.dku[2]) * dk.x + mk3(P.dkv[0], P.dkv[1], P.dkv[2]) * dk.y;
    o = o + off;
    d = d - off;
  }
  ro = {o.x, o.y, o.z, rt_unit_f(r.v[2])};
  rd = {d.x, d.y, d.z, 0.0f};
}

RT_D void start_sample(const Params& P, uint32_t slot, uint32_t chunk, uint32_t j) {
  Ids id = chunk_ids(P, chunk);
  F4 ro, rd;
  camera_ray(P, id, id.sample0 + j, ro, rd);
  P.ray_o[slot] = ro;
  P.ray_d[slot] = rd;
  P.path[slot] = make_uint2(chunk, pack_path(j, 0, 0, 0));
}

// ------------------------------------------------------------- traversal ---
struct Hit {
  float t, u, v;
  uint32_t ref;
};

RT_D void slab(const F4& lo, const F4& hi, f3 o, f3 inv, float tmin, float tmax, bool& hit,
               float& tnear) {
  float tx0 = (lo.x - o.x) * inv.x, tx1 = (hi.x - o.x) * inv.x;
  float ty0 = (lo.y - o.y) * inv.y, ty1 = (hi.y - o.y) * inv.y;
  float tz0 = (lo.z - o.z) * inv.z, tz1 = (hi.z - o.z) * inv.z;
  float t0 = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), tmin));
  float t1 = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax));
  hit = t0 <= t1 * 1.00000024f;  // 2 ulp slack: conservative for flat boxes
  tnear = t0;
}

// Closest hit over the world BVH (replaces BVHNode.Hit bvh.go:69-82 +
// HittableList.Hit hittable.go:122-138 + AABB.Hit aabb.go:90-113).
RT_D void trace_world(const DevScene& sc, const F4* lnodes, int nl, f3 o, f3 d, float time,
                      float tmin, Hit& best) {
  if (sc.root == PRIM_NONE) return;
  f3 inv = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  uint32_t stack[kStack];
  int sp = 0;
  uint32_t cur = sc.root;
  for (;;) {
    if (!(cur & LEAF_BIT)) {
      F4 a0, a1, b0, b1;
      if ((int)cur < nl) {
        a0 = lnodes[4 * cur + 0];
        a1 = lnodes[4 * cur + 1];
        b0 = lnodes[4 * cur + 2];
        b1 = lnodes[4 * cur + 3];
      } else {
        const F4* g = sc.nodes + 4 * (size_t)cur;
        a0 = g[0];
        a1 = g[1];
        b0 = g[2];
        b1 = g[3];
      }
      bool h0, h1;
      float t0, t1;
      slab(a0, a1, o, inv, tmin, best.t, h0, t0);
      slab(b0, b1, o, inv, tmin, best.t, h1, t1);
      uint32_t c0 = fbits(a0.w), c1 = fbits(a1.w);
      if (h0 && h1) {
        uint32_t nearc = t0 <= t1 ? c0 : c1, farc = t0 <= t1 ? c1 : c0;
        if (sp < kStack) stack[sp++] = farc;
        cur = nearc;
        continue;
      }
      if (h0) {
        cur = c0;
        continue;
      }
      if (h1) {
        cur = c1;
        continue;
      }
    } else {
      uint32_t first = (cur >> 4) & 0x7FFFFFFu, count = (cur & 15u) + 1u;
      for (uint32_t k = 0; k < count; ++k) {
        uint32_t ref = sc.refs[first + k];
        float t, u, v;
        if (hit_prim(sc, ref, o, d, time, tmin, best.t, t, u, v)) {
          best.t = t;
          best.u = u;
          best.v = v;
          best.ref = ref;
        }
      }
    }
    if (sp == 0) break;
    cur = stack[--sp];
  }
}

// closest boundary hit over (lo, hi) with each prim's own interval semantics
RT_D bool boundary_hit(const DevScene& sc, const DevMedium& m, f3 o, f3 d, float time, double lo,
                       double hi, double& t_out) {
  bool any = false;
  double best = hi;
  for (uint32_t k = 0; k < m.bcount; ++k) {
    double t;
    if (hit_prim_d(sc, sc.medium_refs[m.bfirst + k], o, d, time, lo, best, t)) {
      any = true;
      best = t;
    }
  }
  t_out = best;
  return any;
}

// constantMedium.Hit medium.go:27-58, as a closest-hit candidate.  A medium
// occurrence with multiplicity m keeps the smallest of m free-flight draws.
RT_D void trace_media(const Params& P, f3 o, f3 d, float time, float tmin, uint32_t gpix,
                      uint32_t sample, uint32_t vertex, Hit& best) {
  const DevScene& sc = P.sc;
  rt_u32x4 r = {{0, 0, 0, 0}};
  int cached_group = -1;
  for (int mi = 0; mi < sc.n_media; ++mi) {
    const DevMedium m = sc.media[mi];
    double t1, t2;
    if (!boundary_hit(sc, m, o, d, time, -(double)kInf, (double)kInf, t1)) continue;
    if (!boundary_hit(sc, m, o, d, time, t1 + 0.0001, (double)kInf, t2)) continue;
    t1 = fmax(t1, (double)tmin);
    if (t1 >= t2) continue;
    t1 = fmax(0.0, t1);
    float ray_len = length(d);
    double inside = (t2 - t1) * (double)ray_len;
    float hd = kInf;
    for (int k = 0; k < m.mult; ++k) {
      int draw = m.draw_base + k;
      int group = 1 + (draw >> 2);
      if (group != cached_group) {
        r = rt_rng_draw(P.seed, gpix, sample, RT_STREAM(vertex, group));
        cached_group = group;
      }
      float u = rt_unit_f(r.v[draw & 3]);
      hd = fminf(hd, m.neg_inv_density * logf(u));
    }
    if ((double)hd > inside) continue;
    float tm = (float)(t1 + (double)(hd / ray_len));
    if (tm < best.t) {
      best.t = tm;
      best.u = 0.0f;
      best.v = 0.0f;
      best.ref = prim_ref(PRIM_MEDIUM, (uint32_t)mi);
    }
  }
}

__global__ __launch_bounds__(256) void k_extend(Params P, int it) {
  __shared__ F4 lnodes[4 * kLdsNodes];
  const int nl = min(P.sc.n_nodes, kLdsNodes);
  for (int i = threadIdx.x; i < 4 * nl; i += blockDim.x) lnodes[i] = P.sc.nodes[i];
  __syncthreads();
  const uint32_t sel = (uint32_t)it & 1u;
  const uint32_t n = P.ctr->cnt[it % kMaxIt];
  const uint32_t* q = P.queue[sel];
  const uint32_t lane = lane_id();
  for (;;) {
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&P.ctr->head[it % kMaxIt], 64u);
    base = __shfl(base, 0);
    if (base >= n) break;
    uint32_t i = base + lane;
    if (lane == 0) atomicAdd(&P.ctr->segments, (unsigned long long)min(64u, n - base));
    if (i < n) {
      uint32_t slot = q[i];
      F4 ro = P.ray_o[slot], rd = P.ray_d[slot];
      f3 o = xyz(ro), d = xyz(rd);
      Hit best = {kInf, 0.0f, 0.0f, PRIM_NONE};
      trace_world(P.sc, lnodes, nl, o, d, ro.w, 0.001f, best);  // camera.go:300
      if (P.sc.n_media > 0 || P.trace) {
        uint2 ps = P.path[slot];
        Ids id = chunk_ids(P, ps.x);
        uint32_t j = ps.y & 0xFFFu, k = (ps.y >> 12) & 0xFFu;
        if (P.sc.n_media > 0) trace_media(P, o, d, ro.w, 0.001f, id.gpix, id.sample0 + j, k, best);
        if (P.trace && id.gpix == P.trace_gpix && id.sample0 + j == P.trace_sample &&
            (int)k < P.trace_cap) {
          P.trace[3 * k + 0] = ro;
          P.trace[3 * k + 1] = {rd.x, rd.y, rd.z, (float)k};
          P.trace[3 * k + 2] = {best.t, best.u, best.v, bitsf(best.ref)};
        }
      }
      P.hit[slot] = {best.t, best.u, best.v, bitsf(best.ref)};
    }
  }
}

// ---------------------------------------------------------------- shading --
// Texture.Value texture.go:10-125 (checker chains resolved iteratively)
RT_D float perlin_noise(const DevPerlin& pl, f3 p) {  // perlin.go:34-54
  float fx = floorf(p.x), fy = floorf(p.y), fz = floorf(p.z);
  float u = p.x - fx, v = p.y - fy, w = p.z - fz;
  int i = (int)fx, j = (int)fy, k = (int)fz;
  float uu = u * u * (3 - 2 * u), vv = v * v * (3 - 2 * v), ww = w * w * (3 - 2 * w);
  float accum = 0.0f;
  for (int di = 0; di < 2; ++di)
    for (int dj = 0; dj < 2; ++dj)
      for (int dk = 0; dk < 2; ++dk) {
        int idx = pl.perm[0][(i + di) & 255] ^ pl.perm[1][(j + dj) & 255] ^ pl.perm[2][(k + dk) & 255];
        F4 g = pl.ranvec[idx];
        f3 wt = mk3(u - (float)di, v - (float)dj, w - (float)dk);
        accum += ((float)di * uu + (float)(1 - di) * (1 - uu)) *
                 ((float)dj * vv + (float)(1 - dj) * (1 - vv)) *
                 ((float)dk * ww + (float)(1 - dk) * (1 - ww)) * dot(xyz(g), wt);
      }
  return accum;
}
RT_D float perlin_turb(const DevPerlin& pl, f3 p, int depth) {  // perlin.go:57-69
  float accum = 0.0f, weight = 1.0f;
  for (int i = 0; i < depth; ++i) {
    accum += weight * perlin_noise(pl, p);
    weight *= 0.5f;
    p = p * 2.0f;
  }
  return fabsf(accum);
}

RT_D f3 tex_value(const DevScene& sc, int tex, float u, float v, f3 p) {
  for (int guard = 0; guard < 64; ++guard) {
    const DevTexture T = sc.texs[tex];
    if (T.kind == RT_TEX_SOLID) return xyz(T.color);
    if (T.kind == RT_TEX_CHECKER) {  // texture.go:50-60
      float inv = T.color.w;
      int x = (int)floorf(inv * p.x), y = (int)floorf(inv * p.y), z = (int)floorf(inv * p.z);
      tex = ((x + y + z) % 2 == 0) ? T.a : T.b;
      continue;
    }
    if (T.kind == RT_TEX_IMAGE) {  // texture.go:70-86 + PixelData imageLoader.go:52-62
      const DevImage im = sc.images[T.a];
      if (im.h <= 0) return mk3(0, 1, 1);
      float uu = fabsf(fmodf(u, 1.0f));
      float vv = 1.0f - fabsf(fmodf(v, 1.0f));
      float fi = uu * (float)(im.w - 1), fj = vv * (float)(im.h - 1);
      int i = isnan(fi) ? 0 : (int)fi, j = isnan(fj) ? 0 : (int)fj;
      i = min(max(i, 0), im.w);
      j = min(max(j, 0), im.h);
      long idx = (long)j * im.w + i;
      if (idx >= (long)im.w * im.h) return mk3(1.0f, 0.0f, 1.0f);  // magenta
      const uint8_t* px = sc.texels + im.offset + 3 * idx;
      const float s = 1.0f / 255.0f;
      return mk3((float)px[0] * s, (float)px[1] * s, (float)px[2] * s);
    }
    // noise, texture.go:112-125
    const DevPerlin& pl = sc.perlins[T.a];
    float scale = T.color.w;
    if (T.variant == RT_NOISE_MARBLE) {
      float s = 0.5f * (1.0f + sinf(scale * p.z + 10.0f * perlin_turb(pl, p, 7)));
      return mk3(s, s, s);
    }
    if (T.variant == RT_NOISE_TURBULENT) {
      float s = perlin_turb(pl, p, 7);
      return mk3(s, s, s);
    }
    float s = 0.5f * (1.0f + perlin_noise(pl, p * scale));
    return mk3(s, s, s);
  }
  return mk3(0, 0, 0);
}

// light PdfValue: sphere objects.go:52-62, quad :152-160, triangle :356-367
RT_D f3 tri_normal(const DevScene& sc, uint32_t idx, float bu, float bv);
RT_D float prim_pdf(const DevScene& sc, uint32_t ref, f3 origin, f3 dir) {
  uint32_t type = ref >> 30, idx = ref & 0x3FFFFFFFu;
  if (type == PRIM_SPHERE) {
    float t;
    if (!hit_sphere(sc, idx, origin, dir, 0.0f, 0.0001f, kInf, t)) return 0.0f;
    const F4 cr = sc.sph_cr[idx];
    f3 oc = xyz(cr) - origin;
    float dist2 = dot(oc, oc);
    float cmax = sqrtf(1.0f - cr.w * cr.w / dist2);
    return 1.0f / (2.0f * kPi * (1.0f - cmax));
  }
  float t, u, v, area;
  f3 n;
  if (type == PRIM_QUAD) {
    if (!hit_quad(sc, idx, origin, dir, 0.001f, kInf, t, u, v)) return 0.0f;
    const F4* q = sc.quad + 5 * (size_t)idx;
    n = xyz(q[3]);
    area = q[1].w;
  } else {
    if (!hit_tri(sc, idx, origin, dir, 0.001f, kInf, t, u, v)) return 0.0f;
    n = tri_normal(sc, idx, u, v);
    area = sc.tri[3 * (size_t)idx + 1].w;
  }
  float dist2 = t * t * dot(dir, dir);
  float cosine = fabsf(dot(dir, n) / length(dir));
  return dist2 / (cosine * area);
}

// Triangle.interpolateNormal objects.go:389-405
RT_D f3 tri_normal(const DevScene& sc, uint32_t idx, float bu, float bv) {
  const F4* at = sc.tri_attr + 6 * (size_t)idx;
  uint32_t flags = fbits(sc.tri[3 * (size_t)idx + 2].w);
  if (!(flags & TRI_HAS_NORMALS)) return xyz(at[0]);
  float w = 1.0f - bu - bv;
  f3 n = xyz(at[1]) * w + xyz(at[2]) * bu + xyz(at[3]) * bv;
  return unit(n);
}

// HittableList.PdfValue hittable.go:89-97 over the flattened light table
RT_D float lights_pdf(const DevScene& sc, f3 origin, f3 dir) {
  float sum = 0.0f;
  for (int i = 0; i < sc.n_lights; ++i) {
    const DevLight L = sc.lights[i];
    if (L.ref == PRIM_NONE) continue;
    sum += L.weight * prim_pdf(sc, L.ref, origin, dir);
  }
  return sum;
}

// HittableList.Random hittable.go:98-103 + sphere/quad/Triangle.Random
RT_D f3 lights_random(const DevScene& sc, f3 origin, const rt_u32x4& r) {
  const float s0 = rt_unit_f(r.v[2]), s1 = rt_unit_f(r.v[3]);
  int lo = 0, hi = sc.n_lights - 1;
  if (sc.n_lights <= 0) return mk3(rt_unit_f(r.v[1]), s0, s1);  // vec.Random()
  const uint32_t u24 = rt_u24(r.v[1]);
  while (lo < hi) {  // last entry with lo24 <= u24
    int mid = (lo + hi + 1) >> 1;
    if (sc.lights[mid].lo24 <= u24) lo = mid;
    else hi = mid - 1;
  }
  const uint32_t ref = sc.lights[lo].ref;
  if (ref == PRIM_NONE) return mk3(rt_unit_f(r.v[1]), s0, s1);
  uint32_t type = ref >> 30, idx = ref & 0x3FFFFFFFu;
  if (type == PRIM_SPHERE) {  // sphere.Random + randomToSphere objects.go:63-80
    const F4 cr = sc.sph_cr[idx];
    f3 dir = xyz(cr) - origin;
    float dist2 = dot(dir, dir);
    Onb b = make_onb(dir);
    float z = 1.0f + s1 * (sqrtf(1.0f - cr.w * cr.w / dist2) - 1.0f);
    float phi = 2.0f * kPi * s0;
    float tt = sqrtf(1.0f - z * z);
    return onb_transform(b, mk3(cosf(phi) * tt, sinf(phi) * tt, z));
  }
  if (type == PRIM_QUAD) {  // quad.Random objects.go:161-165
    const F4* q = sc.quad + 5 * (size_t)idx;
    return (xyz(q[0]) + xyz(q[1]) * s0 + xyz(q[2]) * s1) - origin;
  }
  // Triangle.Random objects.go:369-385 (non-uniform barycentrics kept)
  const F4* tr = sc.tri + 3 * (size_t)idx;
  float r1 = s0, r2 = s1 * (1.0f - r1);
  f3 v0 = xyz(tr[0]), v1 = v0 + xyz(tr[1]), v2 = v0 + xyz(tr[2]);
  f3 p = v0 * (1.0f - r1 - r2) + v1 * r1 + v2 * r2;
  return p - origin;
}

enum { OUT_DEAD = 0, OUT_ALIVE = 1, OUT_NEED_CHUNK = 2 };

RT_D void flush_chunk(const Params& P, uint32_t chunk, f3 acc) {
  const uint32_t lp = chunk % P.npix;
  const float c[3] = {acc.x, acc.y, acc.z};
  for (int ch = 0; ch < 3; ++ch) {
    float v = c[ch];
    if (isnan(v)) {
      atomicOr(&P.pflags[lp], 1u << ch);
    } else if (isinf(v)) {
      atomicOr(&P.pflags[lp], 8u << ch);
    } else {
      float cl = fminf(fmaxf(v, -2147483648.0f), 2147483520.0f);
      long long fx = (long long)(cl * 4294967296.0f);
      atomicAdd(&P.accum[(size_t)ch * P.npix + lp], (unsigned long long)fx);
    }
  }
}

// One vertex of rayColor (camera.go:293-331) for the path in `slot`.
RT_D int shade_path(const Params& P, uint32_t slot) {
  const DevScene& sc = P.sc;
  const F4 h = P.hit[slot];
  const F4 ro = P.ray_o[slot], rd = P.ray_d[slot];
  const uint2 ps = P.path[slot];
  const uint32_t chunk = ps.x;
  uint32_t j = ps.y & 0xFFFu, k = (ps.y >> 12) & 0xFFu, nst = (ps.y >> 20) & 0xFFu,
           flags = ps.y >> 28;
  const f3 o = xyz(ro), d = xyz(rd);
  const float time = ro.w;
  const uint32_t ref = fbits(h.w);

  f3 lterm = mk3(0, 0, 0);
  bool term = false;
  if (ref == PRIM_NONE) {
    lterm = mk3(P.bg[0], P.bg[1], P.bg[2]);  // camera.go:300-302
    term = true;
  } else {
    const float t = h.x;
    const f3 p = o + d * t;  // r.At(t)
    const uint32_t type = ref >> 30, idx = ref & 0x3FFFFFFFu;
    f3 nout;
    float u = h.y, v = h.z;
    int mat;
    bool ff = true;
    f3 n;
    if (type == PRIM_SPHERE) {
      const F4 cr = sc.sph_cr[idx], mv = sc.sph_mv[idx];
      f3 cc = xyz(cr) + xyz(mv) * time;
      nout = (p - cc) * (1.0f / cr.w);
      mat = (int)fbits(mv.w);
      ff = dot(d, nout) < 0;  // setFaceNormal hittable.go:27-34
      n = ff ? nout : -nout;
      const DevMaterial M = sc.mats[mat];
      if (M._pad != 0.0f) {  // texture reads u,v: calculateSphereUV objects.go:44-50
        const F2 rs = sc.sph_uv[idx];
        f3 no = mk3(rs.x * nout.x - rs.y * nout.z, nout.y, rs.y * nout.x + rs.x * nout.z);
        float theta = acosf(-no.y);
        float phi = atan2f(-no.z, no.x) + kPi;
        u = phi / (2.0f * kPi);
        v = theta / kPi;
      }
    } else if (type == PRIM_QUAD) {
      const F4* q = sc.quad + 5 * (size_t)idx;
      nout = xyz(q[3]);
      mat = (int)fbits(q[2].w);
      ff = dot(d, nout) < 0;
      n = ff ? nout : -nout;
    } else if (type == PRIM_TRI) {
      nout = tri_normal(sc, idx, u, v);
      mat = (int)fbits(sc.tri[3 * (size_t)idx].w);
      ff = dot(d, nout) < 0;
      n = ff ? nout : -nout;
      uint32_t tf = fbits(sc.tri[3 * (size_t)idx + 2].w);
      if (tf & TRI_HAS_UV) {  // objects.go:437-446
        const F4* at = sc.tri_attr + 6 * (size_t)idx;
        float w = 1.0f - u - v;
        float tu = w * at[4].x + u * at[4].z + v * at[5].x;
        float tv = w * at[4].y + u * at[4].w + v * at[5].y;
        u = tu;
        v = tv;
      }
    } else {  // medium hit medium.go:162-166: normal (1,0,0), front face
      const DevMedium m = sc.media[idx];
      mat = m.phase_mat;
      n = mk3(1, 0, 0);
      ff = true;
      u = v = 0.0f;
    }
    const DevMaterial M = sc.mats[mat];
    if (M.kind == RT_MAT_DIFFUSE_LIGHT) {  // Emitted materials.go:150-155; Scatter false
      lterm = ff ? tex_value(sc, M.tex, u, v, p) : mk3(0, 0, 0);
      term = true;
    } else {
      const Ids id = chunk_ids(P, chunk);
      const rt_u32x4 r = rt_rng_draw(P.seed, id.gpix, id.sample0 + j, RT_STREAM(k, 0));
      f3 ndir;
      bool clamp_vertex = false;
      f3 weight;
      if (M.kind == RT_MAT_METAL) {  // materials.go:70-79
        f3 refl = unit(reflect(d, n));
        ndir = refl + uniform_sphere(rt_unit_f(r.v[2]), rt_unit_f(r.v[3])) * M.param;
        weight = xyz(M.albedo);
      } else if (M.kind == RT_MAT_DIELECTRIC) {  // materials.go:94-130
        float ior = M.param;
        float ri = ff ? 1.0f / ior : ior;
        f3 ud = unit(d);
        float cs = fminf(dot(-ud, n), 1.0f);
        float sn = sqrtf(1.0f - cs * cs);
        bool cannot = ri * sn > 1.0f;
        bool refl = cannot;
        if (!cannot) {
          float r0 = (1.0f - ior) / (1.0f + ior);
          r0 = r0 * r0;
          float refl_p = r0 + (1.0f - r0) * powf(1.0f - cs, 5.0f);
          refl = refl_p > rt_unit_f(r.v[0]);
        }
        ndir = refl ? reflect(ud, n) : refract(ud, n, ri);
        weight = mk3(1, 1, 1);
      } else {  // lambertian materials.go:45-57 / isotropic :157-177 + mixture pdf.go:58-74
        const bool iso = M.kind == RT_MAT_ISOTROPIC;
        f3 att = tex_value(sc, M.tex, u, v, p);
        Onb b;
        if (!iso) b = make_onb(n);
        if (rt_unit_f(r.v[0]) < 0.5f) {
          ndir = lights_random(sc, p, r);
        } else if (iso) {
          ndir = uniform_sphere(rt_unit_f(r.v[2]), rt_unit_f(r.v[3]));
        } else {
          ndir = onb_transform(b, cosine_direction(rt_unit_f(r.v[2]), rt_unit_f(r.v[3])));
        }
        float bsdf_pdf, spdf;
        if (iso) {
          bsdf_pdf = 1.0f / (4.0f * kPi);
          spdf = 1.0f / (4.0f * kPi);
        } else {
          f3 ud = unit(ndir);
          bsdf_pdf = fmaxf(0.0f, dot(ud, b.w) / kPi);
          float ct = dot(n, ud);
          spdf = ct < 0.0f ? 0.0f : ct / kPi;
        }
        float pdf = 0.5f * lights_pdf(sc, p, ndir) + 0.5f * bsdf_pdf;
        weight = (att * spdf) * (1.0f / pdf);
        clamp_vertex = true;
      }
      // vertex bookkeeping (H1: clamp is folded backwards at termination)
      if (clamp_vertex) {
        if (flags & F_PEND) {
          P.stack[(size_t)nst * P.P + slot] = P.pend[slot];
          ++nst;
          atomicAdd(&P.ctr->pushes, 1ull);
        }
        P.pend[slot] = {weight.x, weight.y, weight.z, 0.0f};
        flags |= F_PEND;
      } else if (flags & F_PEND) {
        F4 w = P.pend[slot];
        P.pend[slot] = {w.x * weight.x, w.y * weight.y, w.z * weight.z, 0.0f};
      } else {
        F4 w = (flags & F_PRE) ? P.pre[slot] : F4{1, 1, 1, 0};
        P.pre[slot] = {w.x * weight.x, w.y * weight.y, w.z * weight.z, 0.0f};
        flags |= F_PRE;
      }
      if (!finite3(weight)) flags |= F_NONFINITE;
      ++k;
      if ((int)k > P.max_depth) {  // rayColor(depth-1 < 0) == black, camera.go:294-296
        term = true;
        lterm = mk3(0, 0, 0);
      } else {
        P.ray_o[slot] = {p.x, p.y, p.z, time};
        P.ray_d[slot] = {ndir.x, ndir.y, ndir.z, 0.0f};
        P.path[slot] = make_uint2(chunk, pack_path(j, k, nst, flags));
        return OUT_ALIVE;
      }
    }
  }
  // ---- termination: backward clamp fold (camera.go:316, :328-330)
  f3 L = lterm;
  const bool zero = lterm.x == 0.0f && lterm.y == 0.0f && lterm.z == 0.0f;
  if (!(zero && !(flags & F_NONFINITE))) {
    if (flags & F_PEND) L = clamp_contribution(xyz(P.pend[slot]) * L, P.maxc);
    for (int kk = (int)nst - 1; kk >= 0; --kk)
      L = clamp_contribution(xyz(P.stack[(size_t)kk * P.P + slot]) * L, P.maxc);
    if (flags & F_PRE) L = xyz(P.pre[slot]) * L;
  } else {
    L = mk3(0, 0, 0);
  }
  f3 acc = L;
  if (j > 0) acc = xyz(P.acc[slot]) + L;
  const Ids id = chunk_ids(P, chunk);
  ++j;
  if (j < id.count) {
    P.acc[slot] = {acc.x, acc.y, acc.z, 0.0f};
    start_sample(P, slot, chunk, j);
    return OUT_ALIVE;
  }
  flush_chunk(P, chunk, acc);
  return OUT_NEED_CHUNK;
}

__global__ __launch_bounds__(256) void k_shade(Params P, int it) {
  const uint32_t sel = (uint32_t)it & 1u;
  const uint32_t n = P.ctr->cnt[it % kMaxIt];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = lane_id();
  const bool active = i < n;
  uint32_t slot = active ? P.queue[sel][i] : 0u;
  int outcome = active ? shade_path(P, slot) : OUT_DEAD;

  // regeneration: lanes whose chunk is done grab new chunks, one atomic per wave
  const bool need = outcome == OUT_NEED_CHUNK;
  const unsigned long long nm = __ballot(need);
  if (nm) {
    const int leader = __ffsll((long long)nm) - 1;
    uint32_t base = 0;
    if ((int)lane == leader) base = atomicAdd(&P.ctr->chunk_head, (uint32_t)__popcll(nm));
    base = __shfl(base, leader);
    if (need) {
      uint32_t c = base + prefix_count(nm);
      if (c < P.n_chunks) {
        start_sample(P, slot, c, 0);
        outcome = OUT_ALIVE;
      } else {
        outcome = OUT_DEAD;
      }
    }
  }
  // compaction of surviving paths into the next queue (ballot + prefix)
  const bool alive = outcome == OUT_ALIVE;
  const unsigned long long am = __ballot(alive);
  if (am) {
    const int leader = __ffsll((long long)am) - 1;
    uint32_t base = 0;
    if ((int)lane == leader)
      base = atomicAdd(&P.ctr->cnt[(it + 1) % kMaxIt], (uint32_t)__popcll(am));
    base = __shfl(base, leader);
    if (alive) P.queue[sel ^ 1u][base + prefix_count(am)] = slot;
  }
}

__global__ __launch_bounds__(256) void k_init(Params P) {
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= P.P) return;
  if (slot < P.n_chunks) {
    start_sample(P, slot, slot, 0);
    P.queue[0][slot] = slot;
  }
  if (slot == 0) {
    P.ctr->cnt[0] = min(P.P, P.n_chunks);
    P.ctr->chunk_head = P.P;
  }
}

// fixed-point sums -> linear mean RGB; Scale(pixelSamplesScale) camera.go:103
__global__ __launch_bounds__(256) void k_resolve(Params P, float* out, double scale) {
  const uint32_t lp = blockIdx.x * blockDim.x + threadIdx.x;
  if (lp >= P.npix) return;
  const uint32_t f = P.pflags[lp];
  for (int ch = 0; ch < 3; ++ch) {
    float v;
    if (f & (1u << ch)) {
      v = __builtin_nanf("");
    } else if (f & (8u << ch)) {
      v = kInf;
    } else {
      long long s = (long long)P.accum[(size_t)ch * P.npix + lp];
      v = (float)((double)s * 2.3283064365386963e-10 * scale);
    }
    out[3 * (size_t)lp + ch] = v;
  }
}

// ==================================================================== host ==
#define HIP_OK(expr)                                                                    \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      return set_error(RT_ERR_DEVICE, "%s failed: %s", #expr, hipGetErrorString(_e));   \
  } while (0)

struct DeviceScene {
  int device = -1;
  std::vector<void*> allocs;
  DevScene d{};
  ~DeviceScene() {
    for (void* p : allocs) (void)hipFree(p);
  }
};

struct RenderState {
  int device = -1;
  uint32_t P = 0;
  int depth_cap = 0;
  uint32_t npix = 0;
  hipStream_t own_stream = nullptr;
  std::vector<void*> allocs;
  F4 *ray_o = nullptr, *ray_d = nullptr, *hit = nullptr, *pend = nullptr, *pre = nullptr,
     *acc = nullptr, *stack = nullptr;
  uint2* path = nullptr;
  uint32_t* queue[2] = {nullptr, nullptr};
  Counters* ctr = nullptr;
  unsigned long long* accum = nullptr;
  uint32_t* pflags = nullptr;
  float* out = nullptr;
  uint32_t out_cap = 0;
  std::vector<hipEvent_t> events;
  int resident_blocks = 0;
  void free_all() {
    for (void* p : allocs) (void)hipFree(p);
    allocs.clear();
  }
  ~RenderState() {
    free_all();
    for (auto e : events) (void)hipEventDestroy(e);
    if (own_stream) (void)hipStreamDestroy(own_stream);
  }
};

void release_device(Scene* s) {
  delete s->dev;
  s->dev = nullptr;
  delete s->state;
  s->state = nullptr;
}

template <typename T>
static int upload(DeviceScene* ds, const std::vector<T>& v, const T** out) {
  *out = nullptr;
  if (v.empty()) return RT_OK;
  void* p = nullptr;
  HIP_OK(hipMalloc(&p, v.size() * sizeof(T)));
  ds->allocs.push_back(p);
  HIP_OK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  *out = (const T*)p;
  return RT_OK;
}

static int ensure_scene(Scene* s, int device) {
  if (s->dev && s->dev->device == device) return RT_OK;
  delete s->dev;
  s->dev = new DeviceScene();
  s->dev->device = device;
  const HostScene& h = s->h;
  DevScene& d = s->dev->d;
  // per-material "texture reads u,v" flag for sphere UV (stored in the pad)
  std::vector<DevMaterial> mats = h.mats;
  for (auto& m : mats) {
    bool needs = false;
    std::vector<int> st;
    if (m.kind != RT_MAT_METAL && m.kind != RT_MAT_DIELECTRIC && m.tex >= 0) st.push_back(m.tex);
    int guard = 0;
    while (!st.empty() && guard++ < 4096) {
      int tx = st.back();
      st.pop_back();
      const DevTexture& T = h.texs[tx];
      if (T.kind == RT_TEX_IMAGE) needs = true;
      if (T.kind == RT_TEX_CHECKER) {
        st.push_back(T.a);
        st.push_back(T.b);
      }
    }
    m._pad = needs ? 1.0f : 0.0f;
  }
  int rc;
#define UP(vec, field)                                      \
  if ((rc = upload(s->dev, vec, &d.field)) != RT_OK) return rc;
  UP(h.sph_cr, sph_cr);
  UP(h.sph_mv, sph_mv);
  UP(h.sph_uv, sph_uv);
  UP(h.quad, quad);
  UP(h.tri, tri);
  UP(h.tri_attr, tri_attr);
  UP(h.nodes, nodes);
  UP(h.refs, refs);
  UP(h.media, media);
  UP(h.medium_refs, medium_refs);
  UP(h.lights, lights);
  UP(mats, mats);
  UP(h.texs, texs);
  UP(h.texels, texels);
  UP(h.images, images);
  UP(h.perlins, perlins);
#undef UP
  d.root = h.root;
  d.n_nodes = (int32_t)(h.nodes.size() / 4);
  d.n_media = (int32_t)h.media.size();
  d.medium_draws = h.medium_draws;
  d.n_lights = (int32_t)h.lights.size();
  return RT_OK;
}

template <typename T>
static int dalloc(RenderState* st, T** p, size_t count) {
  void* q = nullptr;
  HIP_OK(hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T)));
  st->allocs.push_back(q);
  *p = (T*)q;
  return RT_OK;
}

static int ensure_state(Scene* s, int device, uint32_t P, int depth_cap, uint32_t npix) {
  RenderState* st = s->state;
  if (st && (st->device != device || st->P < P || st->depth_cap < depth_cap || st->npix < npix)) {
    delete st;
    st = s->state = nullptr;
  }
  if (st) return RT_OK;
  st = s->state = new RenderState();
  st->device = device;
  st->P = P;
  st->depth_cap = depth_cap;
  st->npix = npix;
  int rc;
  if ((rc = dalloc(st, &st->ray_o, P)) || (rc = dalloc(st, &st->ray_d, P)) ||
      (rc = dalloc(st, &st->hit, P)) || (rc = dalloc(st, &st->pend, P)) ||
      (rc = dalloc(st, &st->pre, P)) || (rc = dalloc(st, &st->acc, P)) ||
      (rc = dalloc(st, &st->stack, (size_t)P * depth_cap)) || (rc = dalloc(st, &st->path, P)) ||
      (rc = dalloc(st, &st->queue[0], P)) || (rc = dalloc(st, &st->queue[1], P)) ||
      (rc = dalloc(st, &st->ctr, 1)) || (rc = dalloc(st, &st->accum, 3 * (size_t)npix)) ||
      (rc = dalloc(st, &st->pflags, npix)) || (rc = dalloc(st, &st->out, 3 * (size_t)npix)))
    return rc;
  int per_cu = 0, cus = 0;
  HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_extend, 256, 0));
  HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  st->resident_blocks = std::max(1, per_cu) * std::max(1, cus);
  return RT_OK;
}

static int render_impl(rt_scene* scene, const rt_camera* cam, const rt_render_opts* opts,
                       float* out_host, float* out_dev, rt_stats* stats) {
  if (!scene || !cam) return set_error(RT_ERR_INVALID, "rt_render: null scene/camera");
  rt_render_opts o{};
  if (opts) o = *opts;
  if (o.nranks <= 0) o.nranks = 1;
  if (o.rank < 0 || o.rank >= o.nranks) return set_error(RT_ERR_INVALID, "rt_render: bad rank");
  rt_camera_derived cd;
  int rc = rt_camera_derive(cam, &cd);
  if (rc) return rc;
  auto t_start = std::chrono::steady_clock::now();

  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return set_error(RT_ERR_DEVICE, "rt_render: no HIP device available");
  if (o.device < 0 || o.device >= ndev)
    return set_error(RT_ERR_INVALID, "rt_render: device %d of %d", o.device, ndev);
  HIP_OK(hipSetDevice(o.device));
  Scene* s = &scene->s;
  if ((rc = ensure_scene(s, o.device))) return rc;

  const uint32_t W = (uint32_t)cd.width, H = (uint32_t)cd.height;
  const uint32_t rows = H > (uint32_t)o.rank ? (H - (uint32_t)o.rank + o.nranks - 1) / o.nranks : 0;
  const uint32_t npix = rows * W;
  const uint32_t ss = (uint32_t)cd.spp_sqrt * (uint32_t)cd.spp_sqrt;
  uint32_t K = o.chunk > 0 ? (uint32_t)o.chunk : std::min<uint32_t>(ss, 32u);
  K = std::min<uint32_t>(std::min(K, ss), 4096u);
  const uint32_t cpp = (ss + K - 1) / K;
  const uint64_t n_chunks64 = (uint64_t)npix * cpp;
  if (n_chunks64 >= 0xFFFFFFFFull) return set_error(RT_ERR_UNSUPPORTED, "too many work chunks");
  const uint32_t n_chunks = (uint32_t)n_chunks64;
  uint32_t P = o.path_slots > 0 ? (uint32_t)o.path_slots : (1u << 20);
  P = std::max<uint32_t>(256u, std::min<uint32_t>(P, std::max<uint32_t>(n_chunks, 256u)));
  P = (P + 255u) & ~255u;
  const int depth_cap = cd.max_depth + 1;
  if ((rc = ensure_state(s, o.device, P, depth_cap, std::max<uint32_t>(npix, 1)))) return rc;
  RenderState* st = s->state;

  hipStream_t stream = (hipStream_t)o.stream;
  if (!stream) {
    if (!st->own_stream) HIP_OK(hipStreamCreateWithFlags(&st->own_stream, hipStreamNonBlocking));
    stream = st->own_stream;
  }

  Params p{};
  p.sc = s->dev->d;
  for (int i = 0; i < 3; ++i) {
    p.p00r[i] = (float)(cd.pixel00[i] - cd.center[i]);
    p.du[i] = (float)cd.delta_u[i];
    p.dv[i] = (float)cd.delta_v[i];
    p.cc[i] = (float)cd.center[i];
    p.dku[i] = (float)cd.defocus_u[i];
    p.dkv[i] = (float)cd.defocus_v[i];
    p.bg[i] = (float)cd.background[i];
  }
  p.recip_s = (float)cd.recip_spp_sqrt;
  p.maxc = (float)cd.max_contribution;
  p.s = cd.spp_sqrt;
  p.defocus = cd.defocus_angle > 0 ? 1 : 0;  // camera.go:262
  p.max_depth = cd.max_depth;
  p.width = (int)W;
  p.rank = o.rank;
  p.nranks = o.nranks;
  p.npix = npix;
  p.K = K;
  p.cpp = cpp;
  p.n_chunks = n_chunks;
  p.P = P;
  p.ss = ss;
  p.seed = o.seed;
  p.ray_o = st->ray_o;
  p.ray_d = st->ray_d;
  p.hit = st->hit;
  p.path = st->path;
  p.pend = st->pend;
  p.pre = st->pre;
  p.acc = st->acc;
  p.stack = st->stack;
  p.queue[0] = st->queue[0];
  p.queue[1] = st->queue[1];
  p.ctr = st->ctr;
  p.accum = st->accum;
  p.pflags = st->pflags;

  F4* dtrace = nullptr;
  if (o.trace_out && o.trace_cap > 0) {
    HIP_OK(hipMalloc(&dtrace, (size_t)o.trace_cap * 3 * sizeof(F4)));
    std::vector<float> init((size_t)o.trace_cap * 12, 0.0f);
    for (int v = 0; v < o.trace_cap; ++v) init[12 * v + 7] = -1.0f;
    HIP_OK(hipMemcpy(dtrace, init.data(), init.size() * 4, hipMemcpyHostToDevice));
    p.trace = dtrace;
    p.trace_gpix = (uint32_t)o.trace_pixel;
    p.trace_sample = (uint32_t)o.trace_sample;
    p.trace_cap = o.trace_cap;
  }
  const bool prof = (o.flags & RT_FLAG_PROFILE) != 0;
  std::vector<std::pair<int, int>> ev_ext, ev_shade;  // event index pairs
  int ev_used = 0;
  auto next_event = [&](hipEvent_t* e) -> int {
    if (ev_used >= (int)st->events.size()) {
      hipEvent_t ne;
      HIP_OK(hipEventCreate(&ne));
      st->events.push_back(ne);
    }
    *e = st->events[ev_used++];
    return RT_OK;
  };

  HIP_OK(hipMemsetAsync(st->ctr, 0, sizeof(Counters), stream));
  if (npix > 0) {
    HIP_OK(hipMemsetAsync(st->accum, 0, 3 * (size_t)npix * sizeof(unsigned long long), stream));
    HIP_OK(hipMemsetAsync(st->pflags, 0, (size_t)npix * sizeof(uint32_t), stream));
  }
  int iterations = 0;
  uint64_t ext_rays = 0;
  int n_ext = 0, n_sh = 0;
  if (n_chunks > 0) {
    hipLaunchKernelGGL(k_init, dim3((P + 255) / 256), dim3(256), 0, stream, p);
    HIP_OK(hipGetLastError());
    uint32_t n_est = std::min(P, n_chunks);
    const int kBatch = 4;
    while (n_est > 0) {
      for (int b = 0; b < kBatch; ++b) {
        if (iterations > 0 && iterations % kMaxIt == 0)
          return set_error(RT_ERR_UNSUPPORTED, "more than %d wavefront iterations", kMaxIt);
        const uint32_t ext_blocks =
            std::max<uint32_t>(1u, std::min<uint32_t>((n_est + 255) / 256, (uint32_t)st->resident_blocks));
        hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;
        if (prof) {
          if ((rc = next_event(&e0)) || (rc = next_event(&e1)) || (rc = next_event(&e2))) return rc;
          HIP_OK(hipEventRecord(e0, stream));
        }
        hipLaunchKernelGGL(k_extend, dim3(ext_blocks), dim3(256), 0, stream, p, iterations);
        if (prof) HIP_OK(hipEventRecord(e1, stream));
        hipLaunchKernelGGL(k_shade, dim3((n_est + 255) / 256), dim3(256), 0, stream, p,
                           iterations);
        if (prof) {
          HIP_OK(hipEventRecord(e2, stream));
          ev_ext.push_back({ev_used - 3, ev_used - 2});
          ev_shade.push_back({ev_used - 2, ev_used - 1});
        }
        HIP_OK(hipGetLastError());
        ++n_ext;
        ++n_sh;
        ++iterations;
      }
      uint32_t n_now = 0;
      HIP_OK(hipMemcpyAsync(&n_now, &st->ctr->cnt[iterations % kMaxIt], 4, hipMemcpyDeviceToHost,
                            stream));
      HIP_OK(hipStreamSynchronize(stream));
      n_est = n_now;
    }
  }
  float* dst = out_dev ? out_dev : st->out;
  if (npix > 0) {
    hipLaunchKernelGGL(k_resolve, dim3((npix + 255) / 256), dim3(256), 0, stream, p, dst,
                       cd.pixel_samples_scale);
    HIP_OK(hipGetLastError());
  }
  if (out_host && npix > 0)
    HIP_OK(hipMemcpyAsync(out_host, dst, 3 * (size_t)npix * sizeof(float), hipMemcpyDeviceToHost,
                          stream));
  HIP_OK(hipStreamSynchronize(stream));
  auto t_end = std::chrono::steady_clock::now();
  if (dtrace) {
    HIP_OK(hipMemcpy(o.trace_out, dtrace, (size_t)o.trace_cap * 3 * sizeof(F4), hipMemcpyDeviceToHost));
    HIP_OK(hipFree(dtrace));
  }

  if (stats) {
    memset(stats, 0, sizeof *stats);
    Counters hc;
    HIP_OK(hipMemcpy(&hc, st->ctr, offsetof(Counters, cnt), hipMemcpyDeviceToHost));
    stats->samples = (uint64_t)npix * ss;
    stats->segments = hc.segments;
    stats->stack_pushes = hc.pushes;
    stats->extend_rays = hc.segments;
    stats->shade_rays = hc.segments;
    stats->ms_total = std::chrono::duration<double, std::milli>(t_end - t_start).count();
    stats->n_extend_launches = n_ext;
    stats->n_shade_launches = n_sh;
    stats->iterations = iterations;
    stats->rows = (int32_t)rows;
    if (prof) {
      double te = 0, ts = 0;
      for (auto& pr : ev_ext) {
        float ms = 0;
        HIP_OK(hipEventElapsedTime(&ms, st->events[pr.first], st->events[pr.second]));
        te += ms;
      }
      for (auto& pr : ev_shade) {
        float ms = 0;
        HIP_OK(hipEventElapsedTime(&ms, st->events[pr.first], st->events[pr.second]));
        ts += ms;
      }
      stats->ms_extend = te;
      stats->ms_shade = ts;
    }
  }
  (void)ext_rays;
  return RT_OK;
}

}  // namespace rt

extern "C" {

int rt_render(rt_scene* s, const rt_camera* cam, const rt_render_opts* opts, float* out_rgb,
              rt_stats* stats) {
  if (!out_rgb) return rt::set_error(RT_ERR_INVALID, "rt_render: null output");
  return rt::render_impl(s, cam, opts, out_rgb, nullptr, stats);
}

int rt_render_device(rt_scene* s, const rt_camera* cam, const rt_render_opts* opts,
                     float* out_rgb_device, rt_stats* stats) {
  if (!out_rgb_device) return rt::set_error(RT_ERR_INVALID, "rt_render_device: null output");
  return rt::render_impl(s, cam, opts, nullptr, out_rgb_device, stats);
}

int rt_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

}  // extern "C"
