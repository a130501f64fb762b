// rt_kernels.h — device-side math, sampling and intersection for the MI355X path.
// Each function cites the reference function it re-implements.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_device.h"
#include "rt_rng.h"

namespace rt {

#define RT_D __device__ __forceinline__

constexpr float kPi = 3.14159265358979323846f;
constexpr float kInf = __builtin_huge_valf();
constexpr float kInvPi = 0.318309886183790671538f;

struct f3 {
  float x, y, z;
};
RT_D f3 mk3(float x, float y, float z) { return {x, y, z}; }
RT_D f3 xyz(const F4& v) { return {v.x, v.y, v.z}; }
RT_D f3 operator+(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
RT_D f3 operator-(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
RT_D f3 operator-(f3 a) { return {-a.x, -a.y, -a.z}; }
RT_D f3 operator*(f3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
RT_D f3 operator*(f3 a, f3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
RT_D float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
RT_D f3 cross(f3 a, f3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// v_sqrt_f32 / v_rcp_f32 (1 ulp): without the denormal-range scaling (sqrtf emits
// ldexp / cndmask around v_sqrt, and a correctly rounded sequence of ~14 ops in some
// contexts).  Arguments here are lengths and [0,1] sampling values; a denormal one
// is off by less than its own size.
RT_D float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
RT_D float length(f3 a) { return fsqrt(dot(a, a)); }
RT_D float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
// UnitVector vec.go:125 as one v_rsq_f32 (1 ulp) instead of v_sqrt + v_rcp (two roundings,
// two transcendental issues at a quarter of the VALU rate)
RT_D f3 unit(f3 a) { return a * __builtin_amdgcn_rsqf(dot(a, a)); }
RT_D bool finite3(f3 a) { return isfinite(a.x) && isfinite(a.y) && isfinite(a.z); }

RT_D uint32_t fbits(float f) { return __float_as_uint(f); }
RT_D float bitsf(uint32_t u) { return __uint_as_float(u); }
RT_D F4 ldg4(const F4* p) { return *p; }

// ------------------------------------------------------------- sampling ----
// cos/sin(2*pi*u) for u in [0,1): v_cos_f32 / v_sin_f32 take their argument in
// revolutions, so the sampling angles need no range reduction.
RT_D float cos2pi(float u) { return __builtin_amdgcn_cosf(u); }
RT_D float sin2pi(float u) { return __builtin_amdgcn_sinf(u); }

// Distribution-identical closed forms of the reference's rejection samplers.
// RandomUnitVector vec.go:159-167 (uniform on the sphere)
RT_D f3 uniform_sphere(float u0, float u1) {
  float z = 1.0f - 2.0f * u0;
  float r = fsqrt(fmaxf(0.0f, 1.0f - z * z));
  return {r * cos2pi(u1), r * sin2pi(u1), z};
}
// RandomUnitDisk vec.go:149-156 (uniform in the disk)
RT_D f3 uniform_disk(float u0, float u1) {
  float r = fsqrt(u0);
  return {r * cos2pi(u1), r * sin2pi(u1), 0.0f};
}
// RandomCosineDirection vec.go:177-186: phi = 2*pi*r1
RT_D f3 cosine_direction(float r1, float r2) {
  float s = fsqrt(r2);
  return {cos2pi(r1) * s, sin2pi(r1) * s, fsqrt(1.0f - r2)};
}

// NewONB onb.go:13-25 — note the 0.9 test is on the un-normalised vector
struct Onb {
  f3 u, v, w;
};
RT_D Onb make_onb(f3 n) {
  Onb o;
  o.w = unit(n);
  f3 a = fabsf(n.x) > 0.9f ? mk3(0, 1, 0) : mk3(1, 0, 0);
  o.v = unit(cross(n, a));
  // unit(cross(n, v)) = cross(n, v) / |n| = cross(w, v): w and v are unit and orthogonal, so
  // the reference's third normalisation (onb.go:23) is the identity up to rounding
  o.u = cross(o.w, o.v);
  return o;
}
// NewONB of a normal that is already unit (every shading normal: quad and triangle normals are
// stored normalised, sphere normals divided by their length): w = n, whose normalisation the
// reference repeats (onb.go:21) and which changes it by at most an ulp here
RT_D Onb make_onb_unit(f3 n) {
  Onb o;
  o.w = n;
  f3 a = fabsf(n.x) > 0.9f ? mk3(0, 1, 0) : mk3(1, 0, 0);
  o.v = unit(cross(n, a));
  o.u = cross(o.w, o.v);
  return o;
}
RT_D f3 onb_transform(const Onb& o, f3 v) { return o.u * v.x + o.v * v.y + o.w * v.z; }  // :38-43

// Reflect / Refract vec.go:136-146
RT_D f3 reflect(f3 v, f3 n) { return v - n * (dot(n, v) * 2.0f); }
RT_D f3 refract(f3 v, f3 n, float eta) {
  float c = fminf(dot(-v, n), 1.0f);
  f3 perp = (v + n * c) * eta;
  f3 par = n * (-fsqrt(fabsf(1.0f - dot(perp, perp))));
  return perp + par;
}

// clampContribution camera.go:334-341
RT_D f3 clamp_contribution(f3 c, float maxv) {
  float intensity = c.x + c.y + c.z;
  if (intensity > maxv) return c * (maxv * rcp(intensity));
  return c;
}

// --------------------------------------------------------- intersection ----
// sphere.Hit objects.go:83-115 — evaluated in fp64 (fp32 cancels in
// |oc|^2 - r^2 for the R=1000 ground and R=5000 fog spheres).  Open interval.
RT_D bool hit_sphere_d(const DevScene& sc, uint32_t i, f3 o, f3 d, float time, double tmin,
                       double tmax, double& t_out) {
  const F4 cr = sc.sph_cr[i];
  const F4 mv = sc.sph_mv[i];
  double cx = (double)cr.x + (double)time * (double)mv.x;
  double cy = (double)cr.y + (double)time * (double)mv.y;
  double cz = (double)cr.z + (double)time * (double)mv.z;
  double ox = cx - (double)o.x, oy = cy - (double)o.y, oz = cz - (double)o.z;
  double dx = d.x, dy = d.y, dz = d.z;
  double a = dx * dx + dy * dy + dz * dz;
  double h = dx * ox + dy * oy + dz * oz;
  double r = cr.w;
  double c = ox * ox + oy * oy + oz * oz - r * r;
  double disc = h * h - a * c;
  if (disc < 0) return false;
  // v_sqrt_f64 / v_rcp_f64 (~2^-23 relative) + one Newton step each (~1e-14):
  // fp64-grade roots (media need |t| ~ 1e4 to 1e-4) without the library sequences
  double sq = __builtin_amdgcn_sqrt(disc);
  sq = disc > 0.0 ? fma(0.5 * fma(-sq, sq, disc), __builtin_amdgcn_rcp(sq), sq) : 0.0;
  double ia = __builtin_amdgcn_rcp(a);
  ia = fma(ia, fma(-a, ia, 1.0), ia);
  double root = (h - sq) * ia;
  if (!(tmin < root && root < tmax)) {
    root = (h + sq) * ia;
    if (!(tmin < root && root < tmax)) return false;
  }
  t_out = root;
  return true;
}
// Both roots of the sphere quadratic, as hit_sphere_d computes them (same
// arithmetic, so identical doubles): r0 <= r1.  False when the ray misses.
RT_D bool sphere_roots_cm(F4 cr, F4 mv, f3 o, f3 d, float time, double& r0, double& r1);
RT_D bool sphere_roots_d(const DevScene& sc, uint32_t i, f3 o, f3 d, float time, double& r0,
                         double& r1) {
  return sphere_roots_cm(sc.sph_cr[i], sc.sph_mv[i], o, d, time, r0, r1);
}
// the same from the sphere's center | radius and motion records
RT_D bool sphere_roots_cm(F4 cr, F4 mv, f3 o, f3 d, float time, double& r0, double& r1) {
  double cx = (double)cr.x + (double)time * (double)mv.x;
  double cy = (double)cr.y + (double)time * (double)mv.y;
  double cz = (double)cr.z + (double)time * (double)mv.z;
  double ox = cx - (double)o.x, oy = cy - (double)o.y, oz = cz - (double)o.z;
  double dx = d.x, dy = d.y, dz = d.z;
  double a = dx * dx + dy * dy + dz * dz;
  double h = dx * ox + dy * oy + dz * oz;
  double r = cr.w;
  double c = ox * ox + oy * oy + oz * oz - r * r;
  double disc = h * h - a * c;
  if (disc < 0) return false;
  double sq = __builtin_amdgcn_sqrt(disc);
  sq = disc > 0.0 ? fma(0.5 * fma(-sq, sq, disc), __builtin_amdgcn_rcp(sq), sq) : 0.0;
  double ia = __builtin_amdgcn_rcp(a);
  ia = fma(ia, fma(-a, ia, 1.0), ia);
  r0 = (h - sq) * ia;
  r1 = (h + sq) * ia;
  return true;
}

RT_D bool hit_sphere(const DevScene& sc, uint32_t i, f3 o, f3 d, float time, float tmin,
                     float tmax, float& t_out) {
  double t;
  if (!hit_sphere_d(sc, i, o, d, time, (double)tmin, (double)tmax, t)) return false;
  t_out = (float)t;
  return true;
}

// quad.Hit objects.go:167-196 + isInterior :198-206 — closed interval
RT_D bool hit_quad(const DevScene& sc, uint32_t i, f3 o, f3 d, float tmin, float tmax,
                   float& t_out, float& a_out, float& b_out) {
  const F4* q = sc.quad + 5 * (size_t)i;
  const F4 Qd = q[0], U = q[1], Vm = q[2], N = q[3], W = q[4];
  f3 n = xyz(N);
  float denom = dot(n, d);
  if (fabsf(denom) < 1e-8f) return false;
  float t = (Qd.w - dot(n, o)) / denom;
  if (!(tmin <= t && t <= tmax)) return false;
  f3 pp = (o + d * t) - xyz(Qd);
  f3 w = xyz(W);
  float alpha = dot(w, cross(pp, xyz(Vm)));
  float beta = dot(w, cross(xyz(U), pp));
  if (!(0.0f <= alpha && alpha <= 1.0f) || !(0.0f <= beta && beta <= 1.0f)) return false;
  t_out = t;
  a_out = alpha;
  b_out = beta;
  return true;
}

// Triangle.Hit objects.go:408-461 (Moller-Trumbore), comparisons kept verbatim
RT_D bool hit_tri(const DevScene& sc, uint32_t i, f3 o, f3 d, float tmin, float tmax,
                  float& t_out, float& u_out, float& v_out) {
  const F4* tr = sc.tri + 3 * (size_t)i;
  const F4 V0 = tr[0], E0 = tr[1], E1 = tr[2];
  f3 e0 = xyz(E0), e1 = xyz(E1);
  f3 pvec = cross(d, e1);
  float det = dot(e0, pvec);
  if (fabsf(det) < 1e-8f) return false;
  float inv = 1.0f / det;
  f3 tvec = o - xyz(V0);
  float u = dot(tvec, pvec) * inv;
  if (u < 0.0f || u > 1.0f) return false;
  f3 qvec = cross(tvec, e0);
  float v = dot(d, qvec) * inv;
  if (v < 0.0f || (u + v) > 1.0f) return false;
  float t = dot(e1, qvec) * inv;
  if (t < tmin || t > tmax) return false;
  t_out = t;
  u_out = u;
  v_out = v;
  return true;
}

// The closest triangle hit's t, u, v re-evaluated in fp64 (Triangle.Hit objects.go:408-461
// on the same fp32 ray and vertex data).  The traversal decides WHICH triangle and
// whether it is hit in fp32; this only refines the values the shading reads.  In
// fp32, u and v carry an absolute error of ~eps * |o - v0| / |edge| (the triple
// products cancel), i.e. ~1e-5 for rays crossing a 1M-triangle mesh: the smooth
// normal interpolated from them is off by that much, and on chains of metal bounces
// the fp32 path drifted away from the fp64 reference's (tools/fork_probe.py: every
// forked sample of C5 forked after 2-14 bounces of accumulated drift).
RT_D void refine_tri_hit(const DevScene& sc, uint32_t idx, f3 o, f3 d, float& t_io, float& u_io,
                         float& v_io) {
  const F4* tr = sc.tri + 3 * (size_t)idx;
  const F4 V0 = tr[0], E0 = tr[1], E1 = tr[2];
  const double dx = d.x, dy = d.y, dz = d.z;
  const double ax = E0.x, ay = E0.y, az = E0.z, bx = E1.x, by = E1.y, bz = E1.z;
  const double px = dy * bz - dz * by, py = dz * bx - dx * bz, pz = dx * by - dy * bx;  // d x e1
  const double det = ax * px + ay * py + az * pz;
  double inv = __builtin_amdgcn_rcp(det);
  inv = fma(inv, fma(-det, inv, 1.0), inv);
  const double tx = (double)o.x - V0.x, ty = (double)o.y - V0.y, tz = (double)o.z - V0.z;
  const double qx = ty * az - tz * ay, qy = tz * ax - tx * az, qz = tx * ay - ty * ax;  // tvec x e0
  u_io = (float)((tx * px + ty * py + tz * pz) * inv);
  v_io = (float)((dx * qx + dy * qy + dz * qz) * inv);
  t_io = (float)((bx * qx + by * qy + bz * qz) * inv);
}

RT_D bool hit_prim(const DevScene& sc, uint32_t ref, f3 o, f3 d, float time, float tmin,
                   float tmax, float& t, float& u, float& v) {
  uint32_t type = ref >> 30, idx = ref & 0x3FFFFFFFu;
  if (type == PRIM_SPHERE) {
    u = v = 0.0f;
    return hit_sphere(sc, idx, o, d, time, tmin, tmax, t);
  }
  if (type == PRIM_QUAD) return hit_quad(sc, idx, o, d, tmin, tmax, t, u, v);
  return hit_tri(sc, idx, o, d, tmin, tmax, t, u, v);
}

// ---- leaf-record tests (traversal; same semantics as the per-type tests) ----
RT_D bool hit_sphere_rec64(const F4 r[4], f3 o, f3 d, float time, float tmin, float tmax,
                           float& t_out) {
  const F4 c0 = r[0], mv = r[1];
  double cx = (double)c0.x + (double)time * (double)mv.x;
  double cy = (double)c0.y + (double)time * (double)mv.y;
  double cz = (double)c0.z + (double)time * (double)mv.z;
  double ox = cx - (double)o.x, oy = cy - (double)o.y, oz = cz - (double)o.z;
  double dx = d.x, dy = d.y, dz = d.z;
  double a = dx * dx + dy * dy + dz * dz;
  double h = dx * ox + dy * oy + dz * oz;
  double rr = mv.w;
  double c = ox * ox + oy * oy + oz * oz - rr * rr;
  double disc = h * h - a * c;
  if (disc < 0) return false;
  // fp64 sqrt as v_sqrt_f64 (~2^-23 relative) + one Newton step (~1e-14): the
  // exact-rounding library sequence is twice as long and buys nothing here
  double sq = __builtin_amdgcn_sqrt(disc);
  sq = disc > 0.0 ? fma(0.5 * fma(-sq, sq, disc), __builtin_amdgcn_rcp(sq), sq) : 0.0;
  // (tmin < (h -/+ sq)/a < tmax) tested as tmin*a < q < tmax*a (a > 0): no division
  double lo = (double)tmin * a, hi = (double)tmax * a;
  double q = h - sq;
  if (!(lo < q && q < hi)) {
    q = h + sq;
    if (!(lo < q && q < hi)) return false;
  }
  t_out = (float)(q * __builtin_amdgcn_rcp(a));  // fp32-level result from fp64 q: float t
  return true;
}
// Measured slower, kept opt-in (-DRT_SPHERE32_LEAVES; C3 +3.6 %, C4 +5.4 %, C5 +3.8 % against
// the fp64 leaves, profiles/r4_sphere_leaves_ab.jsonl): the BVH's sphere leaves (radius
// < kBigSphereR) in fp32 with the numerically robust discriminant r^2 - |oc - (h/a) d|^2
// (no cancellation of |oc|^2 against r^2), falling back to the fp64 test where the fp32
// result is uncertain: the discriminant within its rounding bound (a grazing ray) or a
// root next to tmin or tmax (a self-hit or a near-tie with the closest hit so far).  The
// winner's t is re-solved in fp64 once per segment (refine_sphere_hit).
RT_D bool hit_sphere_rec32(const F4 r[4], f3 o, f3 d, float time, float tmin, float tmax,
                           float& t_out) {
  const F4 c0 = r[0], mv = r[1];
  const f3 oc = mk3(fmaf(time, mv.x, c0.x), fmaf(time, mv.y, c0.y), fmaf(time, mv.z, c0.z)) - o;
  const float a = dot(d, d), ia = rcp(a), h = dot(d, oc);
  const float s = h * ia;  // the ray's closest approach to the center
  const f3 f = mk3(fmaf(-s, d.x, oc.x), fmaf(-s, d.y, oc.y), fmaf(-s, d.z, oc.z));
  const float ff = dot(f, f), rr = mv.w * mv.w, q = rr - ff;  // disc / a
  // rounding of f ~ eps |oc| per component: |ff| off by ~4 eps |f| |oc|
  const float err = 6.0e-7f * (rr + fsqrt(ff * dot(oc, oc)));
  if (fabsf(q) <= err) return hit_sphere_rec64(r, o, d, time, tmin, tmax, t_out);
  if (q < 0.0f) return false;
  const float sq = fsqrt(q * ia);  // sqrt(disc) / a
  float root = s - sq;
  const float tol = 1.0e-5f * (fabsf(root) + tmin);
  if (fabsf(root - tmin) <= tol || fabsf(root - tmax) <= 1.0e-5f * fabsf(root))
    return hit_sphere_rec64(r, o, d, time, tmin, tmax, t_out);
  if (!(tmin < root && root < tmax)) {
    root = s + sq;
    if (fabsf(root - tmin) <= 1.0e-5f * (fabsf(root) + tmin) ||
        fabsf(root - tmax) <= 1.0e-5f * fabsf(root))
      return hit_sphere_rec64(r, o, d, time, tmin, tmax, t_out);
    if (!(tmin < root && root < tmax)) return false;
  }
  t_out = root;
  return true;
}
RT_D bool hit_sphere_rec(const F4 r[4], f3 o, f3 d, float time, float tmin, float tmax,
                         float& t_out) {
#ifdef RT_SPHERE32_LEAVES
  return hit_sphere_rec32(r, o, d, time, tmin, tmax, t_out);
#else
  return hit_sphere_rec64(r, o, d, time, tmin, tmax, t_out);
#endif
}
// The winning sphere's t re-solved in fp64 (hit_sphere_d's quadratic on the same fp32
// ray): the root nearest to the fp32 test's, so the refinement never changes which root
// (entering or leaving) the traversal chose
RT_D void refine_sphere_hit(const DevScene& sc, uint32_t idx, f3 o, f3 d, float time, float& t_io) {
  double r0, r1;
  if (!sphere_roots_d(sc, idx, o, d, time, r0, r1)) return;  // fp32 hit, fp64 grazing miss
  const double t = (double)t_io;
  t_io = (float)(fabs(r0 - t) <= fabs(r1 - t) ? r0 : r1);
}
RT_D bool hit_quad_rec(const F4 r[4], f3 o, f3 d, float tmin, float tmax, float& t_out,
                       float& a_out, float& b_out) {
  const F4 Q = r[0], N = r[1], A = r[2], B = r[3];
  f3 n = xyz(N);
  float denom = dot(n, d);
  if (fabsf(denom) < 1e-8f) return false;
  float t = (N.w - dot(n, o)) * rcp(denom);
  if (!(tmin <= t && t <= tmax)) return false;
  f3 pp = (o + d * t) - xyz(Q);
  float alpha = dot(pp, xyz(A));
  float beta = dot(pp, xyz(B));
  // 0 <= alpha, beta <= 1 as one unsigned max + compare (non-negative floats order like
  // their bits; negatives and NaN exceed 1.0f's bits; -0.0f is rejected where the
  // reference accepts it: an exactly-zero coordinate of negative sign, measure zero)
  if (max(__float_as_uint(alpha), __float_as_uint(beta)) > 0x3F800000u) return false;
  t_out = t;
  a_out = alpha;
  b_out = beta;
  return true;
}
RT_D bool hit_tri_rec(const F4 r[4], f3 o, f3 d, float tmin, float tmax, float& t_out,
                      float& u_out, float& v_out) {
  const F4 V0 = r[0], E0 = r[1], E1 = r[2];
  f3 e0 = xyz(E0), e1 = xyz(E1);
  f3 pvec = cross(d, e1);
  float det = dot(e0, pvec);
  if (fabsf(det) < 1e-8f) return false;
  float inv = rcp(det);
  f3 tvec = o - xyz(V0);
  float u = dot(tvec, pvec) * inv;
  if (u < 0.0f || u > 1.0f) return false;
  f3 qvec = cross(tvec, e0);
  float v = dot(d, qvec) * inv;
  if (v < 0.0f || (u + v) > 1.0f) return false;
  float t = dot(e1, qvec) * inv;
  if (t < tmin || t > tmax) return false;
  t_out = t;
  u_out = u;
  v_out = v;
  return true;
}
// A box leaf (rt_device.h "box leaf"): NewBox's six quads (objects.go:208-240, closed
// intervals like quad.Hit :167-196) as one slab test in the box's frame, the frame of
// rotateY.Hit (transformation.go:94-107): x' = (o - C).a + t d.a, z' likewise, y as is;
// the faces are the planes x' = 0 / 1, y = ylo / yhi, z' = 0 / 1.  The closest face with
// t in [tmin, tmax] is the entering one when t_near >= tmin, else the leaving one (a ray
// that starts inside).  ref = that face's quad ref; u = -1 marks (alpha, beta) as not
// computed: shade_core derives them from the face's quad record when its material reads
// them (only image textures do).  iy = 1 / d.y (the traversal's).
RT_D bool hit_box_rec(const F4 r[4], f3 o, f3 d, float iy, float tmin, float tmax, float& t_out,
                      uint32_t& ref) {
  const float ex = o.x - r[0].x, ez = o.z - r[0].y;
  const float lx = fmaf(ez, r[1].y, ex * r[1].x), lz = fmaf(ez, r[1].w, ex * r[1].z);
  const float ix = rcp(fmaf(d.z, r[1].y, d.x * r[1].x)), iz = rcp(fmaf(d.z, r[1].w, d.x * r[1].z));
  // (1 - l) * i, not fma(-l, i, i): a ray parallel to the slab (i = inf) inside it
  // must get +-inf for both planes, not -inf + inf = NaN
  const float tx0 = -lx * ix, tx1 = (1.0f - lx) * ix;
  const float tz0 = -lz * iz, tz1 = (1.0f - lz) * iz;
  const float ty0 = (r[0].z - o.y) * iy, ty1 = (r[2].x - o.y) * iy;
  const float nx = fminf(tx0, tx1), ny = fminf(ty0, ty1), nz = fminf(tz0, tz1);
  const float fx = fmaxf(tx0, tx1), fy = fmaxf(ty0, ty1), fz = fmaxf(tz0, tz1);
  const float tn = fmaxf(fmaxf(nx, ny), nz), tf = fminf(fminf(fx, fy), fz);
  const bool enter = tn >= tmin;
  const float t = enter ? tn : tf;
  if (!(tn <= tf && t >= tmin && t <= tmax)) return false;
  // the face: the slab whose plane gave t, and which of its two planes
  int slot;
  if (enter)
    slot = tn == nx ? (tx1 < tx0 ? 1 : 0) : tn == ny ? (ty1 < ty0 ? 3 : 2) : (tz1 < tz0 ? 5 : 4);
  else
    slot = tf == fx ? (tx1 > tx0 ? 1 : 0) : tf == fy ? (ty1 > ty0 ? 3 : 2) : (tz1 > tz0 ? 5 : 4);
  const float fr[6] = {r[2].y, r[2].z, r[2].w, r[3].x, r[3].y, r[3].z};
  float f = fr[0];
#pragma unroll
  for (int k = 1; k < 6; ++k) f = slot == k ? fr[k] : f;
  ref = fbits(f);
  t_out = t;
  return true;
}

// ---- the same tests, branch-free, returning a reject mask (all ones: no hit) -------
// Each comparison of the boolean tests becomes the sign of a difference (>= 0 exactly when
// the comparison holds, equal values giving +0), OR-ed and spread by an arithmetic shift:
// full-rate v_sub / v_bitop3 / v_ashr instead of v_cmp + exec-mask branches (v_cmp issues
// at half rate on gfx950 and the hazard s_nops before its v_cndmask, profiles/
// r4_instr_rate.jsonl).  The same hits, except that an exactly -0.0 barycentric (reference:
// accepted) is rejected, as the record loop already does (unit_ab).
RT_D uint32_t sign_any3(float a, float b, float c) {
  return __builtin_amdgcn_bitop3_b32(fbits(a), fbits(b), fbits(c), 0xFE);
}
RT_D uint32_t spread_sign(uint32_t x) { return (uint32_t)((int32_t)x >> 31); }
// !unit_ab(a, b) in the sign bit: with m = max(bits(a), bits(b)), m > 1.0f's bits exactly
// when (1.0f's bits - m) wraps negative (m in (0x3F800000, 0xBF800000]) or m itself has the
// sign set (values below -1 and negative NaNs, where the difference wraps back positive)
RT_D uint32_t unit_ab_rej(float a, float b) {
  const uint32_t m = max(__float_as_uint(a), __float_as_uint(b));
  return (0x3F800000u - m) | m;
}
// Triangle.Hit objects.go:408-461 (hit_tri_rec's arithmetic)
RT_D uint32_t hit_tri_rec_m(const F4 r[4], f3 o, f3 d, float tmin, float tmax, float& t_out,
                            float& u_out, float& v_out, bool& near) {
  const f3 e0 = xyz(r[1]), e1 = xyz(r[2]);
  const f3 pvec = cross(d, e1);
  const float det = dot(e0, pvec);
  const float inv = rcp(det);
  const f3 tvec = o - xyz(r[0]);
  const float u = dot(tvec, pvec) * inv;
  const f3 qvec = cross(tvec, e0);
  const float v = dot(d, qvec) * inv;
  const float t = dot(e1, qvec) * inv;
  t_out = t;
  u_out = u;
  v_out = v;
  // |det| >= 1e-8, 0 <= u <= 1, v >= 0, u + v <= 1, tmin <= t <= tmax
  const uint32_t a = sign_any3(fabsf(det) - 1e-8f, u, 1.0f - u);
  const float w = 1.0f - (u + v);
  const uint32_t b = sign_any3(v, w, t - tmin);
  uint32_t rej = spread_sign(__builtin_amdgcn_bitop3_b32(a, b, fbits(tmax - t), 0xFE));
#ifdef RT_TRI_EDGE64  // opt-in build (DESIGN.md §7 "Triangle edges"): +5.6 % C5 time, parity unchanged
  // Near-edge rejections.  In fp32, u, v and w carry an absolute error of
  // a few eps * |o - v0| * |d| * |e| / |det| (the triple products cancel: ~1e-4 for camera rays
  // 14 units from the 1M-triangle mesh's 0.01-unit triangles; tools/tri_edge_error.py measures
  // at most 6.2 times that bound).  Two triangles sharing an edge compute their edge functions
  // from different vertices, so their errors differ, and a ray within that error of the edge
  // can be rejected by both: a hole, through which the GPU saw the mesh behind where the fp64
  // oracle hit it (C5's vertex-0 forks: u = 2e-4 against an fp32 error of ~2e-4).  A test
  // rejected only by a barycentric that is within 8 times the bound below 0 is flagged
  // `near`; the traversal keeps it (trav_steps `pend`) and tri_hit64 repeats Triangle.Hit in
  // fp64 on the same fp32 ray and vertices after the round (retest_near).  Below the band the
  // fp64 test rejects too, so every triangle the fp64 test accepts is accepted: no hole.
  // (fp32 acceptances just inside an edge stay: they cover the surface twice, never open it.)
  const float amax = fmaxf(fmaxf(fabsf(e0.x), fabsf(e0.y)), fmaxf(fabsf(e0.z), fabsf(e1.x)));
  const float emax = fmaxf(amax, fmaxf(fabsf(e1.y), fabsf(e1.z)));
  const float tmax3 = fmaxf(fmaxf(fabsf(tvec.x), fabsf(tvec.y)), fabsf(tvec.z));
  const float dmax3 = fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fabsf(d.z));
  const float bnd = 0x1p-21f * tmax3 * dmax3 * emax * fabsf(inv);
  const float bmin = fminf(fminf(u, v), w);
  // rejected with det and t in range (signs clear): by a barycentric, the smallest in the band
  const uint32_t other = sign_any3(fabsf(det) - 1e-8f, t - tmin, tmax - t);
  near = rej != 0u && (int32_t)other >= 0 && bmin + bnd >= 0.0f;
#else
  near = false;
#endif
  return rej;
}
// Triangle.Hit (objects.go:408-461) in fp64 on the fp32 ray and the triangle's fp32 vertex
// data (sc.tri: the same v0, e0, e1 as its leaf record), closed interval [tmin, tmax]: the
// re-test of a near-edge rejection (hit_tri_rec_m `near`)
RT_D bool tri_hit64(const DevScene& sc, uint32_t idx, f3 o, f3 d, float tmin, float tmax,
                    float& t_out, float& u_out, float& v_out) {
  const F4* tr = sc.tri + 3 * (size_t)idx;
  const F4 V0 = tr[0], E0 = tr[1], E1 = tr[2];
  const double ax = E0.x, ay = E0.y, az = E0.z, bx = E1.x, by = E1.y, bz = E1.z;
  const double dx = d.x, dy = d.y, dz = d.z;
  const double px = dy * bz - dz * by, py = dz * bx - dx * bz, pz = dx * by - dy * bx;
  const double det = ax * px + ay * py + az * pz;
  if (!(fabs(det) >= 1e-8)) return false;
  double inv = __builtin_amdgcn_rcp(det);  // + one Newton step (refine_tri_hit's)
  inv = fma(inv, fma(-det, inv, 1.0), inv);
  const double tx = (double)o.x - V0.x, ty = (double)o.y - V0.y, tz = (double)o.z - V0.z;
  const double u = (tx * px + ty * py + tz * pz) * inv;
  if (u < 0.0 || u > 1.0) return false;
  const double qx = ty * az - tz * ay, qy = tz * ax - tx * az, qz = tx * ay - ty * ax;
  const double v = (dx * qx + dy * qy + dz * qz) * inv;
  if (v < 0.0 || u + v > 1.0) return false;
  const double t = (bx * qx + by * qy + bz * qz) * inv;
  if (t < (double)tmin || t > (double)tmax) return false;
  t_out = (float)t;
  u_out = (float)u;
  v_out = (float)v;
  return true;
}
// quad.Hit objects.go:167-196 (hit_quad_rec's arithmetic)
RT_D uint32_t hit_quad_rec_m(const F4 r[4], f3 o, f3 d, float tmin, float tmax, float& t_out,
                             float& a_out, float& b_out) {
  const F4 Q = r[0], N = r[1], A = r[2], B = r[3];
  const f3 n = xyz(N);
  const float denom = dot(n, d);
  const float t = (N.w - dot(n, o)) * rcp(denom);
  const f3 pp = (o + d * t) - xyz(Q);
  const float alpha = dot(pp, xyz(A)), beta = dot(pp, xyz(B));
  t_out = t;
  a_out = alpha;
  b_out = beta;
  // |n.d| >= 1e-8, tmin <= t <= tmax, 0 <= alpha, beta <= 1 (unit_ab)
  const uint32_t ab = unit_ab_rej(alpha, beta);
  const uint32_t x = sign_any3(fabsf(denom) - 1e-8f, t - tmin, tmax - t);
  return spread_sign(x | ab);
}

#define HAS(f) ((FT & (f)) != 0u)
template <uint32_t FT>
RT_D bool hit_record(const F4 r[4], f3 o, f3 d, float iy, float time, float tmin, float tmax,
                     float& t, float& u, float& v, uint32_t& ref) {
  ref = fbits(r[0].w);
  const uint32_t type = ref >> 30;
  if (HAS(FT_BOX) && type == PRIM_BOX) {
    u = -1.0f;  // (alpha, beta) deferred to shade_core
    v = 0.0f;
    return hit_box_rec(r, o, d, iy, tmin, tmax, t, ref);
  }
  if (!HAS(FT_SPHERE | FT_TRI) || type == PRIM_QUAD) return hit_quad_rec(r, o, d, tmin, tmax, t, u, v);
  if (HAS(FT_TRI) && (!HAS(FT_SPHERE) || type == PRIM_TRI))
    return hit_tri_rec(r, o, d, tmin, tmax, t, u, v);
  u = v = 0.0f;
  return hit_sphere_rec(r, o, d, time, tmin, tmax, t);
}

// hit_record as a reject mask (the traversal's closest-hit update is then v_bitop3 selects)
template <uint32_t FT>
RT_D uint32_t hit_record_m(const F4 r[4], f3 o, f3 d, float iy, float time, float tmin, float tmax,
                           float& t, float& u, float& v, uint32_t& ref, bool& near) {
  near = false;
  ref = fbits(r[0].w);
  const uint32_t type = ref >> 30;
  if (HAS(FT_BOX) && type == PRIM_BOX) {
    u = -1.0f;
    v = 0.0f;
    return hit_box_rec(r, o, d, iy, tmin, tmax, t, ref) ? 0u : ~0u;
  }
  if (!HAS(FT_SPHERE | FT_TRI) || type == PRIM_QUAD) return hit_quad_rec_m(r, o, d, tmin, tmax, t, u, v);
  if (HAS(FT_TRI) && (!HAS(FT_SPHERE) || type == PRIM_TRI)) return hit_tri_rec_m(r, o, d, tmin, tmax, t, u, v, near);
  u = v = 0.0f;
  return hit_sphere_rec(r, o, d, time, tmin, tmax, t) ? 0u : ~0u;
}

// same, with fp64 interval bounds and result (medium boundaries: the reference
// searches (t1 + 1e-4, inf) with |t1| up to ~1e4, below fp32 resolution)
RT_D bool hit_prim_d(const DevScene& sc, uint32_t ref, f3 o, f3 d, float time, double tmin,
                     double tmax, double& t) {
  uint32_t type = ref >> 30, idx = ref & 0x3FFFFFFFu;
  if (type == PRIM_SPHERE) return hit_sphere_d(sc, idx, o, d, time, tmin, tmax, t);
  float tf, u, v;
  bool h = type == PRIM_QUAD ? hit_quad(sc, idx, o, d, -kInf, kInf, tf, u, v)
                             : hit_tri(sc, idx, o, d, -kInf, kInf, tf, u, v);
  if (!h) return false;
  t = (double)tf;
  if (type == PRIM_QUAD) return tmin <= t && t <= tmax;  // Contains
  return !(t < tmin || t > tmax);                        // Triangle.Hit :433
}

}  // namespace rt
