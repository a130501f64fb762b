// oracle.cpp — CPU restatement of nsp5488/go_raytracer's render path.
// TEST INFRASTRUCTURE ONLY (see oracle.h).  Every function cites the Go code it
// restates.  Random draws come from include/rt_rng.h at the dimensions listed
// there; the reference's rejection samplers (RandomUnitVector vec.go:159-167,
// RandomUnitDisk :149-156) are replaced by distribution-identical closed forms,
// exactly as on the device, so both sides consume identical uniforms.
#include "oracle.h"

#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <thread>
#include <vector>

#include "rt_rng.h"

namespace orc {

template <typename R>
struct Vec3 {  // vec.go:12-195
  R e[3];
  Vec3() : e{0, 0, 0} {}
  Vec3(R x, R y, R z) : e{x, y, z} {}
  R x() const { return e[0]; }
  R y() const { return e[1]; }
  R z() const { return e[2]; }
  Vec3 operator-() const { return {-e[0], -e[1], -e[2]}; }
  Vec3 add(const Vec3& o) const { return {e[0] + o.e[0], e[1] + o.e[1], e[2] + o.e[2]}; }
  Vec3 sub(const Vec3& o) const { return {e[0] - o.e[0], e[1] - o.e[1], e[2] - o.e[2]}; }
  Vec3 mul(const Vec3& o) const { return {e[0] * o.e[0], e[1] * o.e[1], e[2] * o.e[2]}; }
  Vec3 div(const Vec3& o) const { return {e[0] / o.e[0], e[1] / o.e[1], e[2] / o.e[2]}; }
  Vec3 scale(R t) const { return {e[0] * t, e[1] * t, e[2] * t}; }
  R len_sq() const { return e[0] * e[0] + e[1] * e[1] + e[2] * e[2]; }
  R len() const { return std::sqrt(len_sq()); }
  R dot(const Vec3& o) const { return e[0] * o.e[0] + e[1] * o.e[1] + e[2] * o.e[2]; }
  Vec3 cross(const Vec3& o) const {
    return {e[1] * o.e[2] - e[2] * o.e[1], e[2] * o.e[0] - e[0] * o.e[2],
            e[0] * o.e[1] - e[1] * o.e[0]};
  }
  Vec3 unit() const { return scale(R(1) / len()); }
  bool near_zero() const {
    R s = R(1e-8);
    return std::fabs(e[0]) < s && std::fabs(e[1]) < s && std::fabs(e[2]) < s;
  }
  Vec3 reflect(const Vec3& n) const { return sub(n.scale(n.dot(*this) * 2)); }  // :136-138
  Vec3 refract(const Vec3& n, R eta) const {                                   // :141-146
    R c = std::min((-*this).dot(n), R(1));
    Vec3 perp = add(n.scale(c)).scale(eta);
    Vec3 par = n.scale(-std::sqrt(std::fabs(R(1) - perp.len_sq())));
    return perp.add(par);
  }
};

template <typename R>
struct Ray {  // ray.go:10-38
  Vec3<R> o, d;
  R time = 0;
  Vec3<R> at(R t) const { return o.add(d.scale(t)); }
};

template <typename R>
struct Interval {  // interval.go
  R min, max;
  bool contains(R x) const { return min <= x && x <= max; }
  bool surrounds(R x) const { return min < x && x < max; }
  R clamp(R x) const { return x < min ? min : (x > max ? max : x); }
  R size() const { return max - min; }
};

// Go's builtin max/min propagate NaN (used in AABB.Hit aabb.go:104-105)
template <typename R>
inline R gomax(R a, R b) {
  if (std::isnan(a) || std::isnan(b)) return NAN;
  return a > b ? a : b;
}
template <typename R>
inline R gomin(R a, R b) {
  if (std::isnan(a) || std::isnan(b)) return NAN;
  return a < b ? a : b;
}

template <typename R>
struct AABB {  // aabb.go
  Interval<R> a[3];
  static AABB make(Interval<R> x, Interval<R> y, Interval<R> z) {
    AABB b;
    b.a[0] = x;
    b.a[1] = y;
    b.a[2] = z;
    b.pad();
    return b;
  }
  void pad() {  // padToMinimum :118-129
    R delta = R(0.0001);
    for (int i = 0; i < 3; ++i)
      if (a[i].size() < delta) a[i] = {a[i].min - delta / 2, a[i].max + delta / 2};
  }
  static AABB empty() {
    Interval<R> e{R(INFINITY), R(-INFINITY)};
    return make(e, e, e);
  }
  static AABB from_points(const Vec3<R>& p, const Vec3<R>& q) {
    Interval<R> iv[3];
    for (int i = 0; i < 3; ++i)
      iv[i] = p.e[i] < q.e[i] ? Interval<R>{p.e[i], q.e[i]} : Interval<R>{q.e[i], p.e[i]};
    return make(iv[0], iv[1], iv[2]);
  }
  static AABB from_boxes(const AABB& p, const AABB& q) {
    Interval<R> iv[3];
    for (int i = 0; i < 3; ++i)
      iv[i] = {std::min(p.a[i].min, q.a[i].min), std::max(p.a[i].max, q.a[i].max)};
    return make(iv[0], iv[1], iv[2]);
  }
  int longest_axis() const {
    if (a[0].size() > a[1].size()) return a[0].size() > a[2].size() ? 0 : 2;
    return a[1].size() > a[2].size() ? 1 : 2;
  }
  bool hit(const Ray<R>& r, Interval<R> rt) const {  // :90-113
    for (int axis = 0; axis < 3; ++axis) {
      R invd = R(1) / r.d.e[axis];
      R t0 = (a[axis].min - r.o.e[axis]) * invd;
      R t1 = (a[axis].max - r.o.e[axis]) * invd;
      if (invd < 0) std::swap(t0, t1);
      rt.min = gomax(t0, rt.min);
      rt.max = gomin(t1, rt.max);
      if (rt.max <= rt.min) return false;
    }
    return true;
  }
};

// ------------------------------------------------------------ RNG context --
struct Ctx {
  uint64_t seed;
  uint32_t gpix, sample;
  uint32_t vertex;
  uint64_t segments = 0;
  std::vector<int> med_calls;  // per medium object: calls during this world.Hit
  rt_u32x4 main{};             // group 0 of the current vertex
  uint32_t spare = 0;          // rt_spare24 of the call that generated the current ray
  float* trace = nullptr;      // oracle_trace records
  int trace_cap = 0, trace_n = 0;
  rt_u32x4 draw(uint32_t stream) const { return rt_rng_draw(seed, gpix, sample, stream); }
};
template <typename R>
inline R U(uint32_t x) {
  return (R)rt_unit_d(x);
}

template <typename R>
Vec3<R> random_unit_vector(uint32_t a, uint32_t b) {  // vec.go:159-167, closed form
  R z = R(1) - R(2) * U<R>(a);
  R r = std::sqrt(std::max(R(0), R(1) - z * z));
  R phi = R(2) * R(M_PI) * U<R>(b);
  return {r * std::cos(phi), r * std::sin(phi), z};
}

template <typename R>
struct Texture;
template <typename R>
struct Material;

template <typename R>
struct HitRecord {  // hittable.go:14-24
  Vec3<R> p, normal;
  R t = 0;
  bool front_face = false;
  R u = 0, v = 0;
  const Material<R>* mat = nullptr;
  void set_face_normal(const Ray<R>& r, const Vec3<R>& n) {  // :27-34
    front_face = r.d.dot(n) < 0;
    normal = front_face ? n : -n;
  }
};

// ---------------------------------------------------------------- textures -
template <typename R>
struct Perlin {  // perlin.go
  Vec3<R> ranvec[256];
  int perm[3][256];
  R noise(const Vec3<R>& p) const {  // :34-54
    R u = p.x() - std::floor(p.x()), v = p.y() - std::floor(p.y()), w = p.z() - std::floor(p.z());
    int i = (int)std::floor(p.x()), j = (int)std::floor(p.y()), k = (int)std::floor(p.z());
    const Vec3<R>* c[2][2][2];
    for (int di = 0; di < 2; ++di)
      for (int dj = 0; dj < 2; ++dj)
        for (int dk = 0; dk < 2; ++dk)
          c[di][dj][dk] =
              &ranvec[perm[0][(i + di) & 255] ^ perm[1][(j + dj) & 255] ^ perm[2][(k + dk) & 255]];
    R uu = u * u * (3 - 2 * u), vv = v * v * (3 - 2 * v), ww = w * w * (3 - 2 * w);  // :93-111
    R acc = 0;
    for (int a = 0; a < 2; ++a)
      for (int b = 0; b < 2; ++b)
        for (int d = 0; d < 2; ++d) {
          Vec3<R> wt(u - (R)a, v - (R)b, w - (R)d);
          acc += ((R)a * uu + (R)(1 - a) * (1 - uu)) * ((R)b * vv + (R)(1 - b) * (1 - vv)) *
                 ((R)d * ww + (R)(1 - d) * (1 - ww)) * c[a][b][d]->dot(wt);
        }
    return acc;
  }
  R turbulence(Vec3<R> p, int depth) const {  // :57-69
    R acc = 0, weight = 1;
    for (int i = 0; i < depth; ++i) {
      acc += weight * noise(p);
      weight *= R(0.5);
      p = p.scale(2);
    }
    return std::fabs(acc);
  }
};

template <typename R>
struct Texture {
  virtual ~Texture() {}
  virtual Vec3<R> value(R u, R v, const Vec3<R>& p) const = 0;
};
template <typename R>
struct SolidColor : Texture<R> {  // texture.go:14-27
  Vec3<R> albedo;
  Vec3<R> value(R, R, const Vec3<R>&) const override { return albedo; }
};
template <typename R>
struct Checker : Texture<R> {  // texture.go:29-60
  R inv_scale;
  const Texture<R>*even, *odd;
  Vec3<R> value(R u, R v, const Vec3<R>& p) const override {
    int x = (int)std::floor(inv_scale * p.x());
    int y = (int)std::floor(inv_scale * p.y());
    int z = (int)std::floor(inv_scale * p.z());
    if ((x + y + z) % 2 == 0) return even->value(u, v, p);
    return odd->value(u, v, p);
  }
};
template <typename R>
struct ImageTex : Texture<R> {  // texture.go:62-86 + imageLoader.go:52-62
  int w, h;
  const uint8_t* rgb;
  Vec3<R> value(R u, R v, const Vec3<R>&) const override {
    if (h <= 0) return {0, 1, 1};
    u = std::fabs(std::fmod(u, R(1)));
    v = R(1) - std::fabs(std::fmod(v, R(1)));
    R fi = u * (R)(w - 1), fj = v * (R)(h - 1);
    int i = std::isnan(fi) ? 0 : (int)fi, j = std::isnan(fj) ? 0 : (int)fj;
    i = std::min(std::max(i, 0), w);
    j = std::min(std::max(j, 0), h);
    long idx = (long)j * w + i;
    if (idx >= (long)w * h || !rgb) return {1, 0, 1};  // magenta
    R s = R(1) / R(255);
    const uint8_t* px = rgb + 3 * idx;
    return {(R)px[0] * s, (R)px[1] * s, (R)px[2] * s};
  }
};
template <typename R>
struct NoiseTex : Texture<R> {  // texture.go:108-125
  const Perlin<R>* noise;
  R scale;
  int variant;
  Vec3<R> value(R, R, const Vec3<R>& p) const override {
    switch (variant) {
      case RT_NOISE_MARBLE:
        return Vec3<R>(.5, .5, .5).scale(1 + std::sin(scale * p.z() + 10 * noise->turbulence(p, 7)));
      case RT_NOISE_TURBULENT:
        return Vec3<R>(1, 1, 1).scale(noise->turbulence(p, 7));
      default:
        return Vec3<R>(1, 1, 1).scale(R(.5) * (R(1) + noise->noise(p.scale(scale))));
    }
  }
};

// -------------------------------------------------------------- hittables --
template <typename R>
struct Hittable {  // hittable.go:60-65
  virtual ~Hittable() {}
  virtual bool hit(const Ray<R>& r, Interval<R> rt, HitRecord<R>& rec, Ctx& c) const = 0;
  virtual AABB<R> bbox() const = 0;
  virtual bool has_pdf() const { return false; }  // defaultPdfImpl: log.Fatal
  virtual R pdf_value(const Vec3<R>&, const Vec3<R>&) const { return 0; }
  virtual Vec3<R> random(const Vec3<R>&, Ctx&, uint32_t) const { return {1, 0, 0}; }
  virtual void walk_media(std::vector<int>&) const {}
};

template <typename R>
struct ONB {  // onb.go:13-43
  Vec3<R> ax[3];
  explicit ONB(const Vec3<R>& n) {
    ax[2] = n.unit();
    Vec3<R> a = std::fabs(n.x()) > R(.9) ? Vec3<R>(0, 1, 0) : Vec3<R>(1, 0, 0);
    ax[1] = n.cross(a).unit();
    ax[0] = n.cross(ax[1]).unit();
  }
  Vec3<R> transform(const Vec3<R>& v) const {
    return ax[0].scale(v.x()).add(ax[1].scale(v.y())).add(ax[2].scale(v.z()));
  }
};

template <typename R>
struct Sphere : Hittable<R> {  // objects.go:14-115
  Ray<R> center;  // motion as a ray
  R radius;
  const Material<R>* mat;
  AABB<R> box;
  Sphere(Vec3<R> c1, Vec3<R> c2, R r, bool moving, const Material<R>* m) : radius(r), mat(m) {
    Vec3<R> rv(r, r, r);
    if (!moving) {
      center = {c1, Vec3<R>(), 0};
      box = AABB<R>::from_points(c1.sub(rv), c1.add(rv));
    } else {
      center = {c1, c2.sub(c1), 0};
      box = AABB<R>::from_boxes(AABB<R>::from_points(center.at(0).sub(rv), center.at(0).add(rv)),
                                AABB<R>::from_points(center.at(1).sub(rv), center.at(1).add(rv)));
    }
  }
  AABB<R> bbox() const override { return box; }
  bool hit(const Ray<R>& r, Interval<R> rt, HitRecord<R>& rec, Ctx&) const override {
    Vec3<R> cur = center.at(r.time);
    Vec3<R> oc = cur.sub(r.o);
    R a = r.d.len_sq();
    R h = r.d.dot(oc);
    R c = oc.len_sq() - radius * radius;
    R disc = h * h - a * c;
    if (disc < 0) return false;
    R sq = std::sqrt(disc);
    R root = (h - sq) / a;
    if (!rt.surrounds(root)) {
      root = (h + sq) / a;
      if (!rt.surrounds(root)) return false;
    }
    rec.t = root;
    rec.p = r.at(root);
    Vec3<R> outward = rec.p.sub(cur).scale(R(1) / radius);
    rec.set_face_normal(r, outward);
    rec.mat = mat;
    // calculateSphereUV :44-50
    R theta = std::acos(-outward.y());
    R phi = std::atan2(-outward.z(), outward.x()) + R(M_PI);
    rec.u = phi / (2 * R(M_PI));
    rec.v = theta / R(M_PI);
    return true;
  }
  bool has_pdf() const override { return true; }
  R pdf_value(const Vec3<R>& origin, const Vec3<R>& dir) const override {  // :52-62
    HitRecord<R> rec;
    Ctx dummy{};
    if (!hit(Ray<R>{origin, dir, 0}, Interval<R>{R(.0001), R(INFINITY)}, rec, dummy)) return 0;
    R dist2 = center.at(0).sub(origin).len_sq();
    R cmax = std::sqrt(1 - radius * radius / dist2);
    R solid = 2 * R(M_PI) * (1 - cmax);
    return 1 / solid;
  }
  Vec3<R> random(const Vec3<R>& origin, Ctx& c, uint32_t) const override {  // :63-69
    Vec3<R> dir = center.at(0).sub(origin);
    R dist2 = dir.len_sq();
    ONB<R> onb(dir);
    return onb.transform(random_to_sphere(radius, dist2, U<R>(c.main.v[2]), U<R>(c.main.v[3])));
  }
  static Vec3<R> random_to_sphere(R rad, R dist2, R r1, R r2) {  // :70-80
    R z = 1 + r2 * (std::sqrt(1 - rad * rad / dist2) - 1);
    R phi = 2 * R(M_PI) * r1;
    R tt = std::sqrt(1 - z * z);
    return {std::cos(phi) * tt, std::sin(phi) * tt, z};
  }
};

template <typename R>
struct Quad : Hittable<R> {  // objects.go:117-206
  Vec3<R> Q, u, v, normal, w;
  R D, area;
  const Material<R>* mat;
  AABB<R> box;
  Quad(Vec3<R> q, Vec3<R> a, Vec3<R> b, const Material<R>* m) : Q(q), u(a), v(b), mat(m) {
    Vec3<R> n = u.cross(v);
    area = n.len();
    normal = n.unit();
    D = normal.dot(Q);
    w = n.scale(R(1) / n.dot(n));
    box = AABB<R>::from_boxes(AABB<R>::from_points(Q, Q.add(u).add(v)),
                              AABB<R>::from_points(Q.add(u), Q.add(v)));
  }
  AABB<R> bbox() const override { return box; }
  bool hit(const Ray<R>& r, Interval<R> rt, HitRecord<R>& rec, Ctx&) const override {
    R denom = normal.dot(r.d);
    if (std::fabs(denom) < R(1e-8)) return false;
    R t = (D - normal.dot(r.o)) / denom;
    if (!rt.contains(t)) return false;
    Vec3<R> p = r.at(t);
    Vec3<R> pp = p.sub(Q);
    R alpha = w.dot(pp.cross(v));
    R beta = w.dot(u.cross(pp));
    Interval<R> unit{0, 1};
    if (!unit.contains(alpha) || !unit.contains(beta)) return false;
    rec.u = alpha;
    rec.v = beta;
    rec.t = t;
    rec.p = p;
    rec.mat = mat;
    rec.set_face_normal(r, normal);
    return true;
  }
  bool has_pdf() const override { return true; }
  R pdf_value(const Vec3<R>& origin, const Vec3<R>& dir) const override {  // :152-160
    HitRecord<R> rec;
    Ctx dummy{};
    if (!hit(Ray<R>{origin, dir, 0}, Interval<R>{R(0.001), R(INFINITY)}, rec, dummy)) return 0;
    R dist2 = rec.t * rec.t * dir.len_sq();
    R cosine = std::fabs(dir.dot(rec.normal) / dir.len());
    return dist2 / (cosine * area);
  }
  Vec3<R> random(const Vec3<R>& origin, Ctx& c, uint32_t) const override {  // :161-165
    Vec3<R> p = Q.add(u.scale(U<R>(c.main.v[2]))).add(v.scale(U<R>(c.main.v[3])));
    return p.sub(origin);
  }
};

template <typename R>
struct Triangle : Hittable<R> {  // objects.go:242-465
  Vec3<R> V[3], N[3], normal;
  R area;
  R tex[3][2];
  bool has_uv, has_vn;
  const Material<R>* mat;
  AABB<R> box;
  Triangle(const rt_tri& t, const Material<R>* m) : mat(m) {
    for (int i = 0; i < 3; ++i) {
      V[i] = Vec3<R>((R)t.v[3 * i], (R)t.v[3 * i + 1], (R)t.v[3 * i + 2]);
      N[i] = Vec3<R>((R)t.n[3 * i], (R)t.n[3 * i + 1], (R)t.n[3 * i + 2]);
      tex[i][0] = (R)t.uv[2 * i];
      tex[i][1] = (R)t.uv[2 * i + 1];
    }
    has_vn = (t.flags & 1) != 0;
    has_uv = (t.flags & 2) != 0;
    Vec3<R> e0 = V[1].sub(V[0]), e1 = V[2].sub(V[0]);
    area = e0.cross(e1).len() / 2;
    normal = e0.cross(e1).unit();
    R mn[3], mx[3];  // SetBbox :317-354
    for (int a = 0; a < 3; ++a) {
      mn[a] = R(INFINITY);
      mx[a] = R(-INFINITY);
      for (int k = 0; k < 3; ++k) {
        mn[a] = std::min(V[k].e[a], mn[a]);
        mx[a] = std::max(V[k].e[a], mx[a]);
      }
      if (mx[a] - mn[a] < R(1e-8)) {
        mx[a] += R(1e-8);
        mn[a] -= R(1e-8);
      }
    }
    box = AABB<R>::make({mn[0], mx[0]}, {mn[1], mx[1]}, {mn[2], mx[2]});
  }
  AABB<R> bbox() const override { return box; }
  Vec3<R> interp_normal(R u, R v) const {  // :389-405
    if (!has_vn) return normal;
    R w = 1 - u - v;
    Vec3<R> n(w * N[0].x() + u * N[1].x() + v * N[2].x(), w * N[0].y() + u * N[1].y() + v * N[2].y(),
              w * N[0].z() + u * N[1].z() + v * N[2].z());
    return n.unit();
  }
  bool hit(const Ray<R>& r, Interval<R> rt, HitRecord<R>& rec, Ctx&) const override {  // :408-461
    Vec3<R> e0 = V[1].sub(V[0]), e1 = V[2].sub(V[0]);
    Vec3<R> pvec = r.d.cross(e1);
    R det = e0.dot(pvec);
    if (std::fabs(det) < R(1e-8)) return false;
    R inv = R(1) / det;
    Vec3<R> tvec = r.o.sub(V[0]);
    R u = tvec.dot(pvec) * inv;
    if (u < 0 || u > 1) return false;
    Vec3<R> qvec = tvec.cross(e0);
    R v = r.d.dot(qvec) * inv;
    if (v < 0 || (u + v) > 1) return false;
    R tl = e1.dot(qvec) * inv;
    if (tl < rt.min || tl > rt.max) return false;
    if (has_uv) {
      R w = 1 - u - v;
      rec.u = w * tex[0][0] + u * tex[1][0] + v * tex[2][0];
      rec.v = w * tex[0][1] + u * tex[1][1] + v * tex[2][1];
    } else {
      rec.u = u;
      rec.v = v;
    }
    rec.t = tl;
    rec.p = r.at(tl);
    rec.set_face_normal(r, has_vn ? interp_normal(u, v) : normal);
    rec.mat = mat;
    return true;
  }
  bool has_pdf() const override { return true; }
  R pdf_value(const Vec3<R>& origin, const Vec3<R>& dir) const override {  // :356-367
    HitRecord<R> rec;
    Ctx dummy{};
    if (!hit(Ray<R>{origin, dir, 0}, Interval<R>{R(0.001), R(INFINITY)}, rec, dummy)) return 0;
    R dist2 = rec.t * rec.t * dir.len_sq();
    R cosine = std::fabs(dir.dot(rec.normal) / dir.len());
    return dist2 / (cosine * area);
  }
  Vec3<R> random(const Vec3<R>& origin, Ctx& c, uint32_t) const override {  // :369-385
    R r1 = U<R>(c.main.v[2]);
    R r2 = U<R>(c.main.v[3]) * (1 - r1);
    R wa = 1 - r1 - r2, wb = r1, wc = r2;
    Vec3<R> p = V[0].scale(wa).add(V[1].scale(wb)).add(V[2].scale(wc));
    return p.sub(origin);
  }
};

template <typename R>
struct HittableList : Hittable<R> {  // hittable.go:77-138
  std::vector<const Hittable<R>*> objs;
  AABB<R> box = AABB<R>::empty();
  void add(const Hittable<R>* o) {
    objs.push_back(o);
    box = AABB<R>::from_boxes(box, o->bbox());
  }
  AABB<R> bbox() const override { return box; }
  bool hit(const Ray<R>& r, Interval<R> rt, HitRecord<R>& rec, Ctx& c) const override {
    HitRecord<R> tmp;
    bool any = false;
    Interval<R> iv{rt.min, rt.max};
    for (auto* o : objs)
      if (o->hit(r, iv, tmp, c)) {
        any = true;
        iv.max = tmp.t;
        rec = tmp;
      }
    return any;
  }
  bool has_pdf() const override {
    for (auto* o : objs)
      if (!o->has_pdf()) return false;
    return true;
  }
  R pdf_value(const Vec3<R>& origin, const Vec3<R>& dir) const override {  // :89-97
    R weight = R(1) / (R)objs.size();
    R sum = 0;
    for (auto* o : objs) sum += weight * o->pdf_value(origin, dir);
    return sum;
  }
  Vec3<R> random(const Vec3<R>& origin, Ctx& c, uint32_t pick) const override {  // :98-103
    if (objs.empty()) return {U<R>(c.main.v[1]), U<R>(c.main.v[2]), U<R>(c.main.v[3])};  // vec.Random()
    uint32_t n = (uint32_t)objs.size();
    return objs[rt_pick(pick, n)]->random(origin, c, rt_pick_residual(pick, n));
  }
  void walk_media(std::vector<int>& cnt) const override {
    for (auto* o : objs) o->walk_media(cnt);
  }
};

template <typename R>
struct BVHNode : Hittable<R> {  // bvh.go
  const Hittable<R>*left, *right;
  AABB<R> box;
  AABB<R> bbox() const override { return box; }
  bool hit(const Ray<R>& r, Interval<R> rt, HitRecord<R>& rec, Ctx& c) const override {  // :69-82
    if (!box.hit(r, rt)) return false;
    bool hl = left->hit(r, rt, rec, c);
    if (hl) rt.max = rec.t;
    bool hr = right->hit(r, rt, rec, c);
    return hr || hl;
  }
  void walk_media(std::vector<int>& cnt) const override {
    left->walk_media(cnt);
    right->walk_media(cnt);
  }
};

template <typename R>
struct Translate : Hittable<R> {  // transformation.go:13-38
  const Hittable<R>* obj;
  Vec3<R> off;
  AABB<R> box;
  AABB<R> bbox() const override { return box; }
  bool hit(const Ray<R>& r, Interval<R> rt, HitRecord<R>& rec, Ctx& c) const override {
    Ray<R> orr{r.o.sub(off), r.d, r.time};
    if (!obj->hit(orr, rt, rec, c)) return false;
    rec.p = rec.p.add(off);
    return true;
  }
  void walk_media(std::vector<int>& cnt) const override { obj->walk_media(cnt); }
};

template <typename R>
struct RotateY : Hittable<R> {  // transformation.go:40-110
  const Hittable<R>* obj;
  R sn, cs;
  AABB<R> box;
  AABB<R> bbox() const override { return box; }
  Vec3<R> to_obj(const Vec3<R>& v) const { return {cs * v.x() - sn * v.z(), v.y(), sn * v.x() + cs * v.z()}; }
  Vec3<R> to_world(const Vec3<R>& v) const { return {cs * v.x() + sn * v.z(), v.y(), -sn * v.x() + cs * v.z()}; }
  bool hit(const Ray<R>& r, Interval<R> rt, HitRecord<R>& rec, Ctx& c) const override {
    Ray<R> rr{to_obj(r.o), to_obj(r.d), r.time};
    if (!obj->hit(rr, rt, rec, c)) return false;
    rec.p = to_world(rec.p);
    rec.normal = to_world(rec.normal);
    return true;
  }
  void walk_media(std::vector<int>& cnt) const override { obj->walk_media(cnt); }
};

template <typename R>
struct ConstantMedium : Hittable<R> {  // medium.go:13-62
  const Hittable<R>* boundary;
  R neg_inv_density;
  const Material<R>* phase;
  int id = 0, draw_base = 0, spare_draw = -1;  // spare_draw: the scene's last draw index
  AABB<R> bbox() const override { return boundary->bbox(); }
  bool hit(const Ray<R>& r, Interval<R> rt, HitRecord<R>& rec, Ctx& c) const override {
    HitRecord<R> h1, h2;
    if (!boundary->hit(r, Interval<R>{R(-INFINITY), R(INFINITY)}, h1, c)) return false;
    if (!boundary->hit(r, Interval<R>{h1.t + R(.0001), R(INFINITY)}, h2, c)) return false;
    h1.t = std::max(h1.t, rt.min);
    h2.t = std::min(h2.t, rt.max);
    if (h1.t >= h2.t) return false;
    h1.t = std::max(R(0), h1.t);
    R len = r.d.len();
    R inside = (h2.t - h1.t) * len;
    int k = c.med_calls[id]++;
    int draw = draw_base + k;
    uint32_t w;
    if (draw == spare_draw) {
      w = c.spare;  // rt_rng.h: the last draw index takes the ray's spare bits
    } else {
      rt_u32x4 q = c.draw(RT_STREAM(c.vertex, 1 + (draw >> 2)));
      w = q.v[draw & 3];
    }
    R hd = neg_inv_density * std::log(U<R>(w));
    if (hd > inside) return false;
    rec.t = h1.t + hd / len;
    rec.p = r.at(rec.t);
    rec.normal = Vec3<R>(1, 0, 0);
    rec.front_face = true;
    rec.mat = phase;
    return true;
  }
  void walk_media(std::vector<int>& cnt) const override { cnt[id]++; }
};

// -------------------------------------------------------------- materials --
template <typename R>
struct Scatter {
  Vec3<R> att;
  int pdf_kind = 0;  // 0 none, 1 cosine, 2 sphere
  bool skip_pdf = false;
  Ray<R> skip_ray;
};

template <typename R>
struct Material {  // materials.go:19-27
  int kind;
  const Texture<R>* tex = nullptr;
  Vec3<R> albedo;
  R fuzz = 0, ior = 1;
  // Scatter
  bool scatter(const Ray<R>& rin, const HitRecord<R>& rec, Scatter<R>& s, Ctx& c) const {
    switch (kind) {
      case RT_MAT_LAMBERTIAN:  // :45-50
        s.att = tex->value(rec.u, rec.v, rec.p);
        s.pdf_kind = 1;
        s.skip_pdf = false;
        return true;
      case RT_MAT_METAL: {  // :70-79
        Vec3<R> refl = rin.d.reflect(rec.normal);
        refl = refl.unit().add(random_unit_vector<R>(c.main.v[2], c.main.v[3]).scale(fuzz));
        s.att = albedo;
        s.skip_pdf = true;
        s.skip_ray = {rec.p, refl, rin.time};
        return true;
      }
      case RT_MAT_DIELECTRIC: {  // :94-120
        s.att = Vec3<R>(1, 1, 1);
        s.skip_pdf = true;
        R ri = rec.front_face ? R(1) / ior : ior;
        Vec3<R> ud = rin.d.unit();
        R ct = std::min((-ud).dot(rec.normal), R(1));
        R st = std::sqrt(R(1) - ct * ct);
        bool cannot = ri * st > R(1);
        Vec3<R> dir;
        if (cannot || reflectance(ct) > U<R>(c.main.v[0]))
          dir = ud.reflect(rec.normal);
        else
          dir = ud.refract(rec.normal, ri);
        s.skip_ray = {rec.p, dir, rin.time};
        return true;
      }
      case RT_MAT_DIFFUSE_LIGHT: return false;  // :146-148
      case RT_MAT_ISOTROPIC:                    // :172-177
        s.att = tex->value(rec.u, rec.v, rec.p);
        s.pdf_kind = 2;
        s.skip_pdf = false;
        return true;
    }
    return false;
  }
  R reflectance(R cosine) const {  // :126-130
    R r0 = (1 - ior) / (1 + ior);
    r0 *= r0;
    return r0 + (1 - r0) * std::pow(1 - cosine, R(5));
  }
  R scattering_pdf(const Ray<R>&, const Ray<R>& out, const HitRecord<R>& rec) const {
    if (kind == RT_MAT_LAMBERTIAN) {  // :51-57
      R ct = rec.normal.dot(out.d.unit());
      return ct < 0 ? R(0) : ct / R(M_PI);
    }
    if (kind == RT_MAT_ISOTROPIC) return R(1) / (4 * R(M_PI));  // :161-163
    return 0;
  }
  bool emissive() const { return kind == RT_MAT_DIFFUSE_LIGHT; }
  Vec3<R> emitted(const HitRecord<R>& rec) const {  // :150-155
    if (!rec.front_face) return {};
    return tex->value(rec.u, rec.v, rec.p);
  }
};

// ------------------------------------------------------------ scene build --
template <typename R>
struct World {
  const rt_tree_view& tv;
  std::vector<std::unique_ptr<Hittable<R>>> pool;
  std::vector<std::unique_ptr<Texture<R>>> textures;
  std::vector<std::unique_ptr<Perlin<R>>> perlins;
  std::vector<std::unique_ptr<Material<R>>> materials;
  std::vector<ConstantMedium<R>*> media;
  const Hittable<R>* world = nullptr;
  const Hittable<R>* lights = nullptr;
  int error = 0;

  explicit World(const rt_tree_view& t) : tv(t) {
    for (int i = 0; i < tv.n_perlins; ++i) {
      auto p = std::make_unique<Perlin<R>>();
      for (int k = 0; k < 256; ++k)
        p->ranvec[k] = Vec3<R>((R)tv.perlins[i].ranvec[k][0], (R)tv.perlins[i].ranvec[k][1],
                               (R)tv.perlins[i].ranvec[k][2]);
      memcpy(p->perm, tv.perlins[i].perm, sizeof p->perm);
      perlins.push_back(std::move(p));
    }
    textures.resize(tv.n_textures);
    for (int i = 0; i < tv.n_textures; ++i) make_tex(i);
    for (int i = 0; i < tv.n_materials; ++i) {
      const rt_material& m = tv.materials[i];
      auto mm = std::make_unique<Material<R>>();
      mm->kind = m.kind;
      mm->tex = m.tex >= 0 ? textures[m.tex].get() : nullptr;
      mm->albedo = Vec3<R>((R)m.albedo[0], (R)m.albedo[1], (R)m.albedo[2]);
      mm->fuzz = (R)m.fuzz;
      mm->ior = (R)m.ior;
      materials.push_back(std::move(mm));
    }
  }
  const Texture<R>* make_tex(int i) {
    if (textures[i]) return textures[i].get();
    const rt_texture& x = tv.textures[i];
    switch (x.kind) {
      case RT_TEX_SOLID: {
        auto t = std::make_unique<SolidColor<R>>();
        t->albedo = Vec3<R>((R)x.color[0], (R)x.color[1], (R)x.color[2]);
        textures[i] = std::move(t);
        break;
      }
      case RT_TEX_CHECKER: {
        auto t = std::make_unique<Checker<R>>();
        t->inv_scale = (R)x.scale;
        t->even = make_tex(x.a);
        t->odd = make_tex(x.b);
        textures[i] = std::move(t);
        break;
      }
      case RT_TEX_IMAGE: {
        auto t = std::make_unique<ImageTex<R>>();
        t->w = tv.images[x.a].w;
        t->h = tv.images[x.a].h;
        t->rgb = tv.images[x.a].rgb;
        textures[i] = std::move(t);
        break;
      }
      default: {
        auto t = std::make_unique<NoiseTex<R>>();
        t->noise = perlins[x.a].get();
        t->scale = (R)x.scale;
        t->variant = x.variant;
        textures[i] = std::move(t);
      }
    }
    return textures[i].get();
  }
  template <typename T>
  T* keep(std::unique_ptr<T> p) {
    T* raw = p.get();
    pool.push_back(std::move(p));
    return raw;
  }
  Vec3<R> v3(const double* p) { return Vec3<R>((R)p[0], (R)p[1], (R)p[2]); }

  // bvhHelper bvh.go:35-61
  const Hittable<R>* bvh_helper(std::vector<const Hittable<R>*>& objs, int start, int end) {
    AABB<R> bb = AABB<R>::empty();
    for (int i = start; i < end; ++i) bb = AABB<R>::from_boxes(bb, objs[i]->bbox());
    int axis = bb.longest_axis();
    int span = end - start;
    auto node = std::make_unique<BVHNode<R>>();
    node->box = bb;
    if (span == 1) {
      node->left = node->right = objs[start];
    } else if (span == 2) {
      node->left = objs[start];
      node->right = objs[start + 1];
    } else {
      std::stable_sort(objs.begin() + start, objs.begin() + end,
                       [axis](const Hittable<R>* a, const Hittable<R>* b) {  // boxCompare :25-32
                         Interval<R> ia = a->bbox().a[axis], ib = b->bbox().a[axis];
                         if (ia.min != ib.min) return ia.min < ib.min;
                         return ia.max < ib.max;
                       });
      int mid = start + span / 2;
      node->left = bvh_helper(objs, start, mid);
      node->right = bvh_helper(objs, mid, end);
    }
    return keep(std::move(node));
  }

  const Hittable<R>* build(int id, bool is_world) {
    const rt_node& n = tv.nodes[id];
    switch (n.kind) {
      case RT_NODE_LIST: {
        auto l = std::make_unique<HittableList<R>>();
        for (int i = 0; i < n.b; ++i) l->add(build(tv.children[n.a + i], is_world));
        return keep(std::move(l));
      }
      case RT_NODE_BVH: {
        std::vector<const Hittable<R>*> objs;
        for (int i = 0; i < n.b; ++i) objs.push_back(build(tv.children[n.a + i], is_world));
        return bvh_helper(objs, 0, (int)objs.size());
      }
      case RT_NODE_SPHERE:
        return keep(std::make_unique<Sphere<R>>(v3(n.p), v3(n.p + 3), (R)n.p[6], n.p[7] != 0,
                                                materials[n.mat].get()));
      case RT_NODE_QUAD:
        return keep(std::make_unique<Quad<R>>(v3(n.p), v3(n.p + 3), v3(n.p + 6), materials[n.mat].get()));
      case RT_NODE_TRIANGLE:
        return keep(std::make_unique<Triangle<R>>(tv.tris[n.a], materials[tv.tris[n.a].mat].get()));
      case RT_NODE_TRANSLATE: {  // Translate transformation.go:20-24
        auto t = std::make_unique<Translate<R>>();
        t->obj = build(n.a, is_world);
        t->off = v3(n.p);
        AABB<R> cb = t->obj->bbox();
        t->box = AABB<R>::make({cb.a[0].min + t->off.x(), cb.a[0].max + t->off.x()},
                               {cb.a[1].min + t->off.y(), cb.a[1].max + t->off.y()},
                               {cb.a[2].min + t->off.z(), cb.a[2].max + t->off.z()});
        return keep(std::move(t));
      }
      case RT_NODE_ROTATE_Y: {  // RotateY :48-77
        auto r = std::make_unique<RotateY<R>>();
        r->obj = build(n.a, is_world);
        R rad = (R)n.p[0] * R(M_PI) / R(180.0);
        r->sn = std::sin(rad);
        r->cs = std::cos(rad);
        AABB<R> bb = r->obj->bbox();
        R mn[3] = {R(INFINITY), R(INFINITY), R(INFINITY)}, mx[3] = {R(-INFINITY), R(-INFINITY), R(-INFINITY)};
        for (int i = 0; i < 2; ++i)
          for (int j = 0; j < 2; ++j)
            for (int k = 0; k < 2; ++k) {
              R x = (R)i * bb.a[0].max + (R)(1 - i) * bb.a[0].min;
              R y = (R)j * bb.a[1].max + (R)(1 - j) * bb.a[1].min;
              R z = (R)k * bb.a[2].max + (R)(1 - k) * bb.a[2].min;
              R tv3[3] = {r->cs * x + r->sn * z, y, -r->sn * x + r->cs * z};
              for (int c = 0; c < 3; ++c) {
                mn[c] = std::min(mn[c], tv3[c]);
                mx[c] = std::max(mx[c], tv3[c]);
              }
            }
        r->box = AABB<R>::from_points(Vec3<R>(mn[0], mn[1], mn[2]), Vec3<R>(mx[0], mx[1], mx[2]));
        return keep(std::move(r));
      }
      case RT_NODE_MEDIUM: {
        auto m = std::make_unique<ConstantMedium<R>>();
        m->id = (int)media.size();
        media.push_back(m.get());
        if (!is_world) error = RT_ERR_UNSUPPORTED;
        m->boundary = build(n.a, false);
        m->neg_inv_density = R(-1) / (R)n.p[0];
        m->phase = materials[n.mat].get();
        return keep(std::move(m));
      }
    }
    error = RT_ERR_INVALID;
    return nullptr;
  }

  void finalize_media() {
    std::vector<int> cnt(media.size(), 0);
    world->walk_media(cnt);
    int base = 0;
    for (size_t i = 0; i < media.size(); ++i) {
      media[i]->draw_base = base;
      base += cnt[i];
    }
    for (auto* m : media) m->spare_draw = base - 1;
  }
};

// ---------------------------------------------------------------- camera ---
struct CamD {  // initialize camera.go:179-253 (fp64)
  int width, height, s, max_depth;
  double scale, recip;
  Vec3<double> center, p00, du, dv, dku, dkv, bg;
  double defocus, maxc;
};

static int init_camera(const rt_camera* c, CamD& o) {
  double aspect = c->aspect_ratio == 0 ? 1.0 : c->aspect_ratio;
  o.width = c->width == 0 ? 100 : c->width;
  int spp = c->samples_per_pixel == 0 ? 100 : c->samples_per_pixel;
  o.max_depth = c->max_depth == 0 ? 10 : c->max_depth;
  double vfov = c->vertical_fov == 0 ? 90 : c->vertical_fov;
  double focus = c->focus_distance == 0 ? 10 : c->focus_distance;
  o.maxc = c->max_contribution == 0 ? 1.5 : c->max_contribution;
  o.height = std::max(1, (int)((double)o.width / aspect));
  o.s = (int)std::sqrt((double)spp);
  if (o.s < 1) return RT_ERR_INVALID;
  o.scale = 1.0 / (double)(o.s * o.s);
  o.recip = 1.0 / (double)o.s;
  Vec3<double> from(0, 0, 0), at(0, 0, -1), vup(0, 1, 0);
  if (c->positioned) {
    from = Vec3<double>(c->look_from[0], c->look_from[1], c->look_from[2]);
    at = Vec3<double>(c->look_at[0], c->look_at[1], c->look_at[2]);
    vup = Vec3<double>(c->vup[0], c->vup[1], c->vup[2]);
  }
  o.center = from;
  double theta = vfov * M_PI / 180.0;
  double h = std::tan(theta / 2);
  double vh = 2.0 * h * focus;
  double vw = vh * ((double)o.width / (double)o.height);
  Vec3<double> w = from.sub(at).unit();
  Vec3<double> u = vup.cross(w).unit();
  Vec3<double> v = w.cross(u);
  Vec3<double> vpu = u.scale(vw), vpv = (-v).scale(vh);
  o.du = vpu.scale(1.0 / (double)o.width);
  o.dv = vpv.scale(1.0 / (double)o.height);
  Vec3<double> tl = o.center.sub(w.scale(focus)).sub(vpu.scale(0.5)).sub(vpv.scale(0.5));
  o.p00 = tl.add(o.du.add(o.dv).scale(0.5));
  double dr = focus * std::tan((c->defocus_angle / 2.0) * M_PI / 180.0);
  o.dku = u.scale(dr);
  o.dkv = v.scale(dr);
  o.defocus = c->defocus_angle;
  o.bg = Vec3<double>(c->background[0], c->background[1], c->background[2]);
  return RT_OK;
}

template <typename R>
struct Renderer {
  const CamD& cd;
  World<R>& W;
  Vec3<R> p00, du, dv, center, dku, dkv, bg;
  R recip, maxc;
  Renderer(const CamD& c, World<R>& w) : cd(c), W(w) {
    auto cv = [](const Vec3<double>& a) { return Vec3<R>((R)a.x(), (R)a.y(), (R)a.z()); };
    p00 = cv(c.p00);
    du = cv(c.du);
    dv = cv(c.dv);
    center = cv(c.center);
    dku = cv(c.dku);
    dkv = cv(c.dkv);
    bg = cv(c.bg);
    recip = (R)c.recip;
    maxc = (R)c.maxc;
  }

  Ray<R> get_ray(int i, int j, int s_i, int s_j, Ctx& c) const {  // camera.go:256-270
    rt_u32x4 r = c.draw(RT_STREAM_CAMERA);
    c.spare = rt_spare24(r);
    R px = (((R)s_i + U<R>(r.v[0])) * recip) - R(.5);  // sampleSquareStratified :277-282
    R py = (((R)s_j + U<R>(r.v[1])) * recip) - R(.5);
    Vec3<R> ps = p00.add(du.scale((R)i + px)).add(dv.scale((R)j + py));
    Vec3<R> origin = center;
    if (cd.defocus > 0) {  // defocusDiskSample :285-290 (RandomUnitDisk, closed form)
      // the disk's two uniforms: the halves of camera word [3] (rt_rng.h)
      const R u0 = sizeof(R) == 4 ? (R)rt_unit16_hi_f(r.v[3]) : (R)rt_unit16_hi_d(r.v[3]);
      const R u1 = sizeof(R) == 4 ? (R)rt_unit16_lo_f(r.v[3]) : (R)rt_unit16_lo_d(r.v[3]);
      R rr = std::sqrt(u0), phi = R(2) * R(M_PI) * u1;
      Vec3<R> p(rr * std::cos(phi), rr * std::sin(phi), 0);
      origin = center.add(dku.scale(p.x())).add(dkv.scale(p.y()));
    }
    return Ray<R>{origin, ps.sub(origin), U<R>(r.v[2])};
  }

  static Vec3<R> clamp_contribution(const Vec3<R>& col, R mx) {  // camera.go:334-341
    R intensity = col.x() + col.y() + col.z();
    if (intensity > mx) return col.scale(mx / intensity);
    return col;
  }

  Vec3<R> ray_color(const Ray<R>& r, int depth, Ctx& c) const {  // camera.go:293-331
    if (depth < 0) return {};
    c.vertex = (uint32_t)(cd.max_depth - depth);
    std::fill(c.med_calls.begin(), c.med_calls.end(), 0);
    ++c.segments;
    HitRecord<R> rec;
    bool any = W.world->hit(r, Interval<R>{R(0.001), R(INFINITY)}, rec, c);
    if (c.trace && c.trace_n < c.trace_cap) {
      float* q = c.trace + 12 * c.trace_n++;
      const float rec12[12] = {(float)r.o.x(), (float)r.o.y(), (float)r.o.z(), (float)r.time,
                               (float)r.d.x(), (float)r.d.y(), (float)r.d.z(), (float)c.vertex,
                               any ? (float)rec.t : INFINITY, (float)rec.u, (float)rec.v,
                               any ? (float)rec.mat->kind : -1.0f};
      memcpy(q, rec12, sizeof rec12);
    }
    if (!any) return bg;
    c.main = c.draw(RT_STREAM(c.vertex, 0));
    c.spare = rt_spare24(c.main);  // the next segment's ray comes from this call
    Vec3<R> emit;
    if (rec.mat->emissive()) emit = rec.mat->emitted(rec);
    Scatter<R> s;
    if (!rec.mat->scatter(r, rec, s, c)) return emit;
    if (s.skip_pdf) return s.att.mul(ray_color(s.skip_ray, depth - 1, c));
    // HittablePdf(P, lights) + MixturePdf(light, srec.Pdf) camera.go:319-320, pdf.go
    const rt_u32x4 m = c.main;
    Vec3<R> dir;
    std::unique_ptr<ONB<R>> onb;
    if (s.pdf_kind == 1) onb = std::make_unique<ONB<R>>(rec.normal);
    if (U<R>(m.v[0]) < R(0.5)) {  // mixturePdf.Generate pdf.go:69-74
      dir = light_random(W.lights, rec.p, c, m.v[1]);
    } else if (s.pdf_kind == 1) {  // cosinePdf.Generate pdf.go:38
      R r1 = U<R>(m.v[2]), r2 = U<R>(m.v[3]);
      R phi = 2 * R(M_PI) * r1;
      Vec3<R> cd3(std::cos(phi) * std::sqrt(r2), std::sin(phi) * std::sqrt(r2), std::sqrt(1 - r2));
      dir = onb->transform(cd3);
    } else {  // SpherePdf.Generate pdf.go:21
      dir = random_unit_vector<R>(m.v[2], m.v[3]);
    }
    Ray<R> scattered{rec.p, dir, r.time};
    R light_pdf = W.lights ? W.lights->pdf_value(rec.p, dir) : R(0);
    R bsdf_pdf;
    if (s.pdf_kind == 1)
      bsdf_pdf = std::max(R(0), dir.unit().dot(onb->ax[2]) / R(M_PI));  // pdf.go:33-36
    else
      bsdf_pdf = R(1) / (4 * R(M_PI));
    R pdf_value = R(0.5) * light_pdf + R(0.5) * bsdf_pdf;
    R spdf = rec.mat->scattering_pdf(r, scattered, rec);
    Vec3<R> sample = ray_color(scattered, depth - 1, c);
    Vec3<R> sc = s.att.scale(spdf).mul(sample).scale(R(1) / pdf_value);
    return clamp_contribution(emit.add(sc), maxc);
  }

  Vec3<R> light_random(const Hittable<R>* L, const Vec3<R>& origin, Ctx& c, uint32_t pick) const {
    if (!L) return {U<R>(c.main.v[1]), U<R>(c.main.v[2]), U<R>(c.main.v[3])};
    // resolve the nested pick to the leaf first (same rule as HittableList.random)
    const Hittable<R>* cur = L;
    uint32_t x = pick;
    for (;;) {
      auto* hl = dynamic_cast<const HittableList<R>*>(cur);
      if (!hl) break;
      if (hl->objs.empty()) return {U<R>(c.main.v[1]), U<R>(c.main.v[2]), U<R>(c.main.v[3])};
      uint32_t n = (uint32_t)hl->objs.size();
      cur = hl->objs[rt_pick(x, n)];
      x = rt_pick_residual(x, n);
    }
    return cur->random(origin, c, x);
  }
};

}  // namespace orc

using namespace orc;

template <typename R>
static int render_t(const rt_tree_view* tv, int world, int lights, const rt_camera* cam,
                    uint64_t seed, int threads, int rank, int nranks, int max_rows, float* out,
                    oracle_stats* st) {
  CamD cd;
  if (init_camera(cam, cd)) return RT_ERR_INVALID;
  World<R> W(*tv);
  W.world = W.build(world, true);
  if (lights >= 0) W.lights = W.build(lights, false);
  if (W.error || !W.world) return W.error ? W.error : RT_ERR_INVALID;
  if (W.lights && !W.lights->has_pdf()) return RT_ERR_UNSUPPORTED;
  W.finalize_media();
  Renderer<R> rd(cd, W);
  const int Wd = cd.width;
  std::vector<int> rows;
  for (int r = rank; r < cd.height; r += nranks) rows.push_back(r);
  if (max_rows > 0 && (int)rows.size() > max_rows) rows.resize(max_rows);
  if (threads <= 0) threads = 1;
  std::atomic<int> next{0};
  std::atomic<uint64_t> segs{0};
  auto t0 = std::chrono::steady_clock::now();
  auto worker = [&]() {  // threadedRenderer / renderRow camera.go:90-132
    Ctx c;
    c.seed = seed;
    c.med_calls.assign(W.media.size(), 0);
    for (;;) {
      int ri = next.fetch_add(1);
      if (ri >= (int)rows.size()) break;
      int row = rows[ri];
      for (int col = 0; col < Wd; ++col) {
        Vec3<R> pc;
        c.gpix = (uint32_t)(row * Wd + col);
        for (int si = 0; si < cd.s; ++si)
          for (int sj = 0; sj < cd.s; ++sj) {
            c.sample = (uint32_t)(si * cd.s + sj);
            Ray<R> r = rd.get_ray(col, row, sj, si, c);
            Vec3<R> v = rd.ray_color(r, cd.max_depth, c);
            pc = pc.add(v);
          }
        pc = pc.scale((R)cd.scale);
        float* o = out + 3 * ((size_t)ri * Wd + col);
        o[0] = (float)pc.x();
        o[1] = (float)pc.y();
        o[2] = (float)pc.z();
      }
    }
    segs += c.segments;
  };
  std::vector<std::thread> pool;
  for (int i = 1; i < threads; ++i) pool.emplace_back(worker);
  worker();
  for (auto& t : pool) t.join();
  auto t1 = std::chrono::steady_clock::now();
  if (st) {
    st->samples = (uint64_t)rows.size() * Wd * cd.s * cd.s;
    st->segments = segs.load();
    st->seconds = std::chrono::duration<double>(t1 - t0).count();
    st->threads = threads;
  }
  return RT_OK;
}

template <typename R>
static int trace_t(const rt_tree_view* tv, int world, int lights, const rt_camera* cam,
                   uint64_t seed, int64_t pixel, int sample, float* out, int cap) {
  CamD cd;
  if (init_camera(cam, cd)) return RT_ERR_INVALID;
  World<R> W(*tv);
  W.world = W.build(world, true);
  if (lights >= 0) W.lights = W.build(lights, false);
  if (W.error || !W.world) return W.error ? W.error : RT_ERR_INVALID;
  W.finalize_media();
  Renderer<R> rd(cd, W);
  Ctx c;
  c.seed = seed;
  c.med_calls.assign(W.media.size(), 0);
  c.trace = out;
  c.trace_cap = cap;
  c.gpix = (uint32_t)pixel;
  c.sample = (uint32_t)sample;
  int row = (int)(pixel / cd.width), col = (int)(pixel % cd.width);
  int si = sample / cd.s, sj = sample % cd.s;
  Ray<R> r = rd.get_ray(col, row, sj, si, c);
  rd.ray_color(r, cd.max_depth, c);
  return c.trace_n;
}

extern "C" {

int oracle_trace(const rt_tree_view* tree, int world, int lights, const rt_camera* cam,
                 uint64_t seed, int precision, int64_t pixel, int sample, float* out, int cap) {
  if (!tree || !cam || !out || cap <= 0) return RT_ERR_INVALID;
  if (precision == 32) return trace_t<float>(tree, world, lights, cam, seed, pixel, sample, out, cap);
  return trace_t<double>(tree, world, lights, cam, seed, pixel, sample, out, cap);
}

int oracle_render(const rt_tree_view* tree, int world, int lights, const rt_camera* cam,
                  uint64_t seed, int precision, int threads, int rank, int nranks, int max_rows,
                  float* out, oracle_stats* stats) {
  if (!tree || !cam || !out || nranks <= 0 || rank < 0 || rank >= nranks) return RT_ERR_INVALID;
  if (world < 0 || world >= tree->n_nodes || lights >= tree->n_nodes) return RT_ERR_INVALID;
  if (precision == 32)
    return render_t<float>(tree, world, lights, cam, seed, threads, rank, nranks, max_rows, out, stats);
  return render_t<double>(tree, world, lights, cam, seed, threads, rank, nranks, max_rows, out, stats);
}

int oracle_vec_op(int op, const double* a, const double* b, double s, double* out) {
  Vec3<double> A(a[0], a[1], a[2]), B;
  if (b) B = Vec3<double>(b[0], b[1], b[2]);
  Vec3<double> r;
  switch (op) {
    case ORACLE_VEC_ADD: r = A.add(B); break;
    case ORACLE_VEC_SUB: r = A.sub(B); break;
    case ORACLE_VEC_MUL: r = A.mul(B); break;
    case ORACLE_VEC_DIV: r = A.div(B); break;
    case ORACLE_VEC_NEG: r = -A; break;
    case ORACLE_VEC_DOT: out[0] = A.dot(B); return RT_OK;
    case ORACLE_VEC_CROSS: r = A.cross(B); break;
    case ORACLE_VEC_SCALE: r = A.scale(s); break;
    case ORACLE_VEC_LEN: out[0] = A.len(); return RT_OK;
    case ORACLE_VEC_LENSQ: out[0] = A.len_sq(); return RT_OK;
    case ORACLE_VEC_UNIT: r = A.unit(); break;
    case ORACLE_VEC_NEARZERO: out[0] = A.near_zero() ? 1 : 0; return RT_OK;
    case ORACLE_VEC_REFLECT: r = A.reflect(B); break;
    case ORACLE_VEC_REFRACT: r = A.refract(B, s); break;
    default: return RT_ERR_INVALID;
  }
  out[0] = r.x();
  out[1] = r.y();
  out[2] = r.z();
  return RT_OK;
}

int oracle_print_color(double r, double g, double b, char* out, int cap) {  // color.go:23-46
  double v[3] = {r, g, b};
  int q[3];
  Interval<double> intensity{0, 0.99999};
  for (int i = 0; i < 3; ++i) {
    double x = std::isnan(v[i]) ? 0.0 : v[i];
    x = x <= 0 ? 0 : std::sqrt(x);  // linearToGamma :11-16
    q[i] = (int)(intensity.clamp(x) * 256);
  }
  return snprintf(out, cap, "%d %d %d\n", q[0], q[1], q[2]);
}

int oracle_interval(int op, double mn, double mx, double x, double* out) {
  Interval<double> iv{mn, mx};
  if (op == 0) *out = iv.contains(x);
  else if (op == 1) *out = iv.surrounds(x);
  else if (op == 2) *out = iv.clamp(x);
  else return RT_ERR_INVALID;
  return RT_OK;
}

int oracle_ray_at(const double* o, const double* d, double t, double* out) {
  Ray<double> r{Vec3<double>(o[0], o[1], o[2]), Vec3<double>(d[0], d[1], d[2]), 0};
  Vec3<double> p = r.at(t);
  out[0] = p.x();
  out[1] = p.y();
  out[2] = p.z();
  return RT_OK;
}

int oracle_camera(const rt_camera* cam, rt_camera_derived* o) {
  CamD cd;
  if (!cam || !o || init_camera(cam, cd)) return RT_ERR_INVALID;
  memset(o, 0, sizeof *o);
  o->width = cd.width;
  o->height = cd.height;
  o->spp_sqrt = cd.s;
  o->max_depth = cd.max_depth;
  o->pixel_samples_scale = cd.scale;
  o->recip_spp_sqrt = cd.recip;
  auto put = [](double* d, const Vec3<double>& v) {
    d[0] = v.x();
    d[1] = v.y();
    d[2] = v.z();
  };
  put(o->center, cd.center);
  put(o->pixel00, cd.p00);
  put(o->delta_u, cd.du);
  put(o->delta_v, cd.dv);
  put(o->defocus_u, cd.dku);
  put(o->defocus_v, cd.dkv);
  put(o->background, cd.bg);
  o->defocus_angle = cd.defocus;
  o->max_contribution = cd.maxc;
  return RT_OK;
}

}  // extern "C"
