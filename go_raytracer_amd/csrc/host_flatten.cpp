// host_flatten.cpp — rt_scene_create: the reference object graph -> flat HBM scene.
//
// * Translate / RotateY (transformation.go:13-110) are baked into world-space
//   spheres, quads and triangles: the wrappers move the ray into object space
//   and the hit back out, so the closest hit (and t) is unchanged by baking.
//   A sphere keeps its accumulated rotation to compute UV in object space
//   (objects.go:110-113 under rotateY.Hit :94-107).
// * constantMedium (medium.go:27-58) is kept out of the closest-hit BVH: its
//   boundary prims are stored separately and the extend kernel tests each
//   medium occurrence after the BVH.  A medium reachable through a span-1 BVH
//   leaf is tested twice per world.Hit (bvh.go:44-46, :69-82), i.e. it draws
//   two free-flight distances and keeps the smaller one; that multiplicity is
//   reproduced here by simulating bvhHelper's topology.
// * The lights Hittable becomes a table of prims with pick intervals that are
//   bit-exact with nested rand.Intn picks (hittable.go:98-103) and weights for
//   the averaged PdfValue (hittable.go:89-97).
#include <math.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <functional>

#include "rt_internal.h"

namespace rt {
namespace {

// ------------------------------------------------------------- fp64 helpers
struct D3 {
  double x, y, z;
};
inline D3 mk(const double* p) { return {p[0], p[1], p[2]}; }
inline D3 operator+(D3 a, D3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline D3 operator-(D3 a, D3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline D3 operator*(D3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
inline double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline D3 cross(D3 a, D3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline double len(D3 a) { return sqrt(dot(a, a)); }
inline double get(D3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

// Rigid transform p_world = Ry(c,s) * p + T  (composition of rotateY/translate)
struct Xf {
  double c = 1, s = 0;
  D3 T{0, 0, 0};
  D3 rot(D3 v) const { return {c * v.x + s * v.z, v.y, -s * v.x + c * v.z}; }  // :87-93
  D3 pt(D3 p) const { return rot(p) + T; }
  Xf translate(D3 off) const {
    Xf r = *this;
    r.T = T + rot(off);
    return r;
  }
  Xf rotate_deg(double deg) const {
    double rad = deg * M_PI / 180.0;
    double cs = cos(rad), sn = sin(rad);
    Xf r = *this;
    r.c = c * cs - s * sn;
    r.s = s * cs + c * sn;
    return r;
  }
};

// --------------------------------------------- reference AABB (aabb.go) ----
struct Iv {
  double mn, mx;
  double size() const { return mx - mn; }
};
struct RBox {
  Iv a[3];
};
inline Iv combine(Iv p, Iv q) { return {std::min(p.mn, q.mn), std::max(p.mx, q.mx)}; }
inline RBox pad(RBox b) {  // padToMinimum aabb.go:118-129
  const double delta = 0.0001;
  for (int i = 0; i < 3; ++i)
    if (b.a[i].size() < delta) b.a[i] = {b.a[i].mn - delta / 2, b.a[i].mx + delta / 2};
  return b;
}
inline RBox empty_box() {
  RBox b;
  for (int i = 0; i < 3; ++i) b.a[i] = {INFINITY, -INFINITY};
  return pad(b);
}
inline RBox from_points(D3 a, D3 b) {  // FromPoints aabb.go:31-51
  RBox r;
  for (int i = 0; i < 3; ++i) {
    double p = get(a, i), q = get(b, i);
    r.a[i] = p < q ? Iv{p, q} : Iv{q, p};
  }
  return pad(r);
}
inline RBox from_boxes(const RBox& p, const RBox& q) {
  RBox r;
  for (int i = 0; i < 3; ++i) r.a[i] = combine(p.a[i], q.a[i]);
  return pad(r);
}
inline int longest_axis(const RBox& b) {  // aabb.go:73-87
  if (b.a[0].size() > b.a[1].size()) return b.a[0].size() > b.a[2].size() ? 0 : 2;
  return b.a[1].size() > b.a[2].size() ? 1 : 2;
}

struct Flattener {
  const Tree& t;
  HostScene& out;
  std::vector<int8_t> has_med;  // memo: subtree contains a medium
  std::vector<int8_t> box_done;
  std::vector<RBox> boxes;

  // world prims for the BVH builder
  std::vector<F4> lo, hi;
  std::vector<uint32_t> world_refs;

  // Box leaves (rt_device.h "box leaf"): a NewBox in the world becomes one leaf ref of
  // type PRIM_BOX; its six quads are emitted as usual (same quad indices) but reached
  // through the box record.  expand_boxes() puts the six face refs back in its place
  // (small scenes, kernels without FT_BOX): then the scene is exactly the per-quad one.
  struct BoxLeaf {
    size_t pos;            // index in world_refs
    uint32_t face_ref[6];  // in the list's order: front, right, back, left, top, bottom
    F4 flo[6], fhi[6];     // their padded bounds
  };
  std::vector<BoxLeaf> box_leaves;
  bool box_leaves_on = true;
  double big_r = kBigSphereR;  // spheres at least this large: out.big_refs

  explicit Flattener(const Tree& tr, HostScene& o) : t(tr), out(o) {
    has_med.assign(t.nodes.size(), -1);
    box_done.assign(t.nodes.size(), 0);
    boxes.resize(t.nodes.size());
  }

  const std::vector<int32_t>& kids(const rt_node& n) const { return t.lists[n.a]; }

  bool subtree_has_medium(int id) {
    if (has_med[id] >= 0) return has_med[id];
    const rt_node& n = t.nodes[id];
    bool r = false;
    switch (n.kind) {
      case RT_NODE_MEDIUM: r = true; break;
      case RT_NODE_LIST:
      case RT_NODE_BVH:
        for (int c : kids(n)) r = r || subtree_has_medium(c);
        break;
      case RT_NODE_TRANSLATE:
      case RT_NODE_ROTATE_Y: r = subtree_has_medium(n.a); break;
      default: break;
    }
    has_med[id] = r;
    return r;
  }

  // Hittable.BBox() of the reference, fp64, bit-faithful
  const RBox& ref_box(int id) {
    if (box_done[id]) return boxes[id];
    const rt_node& n = t.nodes[id];
    RBox b = empty_box();
    switch (n.kind) {
      case RT_NODE_SPHERE: {
        D3 c1 = mk(n.p), c2 = mk(n.p + 3), rv = {n.p[6], n.p[6], n.p[6]};
        if (n.p[7] == 0) {
          b = from_points(c1 - rv, c1 + rv);  // NewSphere objects.go:23-27
        } else {                              // NewMotionSphere :30-37
          D3 dir = c2 - c1;
          D3 a0 = c1 + dir * 0.0, a1 = c1 + dir * 1.0;
          b = from_boxes(from_points(a0 - rv, a0 + rv), from_points(a1 - rv, a1 + rv));
        }
        break;
      }
      case RT_NODE_QUAD: {  // setBBox objects.go:142-146
        D3 Q = mk(n.p), u = mk(n.p + 3), v = mk(n.p + 6);
        b = from_boxes(from_points(Q, Q + u + v), from_points(Q + u, Q + v));
        break;
      }
      case RT_NODE_TRIANGLE: {  // SetBbox objects.go:317-354
        const rt_tri& tr = t.tris[n.a];
        double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int v = 0; v < 3; ++v)
          for (int i = 0; i < 3; ++i) {
            mn[i] = std::min(tr.v[3 * v + i], mn[i]);
            mx[i] = std::max(tr.v[3 * v + i], mx[i]);
          }
        for (int i = 0; i < 3; ++i) {
          if (mx[i] - mn[i] < 1e-8) {
            mx[i] += 1e-8;
            mn[i] -= 1e-8;
          }
          b.a[i] = {mn[i], mx[i]};
        }
        b = pad(b);
        break;
      }
      case RT_NODE_LIST:
      case RT_NODE_BVH:
        for (int c : kids(n)) b = from_boxes(b, ref_box(c));
        break;
      case RT_NODE_TRANSLATE: {  // VecOffset aabb.go:131
        const RBox& cb = ref_box(n.a);
        for (int i = 0; i < 3; ++i) b.a[i] = {cb.a[i].mn + n.p[i], cb.a[i].mx + n.p[i]};
        b = pad(b);
        break;
      }
      case RT_NODE_ROTATE_Y: {  // RotateY transformation.go:48-77
        const RBox& cb = ref_box(n.a);
        double rad = n.p[0] * M_PI / 180.0, sn = sin(rad), cs = cos(rad);
        double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = 0; i < 2; ++i)
          for (int j = 0; j < 2; ++j)
            for (int k = 0; k < 2; ++k) {
              double x = i * cb.a[0].mx + (1 - i) * cb.a[0].mn;
              double y = j * cb.a[1].mx + (1 - j) * cb.a[1].mn;
              double z = k * cb.a[2].mx + (1 - k) * cb.a[2].mn;
              double tv[3] = {cs * x + sn * z, y, -sn * x + cs * z};
              for (int c = 0; c < 3; ++c) {
                mn[c] = std::min(mn[c], tv[c]);
                mx[c] = std::max(mx[c], tv[c]);
              }
            }
        b = from_points({mn[0], mn[1], mn[2]}, {mx[0], mx[1], mx[2]});
        break;
      }
      case RT_NODE_MEDIUM: b = ref_box(n.a); break;
    }
    boxes[id] = b;
    box_done[id] = 1;
    return boxes[id];
  }

  // bvhHelper (bvh.go:35-61) topology: how many leaf slots each child occupies
  void bvh_mult(std::vector<int32_t>& objs, std::vector<int32_t>& orig_pos, int start, int end,
                std::vector<int>& mult) {
    RBox bb = empty_box();
    for (int i = start; i < end; ++i) bb = from_boxes(bb, ref_box(objs[i]));
    int axis = longest_axis(bb);
    int span = end - start;
    if (span == 1) {
      mult[orig_pos[start]] += 2;  // left == right == objects[start]
    } else if (span == 2) {
      mult[orig_pos[start]] += 1;
      mult[orig_pos[start + 1]] += 1;
    } else {
      std::vector<std::pair<int32_t, int32_t>> sub;
      for (int i = start; i < end; ++i) sub.push_back({objs[i], orig_pos[i]});
      std::stable_sort(sub.begin(), sub.end(), [&](auto& A, auto& B) {
        const Iv& a = ref_box(A.first).a[axis];
        const Iv& b = ref_box(B.first).a[axis];
        if (a.mn != b.mn) return a.mn < b.mn;  // boxCompare bvh.go:25-32
        return a.mx < b.mx;
      });
      for (int i = start; i < end; ++i) {
        objs[i] = sub[i - start].first;
        orig_pos[i] = sub[i - start].second;
      }
      int mid = start + span / 2;
      bvh_mult(objs, orig_pos, start, mid, mult);
      bvh_mult(objs, orig_pos, mid, end, mult);
    }
  }

  // ------------------------------------------------------------ emission
  static void padded_bounds(D3 mn, D3 mx, F4* lp, F4* hp) {
    // conservative fp32 box: round outward, then pad by a relative epsilon
    double ext = std::max({mx.x - mn.x, mx.y - mn.y, mx.z - mn.z, 0.0});
    double m = std::max({fabs(mn.x), fabs(mn.y), fabs(mn.z), fabs(mx.x), fabs(mx.y), fabs(mx.z)});
    double e = 1e-6 * ext + 4e-7 * m + 1e-7;
    F4 l = {(float)(mn.x - e), (float)(mn.y - e), (float)(mn.z - e), 0};
    F4 h = {(float)(mx.x + e), (float)(mx.y + e), (float)(mx.z + e), 0};
    l.x = nextafterf(l.x, -INFINITY);
    l.y = nextafterf(l.y, -INFINITY);
    l.z = nextafterf(l.z, -INFINITY);
    h.x = nextafterf(h.x, INFINITY);
    h.y = nextafterf(h.y, INFINITY);
    h.z = nextafterf(h.z, INFINITY);
    *lp = l;
    *hp = h;
  }
  void add_bounds(uint32_t ref, D3 mn, D3 mx) {
    F4 l, h;
    padded_bounds(mn, mx, &l, &h);
    lo.push_back(l);
    hi.push_back(h);
    world_refs.push_back(ref);
  }

  // The BVH node rt_new_box builds (NewBox objects.go:208-240, host_tree.cpp): six quad
  // children, exactly front, right, back, left, top, bottom of the box [mn, mx] with the
  // edge vectors computed as rt_new_box computes them.  Exact comparisons: a user list
  // that only looks like a box (or a degenerate one) stays six quads.
  bool is_newbox(const rt_node& n, D3* pmn, D3* pmx) const {
    if (n.kind != RT_NODE_BVH) return false;
    const auto& ch = kids(n);
    if (ch.size() != 6) return false;
    for (int c : ch)
      if (t.nodes[c].kind != RT_NODE_QUAD) return false;
    auto Q = [&](int k) { return mk(t.nodes[ch[k]].p); };
    auto U = [&](int k) { return mk(t.nodes[ch[k]].p + 3); };
    auto V = [&](int k) { return mk(t.nodes[ch[k]].p + 6); };
    const D3 mn = Q(5);
    const D3 mx = {Q(1).x, Q(4).y, Q(0).z};
    const double dx = mx.x - mn.x, dy = mx.y - mn.y, dz = mx.z - mn.z;
    if (!(dx > 0.0 && dy > 0.0 && dz > 0.0)) return false;
    auto eq = [](D3 a, D3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; };
    const D3 ex = {dx, 0, 0}, ey = {0, dy, 0}, ez = {0, 0, dz}, nx = {-dx, 0, 0}, nz = {0, 0, -dz};
    const bool ok = eq(Q(0), D3{mn.x, mn.y, mx.z}) && eq(U(0), ex) && eq(V(0), ey) &&
                    eq(Q(1), D3{mx.x, mn.y, mx.z}) && eq(U(1), nz) && eq(V(1), ey) &&
                    eq(Q(2), D3{mx.x, mn.y, mn.z}) && eq(U(2), nx) && eq(V(2), ey) &&
                    eq(Q(3), mn) && eq(U(3), ez) && eq(V(3), ey) &&
                    eq(Q(4), D3{mn.x, mx.y, mx.z}) && eq(U(4), ex) && eq(V(4), nz) &&
                    eq(Q(5), mn) && eq(U(5), ex) && eq(V(5), ez);
    if (ok) *pmn = mn, *pmx = mx;
    return ok;
  }

  // one box leaf: the six faces as quads (in list order, as the per-quad walk would emit
  // them), the box record and one world ref over their union
  void emit_box(const rt_node& n, const Xf& xf, D3 mn, D3 mx) {
    const auto& ch = kids(n);
    BoxLeaf bl{};
    bl.pos = world_refs.size();
    D3 bmn = {INFINITY, INFINITY, INFINITY}, bmx = {-INFINITY, -INFINITY, -INFINITY};
    for (int k = 0; k < 6; ++k) {
      D3 a, b;
      bl.face_ref[k] = emit_quad(t.nodes[ch[k]], xf, &a, &b);
      padded_bounds(a, b, &bl.flo[k], &bl.fhi[k]);
      bmn = {std::min(bmn.x, a.x), std::min(bmn.y, a.y), std::min(bmn.z, a.z)};
      bmx = {std::max(bmx.x, b.x), std::max(bmx.y, b.y), std::max(bmx.z, b.z)};
    }
    // frame: C = the min corner, A / B = the x / z edges (horizontal: rotations are about y)
    const D3 C = xf.pt(mn), A = xf.rot(D3{mx.x - mn.x, 0, 0}), B = xf.rot(D3{0, 0, mx.z - mn.z});
    const double a2 = A.x * A.x + A.z * A.z, b2 = B.x * B.x + B.z * B.z;
    // face slots by plane: x' = 0 left, x' = 1 right, y = lo bottom, y = hi top,
    // z' = 0 back, z' = 1 front
    const uint32_t* f = bl.face_ref;
    const uint32_t slot[6] = {f[3], f[1], f[5], f[4], f[2], f[0]};
    const uint32_t idx = (uint32_t)(out.box_recs.size() / 4);
    out.box_recs.push_back({(float)C.x, (float)C.z, (float)C.y, 0.0f});  // .w: the ref (make_record)
    out.box_recs.push_back({(float)(A.x / a2), (float)(A.z / a2), (float)(B.x / b2), (float)(B.z / b2)});
    out.box_recs.push_back({(float)xf.pt(mx).y, as_f(slot[0]), as_f(slot[1]), as_f(slot[2])});
    out.box_recs.push_back({as_f(slot[3]), as_f(slot[4]), as_f(slot[5]), 0.0f});
    box_leaves.push_back(bl);
    add_bounds(prim_ref(PRIM_BOX, idx), bmn, bmx);
  }

  // every box leaf back to its six face refs, in place (world order as without boxes)
  void expand_boxes() {
    if (box_leaves.empty()) return;
    std::vector<F4> nlo, nhi;
    std::vector<uint32_t> nrefs;
    size_t b = 0;
    for (size_t i = 0; i < world_refs.size(); ++i) {
      if (b < box_leaves.size() && box_leaves[b].pos == i) {
        for (int k = 0; k < 6; ++k) {
          nrefs.push_back(box_leaves[b].face_ref[k]);
          nlo.push_back(box_leaves[b].flo[k]);
          nhi.push_back(box_leaves[b].fhi[k]);
        }
        ++b;
      } else {
        nrefs.push_back(world_refs[i]);
        nlo.push_back(lo[i]);
        nhi.push_back(hi[i]);
      }
    }
    world_refs.swap(nrefs);
    lo.swap(nlo);
    hi.swap(nhi);
    box_leaves.clear();
    out.box_recs.clear();
  }

  static uint32_t fbits(int32_t v) {
    uint32_t u;
    memcpy(&u, &v, 4);
    return u;
  }
  static float as_f(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
  }

  uint32_t emit_sphere(const rt_node& n, const Xf& xf, D3* bmn, D3* bmx) {
    D3 c1 = xf.pt(mk(n.p)), mv = xf.rot(mk(n.p + 3) - mk(n.p));
    double r = n.p[6];
    uint32_t idx = (uint32_t)out.sph_cr.size();
    out.sph_cr.push_back({(float)c1.x, (float)c1.y, (float)c1.z, (float)r});
    out.sph_mv.push_back({(float)mv.x, (float)mv.y, (float)mv.z, as_f(fbits(n.mat))});
    out.sph_uv.push_back({(float)xf.c, (float)xf.s});
    if (bmn) {
      D3 c2 = c1 + mv;
      double ar = fabs(r);
      *bmn = {std::min(c1.x, c2.x) - ar, std::min(c1.y, c2.y) - ar, std::min(c1.z, c2.z) - ar};
      *bmx = {std::max(c1.x, c2.x) + ar, std::max(c1.y, c2.y) + ar, std::max(c1.z, c2.z) + ar};
    }
    return prim_ref(PRIM_SPHERE, idx);
  }

  uint32_t emit_quad(const rt_node& n, const Xf& xf, D3* bmn, D3* bmx) {
    D3 Q = xf.pt(mk(n.p)), u = xf.rot(mk(n.p + 3)), v = xf.rot(mk(n.p + 6));
    // NewQuad objects.go:129-140
    D3 nn = cross(u, v);
    double area = len(nn);
    D3 normal = nn * (1.0 / area);
    double D = dot(normal, Q);
    D3 w = nn * (1.0 / dot(nn, nn));
    uint32_t idx = (uint32_t)(out.quad.size() / 5);
    out.quad.push_back({(float)Q.x, (float)Q.y, (float)Q.z, (float)D});
    out.quad.push_back({(float)u.x, (float)u.y, (float)u.z, (float)area});
    out.quad.push_back({(float)v.x, (float)v.y, (float)v.z, as_f(fbits(n.mat))});
    out.quad.push_back({(float)normal.x, (float)normal.y, (float)normal.z, 0});
    out.quad.push_back({(float)w.x, (float)w.y, (float)w.z, 0});
    if (bmn) {
      D3 pts[4] = {Q, Q + u, Q + v, Q + u + v};
      *bmn = *bmx = pts[0];
      for (auto& p : pts) {
        *bmn = {std::min(bmn->x, p.x), std::min(bmn->y, p.y), std::min(bmn->z, p.z)};
        *bmx = {std::max(bmx->x, p.x), std::max(bmx->y, p.y), std::max(bmx->z, p.z)};
      }
    }
    return prim_ref(PRIM_QUAD, idx);
  }

  uint32_t emit_tri(const rt_node& n, const Xf& xf, D3* bmn, D3* bmx) {
    const rt_tri& tr = t.tris[n.a];
    D3 v0 = xf.pt(mk(tr.v)), v1 = xf.pt(mk(tr.v + 3)), v2 = xf.pt(mk(tr.v + 6));
    D3 e0 = v1 - v0, e1 = v2 - v0;
    D3 cr = cross(e0, e1);
    double area = len(cr) / 2.0;
    D3 fn = cr * (1.0 / len(cr));
    uint32_t idx = (uint32_t)(out.tri.size() / 3);
    out.tri.push_back({(float)v0.x, (float)v0.y, (float)v0.z, as_f(fbits(tr.mat))});
    out.tri.push_back({(float)e0.x, (float)e0.y, (float)e0.z, (float)area});
    out.tri.push_back({(float)e1.x, (float)e1.y, (float)e1.z, as_f((uint32_t)tr.flags)});
    out.tri_attr.push_back({(float)fn.x, (float)fn.y, (float)fn.z, 0});
    for (int k = 0; k < 3; ++k) {
      D3 nk = (tr.flags & 1) ? xf.rot(mk(tr.n + 3 * k)) : D3{0, 0, 0};
      out.tri_attr.push_back({(float)nk.x, (float)nk.y, (float)nk.z, 0});
    }
    out.tri_attr.push_back({(float)tr.uv[0], (float)tr.uv[1], (float)tr.uv[2], (float)tr.uv[3]});
    out.tri_attr.push_back({(float)tr.uv[4], (float)tr.uv[5], 0, 0});
    if (bmn) {
      *bmn = {std::min({v0.x, v1.x, v2.x}), std::min({v0.y, v1.y, v2.y}),
              std::min({v0.z, v1.z, v2.z})};
      *bmx = {std::max({v0.x, v1.x, v2.x}), std::max({v0.y, v1.y, v2.y}),
              std::max({v0.z, v1.z, v2.z})};
    }
    return prim_ref(PRIM_TRI, idx);
  }

  uint32_t emit_prim(const rt_node& n, const Xf& xf, D3* bmn, D3* bmx) {
    if (n.kind == RT_NODE_SPHERE) return emit_sphere(n, xf, bmn, bmx);
    if (n.kind == RT_NODE_QUAD) return emit_quad(n, xf, bmn, bmx);
    return emit_tri(n, xf, bmn, bmx);
  }

  // role: 0 = world (BVH prims + media), 1 = medium boundary
  int walk(int id, const Xf& xf, int mult, int role) {
    const rt_node& n = t.nodes[id];
    switch (n.kind) {
      case RT_NODE_SPHERE:
      case RT_NODE_QUAD:
      case RT_NODE_TRIANGLE: {
        if (role == 0) {
          D3 mn, mx;
          uint32_t ref = emit_prim(n, xf, &mn, &mx);
          if (n.kind == RT_NODE_SPHERE && fabs(n.p[6]) >= big_r)
            out.big_refs.push_back(ref);  // tested before the BVH, in fp64 (trav_init)
          else
            add_bounds(ref, mn, mx);
        } else {
          out.medium_refs.push_back(emit_prim(n, xf, nullptr, nullptr));
        }
        return RT_OK;
      }
      case RT_NODE_LIST:
        for (int c : kids(n)) {
          int rc = walk(c, xf, mult, role);
          if (rc) return rc;
        }
        return RT_OK;
      case RT_NODE_BVH: {
        const auto& ch = kids(n);
        D3 bmn, bmx;
        if (role == 0 && box_leaves_on && is_newbox(n, &bmn, &bmx)) {
          emit_box(n, xf, bmn, bmx);
          return RT_OK;
        }
        if (role == 0 && subtree_has_medium(id)) {
          std::vector<int32_t> objs(ch.begin(), ch.end()), pos(ch.size());
          for (size_t i = 0; i < ch.size(); ++i) pos[i] = (int32_t)i;
          std::vector<int> m(ch.size(), 0);
          bvh_mult(objs, pos, 0, (int)ch.size(), m);
          for (size_t i = 0; i < ch.size(); ++i) {
            int rc = walk(ch[i], xf, mult * m[i], role);
            if (rc) return rc;
          }
          return RT_OK;
        }
        for (int c : ch) {
          int rc = walk(c, xf, mult, role);
          if (rc) return rc;
        }
        return RT_OK;
      }
      case RT_NODE_TRANSLATE: return walk(n.a, xf.translate(mk(n.p)), mult, role);
      case RT_NODE_ROTATE_Y: return walk(n.a, xf.rotate_deg(n.p[0]), mult, role);
      case RT_NODE_MEDIUM: {
        if (role != 0)
          return set_error(RT_ERR_UNSUPPORTED, "medium %d nested inside a medium boundary", id);
        DevMedium m{};
        m.bfirst = (uint32_t)out.medium_refs.size();
        int rc = walk(n.a, xf, 1, 1);
        if (rc) return rc;
        m.bcount = (uint32_t)out.medium_refs.size() - m.bfirst;
        m.neg_inv_density = (float)(-1.0 / n.p[0]);  // medium.go:20-25
        m.phase_mat = n.mat;
        m.draw_base = out.medium_draws;
        m.mult = mult;
        out.medium_draws += mult;
        out.media.push_back(m);
        return RT_OK;
      }
    }
    return set_error(RT_ERR_INVALID, "node %d has unknown kind %d", id, n.kind);
  }

  // lights: HittableList nesting -> weighted leaves with exact pick intervals
  int walk_lights(int id, unsigned __int128 P, unsigned __int128 C, double weight, uint32_t lo24) {
    const rt_node& n = t.nodes[id];
    if (n.kind == RT_NODE_SPHERE || n.kind == RT_NODE_QUAD || n.kind == RT_NODE_TRIANGLE) {
      DevLight L{};
      L.ref = emit_prim(n, Xf{}, nullptr, nullptr);
      L.lo24 = lo24;
      L.weight = (float)weight;
      out.lights.push_back(L);
      return RT_OK;
    }
    if (n.kind != RT_NODE_LIST)
      return set_error(RT_ERR_UNSUPPORTED,
                       "light node %d (kind %d) has no PdfValue in the reference "
                       "(defaultPdfImpl, hittable.go:69-72)",
                       id, n.kind);
    const auto& ch = kids(n);
    if (ch.empty()) {  // Random -> vec.Random(), PdfValue -> 0 (hittable.go:89-103)
      DevLight L{};
      L.ref = PRIM_NONE;
      L.lo24 = lo24;
      L.weight = 0.0f;
      out.lights.push_back(L);
      return RT_OK;
    }
    const unsigned __int128 n_ = ch.size();
    const unsigned __int128 ONE = (unsigned __int128)1 << 24;
    for (size_t i = 0; i < ch.size(); ++i) {
      // child i <=> u24 >= ceil((C*n + i*2^24) / (P*n))
      unsigned __int128 num = C * n_ + (unsigned __int128)i * ONE, den = P * n_;
      uint32_t lo = (uint32_t)((num + den - 1) / den);
      int rc = walk_lights(ch[i], P * n_, num, weight / (double)ch.size(), lo);
      if (rc) return rc;
    }
    return RT_OK;
  }
};

}  // namespace

int flatten_scene(const Tree& t, int world, int lights, HostScene& out) {
  out = HostScene();
  if (world < 0 || world >= (int)t.nodes.size())
    return set_error(RT_ERR_INVALID, "rt_scene_create: bad world handle %d", world);
  if (lights >= (int)t.nodes.size())
    return set_error(RT_ERR_INVALID, "rt_scene_create: bad lights handle %d", lights);
  const bool timing = tune_int("RT_TIMING", 0) != 0;
  auto t0 = std::chrono::steady_clock::now();
  Flattener f(t, out);
  f.box_leaves_on = tune_int("RT_BOX_LEAVES", 1) != 0;
  f.big_r = tune_num("RT_BIG_SPHERE_R", kBigSphereR);  // A/B: a huge value keeps every sphere in the BVH
  int rc = f.walk(world, Xf{}, 1, 0);
  if (timing)
    fprintf(stderr, "[rt] flatten walk %.3f s\n",
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  if (rc) return rc;
  if (lights >= 0) {
    rc = f.walk_lights(lights, 1, 0, 1.0, 0);
    if (rc) return rc;
  }
  // materials / textures / images / perlin tables: indices kept identical to the tree
  for (const auto& m : t.materials) {
    DevMaterial d{};
    d.kind = m.kind;
    d.tex = m.tex;
    d.param = (float)(m.kind == RT_MAT_METAL ? m.fuzz : m.ior);
    d.albedo = {(float)m.albedo[0], (float)m.albedo[1], (float)m.albedo[2], 0};
    out.mats.push_back(d);
  }
  for (const auto& x : t.textures) {
    DevTexture d{};
    d.kind = x.kind;
    d.a = x.a;
    d.b = x.b;
    d.variant = x.variant;
    d.color = {(float)x.color[0], (float)x.color[1], (float)x.color[2], (float)x.scale};
    out.texs.push_back(d);
  }
  for (size_t i = 0; i < t.images.size(); ++i) {
    DevImage d{};
    d.offset = out.texels.size();
    d.w = t.images[i].w;
    d.h = t.images[i].h;
    out.texels.insert(out.texels.end(), t.image_data[i].begin(), t.image_data[i].end());
    out.images.push_back(d);
  }
  while (out.texels.size() % 16) out.texels.push_back(0);
  for (const auto& p : t.perlins) {
    DevPerlin d{};
    for (int i = 0; i < 256; ++i)
      d.ranvec[i] = {(float)p.ranvec[i][0], (float)p.ranvec[i][1], (float)p.ranvec[i][2], 0};
    for (int a = 0; a < 3; ++a)  // values are 0..255 (checked at rt_tex_noise_tables)
      for (int i = 0; i < 256; ++i) d.perm[a][i] = (uint8_t)p.perm[a][i];
    out.perlins.push_back(d);
  }
  // Box leaves stay only in large scenes (a tree read through L1/L2: the record loop
  // and the LDS trees of small scenes test quads) whose kernel set has FT_BOX anyway,
  // so they never move a scene to a bigger kernel (DESIGN.md §4 "Box leaves").
  if (!f.box_leaves.empty()) {
    out.refs = f.world_refs;  // features as they would be with the faces as quads
    bool nt0 = true;
    const uint32_t feats = scene_features(out, &nt0) & ~FT_BOX;
    out.refs.clear();
    const size_t n_faces = f.world_refs.size() + 5 * f.box_leaves.size();
    const uint32_t set = (feats & FT_NOISE) && !nt0 ? FT_ALL : pick_ft_set(feats);
    if (n_faces <= kBoxLeafMinPrims || !(set & FT_BOX)) f.expand_boxes();
  }
  out.n_world_prims = (int32_t)f.world_refs.size();
  // keep prim bounds for export, in the BVH's final ref order (set by build_bvh)
  t0 = std::chrono::steady_clock::now();
  // large scenes: PLOC on the GPU (rt_build.hip) when a device is present
  std::string builder = "auto";
  tune_str("RT_BVH_BUILDER", &builder);
  const size_t dev_min = (size_t)tune_num("RT_BVH_DEVICE_MIN", 65536.0);
  const bool on_device =
      f.world_refs.size() >= 2 &&
      (builder == "device" || (builder == "auto" && f.world_refs.size() >= dev_min)) &&
      bvh_device_available();
  if (builder == "device" && !on_device && f.world_refs.size() >= 2)
    return set_error(RT_ERR_DEVICE, "RT_BVH_BUILDER device: no HIP device is available");
  out.bvh_builder = on_device ? 1 : 0;
  rc = on_device ? build_bvh_device(out, f.lo, f.hi, f.world_refs, -1)  // current device
                 : build_bvh(out, f.lo, f.hi, f.world_refs);
  if (timing)
    fprintf(stderr, "[rt] build_bvh (%s) %.3f s\n", on_device ? "device" : "host",
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  if (rc != RT_OK) return rc;
  // the wide tree (host_bvh8.cpp), opt-in: RT_BVH8=1 at scene creation.  Measured
  // slower than the BVH4 on C4/C5, kept for A/B and further work
  if (tune_int("RT_BVH8", 0) != 0 && out.refs.size() >= kBvh8MinRefs) {
    t0 = std::chrono::steady_clock::now();
    rc = build_bvh8(out);
    if (rc != RT_OK) {
      // an opt-in performance path never fails a valid scene: keep the BVH4
      fprintf(stderr, "[rt] RT_BVH8: %s; keeping the BVH4\n", rt_last_error());
      out.nodes8.clear();
      out.refs8.clear();
      rc = RT_OK;
    }
    if (timing)
      fprintf(stderr, "[rt] build_bvh8 %.3f s (%zu nodes)\n",
              std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(),
              out.nodes8.size() / 8);
  }
  return rc;
}

}  // namespace rt
