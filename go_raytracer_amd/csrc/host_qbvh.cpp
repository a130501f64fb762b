// host_qbvh.cpp — the BVH4 of a large scene re-encoded with 64-B nodes (rt_device.h
// "compressed BVH4 node"), for the fused kernels that read the tree through L1/L2.
//
// The traversal of C3-C5 is bound by the CU's vector-memory data return (C5: TD busy 98 %,
// DESIGN.md §5): every node step moved 112 B per lane (the codes and six plane vectors of a
// 128-B node), every leaf step 64 B.  Here a node is 64 B: its box corner in fp32, and the
// children's planes as fp16 offsets from it (conservatively rounded outwards and widened by
// eps, so every box contains the fp32 box it encodes), plus one word naming its children:
// they sit together, as four consecutive 64-B items of ONE array, each either a node of
// this format or the 64-B leaf record of one prim (rt_device.h "leaf records"; a BVH4 leaf
// of 2-4 prims becomes a node over its prims, boxed by their prim_bounds).
// A node step and a leaf step both load one 64-B item.  The kernel turns an offset into a
// slab distance with one v_fma_mix_f32 (fp16 operand, fp32 arithmetic), t = off * inv +
// (corner - o) * inv, so the planes cost no conversion instructions.
//
// Images: the closest hit is the same as with the 128-B nodes, because every child box
// tested here contains the one tested there (its culling only visits more), and the leaf
// tests are the same code on the same records.
#include <math.h>
#include <string.h>

#include <deque>
#include <vector>

#include "rt_internal.h"

namespace rt {

namespace {

// fp16 bits of the largest half <= x (x >= 0, finite), and of the smallest half >= x
// (x >= 0; overflow gives +inf), exact for every double (frexp / ldexp are exact)
uint16_t half_bits(double x, bool up) {
  if (!(x > 0.0)) return 0;                        // +0 (x == 0)
  if (x > 65504.0) return up ? 0x7C00 : 0x7BFF;    // above the largest finite half
  int e;
  frexp(x, &e);                                    // x = m * 2^e, m in [0.5, 1)
  int ex = e - 1;                                  // x in [2^ex, 2^(ex+1))
  if (ex < -14) ex = -14;                          // subnormals share the 2^-24 step
  const double step = ldexp(1.0, ex - 10);         // the half spacing at x
  double q = x / step;                             // exact: a power-of-two division
  q = up ? ceil(q) : floor(q);
  // q * step is the result; encode it (q may reach 2048 on rounding up: next binade)
  double v = q * step;
  if (v > 65504.0) return 0x7C00;
  if (v == 0.0) return 0;
  frexp(v, &e);
  ex = e - 1;
  if (ex < -14) return (uint16_t)(v / ldexp(1.0, -24));  // subnormal: v / 2^-24
  const uint32_t mant = (uint32_t)(v / ldexp(1.0, ex - 10)) - 1024u;
  return (uint16_t)(((uint32_t)(ex + 15) << 10) | mant);
}

float fbits_f(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}
uint32_t fbits_u(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}

}  // namespace

int build_qbvh(const HostScene& h, const std::vector<F4>& recs, std::vector<F4>* out,
               size_t* n_items) {
  out->clear();
  *n_items = 0;
  if (h.nodes4.empty() || h.root4 == PRIM_NONE || (h.root4 & LEAF_BIT) || h.max_leaf > 4 ||
      h.prim_bounds.size() != 6 * h.refs.size())
    return RT_OK;  // not encodable here (tiny trees, leaves of > 4 prims): the 128-B nodes
  const size_t n4 = h.nodes4.size() / 8;
  // A queue entry is a BVH4 node, or a leaf of 2-4 prims, which becomes a node of its own
  // whose children are its single prims (their boxes: prim_bounds, refs order)
  struct Job {
    uint32_t node;   // BVH4 node, or the leaf's first prim when count > 0
    uint32_t count;  // 0: a BVH4 node; else the leaf's prim count
    uint32_t item;
  };
  std::vector<F4> U(4, F4{0, 0, 0, 0});  // item 0: the root node
  std::deque<Job> q = {{0u, 0u, 0u}};
  while (!q.empty()) {
    const Job job = q.front();
    q.pop_front();
    // the four children: box, BVH4 code (CHILD_EMPTY for an empty slot)
    float cl[4][3], chi[4][3];
    uint32_t code[4];
    if (job.count == 0) {
      if (job.node >= n4) return set_error(RT_ERR_INVALID, "qbvh: node %u of %zu", job.node, n4);
      const float* nd = &h.nodes4[8 * (size_t)job.node].x;  // [field][child]: codes, lo.x, hi.x, ...
      for (int k = 0; k < 4; ++k) {
        code[k] = fbits_u(nd[k]);
        for (int a = 0; a < 3; ++a) {
          cl[k][a] = nd[4 * (1 + 2 * a) + k];
          chi[k][a] = nd[4 * (2 + 2 * a) + k];
        }
      }
    } else {
      for (int k = 0; k < 4; ++k) {
        code[k] = (uint32_t)k < job.count ? leaf_code(job.node + (uint32_t)k, 1u) : CHILD_EMPTY;
        for (int a = 0; a < 3; ++a) {
          cl[k][a] = (uint32_t)k < job.count ? h.prim_bounds[6 * ((size_t)job.node + k) + a] : INFINITY;
          chi[k][a] = (uint32_t)k < job.count ? h.prim_bounds[6 * ((size_t)job.node + k) + 3 + a] : -INFINITY;
        }
      }
    }
    const size_t base = U.size() / 4;
    if (base + 4 >= (1u << 28)) return set_error(RT_ERR_UNSUPPORTED, "qbvh: tree too large");
    U.resize(U.size() + 16, F4{0, 0, 0, 0});
    bool empty[4];
    for (int k = 0; k < 4; ++k)
      empty[k] = code[k] == CHILD_EMPTY ||
                 !(cl[k][0] <= chi[k][0] && cl[k][1] <= chi[k][1] && cl[k][2] <= chi[k][2]);
    // the corner: the node's box lo (over its non-empty children), widened by eps and
    // rounded down in fp32; eps covers the device's two roundings in (corner - o) * inv
    // beyond the slab test's 2-ulp slack (2^-19 of the box's magnitude)
    double lo[3] = {INFINITY, INFINITY, INFINITY}, mag = 0.0;
    bool any = false;
    for (int k = 0; k < 4; ++k) {
      if (empty[k]) continue;
      any = true;
      for (int a = 0; a < 3; ++a) {
        lo[a] = fmin(lo[a], (double)cl[k][a]);
        mag = fmax(mag, fmax(fabs((double)cl[k][a]), fabs((double)chi[k][a])));
      }
    }
    if (!any) return set_error(RT_ERR_INVALID, "qbvh: node %u without children", job.node);
    const double eps = ldexp(mag, -19) + 1e-30;
    float corner[3];
    for (int a = 0; a < 3; ++a) {
      float c = (float)(lo[a] - eps);
      if ((double)c > lo[a] - eps) c = nextafterf(c, -INFINITY);
      corner[a] = c;
    }
    uint16_t planes[3][2][4];  // [axis][lo, hi][child]
    uint32_t leafmask = 0;
    for (int k = 0; k < 4; ++k) {
      for (int a = 0; a < 3; ++a) {
        if (empty[k]) {  // an inverted infinite box: never hit (rt_path.h trav_steps)
          planes[a][0][k] = 0x7C00;
          planes[a][1][k] = 0xFC00;
        } else {
          planes[a][0][k] = half_bits(((double)cl[k][a] - eps) - (double)corner[a], false);
          planes[a][1][k] = half_bits(((double)chi[k][a] + eps) - (double)corner[a], true);
        }
      }
      if (empty[k]) continue;
      const uint32_t item = (uint32_t)(base + k);
      if (code[k] & LEAF_BIT) {
        const uint32_t first = (code[k] >> 4) & 0x7FFFFFFu, count = (code[k] & 15u) + 1u;
        if ((size_t)first + count > h.refs.size() || 4 * ((size_t)first + count) > recs.size())
          return set_error(RT_ERR_INVALID, "qbvh: leaf %u x %u", first, count);
        if (count == 1u) {
          for (int e = 0; e < 4; ++e) U[4 * (size_t)item + e] = recs[4 * (size_t)first + e];
          leafmask |= 1u << k;
        } else {
          q.push_back({first, count, item});  // a node over its prims
        }
      } else {
        q.push_back({code[k], 0u, item});
      }
    }
    F4* node = &U[4 * (size_t)job.item];
    node[0] = {corner[0], corner[1], corner[2], fbits_f((uint32_t)base | (leafmask << 28))};
    for (int a = 0; a < 3; ++a) {
      uint32_t w[4];
      for (int j = 0; j < 2; ++j) {  // lo pair (children 0,1), (2,3); then hi
        w[2 * j + 0] = (uint32_t)planes[a][j][0] | ((uint32_t)planes[a][j][1] << 16);
        w[2 * j + 1] = (uint32_t)planes[a][j][2] | ((uint32_t)planes[a][j][3] << 16);
      }
      node[1 + a] = {fbits_f(w[0]), fbits_f(w[1]), fbits_f(w[2]), fbits_f(w[3])};
    }
  }
  *n_items = U.size() / 4;
  out->swap(U);
  return RT_OK;
}

}  // namespace rt
