// host_bvh8.cpp — the wide tree of large scenes: BVH8 with 16-bit quantised child
// boxes, one 128-B node per L2 line, leaf records regrouped per node.
//
// The closest hit does not depend on the tree (bvh.go:69-82 visits everything that
// may hold it), so this is a different tree over the same leaves: the binary tree
// (host SAH or device PLOC, s.nodes) collapsed to 8 children per node by expanding
// the largest-area inner child until eight, as the BVH4 collapse does with four.
// A BVH4 step over a 1M-triangle mesh resolves 2 tree levels per dependent fetch;
// a BVH8 step resolves 3 in the same 128 B, because the boxes are stored relative
// to the node's own box in 16 bits per plane instead of 32.
//
// Node (8 x F4 = 128 B, rt_device.h "BVH8 node"):
//   [0] origin.xyz (the node's box lo, fp32) | biased exponents ex, ey, ez (bytes 0-2)
//   [1] x child_base (inner children are nodes child_base + rank, in slot order)
//       y leaf_base (leaf children's records start there, in slot order)
//       z meta of slots 0-3, w meta of slots 4-7 (one byte each):
//         0xFF empty, 0x80 | rank inner child, else a leaf: record offset (bits 0-4)
//         from leaf_base and count - 1 (bits 5-6)
//   [2..7] qlo.x, qhi.x, qlo.y, qhi.y, qlo.z, qhi.z: eight uint16 each (slot k in
//       halfword k); child box plane = origin + q * 2^(e - 127), conservative
//       (verified here in fp32 with the device's arithmetic, plus one quantum).
#include <math.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <vector>

#include "rt_internal.h"

namespace rt {

namespace {

struct CBox {
  float lo[3], hi[3];
  double area() const {
    double d[3];
    for (int i = 0; i < 3; ++i) d[i] = std::max(0.0, (double)hi[i] - (double)lo[i]);
    return 2.0 * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
  }
};
struct Child {
  CBox box;
  uint32_t code;  // BVH2 inner node index or leaf code (refs)
};

inline uint32_t fbits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
inline float bitsf(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}
// the device's dequantised plane: origin + q * s, q * s exact (s a power of two)
inline float plane(float origin, uint32_t q, float s) { return origin + (float)q * s; }

// biased exponent E (s = 2^(E-127)) so that the extent spans at most 65000 quanta
// (room for the one-quantum padding on either side)
int pick_exponent(float lo, float hi) {
  const double ext = (double)hi - (double)lo;
  int e = -100;
  if (ext > 0) e = std::max(-100, (int)ceil(log2(ext / 65000.0)));
  while (ldexp(65000.0, e) < ext) ++e;
  return e + 127;
}

}  // namespace

int build_bvh8(HostScene& s) {
  s.nodes8.clear();
  s.refs8.clear();
  if (s.nodes.empty() || (s.root & LEAF_BIT)) return RT_OK;  // no inner node: no tree
  auto child_of = [&](uint32_t node, int k) -> Child {
    const F4* nd = &s.nodes[4 * (size_t)node];
    Child c;
    const F4 mn = nd[2 * k], mx = nd[2 * k + 1];
    c.box = {{mn.x, mn.y, mn.z}, {mx.x, mx.y, mx.z}};
    c.code = fbits(k == 0 ? nd[0].w : nd[1].w);
    return c;
  };
  auto is_inner = [](uint32_t code) { return (code & LEAF_BIT) == 0u; };
  // BFS: queue entries are BVH2 inner nodes, each becomes one BVH8 node
  std::vector<uint32_t> queue = {s.root};
  std::vector<CBox> qbox(1);
  {
    const Child a = child_of(s.root, 0), b = child_of(s.root, 1);
    for (int i = 0; i < 3; ++i) {
      qbox[0].lo[i] = std::min(a.box.lo[i], b.box.lo[i]);
      qbox[0].hi[i] = std::max(a.box.hi[i], b.box.hi[i]);
    }
  }
  s.nodes8.reserve(8 * (s.nodes.size() / 4 / 3 + 1));
  for (size_t head = 0; head < queue.size(); ++head) {
    std::vector<Child> ch = {child_of(queue[head], 0), child_of(queue[head], 1)};
    while (ch.size() < 8) {
      int best = -1;
      double best_area = -1;
      for (int k = 0; k < (int)ch.size(); ++k)
        if (is_inner(ch[k].code) && ch[k].box.area() > best_area) {
          best_area = ch[k].box.area();
          best = k;
        }
      if (best < 0) break;
      const uint32_t v = ch[best].code;
      ch[best] = child_of(v, 0);
      ch.push_back(child_of(v, 1));
    }
    const CBox nb = qbox[head];
    F4 node[8];
    memset(node, 0, sizeof node);
    // quantisation frame: origin = the node's box lo, one exponent per axis
    int E[3];
    float sc[3];
    for (int a = 0; a < 3; ++a) {
      E[a] = pick_exponent(nb.lo[a], nb.hi[a]);
      sc[a] = bitsf((uint32_t)E[a] << 23);
    }
    uint16_t q[6][8];
    for (int f = 0; f < 6; ++f)
      for (int k = 0; k < 8; ++k) q[f][k] = (f & 1) ? 0 : 0xFFFF;  // empty slots: inverted box
    uint8_t meta[8];
    memset(meta, 0xFF, sizeof meta);
    const uint32_t child_base = (uint32_t)queue.size();
    const uint32_t leaf_base = (uint32_t)s.refs8.size();
    uint32_t rank = 0, offset = 0;
    for (int k = 0; k < (int)ch.size(); ++k) {
      const Child& c = ch[k];
      for (int a = 0; a < 3; ++a) {
        const float o = nb.lo[a], st = sc[a];
        // conservative 16-bit planes, verified with the device's fp32 dequantisation
        double fl = floor(((double)c.box.lo[a] - o) / st) - 1.0;
        double fh = ceil(((double)c.box.hi[a] - o) / st) + 1.0;
        uint32_t ql = (uint32_t)std::min(65535.0, std::max(0.0, fl));
        uint32_t qh = (uint32_t)std::min(65535.0, std::max(0.0, fh));
        while (ql > 0 && plane(o, ql, st) > c.box.lo[a]) --ql;
        while (qh < 65535 && plane(o, qh, st) < c.box.hi[a]) ++qh;
        if (plane(o, ql, st) > c.box.lo[a] || plane(o, qh, st) < c.box.hi[a])
          return set_error(RT_ERR_INVALID, "bvh8: child box outside its node's frame");
        q[2 * a][k] = (uint16_t)ql;
        q[2 * a + 1][k] = (uint16_t)qh;
      }
      if (is_inner(c.code)) {
        meta[k] = (uint8_t)(0x80u | rank++);
        queue.push_back(c.code);
        qbox.push_back(c.box);
      } else {
        const uint32_t first = (c.code >> 4) & 0x7FFFFFFu, count = (c.code & 15u) + 1u;
        if (count > 4u || offset + count > 32u)
          return set_error(RT_ERR_UNSUPPORTED, "bvh8: leaf of %u prims (max 4)", count);
        meta[k] = (uint8_t)(offset | ((count - 1u) << 5));
        for (uint32_t i = 0; i < count; ++i) s.refs8.push_back(s.refs[first + i]);
        offset += count;
      }
    }
    node[0] = {nb.lo[0], nb.lo[1], nb.lo[2], bitsf((uint32_t)E[0] | ((uint32_t)E[1] << 8) |
                                                   ((uint32_t)E[2] << 16))};
    uint32_t m0 = 0, m1 = 0;
    for (int k = 0; k < 4; ++k) {
      m0 |= (uint32_t)meta[k] << (8 * k);
      m1 |= (uint32_t)meta[k + 4] << (8 * k);
    }
    node[1] = {bitsf(child_base), bitsf(leaf_base), bitsf(m0), bitsf(m1)};
    for (int f = 0; f < 6; ++f) {
      uint32_t w[4];
      for (int j = 0; j < 4; ++j) w[j] = (uint32_t)q[f][2 * j] | ((uint32_t)q[f][2 * j + 1] << 16);
      node[2 + f] = {bitsf(w[0]), bitsf(w[1]), bitsf(w[2]), bitsf(w[3])};
    }
    s.nodes8.insert(s.nodes8.end(), node, node + 8);
  }
  return RT_OK;
}

}  // namespace rt
