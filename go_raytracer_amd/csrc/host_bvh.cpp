// host_bvh.cpp — the device BVH: binned-SAH BVH2, nodes in BFS order so the top
// of the tree is one contiguous block that the extend kernel stages in LDS.
//
// The reference builds a median-split binary tree over interface values and
// visits both children of every node, left first (bvh.go:21-82).  The closest
// hit does not depend on the topology (ties aside), so the device tree is our
// own: SAH splits, leaves of up to 4 prims, near-child-first traversal.
#include <stdlib.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <stdio.h>

#include <atomic>
#include <chrono>
#include <deque>
#include <thread>
#include <vector>

#include "rt_internal.h"

namespace rt {
namespace {

struct Box {
  float mn[3] = {INFINITY, INFINITY, INFINITY};
  float mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const Box& b) {
    for (int i = 0; i < 3; ++i) {
      mn[i] = std::min(mn[i], b.mn[i]);
      mx[i] = std::max(mx[i], b.mx[i]);
    }
  }
  void grow_pt(const float* p) {
    for (int i = 0; i < 3; ++i) {
      mn[i] = std::min(mn[i], p[i]);
      mx[i] = std::max(mx[i], p[i]);
    }
  }
  double area() const {
    double d[3];
    for (int i = 0; i < 3; ++i) d[i] = std::max(0.0, (double)mx[i] - (double)mn[i]);
    return 2.0 * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
  }
};

struct TmpNode {
  Box box;
  int first = 0, count = 0;  // prim range (leaf)
  int left = -1, right = -1; // children (inner)
  int depth = 0;
};

constexpr int kBins = 16;
// SAH leaf/split trade-off; the knobs RT_BVH_LEAF / RT_BVH_CT / RT_BVH_CI override (rt_tune_set)

}  // namespace

int build_bvh(HostScene& s, const std::vector<F4>& lo, const std::vector<F4>& hi,
              const std::vector<uint32_t>& prims) {
  const int n = (int)prims.size();
  // SAH may stop at <= kLeafTarget prims.  Measured (tools/bvh_sweep.sh, tools/leaf_ab.sh,
  // profiles/): small scenes, whose tree and leaves sit in LDS, are fastest with leaves
  // of up to 4; trees read through L1/L2 (C3 485 prims, C4 3.4k, C5 1M) with single-prim
  // leaves (C4/C5 -11 %, C3 -1.6 %), the parent's child box culling each prim before its
  // record is fetched.  Above 256 prims a tree no longer fits the LDS cache.
  const int kLeafTarget = std::min(tune_int("RT_BVH_LEAF", n > 256 ? 1 : 4), MAX_LEAF);
  const double kCostTrav = tune_num("RT_BVH_CT", 1.0), kCostIsect = tune_num("RT_BVH_CI", 1.0);
  s.nodes.clear();
  s.refs.clear();
  s.prim_bounds.clear();
  s.bvh_depth = 0;
  s.max_leaf = 0;
  if (n == 0) {
    s.root = PRIM_NONE;
    return RT_OK;
  }
  if ((uint32_t)n > 0x7FFFFFFu) return set_error(RT_ERR_UNSUPPORTED, "too many prims (%d)", n);

  std::vector<Box> pb(n);
  std::vector<float> cen(3 * (size_t)n);
  for (int i = 0; i < n; ++i) {
    pb[i].mn[0] = lo[i].x;
    pb[i].mn[1] = lo[i].y;
    pb[i].mn[2] = lo[i].z;
    pb[i].mx[0] = hi[i].x;
    pb[i].mx[1] = hi[i].y;
    pb[i].mx[2] = hi[i].z;
    for (int a = 0; a < 3; ++a) cen[3 * (size_t)i + a] = 0.5f * (pb[i].mn[a] + pb[i].mx[a]);
  }
  std::vector<int> idx(n);
  for (int i = 0; i < n; ++i) idx[i] = i;
  const bool timing = tune_int("RT_TIMING", 0) != 0;
  auto tic = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!timing) return;
    auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[rt]   bvh %s %.3f s\n", what, std::chrono::duration<double>(now - tic).count());
    tic = now;
  };

  // Node split: bounds, binned SAH over three axes, partition of idx[first,
  // first+count).  Box growth is min/max and bin counts are integers, so running
  // the loops on T threads (large nodes) gives bit-identical trees.
  // (bit-identical for any thread count: 16, the GPU box's CPU share, unless RT_THREADS is set)
  const int threads = std::max(1, std::min(tune_int("RT_THREADS", 16),
                                           (int)std::max(1u, std::thread::hardware_concurrency())));
  auto par = [&](int T, int first, int count, auto&& fn) {  // fn(t, lo, hi)
    if (T <= 1) {
      fn(0, first, first + count);
      return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) {
      const int lo = first + (int)((int64_t)count * t / T), hi = first + (int)((int64_t)count * (t + 1) / T);
      th.emplace_back([&fn, t, lo, hi] { fn(t, lo, hi); });
    }
    for (auto& x : th) x.join();
  };
  // returns true and fills L, R when nd is split (nd.box is always set)
  auto split_node = [&](TmpNode& nd, int T, TmpNode& L, TmpNode& R) -> bool {
    // per-thread partials: on the stack for the one-thread case (every node below
    // the top levels), on the heap otherwise (few, large nodes)
    Box pbb1[1], pcb1[1];
    std::array<Box, 3 * kBins> tbins1[1];
    std::array<int, 3 * kBins> tcnt1[1];
    std::vector<Box> pbbv, pcbv;
    std::vector<std::array<Box, 3 * kBins>> tbinsv;
    std::vector<std::array<int, 3 * kBins>> tcntv;
    if (T > 1) {
      pbbv.resize(T), pcbv.resize(T), tbinsv.resize(T), tcntv.resize(T);
    }
    Box* pbb = T > 1 ? pbbv.data() : pbb1;
    Box* pcb = T > 1 ? pcbv.data() : pcb1;
    std::array<Box, 3 * kBins>* tbins = T > 1 ? tbinsv.data() : tbins1;
    std::array<int, 3 * kBins>* tcnt = T > 1 ? tcntv.data() : tcnt1;
    par(T, nd.first, nd.count, [&](int t, int lo, int hi) {
      Box bb, cb;
      for (int i = lo; i < hi; ++i) {
        bb.grow(pb[idx[i]]);
        cb.grow_pt(&cen[3 * (size_t)idx[i]]);
      }
      pbb[t] = bb;
      pcb[t] = cb;
    });
    Box bb, cb;
    for (int t = 0; t < T; ++t) {
      bb.grow(pbb[t]);
      cb.grow(pcb[t]);
    }
    nd.box = bb;
    if (nd.count <= 1) return false;

    // binned SAH over all three axes
    float kinv[3];
    for (int a = 0; a < 3; ++a) {
      const float ext = cb.mx[a] - cb.mn[a];
      kinv[a] = ext > 0 ? kBins / ext : 0.0f;
    }
    par(T, nd.first, nd.count, [&](int t, int lo, int hi) {
      auto& bins = tbins[t];
      auto& cnt = tcnt[t];
      cnt.fill(0);
      for (int i = lo; i < hi; ++i) {
        const int p = idx[i];
        for (int a = 0; a < 3; ++a) {
          if (!(kinv[a] > 0)) continue;
          int b = (int)((cen[3 * (size_t)p + a] - cb.mn[a]) * kinv[a]);
          b = std::min(std::max(b, 0), kBins - 1);
          cnt[a * kBins + b]++;
          bins[a * kBins + b].grow(pb[p]);
        }
      }
    });
    double best_cost = INFINITY;
    int best_axis = -1, best_split = -1;
    for (int a = 0; a < 3; ++a) {
      if (!(kinv[a] > 0)) continue;
      Box bins[kBins];
      int cnt[kBins] = {0};
      for (int t = 0; t < T; ++t)
        for (int b = 0; b < kBins; ++b) {
          bins[b].grow(tbins[t][a * kBins + b]);
          cnt[b] += tcnt[t][a * kBins + b];
        }
      double left_area[kBins];
      int left_cnt[kBins];
      Box acc;
      int c = 0;
      for (int b = 0; b < kBins - 1; ++b) {
        acc.grow(bins[b]);
        c += cnt[b];
        left_area[b] = acc.area();
        left_cnt[b] = c;
      }
      acc = Box();
      c = 0;
      for (int b = kBins - 1; b > 0; --b) {
        acc.grow(bins[b]);
        c += cnt[b];
        int lc = left_cnt[b - 1];
        if (lc == 0 || c == 0) continue;
        double cost = left_area[b - 1] * lc + acc.area() * c;
        if (cost < best_cost) {
          best_cost = cost;
          best_axis = a;
          best_split = b;
        }
      }
    }
    double parent_area = std::max(bb.area(), 1e-30);
    double split_cost = kCostTrav + kCostIsect * best_cost / parent_area;
    double leaf_cost = kCostIsect * nd.count;
    int mid;
    if (best_axis >= 0 && !(nd.count <= kLeafTarget && leaf_cost <= split_cost)) {
      const float k = kinv[best_axis];
      auto it = std::partition(idx.begin() + nd.first, idx.begin() + nd.first + nd.count, [&](int p) {
        int b = (int)((cen[3 * (size_t)p + best_axis] - cb.mn[best_axis]) * k);
        b = std::min(std::max(b, 0), kBins - 1);
        return b < best_split;
      });
      mid = (int)(it - idx.begin());
    } else if (nd.count <= kLeafTarget) {
      return false;  // leaf
    } else {
      // no usable SAH split (coincident centroids): median split by index
      if (nd.count <= MAX_LEAF && best_axis < 0) return false;
      int a = 0;
      float e = -1;
      for (int q = 0; q < 3; ++q)
        if (cb.mx[q] - cb.mn[q] > e) {
          e = cb.mx[q] - cb.mn[q];
          a = q;
        }
      mid = nd.first + nd.count / 2;
      std::nth_element(idx.begin() + nd.first, idx.begin() + mid, idx.begin() + nd.first + nd.count,
                       [&](int p, int q) { return cen[3 * (size_t)p + a] < cen[3 * (size_t)q + a]; });
    }
    if (mid == nd.first || mid == nd.first + nd.count) mid = nd.first + nd.count / 2;
    L = TmpNode();
    R = TmpNode();
    L.first = nd.first;
    L.count = mid - nd.first;
    R.first = mid;
    R.count = nd.first + nd.count - mid;
    L.depth = R.depth = nd.depth + 1;
    return true;
  };
  // depth-first build of the subtree under tn_local[0] (one thread)
  auto build_sub = [&](std::vector<TmpNode>& tl) {
    std::vector<int> work = {0};
    while (!work.empty()) {
      const int ni = work.back();
      work.pop_back();
      TmpNode L, R;
      TmpNode nd = tl[ni];
      const bool sp = split_node(nd, 1, L, R);
      tl[ni].box = nd.box;
      if (!sp) continue;
      const int li = (int)tl.size();
      tl.push_back(L);
      tl.push_back(R);
      tl[ni].left = li;
      tl[ni].right = li + 1;
      work.push_back(li + 1);
      work.push_back(li);
    }
  };

  std::vector<TmpNode> tn;
  tn.reserve(2 * (size_t)n / kLeafTarget + 16);
  tn.push_back(TmpNode());
  tn[0].first = 0;
  tn[0].count = n;
  // top of the tree: large nodes one at a time with threaded loops; subtrees
  // below kSub prims are deferred and built in parallel, one per thread
  const int kSub = threads > 1 ? std::max(4096, n / (8 * threads)) : n + 1;
  std::vector<int> deferred;
  {
    std::vector<int> work = {0};
    while (!work.empty()) {
      const int ni = work.back();
      work.pop_back();
      if (tn[ni].count < kSub) {
        deferred.push_back(ni);
        continue;
      }
      TmpNode L, R;
      TmpNode nd = tn[ni];
      const int T = std::min(threads, std::max(1, nd.count / 16384));
      const bool sp = split_node(nd, T, L, R);
      tn[ni].box = nd.box;
      if (!sp) continue;
      const int li = (int)tn.size();
      tn.push_back(L);
      tn.push_back(R);
      tn[ni].left = li;
      tn[ni].right = li + 1;
      work.push_back(li + 1);
      work.push_back(li);
    }
  }
  lap("top levels");
  if (!deferred.empty()) {
    std::vector<std::vector<TmpNode>> sub(deferred.size());
    std::atomic<size_t> next{0};
    auto worker = [&] {
      for (size_t k; (k = next.fetch_add(1)) < deferred.size();) {
        sub[k].reserve(2 * (size_t)tn[deferred[k]].count / kLeafTarget + 4);
        sub[k].push_back(tn[deferred[k]]);
        build_sub(sub[k]);
      }
    };
    std::vector<std::thread> th;
    const int T = std::min<int>(threads, (int)deferred.size());
    for (int t = 1; t < T; ++t) th.emplace_back(worker);
    worker();
    for (auto& x : th) x.join();
    // splice the subtrees in deferred order (the output order is BFS anyway)
    for (size_t k = 0; k < deferred.size(); ++k) {
      const std::vector<TmpNode>& v = sub[k];
      const int base = (int)tn.size() - 1;  // local index i >= 1 -> base + i
      TmpNode root = v[0];
      if (root.left >= 0) {
        root.left += base;
        root.right += base;
      }
      tn[deferred[k]] = root;
      for (size_t i = 1; i < v.size(); ++i) {
        TmpNode x = v[i];
        if (x.left >= 0) {
          x.left += base;
          x.right += base;
        }
        tn.push_back(x);
      }
    }
  }
  for (const auto& x : tn) s.bvh_depth = std::max(s.bvh_depth, x.depth);
  lap("subtrees");

  // permuted refs + bounds
  s.refs.resize(n);
  s.prim_bounds.resize(6 * (size_t)n);
  for (int i = 0; i < n; ++i) {
    s.refs[i] = prims[idx[i]];
    for (int a = 0; a < 3; ++a) {
      s.prim_bounds[6 * (size_t)i + a] = pb[idx[i]].mn[a];
      s.prim_bounds[6 * (size_t)i + 3 + a] = pb[idx[i]].mx[a];
    }
  }
  auto leaf_of = [&](const TmpNode& x) -> uint32_t {
    s.max_leaf = std::max(s.max_leaf, x.count);
    return leaf_code((uint32_t)x.first, (uint32_t)x.count);
  };
  for (const auto& x : tn)
    if (x.left < 0 && x.count > MAX_LEAF)
      return set_error(RT_ERR_UNSUPPORTED, "BVH leaf of %d prims exceeds %d", x.count, MAX_LEAF);

  if (tn[0].left < 0) {
    s.root = s.root4 = leaf_of(tn[0]);
    s.nodes4.clear();
    return RT_OK;
  }
  // BFS numbering of inner nodes
  std::vector<int> order;
  std::vector<int> out_index(tn.size(), -1);
  std::deque<int> q = {0};
  while (!q.empty()) {
    int i = q.front();
    q.pop_front();
    out_index[i] = (int)order.size();
    order.push_back(i);
    for (int c : {tn[i].left, tn[i].right})
      if (tn[c].left >= 0) q.push_back(c);
  }
  s.nodes.assign(4 * order.size(), F4{0, 0, 0, 0});
  auto bits = [](uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
  };
  for (size_t o = 0; o < order.size(); ++o) {
    const TmpNode& nd = tn[order[o]];
    const TmpNode& a = tn[nd.left];
    const TmpNode& b = tn[nd.right];
    uint32_t ca = a.left >= 0 ? (uint32_t)out_index[nd.left] : leaf_of(a);
    uint32_t cbits = b.left >= 0 ? (uint32_t)out_index[nd.right] : leaf_of(b);
    s.nodes[4 * o + 0] = {a.box.mn[0], a.box.mn[1], a.box.mn[2], bits(ca)};
    s.nodes[4 * o + 1] = {a.box.mx[0], a.box.mx[1], a.box.mx[2], bits(cbits)};
    s.nodes[4 * o + 2] = {b.box.mn[0], b.box.mn[1], b.box.mn[2], 0};
    s.nodes[4 * o + 3] = {b.box.mx[0], b.box.mx[1], b.box.mx[2], 0};
  }
  s.root = 0;

  // BVH4 by collapsing the binary tree: a BVH4 node starts from a BVH2 inner
  // node's two children and keeps replacing its largest-area inner child by
  // that child's two children until it has four or only leaves are left.
  // Leaves (and so the leaf records) are shared with the BVH2.
  std::vector<std::array<int, 4>> kids;
  std::vector<int> nkids;
  std::deque<int> q4 = {0};
  std::vector<int> out4(tn.size(), -1);
  std::vector<int> order4;
  while (!q4.empty()) {
    int i = q4.front();
    q4.pop_front();
    out4[i] = (int)order4.size();
    order4.push_back(i);
    std::array<int, 4> ch = {tn[i].left, tn[i].right, -1, -1};
    int nc = 2;
    while (nc < 4) {
      int best = -1;
      double best_area = -1;
      for (int k = 0; k < nc; ++k)
        if (tn[ch[k]].left >= 0 && tn[ch[k]].box.area() > best_area) {
          best_area = tn[ch[k]].box.area();
          best = k;
        }
      if (best < 0) break;
      const int c = ch[best];
      ch[best] = tn[c].left;
      ch[nc++] = tn[c].right;
    }
    for (int k = 0; k < nc; ++k)
      if (tn[ch[k]].left >= 0) q4.push_back(ch[k]);
    kids.push_back(ch);
    nkids.push_back(nc);
  }
  s.nodes4.assign(8 * order4.size(), F4{0, 0, 0, 0});
  for (size_t o = 0; o < order4.size(); ++o) {
    F4* nd = &s.nodes4[8 * o];
    float* lx = &nd[0].x;  // the 8 F4 as 32 floats: [field][child]
    for (int k = 0; k < 4; ++k) {
      uint32_t code = CHILD_EMPTY;
      // empty slot: an inverted infinite box (lo = +inf, hi = -inf), which the
      // sign-selected slab test (rt_path.h trav_steps) never hits; the min/max slab
      // tests (LDS trees) skip it by its code
      Box b;
      for (int a = 0; a < 3; ++a) b.mn[a] = INFINITY, b.mx[a] = -INFINITY;
      if (k < nkids[o]) {
        const TmpNode& c = tn[kids[o][k]];
        b = c.box;
        code = c.left >= 0 ? (uint32_t)out4[kids[o][k]] : leaf_of(c);
      }
      for (int a = 0; a < 3; ++a) {  // rt_device.h "BVH4 node": codes, then the planes
        lx[(1 + 2 * a) * 4 + k] = b.mn[a];
        lx[(2 + 2 * a) * 4 + k] = b.mx[a];
      }
      lx[k] = bits(code);
    }
  }
  s.root4 = 0;
  lap("numbering + BVH4");
  return RT_OK;
}

}  // namespace rt
