// rt_build.hip — BVH construction on the MI355X for large scenes (C5's 1M-triangle
// mesh; the reference builds its median-split tree in Go, bvh.go:21-61, after
// objLoader.go:489-512 collected the triangles).
//
// PLOC (Meister & Bittner, "Parallel Locally-Ordered Clustering for Bounding
// Volume Hierarchy Construction", IEEE TVCG 2018): primitives sorted along a
// 63-bit Morton curve start as singleton clusters; every iteration each cluster
// finds its nearest neighbour -- the cluster within R positions whose merged box
// has the smallest surface area -- and mutual nearest neighbours merge into a new
// inner node.  The survivors are compacted in curve order and the loop repeats
// until one cluster (the root) is left.  Trees are close to a full SAH sweep in
// traversal cost (the paper's r = 16..25) at a few milliseconds for 1M primitives.
//
// Device side: one kernel per step (bounds, Morton codes, nearest neighbour with
// the window in LDS, merge, emit), hipCUB radix sort and scans between them, all
// on one stream; each iteration reads back one counter.  Host side: BFS numbering
// of the binary tree into the HostScene layout (BVH2 export nodes + the BVH4 the
// kernels traverse, exactly as host_bvh.cpp lays it out), so rt_scene_create's
// other outputs are unchanged.  The result is deterministic: the sort is stable,
// ties pick the lower index, and node ids come from prefix sums, not atomics.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <vector>

#include "rt_internal.h"

namespace rt {
namespace {

#ifndef PLOC_R
#define PLOC_R 16
#endif
constexpr int kR = PLOC_R;  // PLOC search radius (clusters on each side)
#ifndef PLOC_TOP
#define PLOC_TOP 16384  // clusters left to the host full SAH sweep: C5 render +2.5 % vs the host tree (1: +6 %)
#endif
constexpr int kBlock = 256;

#define B_OK(expr)                                                                       \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      return set_error(RT_ERR_DEVICE, "bvh build: %s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

__device__ __forceinline__ float4 fmin4(float4 a, float4 b) {
  return make_float4(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z), 0.0f);
}
__device__ __forceinline__ float4 fmax4(float4 a, float4 b) {
  return make_float4(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), 0.0f);
}
__device__ __forceinline__ float half_area(float4 lo, float4 hi) {
  const float dx = hi.x - lo.x, dy = hi.y - lo.y, dz = hi.z - lo.z;
  return dx * dy + dy * dz + dz * dx;
}

// centroid bounds, per block -> part[2 * block] (lo, hi)
__global__ __launch_bounds__(kBlock) void k_bounds(const float4* lo, const float4* hi, int n,
                                                  float4* part) {
  __shared__ float4 slo[kBlock], shi[kBlock];
  float4 a = make_float4(INFINITY, INFINITY, INFINITY, 0), b = make_float4(-INFINITY, -INFINITY, -INFINITY, 0);
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const float4 l = lo[i], h = hi[i];
    const float4 c = make_float4(0.5f * (l.x + h.x), 0.5f * (l.y + h.y), 0.5f * (l.z + h.z), 0);
    a = fmin4(a, c);
    b = fmax4(b, c);
  }
  slo[threadIdx.x] = a;
  shi[threadIdx.x] = b;
  __syncthreads();
  for (int s = kBlock / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      slo[threadIdx.x] = fmin4(slo[threadIdx.x], slo[threadIdx.x + s]);
      shi[threadIdx.x] = fmax4(shi[threadIdx.x], shi[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = slo[0];
    part[2 * blockIdx.x + 1] = shi[0];
  }
}

__device__ __forceinline__ uint64_t spread21(uint64_t x) {  // 21 bits -> every third bit
  x &= 0x1FFFFFull;
  x = (x | x << 32) & 0x1F00000000FFFFull;
  x = (x | x << 16) & 0x1F0000FF0000FFull;
  x = (x | x << 8) & 0x100F00F00F00F00Full;
  x = (x | x << 4) & 0x10C30C30C30C30C3ull;
  x = (x | x << 2) & 0x1249249249249249ull;
  return x;
}

// 63-bit Morton code of each centroid (bounds reduced from the block partials)
__global__ __launch_bounds__(kBlock) void k_morton(const float4* lo, const float4* hi, int n,
                                                  const float4* part, int nparts, uint64_t* key,
                                                  uint32_t* val) {
  __shared__ float4 cb[2];
  if (threadIdx.x == 0) {
    float4 a = part[0], b = part[1];
    for (int p = 1; p < nparts; ++p) {
      a = fmin4(a, part[2 * p]);
      b = fmax4(b, part[2 * p + 1]);
    }
    cb[0] = a;
    cb[1] = b;
  }
  __syncthreads();
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const float4 a = cb[0], b = cb[1];
  const float4 l = lo[i], h = hi[i];
  const float c[3] = {0.5f * (l.x + h.x), 0.5f * (l.y + h.y), 0.5f * (l.z + h.z)};
  const float mn[3] = {a.x, a.y, a.z}, ext[3] = {b.x - a.x, b.y - a.y, b.z - a.z};
  uint64_t code = 0;
  for (int k = 0; k < 3; ++k) {
    const float t = ext[k] > 0.0f ? (c[k] - mn[k]) / ext[k] : 0.0f;
    const uint64_t q = (uint64_t)fminf(fmaxf(t * 2097152.0f, 0.0f), 2097151.0f);
    code |= spread21(q) << (2 - k);
  }
  key[i] = code;
  val[i] = (uint32_t)i;
}

// leaves in curve order: node k = prim val[k]; clusters start as the leaves
__global__ __launch_bounds__(kBlock) void k_leaves(const float4* lo, const float4* hi, int n,
                                                  const uint32_t* order, float4* nlo, float4* nhi,
                                                  int* cl, float4* clo, float4* chi) {
  const int k = blockIdx.x * kBlock + threadIdx.x;
  if (k >= n) return;
  const uint32_t p = order[k];
  float4 l = lo[p], h = hi[p];
  l.w = __int_as_float(-1);  // no children
  h.w = __int_as_float(-1);
  nlo[k] = l;
  nhi[k] = h;
  cl[k] = k;
  clo[k] = l;
  chi[k] = h;
}

// nearest neighbour of every cluster within kR positions (window staged in LDS);
// ties go to the lower index, so the choice is symmetric and deterministic
__global__ __launch_bounds__(kBlock) void k_nn(const float4* clo, const float4* chi, int m, int* nn) {
  __shared__ float4 slo[kBlock + 2 * kR], shi[kBlock + 2 * kR];
  const int base = blockIdx.x * kBlock;
  for (int t = threadIdx.x; t < kBlock + 2 * kR; t += kBlock) {
    const int g = base - kR + t;
    if (g >= 0 && g < m) {
      slo[t] = clo[g];
      shi[t] = chi[g];
    }
  }
  __syncthreads();
  const int i = base + threadIdx.x;
  if (i >= m) return;
  const float4 a = slo[threadIdx.x + kR], b = shi[threadIdx.x + kR];
  float best = INFINITY;
  int bj = -1;
  const int j0 = max(0, i - kR), j1 = min(m - 1, i + kR);
  for (int j = j0; j <= j1; ++j) {
    if (j == i) continue;
    const int t = j - base + kR;
    const float ar = half_area(fmin4(a, slo[t]), fmax4(b, shi[t]));
    if (ar < best) {
      best = ar;
      bj = j;
    }
  }
  nn[i] = bj;
}

// create: the lower of a mutual pair makes the new node; valid: survives into the
// next cluster list (everything but the upper of a mutual pair).  `force` (no
// mutual pair found last time: never observed, kept as a guarantee of progress)
// pairs clusters 2k, 2k+1.
__global__ __launch_bounds__(kBlock) void k_flags(const int* nn, int m, int force, int* create,
                                                 int* valid) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= m) return;
  int j = nn[i];
  if (force) j = (i ^ 1) < m ? (i ^ 1) : -1;
  const bool mutual = j >= 0 && (force ? true : nn[j] == i);
  create[i] = mutual && i < j;
  valid[i] = !(mutual && i > j);
}

__global__ __launch_bounds__(kBlock) void k_emit(const int* nn, int m, int force, const int* create,
                                                const int* valid, const int* sc, const int* sv,
                                                int node_base, const int* cl, const float4* clo,
                                                const float4* chi, float4* nlo, float4* nhi,
                                                int* cl2, float4* clo2, float4* chi2, int* counts) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= m) return;
  if (i == m - 1) {
    counts[0] = sv[i] + valid[i];   // clusters left
    counts[1] = sc[i] + create[i];  // nodes made
  }
  if (!valid[i]) return;
  const int o = sv[i];
  if (create[i]) {
    const int j = force ? (i ^ 1) : nn[i];
    const int id = node_base + sc[i];
    float4 l = fmin4(clo[i], clo[j]), h = fmax4(chi[i], chi[j]);
    clo2[o] = l;
    chi2[o] = h;
    l.w = __int_as_float(cl[i]);
    h.w = __int_as_float(cl[j]);
    nlo[id] = l;
    nhi[id] = h;
    cl2[o] = id;
  } else {
    cl2[o] = cl[i];
    clo2[o] = clo[i];
    chi2[o] = chi[i];
  }
}

struct DevBuf {
  std::vector<void*> p;
  ~DevBuf() {
    for (void* q : p) (void)hipFree(q);
  }
  template <typename T>
  int alloc(T** out, size_t n) {
    void* q = nullptr;
    B_OK(hipMalloc(&q, std::max<size_t>(n, 1) * sizeof(T)));
    p.push_back(q);
    *out = (T*)q;
    return RT_OK;
  }
};

double area_of(const F4& lo, const F4& hi) {
  const double dx = (double)hi.x - lo.x, dy = (double)hi.y - lo.y, dz = (double)hi.z - lo.z;
  return 2.0 * (std::max(0.0, dx) * std::max(0.0, dy) + std::max(0.0, dy) * std::max(0.0, dz) +
                std::max(0.0, dz) * std::max(0.0, dx));
}

}  // namespace

// Top of the tree over the last PLOC clusters: a full SAH sweep (sort by centroid
// on each axis, prefix/suffix areas), recursing down to single clusters.  Nodes are
// created in post-order from node_base, so the root is the last node (2n-2).
static int top_sah(std::vector<int>& ids, std::vector<F4>& blo, std::vector<F4>& bhi, int first,
                   int count, std::vector<F4>& nlo, std::vector<F4>& nhi, int& node_base) {
  if (count == 1) return ids[first];
  std::vector<int> perm(count), best_perm;
  double best = INFINITY;
  int best_k = count / 2, best_axis = -1;
  std::vector<double> left(count);
  auto sort_axis = [&](int axis) {
    for (int i = 0; i < count; ++i) perm[i] = first + i;
    auto cen = [&](int i) {
      const float* a = &blo[i].x;
      const float* b = &bhi[i].x;
      return a[axis] + b[axis];
    };
    std::stable_sort(perm.begin(), perm.end(), [&](int a, int b) { return cen(a) < cen(b); });
  };
  for (int axis = 0; axis < 3; ++axis) {
    sort_axis(axis);
    F4 lo = {INFINITY, INFINITY, INFINITY, 0}, hi = {-INFINITY, -INFINITY, -INFINITY, 0};
    for (int i = 0; i < count; ++i) {
      const F4 &a = blo[perm[i]], &b = bhi[perm[i]];
      lo = {std::min(lo.x, a.x), std::min(lo.y, a.y), std::min(lo.z, a.z), 0};
      hi = {std::max(hi.x, b.x), std::max(hi.y, b.y), std::max(hi.z, b.z), 0};
      left[i] = area_of(lo, hi) * (i + 1);
    }
    lo = {INFINITY, INFINITY, INFINITY, 0}, hi = {-INFINITY, -INFINITY, -INFINITY, 0};
    for (int i = count - 1; i > 0; --i) {
      const F4 &a = blo[perm[i]], &b = bhi[perm[i]];
      lo = {std::min(lo.x, a.x), std::min(lo.y, a.y), std::min(lo.z, a.z), 0};
      hi = {std::max(hi.x, b.x), std::max(hi.y, b.y), std::max(hi.z, b.z), 0};
      const double c = left[i - 1] + area_of(lo, hi) * (count - i);
      if (c < best) {
        best = c;
        best_k = i;
        best_axis = axis;
      }
    }
  }
  if (best_axis >= 0) {
    sort_axis(best_axis);
    best_perm = perm;
  } else {  // NaN boxes: keep the curve order
    best_perm.resize(count);
    for (int i = 0; i < count; ++i) best_perm[i] = first + i;
  }
  std::vector<int> ids2(count);
  std::vector<F4> lo2(count), hi2(count);
  for (int i = 0; i < count; ++i) {
    ids2[i] = ids[best_perm[i]];
    lo2[i] = blo[best_perm[i]];
    hi2[i] = bhi[best_perm[i]];
  }
  std::copy(ids2.begin(), ids2.end(), ids.begin() + first);
  std::copy(lo2.begin(), lo2.end(), blo.begin() + first);
  std::copy(hi2.begin(), hi2.end(), bhi.begin() + first);
  const int a = top_sah(ids, blo, bhi, first, best_k, nlo, nhi, node_base);
  const int b = top_sah(ids, blo, bhi, first + best_k, count - best_k, nlo, nhi, node_base);
  const int id = node_base++;
  F4 l = {std::min(nlo[a].x, nlo[b].x), std::min(nlo[a].y, nlo[b].y), std::min(nlo[a].z, nlo[b].z), 0};
  F4 h = {std::max(nhi[a].x, nhi[b].x), std::max(nhi[a].y, nhi[b].y), std::max(nhi[a].z, nhi[b].z), 0};
  memcpy(&l.w, &a, 4);
  memcpy(&h.w, &b, 4);
  nlo[id] = l;
  nhi[id] = h;
  return id;
}
static void build_top_sah(std::vector<int>& ids, std::vector<F4>& blo, std::vector<F4>& bhi,
                          std::vector<F4>& nlo, std::vector<F4>& nhi, int& node_base) {
  top_sah(ids, blo, bhi, 0, (int)ids.size(), nlo, nhi, node_base);
}

// The device tree (nodes 0..n-1 leaves in curve order, n..2n-2 inner, root 2n-2)
// -> HostScene's refs, prim_bounds, BVH2 export nodes and BVH4 (host_bvh.cpp layout:
// BFS order, leaves shared, BVH4 by expanding the largest-area inner child).
static int finalize_tree(HostScene& s, const std::vector<F4>& nlo, const std::vector<F4>& nhi,
                         const std::vector<uint32_t>& order, const std::vector<F4>& lo,
                         const std::vector<F4>& hi, const std::vector<uint32_t>& prims) {
  const int n = (int)order.size();
  const int root = n == 1 ? 0 : 2 * n - 2;
  auto left = [&](int v) { int c; memcpy(&c, &nlo[v].w, 4); return c; };
  auto right = [&](int v) { int c; memcpy(&c, &nhi[v].w, 4); return c; };
  auto is_inner = [&](int v) { return v >= n; };
  auto bits = [](uint32_t u) { float f; memcpy(&f, &u, 4); return f; };
  s.refs.resize(n);
  s.prim_bounds.resize(6 * (size_t)n);
  for (int k = 0; k < n; ++k) {
    const uint32_t p = order[k];
    s.refs[k] = prims[p];
    const float b[6] = {lo[p].x, lo[p].y, lo[p].z, hi[p].x, hi[p].y, hi[p].z};
    memcpy(&s.prim_bounds[6 * (size_t)k], b, sizeof b);
  }
  s.max_leaf = 1;
  if (n == 1) {
    s.root = s.root4 = leaf_code(0, 1);
    s.nodes.clear();
    s.nodes4.clear();
    s.bvh_depth = 0;
    return RT_OK;
  }
  auto code_of = [&](int v, const std::vector<int>& idx) -> uint32_t {
    return is_inner(v) ? (uint32_t)idx[v - n] : leaf_code((uint32_t)v, 1u);
  };
  // BVH2: BFS over inner nodes (vector queue), depth per level
  std::vector<int> bfs;
  bfs.reserve(n - 1);
  std::vector<int> idx2(n - 1, -1);
  bfs.push_back(root);
  int depth = 0;
  for (size_t head = 0, level_end = 1; head < bfs.size(); ++head) {
    if (head == level_end) {
      ++depth;
      level_end = bfs.size();
    }
    const int v = bfs[head];
    idx2[v - n] = (int)head;
    for (int c : {left(v), right(v)})
      if (is_inner(c)) bfs.push_back(c);
  }
  s.bvh_depth = depth + 1;
  s.nodes.assign(4 * bfs.size(), F4{0, 0, 0, 0});
  for (size_t o = 0; o < bfs.size(); ++o) {
    const int v = bfs[o], a = left(v), b = right(v);
    s.nodes[4 * o + 0] = {nlo[a].x, nlo[a].y, nlo[a].z, bits(code_of(a, idx2))};
    s.nodes[4 * o + 1] = {nhi[a].x, nhi[a].y, nhi[a].z, bits(code_of(b, idx2))};
    s.nodes[4 * o + 2] = {nlo[b].x, nlo[b].y, nlo[b].z, 0};
    s.nodes[4 * o + 3] = {nhi[b].x, nhi[b].y, nhi[b].z, 0};
  }
  s.root = 0;
  // BVH4: expand the largest-area inner child until four children (BFS order)
  std::vector<int> q4;
  q4.reserve(n / 2 + 1);
  std::vector<int> idx4(n - 1, -1);
  std::vector<std::array<int, 4>> kids;
  kids.reserve(n / 2 + 1);
  q4.push_back(root);
  for (size_t head = 0; head < q4.size(); ++head) {
    const int v = q4[head];
    idx4[v - n] = (int)head;
    std::array<int, 4> ch = {left(v), right(v), -1, -1};
    int nc = 2;
    while (nc < 4) {
      int best = -1;
      double best_area = -1;
      for (int k = 0; k < nc; ++k)
        if (is_inner(ch[k])) {
          const double a = area_of(nlo[ch[k]], nhi[ch[k]]);
          if (a > best_area) {
            best_area = a;
            best = k;
          }
        }
      if (best < 0) break;
      const int c = ch[best];
      ch[best] = left(c);
      ch[nc++] = right(c);
    }
    for (int k = 0; k < nc; ++k)
      if (is_inner(ch[k])) q4.push_back(ch[k]);
    kids.push_back(ch);
  }
  s.nodes4.assign(8 * q4.size(), F4{0, 0, 0, 0});
  for (size_t o = 0; o < q4.size(); ++o) {
    float* lx = &s.nodes4[8 * o].x;  // [field][child]
    for (int k = 0; k < 4; ++k) {
      const int c = kids[o][k];
      uint32_t code = CHILD_EMPTY;
      // an empty slot's box is inverted and infinite (lo = +inf, hi = -inf): the
      // sign-selected slab test (rt_path.h trav_steps) never hits it
      float b[6] = {INFINITY, -INFINITY, INFINITY, -INFINITY, INFINITY, -INFINITY};
      if (c >= 0) {
        code = code_of(c, idx4);
        const float t[6] = {nlo[c].x, nhi[c].x, nlo[c].y, nhi[c].y, nlo[c].z, nhi[c].z};
        memcpy(b, t, sizeof t);
      }
      for (int f = 0; f < 6; ++f) lx[(1 + f) * 4 + k] = b[f];  // rt_device.h "BVH4 node"
      lx[k] = bits(code);
    }
  }
  s.root4 = 0;
  return RT_OK;
}

bool bvh_device_available() {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess && n > 0;
}

int build_bvh_device(HostScene& s, const std::vector<F4>& lo, const std::vector<F4>& hi,
                     const std::vector<uint32_t>& prims, int device) {
  const int n = (int)prims.size();
  if (n < 2) return set_error(RT_ERR_INVALID, "build_bvh_device: needs 2+ prims");
  if ((uint32_t)n > 0x7FFFFFFu) return set_error(RT_ERR_UNSUPPORTED, "too many prims (%d)", n);
  const bool timing = tune_int("RT_TIMING", 0) != 0;
  auto t0 = std::chrono::steady_clock::now();
  // device < 0: the calling thread's current device (one process per GPU builds on its
  // own GPU); the caller's current device is restored on return
  int prev = 0;
  B_OK(hipGetDevice(&prev));
  if (device < 0) device = prev;
  struct DeviceGuard {
    int d;
    ~DeviceGuard() { (void)hipSetDevice(d); }
  } dg{prev};
  B_OK(hipSetDevice(device));
  hipStream_t st;
  B_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  struct StreamGuard {
    hipStream_t s;
    ~StreamGuard() { (void)hipStreamDestroy(s); }
  } sg{st};
  DevBuf B;
  float4 *dlo, *dhi, *part, *nlo, *nhi, *clo[2], *chi[2];
  uint64_t *key, *key2;
  uint32_t *val, *val2;
  int *cl[2], *nn, *create, *valid, *sc, *sv, *counts;
  const int nodes = 2 * n - 1;
  const int nb = (n + kBlock - 1) / kBlock, nparts = std::min(nb, 1024);
  int rc;
  if ((rc = B.alloc(&dlo, n)) || (rc = B.alloc(&dhi, n)) || (rc = B.alloc(&part, 2 * nparts)) ||
      (rc = B.alloc(&nlo, nodes)) || (rc = B.alloc(&nhi, nodes)) || (rc = B.alloc(&clo[0], n)) ||
      (rc = B.alloc(&chi[0], n)) || (rc = B.alloc(&clo[1], n)) || (rc = B.alloc(&chi[1], n)) ||
      (rc = B.alloc(&key, n)) || (rc = B.alloc(&key2, n)) || (rc = B.alloc(&val, n)) ||
      (rc = B.alloc(&val2, n)) || (rc = B.alloc(&cl[0], n)) || (rc = B.alloc(&cl[1], n)) ||
      (rc = B.alloc(&nn, n)) || (rc = B.alloc(&create, n)) || (rc = B.alloc(&valid, n)) ||
      (rc = B.alloc(&sc, n)) || (rc = B.alloc(&sv, n)) || (rc = B.alloc(&counts, 2)))
    return rc;
  static_assert(sizeof(F4) == sizeof(float4), "F4 layout");
  B_OK(hipMemcpyAsync(dlo, lo.data(), n * sizeof(float4), hipMemcpyHostToDevice, st));
  B_OK(hipMemcpyAsync(dhi, hi.data(), n * sizeof(float4), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_bounds, dim3(nparts), dim3(kBlock), 0, st, dlo, dhi, n, part);
  hipLaunchKernelGGL(k_morton, dim3(nb), dim3(kBlock), 0, st, dlo, dhi, n, part, nparts, key, val);
  B_OK(hipGetLastError());
  // stable radix sort of (code, index) pairs
  size_t tmp_sort = 0, tmp_scan = 0;
  B_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_sort, key, key2, val, val2, n, 0, 63, st));
  B_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_scan, create, sc, n, st));
  void* tmp = nullptr;
  {
    char* t8;
    if ((rc = B.alloc(&t8, std::max(tmp_sort, tmp_scan)))) return rc;
    tmp = t8;
  }
  size_t tb = tmp_sort;
  B_OK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, key, key2, val, val2, n, 0, 63, st));
  hipLaunchKernelGGL(k_leaves, dim3(nb), dim3(kBlock), 0, st, dlo, dhi, n, val2, nlo, nhi, cl[0],
                     clo[0], chi[0]);
  B_OK(hipGetLastError());
  // PLOC iterations down to `top` clusters; the top of the tree is then built on
  // the host by a full SAH sweep over those clusters (PLOC's radius-limited merges
  // are weakest where few large clusters remain)
  const int top = std::max(1, tune_int("RT_BVH_TOP", PLOC_TOP));
  int m = n, node_base = n, cur = 0, iters = 0, force = 0;
  while (m > top) {
    if (++iters > 4 * 64 + n) return set_error(RT_ERR_DEVICE, "bvh build: no progress");
    const int g = (m + kBlock - 1) / kBlock;
    if (!force) hipLaunchKernelGGL(k_nn, dim3(g), dim3(kBlock), 0, st, clo[cur], chi[cur], m, nn);
    hipLaunchKernelGGL(k_flags, dim3(g), dim3(kBlock), 0, st, nn, m, force, create, valid);
    tb = tmp_scan;
    B_OK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, create, sc, m, st));
    tb = tmp_scan;
    B_OK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, valid, sv, m, st));
    hipLaunchKernelGGL(k_emit, dim3(g), dim3(kBlock), 0, st, nn, m, force, create, valid, sc, sv,
                       node_base, cl[cur], clo[cur], chi[cur], nlo, nhi, cl[cur ^ 1], clo[cur ^ 1],
                       chi[cur ^ 1], counts);
    B_OK(hipGetLastError());
    int hc[2];
    B_OK(hipMemcpyAsync(hc, counts, sizeof hc, hipMemcpyDeviceToHost, st));
    B_OK(hipStreamSynchronize(st));
    force = hc[1] == 0;  // no mutual pair: pair neighbours next time (guaranteed progress)
    node_base += hc[1];
    m = hc[0];
    cur ^= 1;
  }
  std::vector<F4> hlo(nodes), hhi(nodes);
  std::vector<uint32_t> order(n);
  std::vector<int> top_ids(m);
  std::vector<F4> top_lo(m), top_hi(m);
  B_OK(hipMemcpyAsync(hlo.data(), nlo, node_base * sizeof(F4), hipMemcpyDeviceToHost, st));
  B_OK(hipMemcpyAsync(hhi.data(), nhi, node_base * sizeof(F4), hipMemcpyDeviceToHost, st));
  B_OK(hipMemcpyAsync(order.data(), val2, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  B_OK(hipMemcpyAsync(top_ids.data(), cl[cur], m * sizeof(int), hipMemcpyDeviceToHost, st));
  B_OK(hipMemcpyAsync(top_lo.data(), clo[cur], m * sizeof(F4), hipMemcpyDeviceToHost, st));
  B_OK(hipMemcpyAsync(top_hi.data(), chi[cur], m * sizeof(F4), hipMemcpyDeviceToHost, st));
  B_OK(hipStreamSynchronize(st));
  if (m > 1) build_top_sah(top_ids, top_lo, top_hi, hlo, hhi, node_base);
  if (node_base != nodes) return set_error(RT_ERR_DEVICE, "bvh build: %d of %d nodes", node_base, nodes);
  auto t1 = std::chrono::steady_clock::now();
  rc = finalize_tree(s, hlo, hhi, order, lo, hi, prims);
  if (timing)
    fprintf(stderr, "[rt]   bvh device (PLOC r=%d, %d iterations, top %d by SAH) %.3f s, layout %.3f s\n", kR, iters, top,
            std::chrono::duration<double>(t1 - t0).count(),
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count());
  return rc;
}

}  // namespace rt
