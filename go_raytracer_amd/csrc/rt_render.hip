// rt_render.hip — MI355X kernels and host orchestration of one render.
//
// Replaces the reference's per-pixel loop (camera.go:90-153) and recursive
// estimator rayColor (camera.go:293-331).  Two execution strategies run the
// same per-vertex code (rt_path.h):
//
//  WAVEFRONT — a queue-driven loop of
//   k_extend : closest hit for every queued ray (BVH top staged in LDS, static
//              work split, no atomics) -> SoA hit records
//   k_shade  : one rayColor vertex per queued path; paths that finish a sample
//              regenerate a camera ray in place; survivors are compacted into
//              the next queue by wave ballot + prefix with one atomic per
//              workgroup on a per-XCD counter
//  FUSED — k_fused: persistent threads, one path per lane kept in registers,
//          trace + shade in a loop, finished lanes refilled from a wave-batched
//          chunk counter (ballot + one atomic per >=64 chunks).
// Both end with k_resolve (fixed-point pixel sums -> linear mean RGB).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "rt_internal.h"
#include "rt_path.h"
#include "rt_fused.h"

namespace rt {

// ------------------------------------------------------------- wavefront ---
// The queue of iteration `it` is kXcd segments; segment x holds cnt[it][x]
// slots at queue[sel][x*P ...].
RT_D uint32_t queue_slot(const Params& P, const uint32_t* q, const uint32_t* cnt, uint32_t i) {
  uint32_t x = 0;
  while (x + 1 < (uint32_t)kXcd && i >= cnt[x]) {
    i -= cnt[x];
    ++x;
  }
  return q[(size_t)x * P.P + i];
}

template <bool LDS>
__global__ __launch_bounds__(256) void k_extend(Params P, int it) {
  __shared__ F4 lnodes[LDS ? 4 * kLdsNodes : 4];
  __shared__ uint32_t lstack[kShortStack * 256];
  const bool recs_lds = LDS && stage_nodes(P, lnodes, 8);
  const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
  const TravStack ts = {&lstack[threadIdx.x], P.ostack + gtid, P.stack_cols, kShortStack};
  const uint32_t sel = (uint32_t)it & 1u;
  uint32_t cnt[kXcd];
  uint32_t n = 0;
  for (int x = 0; x < kXcd; ++x) {
    cnt[x] = P.ctr->cnt[it % kMaxIt][x];
    n += cnt[x];
  }
  const uint32_t* q = P.queue[sel];
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t slot = queue_slot(P, q, cnt, i);
    Path s;
    load_path(P, slot, s);
    Hit best;
    trace_world<LDS, FT_ALL>(P.sc, lnodes, recs_lds, ts, s.o, s.d, s.time, 0.001f, best);
    finish_hit<FT_ALL>(P, s, best);
    P.hit[slot] = {best.t, best.u, best.v, bitsf(best.ref)};
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&P.ctr->segments, (unsigned long long)n);
}

__global__ __launch_bounds__(256) void k_shade(Params P, int it) {
  __shared__ uint32_t wave_cnt[4], wave_base[4], block_base;
  stage_perlin(P.sc);
  __syncthreads();
  const uint32_t sel = (uint32_t)it & 1u;
  uint32_t cnt[kXcd];
  uint32_t n = 0;
  for (int x = 0; x < kXcd; ++x) {
    cnt[x] = P.ctr->cnt[it % kMaxIt][x];
    n += cnt[x];
  }
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = i < n;
  const uint32_t slot = active ? queue_slot(P, P.queue[sel], cnt, i) : 0u;
  bool alive = false;
  if (active) {
    Path s;
    load_path(P, slot, s);
    const F4 hv = P.hit[slot];
    const Hit h = {hv.x, hv.y, hv.z, fbits(hv.w)};
    const WStack ws = {nullptr, 0};  // the weight stack outlives the launch: HBM only
    const SampleAcc sa = {nullptr};  // every sample straight to its pixel
    int out = shade_core<true, FT_ALL>(P, slot, s, h, ws, sa);
    if (out == OUT_NEED_CHUNK) {
      // static work split: slot s renders chunks s, s+P, s+2P, ... (no atomics)
      const uint32_t c = s.chunk + P.P;
      if (c < P.n_chunks) {
        start_sample<true>(P, slot, s, c, 0);
        out = OUT_ALIVE;
      }
    }
    alive = out == OUT_ALIVE;
  }
  // compaction: wave ballot + prefix, block-level sum, one atomic per block
  const unsigned long long am = __ballot(alive);
  const uint32_t w = threadIdx.x >> 6, lane = lane_id();
  if (lane == 0) wave_cnt[w] = (uint32_t)__popcll(am);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (int k = 0; k < 4; ++k) {
      wave_base[k] = tot;
      tot += wave_cnt[k];
    }
    const uint32_t x = blockIdx.x % kXcd;
    block_base = tot ? atomicAdd(&P.ctr->cnt[(it + 1) % kMaxIt][x], tot) : 0u;
  }
  __syncthreads();
  if (alive) {
    const uint32_t x = blockIdx.x % kXcd;
    P.queue[sel ^ 1u][(size_t)x * P.P + block_base + wave_base[w] + prefix_count(am)] = slot;
  }
}

__global__ __launch_bounds__(256) void k_init(Params P) {
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= P.P) return;
  if (slot < P.n_chunks) {
    Path s;
    start_sample<true>(P, slot, s, slot, 0);
    P.queue[0][slot] = slot;  // segment 0 holds the whole first queue
  }
  if (slot == 0) {
    P.ctr->cnt[0][0] = min(P.P, P.n_chunks);
    P.ctr->chunk_head = P.P;
  }
}

// fixed-point sums -> linear mean RGB; Scale(pixelSamplesScale) camera.go:103
__global__ __launch_bounds__(256) void k_resolve(Params P, float* out, double scale) {
  const uint32_t lp = blockIdx.x * blockDim.x + threadIdx.x;
  if (lp >= P.npix) return;
  const uint32_t f = P.pflags[lp];
  // the fused kernel's per-chunk sums (SampleAcc::flush): this pixel's chunks are
  // q * gchunks + sub * gpix + r for its group q, its place r in the group and every
  // sample block sub (chunk_pixel), summed mod 2^64 like the atomics they replace
  unsigned long long cs[3] = {0ull, 0ull, 0ull};
  if (P.csum) {
    const uint32_t gpix = P.fd_gpix.d, g = fdiv(lp, P.fd_gpix), r = lp - g * gpix;
#ifdef RT_SWEEP_ORDER
    const uint32_t q = (g ^ P.gflip) + P.gbase;  // the group's sweep position (an involution)
#else
    const uint32_t q = g;
#endif
    for (int ph = 0; ph < 2; ++ph) {  // the first phase's chunks, then the tail's (if any)
      const uint32_t gch = ph ? P.fd_gchunks2.d : P.fd_gchunks.d;
      const uint32_t cpp = ph && P.S1 >= P.ss ? 0u : gch / gpix;
      const unsigned long long* rec = P.csum + 4 * ((ph ? (size_t)P.n1 : 0) + (size_t)q * gch + r);
      // unrolled: eight records' loads in flight per thread before the adds wait (one at a
      // time, the 655 MB of C2's records were read at ~3.5 TB/s)
#pragma unroll 8
      for (uint32_t sb = 0; sb < cpp; ++sb, rec += 4 * (size_t)gpix) {
        cs[0] += rec[0];
        cs[1] += rec[1];
        cs[2] += rec[2];
      }
    }
  }
  for (int ch = 0; ch < 3; ++ch) {
    const bool nan = (f & (1u << ch)) != 0, pinf = (f & (8u << ch)) != 0,
               ninf = (f & (64u << ch)) != 0;
    float v;
    if (nan || (pinf && ninf)) {  // Inf + -Inf = NaN, as in the fp64 sum
      v = __builtin_nanf("");
    } else if (pinf || ninf) {
      v = pinf ? kInf : -kInf;
    } else {
      const size_t i = (size_t)ch * P.npix + lp;
      const long long sum = (long long)(P.accum[i] + cs[ch]);
      v = (float)(((double)sum * 2.3283064365386963e-10 + P.side[i]) * scale);
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
  DevScene d{};                 // nodes = BVH4
  const F4* nodes2 = nullptr;   // BVH2 of the same leaves (tiny scenes)
  const F4* brute_pairs = nullptr;  // quad records in pairs, largest first (record loop)
  size_t brute_slots = 0;           // records in brute_pairs, pads included (even)
  int32_t shade_n = 0;              // F4s of the lean shade table after the pairs (0: none)
  int32_t brute_boxes = 0;          // boxes among them tested as slabs (rt_path.h brute_box)
  uint32_t root2 = PRIM_NONE;
  int32_t n_nodes2 = 0;
  const F4* qnodes = nullptr;       // compressed BVH4 (host_qbvh.cpp): 64-B items, root item 0
  size_t qitems = 0;
  std::mutex qmu;                   // ensure_qbvh: the first render that needs it uploads it
  bool q_done = false;
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
     *stack = nullptr;
  uint2* path = nullptr;
  uint32_t* queue[2] = {nullptr, nullptr};
  Counters* ctr = nullptr;
  unsigned long long* accum = nullptr;
  unsigned long long* csum = nullptr;  // fused: per-chunk sums (4 x u64 per chunk)
  size_t csum_chunks = 0;
  double* side = nullptr;
  uint32_t* pflags = nullptr;
  uint32_t* ostack = nullptr;
  uint32_t ostack_cols = 0;
  float* out = nullptr;
  uint32_t out_cap = 0;
  std::vector<hipEvent_t> events;
  std::vector<hipEvent_t> prog_events;  // one per progress slice (rt_progress)
  int resident_blocks = 0;
  void free_all() {
    for (void* p : allocs) (void)hipFree(p);
    allocs.clear();
  }
  ~RenderState() {
    free_all();
    for (auto e : events) (void)hipEventDestroy(e);
    for (auto e : prog_events) (void)hipEventDestroy(e);
    if (own_stream) (void)hipStreamDestroy(own_stream);
  }
};

// Restores the calling thread's current device on scope exit: every ABI entry that
// switches devices leaves the caller's (e.g. torch's) current device as it found it.
struct DeviceGuard {
  int prev = -1;
  DeviceGuard() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// rt_render_multi's RCCL gather (RT_FLAG_GATHER_RCCL): one communicator per device of
// the list (ncclCommInitAll), a stream and a padded send buffer per share, kept while
// the device list and the share size stay the same
struct RcclGather {
  std::vector<int> devs;
  std::vector<ncclComm_t> comms;
  std::vector<hipStream_t> streams;
  std::vector<float*> send;
  size_t send_floats = 0;
  void release() {
    for (size_t i = 0; i < comms.size(); ++i) {
      (void)hipSetDevice(devs[i]);
      if (send.size() > i && send[i]) (void)hipFree(send[i]);
      if (streams.size() > i && streams[i]) (void)hipStreamDestroy(streams[i]);
      (void)ncclCommDestroy(comms[i]);
    }
    devs.clear();
    comms.clear();
    streams.clear();
    send.clear();
    send_floats = 0;
  }
};

void release_device(Scene* s) {
  DeviceGuard dg;
  if (s->rccl) {
    static_cast<RcclGather*>(s->rccl)->release();
    delete static_cast<RcclGather*>(s->rccl);
    s->rccl = nullptr;
  }
  std::lock_guard<std::mutex> lk(s->mu);
  for (auto& kv : s->slots) {
    if (kv.second->st) {
      (void)hipSetDevice(kv.first.first);
      delete kv.second->st;
    }
    delete kv.second;
  }
  s->slots.clear();
  for (auto& kv : s->devs) {
    if (kv.second->ds) {
      (void)hipSetDevice(kv.first);
      delete kv.second->ds;
    }
    delete kv.second;
  }
  s->devs.clear();
  if (s->multi_buf) {
    (void)hipSetDevice(s->multi_dev);
    (void)hipFree(s->multi_buf);
    s->multi_buf = nullptr;
  }
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

// scheduling knobs of the fused kernel (A/B experiments; defaults measured): rt_tune_set
// only, never the process environment (host_tune.cpp)
static int env_int(const char* name, int dflt) { return tune_int(name, dflt); }


static FastDiv make_fastdiv(uint32_t d) {
  FastDiv f{1u, 0u, 0u, d};
  if (d <= 1) return f;  // d == 1: t = 0, q = n
  const uint32_t l = 32u - (uint32_t)__builtin_clz(d - 1u);
  f.m = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d + 1u);
  f.s1 = 1u;
  f.s2 = l - 1u;
  return f;
}

// the traversal's leaf records (rt_device.h "leaf records"), in refs order
static void make_record(const HostScene& h, uint32_t ref, F4* r);
static void build_leaf_records(const HostScene& h, std::vector<F4>& recs) {
  recs.assign(4 * h.refs.size(), F4{0, 0, 0, 0});
  for (size_t i = 0; i < h.refs.size(); ++i) make_record(h, h.refs[i], &recs[4 * i]);
}
// light table entries: quad lights as leaf records with the area in [2].w (prim_pdf)
static void build_light_records(const HostScene& h, std::vector<F4>& recs) {
  recs.assign(8 * std::max<size_t>(h.lights.size(), 1), F4{0, 0, 0, 0});
  for (size_t i = 0; i < h.lights.size(); ++i) {
    const uint32_t ref = h.lights[i].ref;
    if (ref == PRIM_NONE || (ref >> 30) != PRIM_QUAD) continue;
    make_record(h, ref, &recs[8 * i]);
    const F4* q = &h.quad[5 * (size_t)(ref & 0x3FFFFFFFu)];  // Q|D, u|area, v|mat, n, w
    recs[8 * i + 2].w = q[1].w;                                // area
    recs[8 * i + 4] = q[0];
    recs[8 * i + 5] = q[1];
    recs[8 * i + 6] = q[2];
  }
}
static void make_record(const HostScene& h, uint32_t ref, F4* r) {
  {
    const uint32_t type = ref >> 30, idx = ref & 0x3FFFFFFFu;
    float rb;
    memcpy(&rb, &ref, 4);
    if (type == PRIM_SPHERE) {
      const F4 cr = h.sph_cr[idx], mv = h.sph_mv[idx];
      r[0] = {cr.x, cr.y, cr.z, rb};
      r[1] = {mv.x, mv.y, mv.z, cr.w};
    } else if (type == PRIM_BOX) {  // box leaf (rt_device.h), built by the flattener
      for (int k = 0; k < 4; ++k) r[k] = h.box_recs[4 * (size_t)idx + k];
      r[0].w = rb;
    } else if (type == PRIM_QUAD) {
      const F4* q = &h.quad[5 * (size_t)idx];  // Q|D, u|area, v|mat, n, w
      const double u[3] = {q[1].x, q[1].y, q[1].z}, v[3] = {q[2].x, q[2].y, q[2].z},
                   w[3] = {q[4].x, q[4].y, q[4].z};
      auto cr = [](const double* a, const double* b, int k) {
        return k == 0 ? a[1] * b[2] - a[2] * b[1] : k == 1 ? a[2] * b[0] - a[0] * b[2]
                                                           : a[0] * b[1] - a[1] * b[0];
      };
      r[0] = {q[0].x, q[0].y, q[0].z, rb};
      r[1] = {q[3].x, q[3].y, q[3].z, q[0].w};
      r[2] = {(float)cr(v, w, 0), (float)cr(v, w, 1), (float)cr(v, w, 2), 0.0f};
      r[3] = {(float)cr(w, u, 0), (float)cr(w, u, 1), (float)cr(w, u, 2), 0.0f};
    } else {
      const F4* t = &h.tri[3 * (size_t)idx];  // v0|mat, e0|area, e1|flags
      r[0] = {t[0].x, t[0].y, t[0].z, rb};
      r[1] = {t[1].x, t[1].y, t[1].z, 0.0f};
      r[2] = {t[2].x, t[2].y, t[2].z, 0.0f};
    }
  }
}

// the scene's device copy on `device` (uploaded on first use, then shared by every
// slot on that device; read-only while rendering).  The scene-wide lock covers the
// map lookup only; the upload holds its device's own lock, so first renders on
// different devices upload concurrently.  Called with `device` current.
static int upload_scene(const Scene* s, DeviceScene* ds);
static int ensure_scene(Scene* s, int device, DeviceScene** out) {
  DeviceSlot* slot;
  {
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceSlot*& sl = s->devs[device];
    if (!sl) sl = new DeviceSlot();
    slot = sl;
  }
  std::lock_guard<std::mutex> up(slot->mu);
  if (slot->ds) {
    *out = slot->ds;
    return RT_OK;
  }
  DeviceScene* ds = new DeviceScene();
  ds->device = device;
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = upload_scene(s, ds);
  if (tune_int("RT_TIMING", 0))
    fprintf(stderr, "[rt] scene upload to device %d %.3f s\n", device,
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  if (rc != RT_OK) {
    delete ds;
    return rc;
  }
  slot->ds = ds;
  *out = ds;
  return RT_OK;
}
static int upload_scene(const Scene* s, DeviceScene* ds) {
  const HostScene& h = s->h;
  DevScene& d = ds->d;
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
  if ((rc = upload(ds, vec, &d.field)) != RT_OK) return rc;
  UP(h.sph_cr, sph_cr);
  UP(h.sph_mv, sph_mv);
  UP(h.sph_uv, sph_uv);
  UP(h.quad, quad);
  UP(h.tri, tri);
  UP(h.tri_attr, tri_attr);
  // the BVH4 nodes and the leaf records in ONE allocation (nodes first): the traversal
  // addresses both as 32-bit byte offsets from the node base (rt_path.h trav_steps)
  std::vector<F4> recs;
  build_leaf_records(h, recs);
  {
    std::vector<F4> tree_buf(h.nodes4);
    tree_buf.resize((tree_buf.size() + 15) / 16 * 16, F4{0, 0, 0, 0});  // records 256-B aligned
    const size_t rec0 = tree_buf.size();
    if ((rec0 + recs.size()) * sizeof(F4) >= ((size_t)1 << 32))
      return set_error(RT_ERR_UNSUPPORTED, "scene: BVH nodes + leaf records exceed 4 GiB");
    tree_buf.insert(tree_buf.end(), recs.begin(), recs.end());
    const F4* base = nullptr;
    if ((rc = upload(ds, tree_buf, &base)) != RT_OK) return rc;
    d.nodes = base;
    d.leafprims = base ? base + rec0 : nullptr;
  }
  // (the compressed BVH4 is built and uploaded on demand: ensure_qbvh)
  // the BVH2 and the record-loop pairs serve tiny scenes only (render_impl's tree
  // choice: <= 64 leaf entries); a 1M-triangle scene would upload 64 MB of BVH2
  const size_t tiny = (size_t)std::max(64, env_int("RT_BRUTE_MAX", kBruteMax));
  const bool small = h.refs.size() <= tiny;
  if (small && (rc = upload(ds, h.nodes, &ds->nodes2)) != RT_OK) return rc;
  ds->root2 = h.root;
  ds->n_nodes2 = small ? (int32_t)(h.nodes.size() / 4) : 0;
  UP(h.refs, refs);
  {
    std::vector<F4> lrecs;
    if (!h.refs8.empty()) {  // the BVH8's records, in its node order
      std::vector<F4> r8(4 * h.refs8.size());
      for (size_t i = 0; i < h.refs8.size(); ++i) make_record(h, h.refs8[i], &r8[4 * i]);
      UP(r8, recs8);
      UP(h.nodes8, nodes8);
    }
    build_light_records(h, lrecs);
    UP(lrecs, light_recs);
    if (!small) goto records_done;
    // record-loop order: largest surface first, so the closest hit tends to be found
    // early and later records fail the interval test before their slower half
    std::vector<size_t> ord(h.refs.size());
    for (size_t i = 0; i < ord.size(); ++i) ord[i] = i;
    auto area = [&](uint32_t ref) -> double {
      const uint32_t type = ref >> 30, idx = ref & 0x3FFFFFFFu;
      if (type == PRIM_QUAD) return h.quad[5 * (size_t)idx + 1].w;
      if (type == PRIM_TRI) return h.tri[3 * (size_t)idx + 1].w;
      const double r = h.sph_cr[idx].w;
      return 4.0 * 3.141592653589793 * r * r;
    };
    std::stable_sort(ord.begin(), ord.end(),
                     [&](size_t a, size_t b) { return area(h.refs[a]) > area(h.refs[b]); });
    // Axis-aligned quads (unit normal +-e_a, A_a = B_a = 0 exactly: Cornell's walls,
    // floor, ceiling and box tops) go in per-axis pair groups after the general
    // pairs; the loop tests them with the in-plane terms only, bit-identical to the
    // general test (rt_path.h brute_axis).  An odd record of a group joins the
    // general list.  RT_BRUTE_AXIS=0 keeps every record general (A/B).
    const bool use_axis = env_int("RT_BRUTE_AXIS", 1) != 0;
    auto axis_of = [&](size_t i) -> int {
      const F4* r = &recs[4 * i];
      if (!use_axis || (h.refs[i] >> 30) != PRIM_QUAD) return -1;
      const float n[3] = {r[1].x, r[1].y, r[1].z}, A[3] = {r[2].x, r[2].y, r[2].z},
                  B[3] = {r[3].x, r[3].y, r[3].z};
      for (int a = 0; a < 3; ++a) {
        const int b = (a + 1) % 3, c = (a + 2) % 3;
        if ((n[a] == 1.0f || n[a] == -1.0f) && n[b] == 0.0f && n[c] == 0.0f && A[a] == 0.0f &&
            B[a] == 0.0f)
          return a;
      }
      return -1;
    };
    // y-parallel quads (n_y = A_y = 0 and B = (0, B_y, 0) exactly: the sides of Cornell's
    // boxes rotated about y) go in a pair group between the general and the axis-aligned
    // ones (rt_path.h brute_vert: the general test without its exact-zero terms, images
    // bit-identical; C2 -1.6 % against RT_BRUTE_VERT=0, which keeps them general).
    const bool use_vert = env_int("RT_BRUTE_VERT", 1) != 0;
    auto vert_of = [&](size_t i) -> int {
      const F4* r = &recs[4 * i];
      if (!use_vert || (h.refs[i] >> 30) != PRIM_QUAD || axis_of(i) >= 0) return -1;
      const float n[3] = {r[1].x, r[1].y, r[1].z}, A[3] = {r[2].x, r[2].y, r[2].z},
                  B[3] = {r[3].x, r[3].y, r[3].z};
      // y only (brute_vert<1>): RotateY is the reference's only rotation
      return n[1] == 0.0f && A[1] == 0.0f && B[0] == 0.0f && B[2] == 0.0f && B[1] != 0.0f ? 1 : -1;
    };
    // Boxes rotated about y (NewBox objects.go:208-240 under RotateY / Translate,
    // transformation.go:13-110; Cornell's two boxes): six quad records whose corners are
    // the eight corners of one box with a horizontal top and bottom.  The loop tests each
    // such box once, as three slabs in the box's own frame -- the reference's rotateY.Hit
    // frame, where each face's quad test is t = (k - o'_a) / d'_a -- instead of its six
    // records (rt_path.h brute_box).  The face records stay in the array (after the box
    // descriptors) for the winner's u, v and ref.  RT_BRUTE_BOX=0 keeps them in the groups.
    struct BoxRec { size_t face[6]; double C[3], ax[3], az[3], H; };
    std::vector<BoxRec> boxes;
    std::vector<char> in_box(h.refs.size(), 0);
    if (env_int("RT_BRUTE_BOX", 1) != 0) {
      auto qd = [&](size_t i, int k, double* out) {  // k: 0 Q, 1 u, 2 v
        const F4& f = h.quad[5 * (size_t)(h.refs[i] & 0x3FFFFFFFu) + k];
        out[0] = f.x, out[1] = f.y, out[2] = f.z;
      };
      auto corners = [&](size_t i, double P[4][3]) {
        double Q[3], u[3], v[3];
        qd(i, 0, Q), qd(i, 1, u), qd(i, 2, v);
        for (int c = 0; c < 3; ++c) {
          P[0][c] = Q[c], P[1][c] = Q[c] + u[c], P[2][c] = Q[c] + v[c];
          P[3][c] = Q[c] + u[c] + v[c];
        }
      };
      std::vector<size_t> quads;
      for (size_t i : ord)
        if ((h.refs[i] >> 30) == PRIM_QUAD) quads.push_back(i);
      // four corners of quad i == the four points F (as sets, within tol)
      auto same_face = [&](size_t i, const double F[4][3], double tol) {
        double P[4][3];
        corners(i, P);
        bool used[4] = {false, false, false, false};
        for (int a = 0; a < 4; ++a) {
          int m = -1;
          for (int b = 0; b < 4 && m < 0; ++b)
            if (!used[b] && fabs(P[a][0] - F[b][0]) <= tol && fabs(P[a][1] - F[b][1]) <= tol &&
                fabs(P[a][2] - F[b][2]) <= tol)
              m = b;
          if (m < 0) return false;
          used[m] = true;
        }
        return true;
      };
      for (size_t i : quads) {
        if (in_box[i]) continue;
        double C[3], ax[3], az[3];
        qd(i, 0, C), qd(i, 1, ax), qd(i, 2, az);
        const double la = sqrt(ax[0] * ax[0] + ax[2] * ax[2]), lb = sqrt(az[0] * az[0] + az[2] * az[2]);
        // a horizontal rectangle: the bottom (or top) face of a candidate box
        if (ax[1] != 0.0 || az[1] != 0.0 || la == 0.0 || lb == 0.0 ||
            fabs(ax[0] * az[0] + ax[2] * az[2]) > 1e-6 * la * lb)
          continue;
        const double tol = 1e-5 * (1.0 + fabs(C[0]) + fabs(C[1]) + fabs(C[2]) + la + lb);
        auto corner = [&](int k, double H, double* out) {  // bit 0: +ax, 1: +az, 2: +H
          for (int c = 0; c < 3; ++c)
            out[c] = C[c] + ((k & 1) ? ax[c] : 0.0) + ((k & 2) ? az[c] : 0.0) + (c == 1 && (k & 4) ? H : 0.0);
        };
        // faces by (axis, side): x' = bit 0, y = bit 2, z' = bit 1
        const int fbit[3] = {1, 4, 2};
        for (size_t j : quads) {
          if (j == i || in_box[j]) continue;
          double Qj[3];
          qd(j, 0, Qj);
          const double H = Qj[1] - C[1];
          if (fabs(H) <= tol) continue;
          BoxRec b{};
          bool ok = true;
          for (int f = 0; f < 6 && ok; ++f) {
            double F[4][3];
            int n = 0;
            for (int k = 0; k < 8; ++k)
              if (((k & fbit[f >> 1]) != 0) == (f & 1)) corner(k, H, F[n++]);
            size_t hit = (size_t)-1;
            if (f == 2) hit = i;
            else if (f == 3) hit = same_face(j, F, tol) ? j : (size_t)-1;
            else
              for (size_t m : quads)
                if (m != i && m != j && !in_box[m] && same_face(m, F, tol)) {
                  bool dup = false;
                  for (int g = 0; g < f; ++g) dup |= b.face[g] == m;
                  if (!dup) { hit = m; break; }
                }
            if (hit == (size_t)-1) ok = false;
            else b.face[f] = hit;
          }
          if (!ok) continue;
          for (int c = 0; c < 3; ++c) b.C[c] = C[c], b.ax[c] = ax[c], b.az[c] = az[c];
          b.H = H;
          for (int f = 0; f < 6; ++f) in_box[b.face[f]] = 1;
          boxes.push_back(b);
          break;
        }
      }
    }
    std::vector<size_t> grp[7];  // 0-2: axis-aligned groups, 3: general, 4-6: axis-parallel
    for (size_t i : ord) {
      if (in_box[i]) continue;
      const int a = axis_of(i);
      const int v = a < 0 ? vert_of(i) : -1;
      grp[a >= 0 ? a : v >= 0 ? 4 + v : 3].push_back(i);
    }
    // The odd records of two axis-aligned groups of different axes form one mixed pair, each
    // half tested on its own axis (rt_path.h brute_mixed: the axis test, bit for bit, ~35 VALU
    // where the general pair was ~85; Cornell's light and back wall).  Any other odd record
    // joins the general list.  (Padding each odd group with a never-hit record instead measured
    // 2.5 % slower on C2: one more loop and its per-axis setup.)  RT_BRUTE_MIXED=0: no mixed pair.
    std::vector<std::pair<int, size_t>> odd_ax;  // (axis, record)
    for (int a : {0, 1, 2, 4, 5, 6})
      if (grp[a].size() & 1) {
        if (a < 3 && env_int("RT_BRUTE_MIXED", 1) != 0) odd_ax.push_back({a, grp[a].back()});
        else grp[3].push_back(grp[a].back());  // the group's smallest record
        grp[a].pop_back();
      }
    if (odd_ax.size() == 3) {  // the third joins the general list
      grp[3].push_back(odd_ax.back().second);
      odd_ax.pop_back();
    }
    if (odd_ax.size() == 1) {
      grp[3].push_back(odd_ax.back().second);
      odd_ax.clear();
    }
    std::stable_sort(grp[3].begin(), grp[3].end(),
                     [&](size_t a, size_t b) { return area(h.refs[a]) > area(h.refs[b]); });
    std::vector<long> slots;  // record per slot in loop order, -1 = pad
    for (size_t i : grp[3]) slots.push_back((long)i);
    if (slots.size() & 1) slots.push_back(-1);
    d.brute_ng = (int32_t)(slots.size() / 2);
    for (int a = 0; a < 3; ++a) {
      for (size_t i : grp[4 + a]) slots.push_back((long)i);
      d.brute_vt[a] = (int32_t)(grp[4 + a].size() / 2);
    }
    const size_t n_general = slots.size();  // general and axis-parallel: the stored D
    for (int a = 0; a < 3; ++a) {
      for (size_t i : grp[a]) slots.push_back((long)i);
      d.brute_ax[a] = (int32_t)(grp[a].size() / 2);
    }
    d.brute_mx = 0;  // the mixed pair (axes a0 < a1): (a0 + 1) | (a1 + 1) << 2
    if (odd_ax.size() == 2) {
      slots.push_back((long)odd_ax[0].second);  // odd_ax is in axis order (0, 1, 2 above)
      slots.push_back((long)odd_ax[1].second);
      d.brute_mx = (odd_ax[0].first + 1) | ((odd_ax[1].first + 1) << 2);
    }
    const size_t n_loop = slots.size();  // records the loop tests one by one
    // box descriptors, two per pair slot (an odd box count repeats the last box: the
    // same t and faces, so the winner is unchanged), then the six face records per box
    const size_t nbp = (boxes.size() + 1) / 2;
    d.brute_box = (int32_t)nbp;
    ds->brute_boxes = (int32_t)boxes.size();
    slots.insert(slots.end(), 2 * nbp, -2);
    const size_t face0 = slots.size();
    for (const BoxRec& b : boxes)
      for (int f = 0; f < 6; ++f) slots.push_back((long)b.face[f]);
    if (slots.empty()) {
      slots.assign(2, -1);
      d.brute_ng = 1;
    }
    // pair layout (rt_device.h): records 2p, 2p+1 interleaved field by field
    std::vector<F4> pairs(4 * slots.size(), F4{0, 0, 0, 0});  // pad: n = 0, never hit
    for (size_t k = 0; k < 2 * nbp; ++k) {
      // rt_path.h brute_box: C.x, C.z, ax/|ax|^2 (x, z), az/|az|^2 (x, z), y range, faces
      const BoxRec& b = boxes[std::min(k, boxes.size() - 1)];
      float* f = (float*)&pairs[4 * (n_loop + k - (k & 1))] + (k & 1);
      const double a2 = b.ax[0] * b.ax[0] + b.ax[2] * b.ax[2], z2 = b.az[0] * b.az[0] + b.az[2] * b.az[2];
      const double y0 = b.C[1], y1 = b.C[1] + b.H;
      const float v[8] = {(float)b.C[0], (float)b.C[2], (float)(b.ax[0] / a2), (float)(b.ax[2] / a2),
                          (float)(b.az[0] / z2), (float)(b.az[2] / z2), (float)std::min(y0, y1),
                          (float)std::max(y0, y1)};
      for (int e = 0; e < 8; ++e) f[2 * e] = v[e];
      for (int fc = 0; fc < 6; ++fc) {
        // face slot by (axis x' / y / z', low / high side); y's low side is the lower face
        const int src = (fc >> 1) == 1 && b.H < 0 ? (fc ^ 1) : fc;
        const uint32_t slot = (uint32_t)(face0 + 6 * std::min(k, boxes.size() - 1) + src);
        memcpy(&f[2 * (8 + fc)], &slot, 4);
      }
    }
    for (size_t i = 0; i < slots.size(); ++i) {
      if (slots[i] < 0) continue;
      const F4* r = &recs[4 * (size_t)slots[i]];  // Q|ref, n|D, A, B
      float* f = (float*)&pairs[8 * (i / 2)] + (i & 1);
      float kb;
      const uint32_t k = (uint32_t)i;
      memcpy(&kb, &k, 4);
      // axis records: D / n_a (= +-D exactly) in the D slot, so t = (D' - o_a) / d_a
      const int a = i >= n_general && i < n_loop ? axis_of((size_t)slots[i]) : -1;
      const float na = a == 0 ? r[1].x : a == 1 ? r[1].y : r[1].z;
      const float Dp = a < 0 ? r[1].w : na * r[1].w;
      const float v[15] = {r[1].x, r[1].y, r[1].z, Dp,     r[0].x, r[0].y, r[0].z, r[2].x,
                           r[2].y, r[2].z, r[3].x, r[3].y, r[3].z, kb,     r[0].w};
      for (int e = 0; e < 15; ++e) f[2 * e] = v[e];
    }
    ds->brute_slots = slots.size();
    // The lean set's shade table, after the pairs: per quad its normal and material kind,
    // and its texture's solid colour (2 F4), so the record-loop kernel shades from LDS
    // instead of three dependent global loads (quad, material, texture) per vertex, whose
    // s_waitcnt vmcnt(0) also waited for the chunk flushes' pixel atomics
    // (profiles/r4_phases_flush_c2.jsonl).  Only when every quad's material is Lambertian
    // or a diffuse light with a solid texture (what the lean kernel shades).
    {
      const size_t nq = h.quad.size() / 5;
      std::vector<F4> tab(2 * nq);
      bool ok = nq > 0;
      for (size_t qi = 0; qi < nq && ok; ++qi) {
        const F4* q = &h.quad[5 * qi];
        uint32_t mb;
        memcpy(&mb, &q[2].w, 4);
        ok = mb < mats.size();
        if (!ok) break;
        const DevMaterial& m = mats[mb];
        ok = (m.kind == RT_MAT_LAMBERTIAN || m.kind == RT_MAT_DIFFUSE_LIGHT) && m.tex >= 0 &&
             (size_t)m.tex < h.texs.size() && h.texs[m.tex].kind == RT_TEX_SOLID;
        if (!ok) break;
        float kb;
        const uint32_t kind = (uint32_t)m.kind;
        memcpy(&kb, &kind, 4);
        tab[2 * qi] = {q[3].x, q[3].y, q[3].z, kb};
        // the colour, and the plane offset D (shade_core puts the hit point on the plane)
        const F4 col = h.texs[m.tex].color;
        tab[2 * qi + 1] = {col.x, col.y, col.z, q[0].w};
      }
      ds->shade_n = ok && env_int("RT_SHADE_LDS", 1) != 0 ? (int32_t)tab.size() : 0;
      if (ds->shade_n) pairs.insert(pairs.end(), tab.begin(), tab.end());
    }
    if ((rc = upload(ds, pairs, &ds->brute_pairs)) != RT_OK) return rc;
  }
records_done:
  UP(h.media, media);
  UP(h.medium_refs, medium_refs);
  {  // spheres tested before the BVH (host_flatten: radius >= kBigSphereR), as leaf records
    std::vector<F4> br(4 * h.big_refs.size());
    for (size_t i = 0; i < h.big_refs.size(); ++i) make_record(h, h.big_refs[i], &br[4 * i]);
    UP(br, big_recs);
    d.n_big = (int32_t)h.big_refs.size();
  }
  UP(h.lights, lights);
  UP(mats, mats);
  UP(h.texs, texs);
  UP(h.texels, texels);
  UP(h.images, images);
  UP(h.perlins, perlins);
#undef UP
  d.root = h.root4;
  d.n_nodes = (int32_t)(h.nodes4.size() / 8);
  d.n_media = (int32_t)h.media.size();
  d.medium_draws = h.medium_draws;
  d.n_lights = (int32_t)h.lights.size();
  // mixture-pdf floor (rt_path.h): only when every light entry is a real prim; an entry of
  // an empty HittableList has pdf 0 by the reference's rules, and its 0/0 NaNs are kept
  d.pdf_floor = h.lights.empty() ? 0.0f : 1e-30f;
  for (const auto& e : h.lights)
    if (e.ref == PRIM_NONE) d.pdf_floor = 0.0f;
  d.n_refs = (int32_t)h.refs.size();
  d.n_perlins = (int32_t)h.perlins.size();
  // the weight merge needs non-negative suffix products: every texture value (solid
  // colours; image and noise values are >= 0 by construction) and metal albedo >= 0
  // (the background is checked per render)
  d.shade_lds = -1;  // set per launch (record-loop kernel with the records in LDS)
  d.shade_n = 0;
  d.merge_ok = 1;
  for (const auto& t : h.texs)
    if (t.kind == RT_TEX_SOLID && !(t.color.x >= 0.0f && t.color.y >= 0.0f && t.color.z >= 0.0f))
      d.merge_ok = 0;
  for (const auto& m : mats)
    if (m.kind == RT_MAT_METAL && !(m.albedo.x >= 0.0f && m.albedo.y >= 0.0f && m.albedo.z >= 0.0f))
      d.merge_ok = 0;
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

// slot-indexed wavefront buffers (only for WAVEFRONT) + the weight stack,
// counters and pixel accumulators (both modes)
static int ensure_state(SlotState* slot, int device, uint32_t P, int depth_cap, uint32_t npix,
                        bool soa) {
  RenderState* st = slot->st;
  if (st && (st->device != device || st->P < P || st->depth_cap < depth_cap || st->npix < npix ||
             (soa && !st->ray_o))) {
    delete st;
    st = slot->st = nullptr;
  }
  if (st) return RT_OK;
  st = slot->st = new RenderState();
  st->device = device;
  st->P = P;
  st->depth_cap = depth_cap;
  st->npix = npix;
  int rc;
  if ((rc = dalloc(st, &st->stack, (size_t)P * depth_cap)) || (rc = dalloc(st, &st->ctr, 1)) ||
      (rc = dalloc(st, &st->accum, 3 * (size_t)npix)) || (rc = dalloc(st, &st->side, 3 * (size_t)npix)) ||
      (rc = dalloc(st, &st->pflags, npix)) ||
      (rc = dalloc(st, &st->out, 3 * (size_t)npix)))
    return rc;
  if (soa &&
      ((rc = dalloc(st, &st->ray_o, P)) || (rc = dalloc(st, &st->ray_d, P)) ||
       (rc = dalloc(st, &st->hit, P)) || (rc = dalloc(st, &st->pend, P)) ||
       (rc = dalloc(st, &st->pre, P)) ||
       (rc = dalloc(st, &st->path, P)) || (rc = dalloc(st, &st->queue[0], (size_t)kXcd * P)) ||
       (rc = dalloc(st, &st->queue[1], (size_t)kXcd * P))))
    return rc;
  return RT_OK;
}

static int occupancy_blocks(const void* kernel, int device, int* out, size_t dyn_lds = 0) {
  int per_cu = 0, cus = 0;
  HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, dyn_lds));
  HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  *out = std::max(1, per_cu) * std::max(1, cus);
  return RT_OK;
}

static_assert(FT_SPHERE == RT_FT_SPHERE && FT_TRI == RT_FT_TRI && FT_METAL == RT_FT_METAL &&
                  FT_DIEL == RT_FT_DIEL && FT_MEDIA == RT_FT_MEDIA && FT_CHECKER == RT_FT_CHECKER &&
                  FT_IMAGE == RT_FT_IMAGE && FT_NOISE == RT_FT_NOISE && FT_BOX == RT_FT_BOX,
              "feature bits: rt_device.h and rt_abi.h disagree");

#define RT_FUSED_EXTERN(L, F, T) extern template __global__ void k_fused<L, F, T>(Params);
RT_FUSED_ILP_KERNELS(RT_FUSED_EXTERN)  // defined in rt_fused_sets.hip
#undef RT_FUSED_EXTERN

template <bool LDS>
static const void* fused_for(uint32_t set) {
  switch (set) {
    case kFtSets[0]: return (const void*)k_fused<LDS, kFtSets[0], 4>;
    case kFtSets[1]: return (const void*)k_fused<LDS, kFtSets[1], 4>;
    case kFtSets[2]: return (const void*)k_fused<LDS, kFtSets[2], 4>;
    case kFtSets[3]: return (const void*)k_fused<LDS, kFtSets[3], 4>;
    case kFtSets[4]: return (const void*)k_fused<LDS, kFtSets[4], 4>;
    default: return (const void*)k_fused<LDS, FT_ALL, 4>;
  }
}
static uint32_t pick_set(uint32_t feats) { return pick_ft_set(feats); }
// BVH2 kernels exist for the two smallest sets with the tree in LDS (tiny scenes)
static const void* pick_fused(bool lds, uint32_t set, int tree) {
  if (tree == 0 && lds && set == kFtSets[0]) return (const void*)k_fused<true, kFtSets[0], 0>;
  if (tree == 0 && lds && set == kFtSets[1]) return (const void*)k_fused<true, kFtSets[1], 0>;
  if (tree == 0 && !lds && set == kFtSets[0]) return (const void*)k_fused<false, kFtSets[0], 0>;
  if (tree == 0 && !lds && set == kFtSets[1]) return (const void*)k_fused<false, kFtSets[1], 0>;
  if (tree == 2 && lds && set == kFtSets[0]) return (const void*)k_fused<true, kFtSets[0], 2>;
  if (tree == 2 && lds && set == kFtSets[1]) return (const void*)k_fused<true, kFtSets[1], 2>;
  if (tree == 8) {
#ifdef RT_BVH8_KERNELS
    // BVH8 (measured slower than the BVH4): A/B builds only.  Large trees
    // read through L1/L2, the three tree sets
    if (!lds && set == kFtSets[2]) return (const void*)k_fused<false, kFtSets[2], 8>;
    if (!lds && set == kFtSets[3]) return (const void*)k_fused<false, kFtSets[3], 8>;
    if (!lds && set == kFtSets[4]) return (const void*)k_fused<false, kFtSets[4], 8>;
#endif
    return nullptr;
  }
  if (tree == 5) {  // the compressed BVH4: trees read through L1/L2
    if (lds) return nullptr;
    switch (set) {
      case kFtSets[2]: return (const void*)k_fused<false, kFtSets[2], 5>;
      case kFtSets[3]: return (const void*)k_fused<false, kFtSets[3], 5>;
      case kFtSets[4]: return (const void*)k_fused<false, kFtSets[4], 5>;
      case FT_ALL: return (const void*)k_fused<false, FT_ALL, 5>;
      default: return nullptr;
    }
  }
  if (tree != 4) return nullptr;  // no such kernel: render_impl never asks (see tree there)
  return lds ? fused_for<true>(set) : fused_for<false>(set);
}

// rt_render_multi's share hand-off: after the resolve, the share's image (rows of
// this rank, [rows][W][3]) is copied to `dst` on device `dst_device` (peer copy over
// xGMI when the devices differ) on the share's stream, before the render returns.
struct Gather {
  float* dst;
  int dst_device;
};

// The compressed BVH4 of a tree read through L1/L2 (render_impl's tree 5), on `device`
// (current): built on the host once per scene and uploaded once per device, by the first
// render whose kernel can traverse it -- not for LDS-resident trees, record-loop scenes or
// RT_QBVH=0 renders (~85 MB of HBM per GPU for the 1M-triangle mesh otherwise).
static int ensure_qbvh(Scene* s, DeviceScene* ds) {
  std::lock_guard<std::mutex> lk(ds->qmu);
  if (ds->q_done) return RT_OK;
  {
    std::lock_guard<std::mutex> hk(s->qb_mu);
    if (!s->qb_built) {
      std::vector<F4> recs;
      build_leaf_records(s->h, recs);
      int rc = build_qbvh(s->h, recs, &s->qb, &s->qb_items);
      if (rc != RT_OK) return rc;
      s->qb_built = true;
    }
  }
  if (s->qb_items) {
    const int rc = upload(ds, s->qb, &ds->qnodes);
    if (rc != RT_OK) return rc;
    ds->qitems = s->qb_items;
  }
  ds->q_done = true;
  return RT_OK;
}

static int render_impl(rt_scene* scene, const rt_camera* cam, const rt_render_opts* opts,
                       float* out_host, float* out_dev, rt_stats* stats, int slot_id = 0,
                       const Gather* gather = nullptr) {
  if (!scene || !cam) return set_error(RT_ERR_INVALID, "rt_render: null scene/camera");
  rt_render_opts o{};
  if (opts) o = *opts;
  if (o.nranks <= 0) o.nranks = 1;
  if (o.rank < 0 || o.rank >= o.nranks) return set_error(RT_ERR_INVALID, "rt_render: bad rank");
  rt_camera_derived cd;
  int rc = rt_camera_derive(cam, &cd);
  if (rc) return rc;
  auto t_start = std::chrono::steady_clock::now();
  const int32_t tuned = tune_count();  // rt_stats.tuned: knobs off their defaults

  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return set_error(RT_ERR_DEVICE, "rt_render: no HIP device available");
  if (o.device < 0 || o.device >= ndev)
    return set_error(RT_ERR_INVALID, "rt_render: device %d of %d", o.device, ndev);
  DeviceGuard dg;  // the caller's current device is restored on every return
  HIP_OK(hipSetDevice(o.device));
  Scene* s = &scene->s;
  DeviceScene* ds = nullptr;
  if ((rc = ensure_scene(s, o.device, &ds))) return rc;
  SlotState* slot = nullptr;
  {
    std::lock_guard<std::mutex> lk(s->mu);
    SlotState*& sl = s->slots[{o.device, slot_id}];
    if (!sl) sl = new SlotState();
    slot = sl;
  }
  std::lock_guard<std::mutex> inflight(slot->mu);  // one render per (scene, device, slot)

  const uint32_t W = (uint32_t)cd.width, H = (uint32_t)cd.height;
  const uint32_t rows = H > (uint32_t)o.rank ? (H - (uint32_t)o.rank + o.nranks - 1) / o.nranks : 0;
  const uint32_t npix = rows * W;
  const uint32_t ss = (uint32_t)cd.spp_sqrt * (uint32_t)cd.spp_sqrt;
  int mode = o.mode;
  if (mode != RT_MODE_WAVEFRONT && mode != RT_MODE_FUSED) mode = RT_MODE_FUSED;
  const int depth_cap = cd.max_depth + 1;
  uint32_t P;
  int fused_blocks = 0;
  const bool lds_nodes = s->h.nodes4.size() / 8 <= (size_t)kLdsNodes / 2;
  const uint32_t feats = s->h.features;
  // the feature-set kernels read perlin table 0 from LDS only: scenes whose noise
  // textures use other tables run the all-features kernel (generic table pointers)
  const uint32_t ft_set = (feats & FT_NOISE) && !s->h.noise_table0 ? FT_ALL : pick_set(feats);
  // The fused kernel's LDS scene cache (stage_nodes): all BVH nodes, then the
  // leaf records when both fit, within the LDS a workgroup may take at the
  // kernel's target waves per SIMD (160 KB per CU, 24 KB of stacks per group).
  // A tree that does not fit runs the global-node instantiation: caching only
  // its top measured 3-6 % slower on C3-C5 than one node source per kernel.
  // Tree width: the fused kernel traverses the BVH4, except for tiny scenes
  // (<= 64 leaf entries, C2's 18 quads) where the BVH2 measured 3 % faster;
  // the wavefront extend kernel always takes the BVH4.
  // BVH2 kernels exist only for the two smallest feature sets with the tree and
  // its records in LDS (pick_fused): anything else takes the BVH4.
  const size_t n_refs = s->h.refs.size();
  auto slots_for = [&](int tr) {
    return std::min<size_t>(kLdsNodes, (160u * 1024u / (unsigned)fused_waves(ft_set, tr) -
                                        fused_static_lds(ft_set, tr) - 512u) / 64u);
  };
  const bool small_set = ft_set == kFtSets[0] || ft_set == kFtSets[1];
  // tree: 0 (no tree: every record tested, <= kBruteMax records in LDS), 2 or 4
  const int env_tree = env_int("RT_TREE", -1);
  int tree = 4;
  const size_t brute_max = (size_t)env_int("RT_BRUTE_MAX", kBruteMax);  // A/B override
  // Record loop vs tree, measured on the Cornell box plus 0-12 extra boxes
  // (tools/brute_sweep.py, profiles/r1_brute_sweep.jsonl): the lockstep loop wins
  // up to ~56 records (18: +33 %, 48: +16 %), reading the records from the LDS
  // cache when they fit (C2 +2 % over scalar loads), with scalar loads otherwise.
  if (mode == RT_MODE_FUSED && small_set && n_refs > 0 && n_refs <= brute_max)
    tree = 0;
  else if (mode == RT_MODE_FUSED && small_set && n_refs <= 64 && !s->h.nodes.empty() &&
           s->h.nodes.size() / 4 + n_refs <= slots_for(2))
    tree = 2;
  if (mode == RT_MODE_FUSED && small_set && (env_tree == 2 || env_tree == 4) &&
      (env_tree == 4 || (!s->h.nodes.empty() && s->h.nodes.size() / 4 + n_refs <= slots_for(2))))
    tree = env_tree;  // A/B override
  const size_t lds_slots = slots_for(tree);
  const size_t brute_slots = ds->brute_slots;  // record-loop pairs, 2 x 64 B each
  const int smem_env = env_int("RT_BRUTE_SMEM", -1);
  const bool brute_smem =
      tree == 0 && (smem_env >= 0 ? smem_env != 0 : brute_slots > lds_slots);
  const bool w4 = tree == 4;
  const size_t n_nodes = tree == 4 ? s->h.nodes4.size() / 8 : tree == 2 ? s->h.nodes.size() / 4 : 0;
  const size_t node_slots = w4 ? 2 : 1;  // 64-B LDS slots per node
  const bool f_lds = node_slots * n_nodes <= lds_slots && !brute_smem;
  // the record loop's pairs, then (lean set) the quads' shade table, 4 F4 per 64-B slot
  // The record-loop LDS kernel reads its records from LDS only (trav_brute<.., SMEM = false>),
  // so with a tree 0 in LDS the records must be staged: brute_smem above guarantees they fit
  // alone, and a shade table that would push them over the budget is left out (the lean
  // kernel then shades from the quad table in HBM).  Found in round 6: a 7-wave build shrank
  // the budget below Cornell's records + table, and the kernel read unstaged LDS.
  bool shade_tab = tree == 0 && ft_set == 0u && ds->shade_n > 0;
  if (shade_tab && f_lds && brute_slots + (size_t)(ds->shade_n + 3) / 4 > lds_slots) shade_tab = false;
  const size_t rec_slots = tree == 0 ? brute_slots + (shade_tab ? (size_t)(ds->shade_n + 3) / 4 : 0) : n_refs;
  const bool f_recs = f_lds && node_slots * n_nodes + rec_slots <= lds_slots;
  if (tree == 0 && f_lds && !f_recs)
    return set_error(RT_ERR_UNSUPPORTED, "internal: record loop in LDS without its records");
  // Trees read through L1/L2 take the BVH8 (host_bvh8.cpp) when the scene has one (built
  // only with RT_BVH8=1) and a kernel exists for its feature set; RT_TREE=4 keeps the BVH4
  if (mode == RT_MODE_FUSED && tree == 4 && !f_lds && !s->h.nodes8.empty() && env_tree != 4 &&
      pick_fused(false, ft_set, 8))
    tree = 8;
  // Trees read through L1/L2 with single-prim leaves take the compressed BVH4 (64-B nodes,
  // host_qbvh.cpp): the same closest hits, half the bytes per node step.  RT_QBVH=0: the
  // 128-B nodes (A/B)
  if (mode == RT_MODE_FUSED && tree == 4 && !f_lds && env_int("RT_QBVH", 1) != 0 &&
      pick_fused(false, ft_set, 5)) {
    if ((rc = ensure_qbvh(s, ds))) return rc;
    if (ds->qnodes) tree = 5;
  }
  const void* fused_kernel = pick_fused(f_lds, ft_set, tree);
  if (!fused_kernel) return set_error(RT_ERR_UNSUPPORTED, "internal: no fused kernel for this scene");
#ifdef RT_QTOP
  const size_t fused_lds = f_lds ? 64 * (node_slots * n_nodes + (f_recs ? rec_slots : 0))
                           : tree == 5 ? 64 * std::min<size_t>(RT_QTOP, ds->qitems) : 0;
#else
  const size_t fused_lds = f_lds ? 64 * (node_slots * n_nodes + (f_recs ? rec_slots : 0)) : 0;
#endif
  if (mode == RT_MODE_FUSED) {
    if ((rc = occupancy_blocks(fused_kernel, o.device, &fused_blocks, fused_lds))) return rc;
    if (o.path_slots > 0) fused_blocks = std::max(1, std::min(fused_blocks, (o.path_slots + 255) / 256));
    P = (uint32_t)fused_blocks * 256u;
  }
  // Samples per chunk.  Fused: the largest K in {32, 16, 8} (64 for C2's record loop, below)
  // that still gives
  // every lane >= 12 chunks (tree in LDS) or >= 100 (tree through L1/L2, whose
  // per-pixel cost varies more), so the last chunks do not leave most lanes idle.
  // Round 4 (partitioned counters, chunk sums as plain stores): C2's 2-, 4- and 8-GPU
  // shares are fastest at K = 32 / 16 / 16 (16.9 / 8.67 / 4.68 ms; K = 8: 18.2 / 9.03 /
  // 4.91, profiles/r4_chunk_probe_csum.jsonl), which 12 chunks per lane picks; 48 picked
  // 16 / 8 / 8.
  // Measured with the row-group order (tools/chunk_probe.py,
  // profiles/r2_chunk_size_*.jsonl): 8-GPU shares of C2/C3/C4/C5 are fastest at
  // K = 8 (C5 -27 % against 32), whole images at K = 32 (C3 -3 % against 8); at 100
  // C3 takes K = 16 (1.5 % behind 32, which is 14 % behind 8 on C5's 8-GPU share).
  uint32_t K = 32u;
  if (o.chunk > 0) {
    K = (uint32_t)o.chunk;
  } else if (mode == RT_MODE_FUSED) {
    // (the mesh set asks 200: the 1M-triangle mesh's 2- / 4- / 8-GPU shares -0.6 / -1.6 /
    // -2.3 % with K halved, its whole image unchanged at K = 32; book1 and book2 gained
    // nothing from it, profiles/r5_model_chunk_share_ab.jsonl, r5_chunk_need200_ab.jsonl)
    // Round 6: book1's set asks 50 and may take K = 24.  Its bar of 100 had been met at K = 16
    // with 4 waves per SIMD; at 5 (round 5) the lanes outnumber it and the rule fell to K = 8:
    // the whole C3 image 72.2 ms at 8, 71.2 at 16, 70.6 at 24, 71.8 at 32; its 2- and 8-GPU
    // shares still get 8 and 4 (profiles/r6_chunk_sweep.jsonl)
    const bool book1_set = ft_set == (FT_SPHERE | FT_TRI | FT_METAL | FT_DIEL | FT_CHECKER);
    const int need_dflt = f_lds ? 12 : ft_set == (FT_SPHERE | FT_TRI | FT_METAL) ? 200 : book1_set ? 50 : 100;
    const uint64_t work = (uint64_t)npix * ss,
                   need = (uint64_t)std::max(1, env_int("RT_CHUNK_NEED", need_dflt)) * P;
    K = f_lds ? 8u : 4u;  // the smallest: C3's 8-GPU share 6 % faster at 4 than 8 (C2's ±1 %)
    // Round 6: the lean record-loop kernel (C2) also takes K = 64 at the same bar (half as
    // many chunk starts and records; k_resolve reads half the bytes): C2 28.44 -> 27.81 ms
    // on the whole image, its 2-GPU share -0.6 %; its 4-GPU share, 6.5 chunks per lane at 64,
    // keeps 32 (7.56-7.65 against 7.81-7.83 ms at 64, profiles/r6_chunk64_share_ab.jsonl),
    // the 8-GPU share 16 (64: 4.62, 32: 4.39 ms against 4.03), and the tree kernels 32 (64:
    // book1 +4 %, C5 +1.9 %, book2 +0.5 %; profiles/r6_chunk64_probe.jsonl)
    if (tree == 0 && ft_set == 0u && work / 64u >= need) {
      K = 64u;
    } else {
      for (uint32_t k : {32u, 24u, 16u, 8u})
        if ((k != 24u || book1_set) && work / k >= need) {
          K = k;
          break;
        }
    }
  }
  K = std::max<uint32_t>(1u, std::min<uint32_t>(std::min(K, ss), 4096u));
  // Tail phase (fused, default chunk sizes): the last ~1/RT_TAIL_FRAC of every pixel's
  // samples in chunks of K / 4 (min 4), after all first-phase chunks (rt_path.h chunk_pixel),
  // by default (1/4) when a lane gets fewer than 40 chunks: the multi-GPU shares.  C2's 2-,
  // 4- and 8-GPU shares -1.0 / -4.0 / -2.3 %, the whole image (52 chunks per lane, no tail)
  // +0.5 % with it (profiles/r4_tail_ab.jsonl)
  uint32_t S1 = ss, K2 = K;
  {
    // (not the record-loop kernel: its chunk starts use the one-phase mapping, chunk_ids<true>)
    const bool one_phase = tree == 0 && ft_set == 0u;
    const bool few = mode == RT_MODE_FUSED && !one_phase &&
                     (uint64_t)npix * ss / std::max<uint32_t>(K, 1u) < 40ull * P;
    // default: with the default chunk size only; an explicit RT_TAIL_FRAC also applies to
    // an explicit chunk size (A/B and tests)
    const int tf_env = env_int("RT_TAIL_FRAC", -1);
    const int tf = tf_env >= 0 ? tf_env : (few && o.chunk <= 0 ? 4 : 0);
    if (mode == RT_MODE_FUSED && !one_phase && tf > 1 && K >= 8u) {
      K2 = std::max<uint32_t>(1u, (uint32_t)env_int("RT_TAIL_K", (int)std::max<uint32_t>(4u, K / 4)));
      const uint32_t s1 = (uint32_t)((uint64_t)ss * (uint32_t)(tf - 1) / (uint32_t)tf) / K * K;
      if (s1 > 0 && s1 < ss && K2 < K) S1 = s1;
      else K2 = K;
    }
  }
  const uint32_t cpp1 = S1 / K + (S1 == ss && ss % K ? 1u : 0u);  // no tail: ceil(ss / K)
  const uint32_t cpp2 = S1 < ss ? (ss - S1 + K2 - 1) / K2 : 0u;
  const uint32_t cpp = cpp1 + cpp2;
  const uint64_t n_chunks64 = (uint64_t)npix * cpp;
  if (n_chunks64 >= 0xF0000000ull) return set_error(RT_ERR_UNSUPPORTED, "too many work chunks");
  const uint32_t n_chunks = (uint32_t)n_chunks64;
  if (mode != RT_MODE_FUSED) {
    P = o.path_slots > 0 ? (uint32_t)o.path_slots : (1u << 20);
    P = std::max<uint32_t>(256u, std::min<uint32_t>(P, std::max<uint32_t>(n_chunks, 256u)));
    P = (P + 255u) & ~255u;
  }
  if ((rc = ensure_state(slot, o.device, P, depth_cap, std::max<uint32_t>(npix, 1),
                         mode == RT_MODE_WAVEFRONT)))
    return rc;
  RenderState* st = slot->st;
  const void* extend_kernel =
      lds_nodes ? (const void*)k_extend<true> : (const void*)k_extend<false>;
  if (mode == RT_MODE_WAVEFRONT && st->resident_blocks == 0 &&
      (rc = occupancy_blocks(extend_kernel, o.device, &st->resident_blocks)))
    return rc;
  // traversal-stack overflow columns: one per launched traversal thread
  {
    const uint32_t cols = mode == RT_MODE_FUSED ? P : (uint32_t)st->resident_blocks * 256u;
    if (st->ostack_cols < cols) {
      if (st->ostack) {
        HIP_OK(hipFree(st->ostack));
        st->allocs.erase(std::find(st->allocs.begin(), st->allocs.end(), (void*)st->ostack));
        st->ostack = nullptr;
      }
      if ((rc = dalloc(st, &st->ostack, (size_t)(kStack - kShortStackMin) * cols))) return rc;
      st->ostack_cols = cols;
    }
  }
  // fused: the per-chunk sums (32 B per chunk, every record stored once per render: no clear).
  // The buffer grows with the sample count, not the image: above its cap (RT_CSUM_MAX_MB,
  // default 16 GiB, and at most half of the device's free memory) or when it cannot be
  // allocated, the render falls back to pixel atomics (P.csum == nullptr: the same integer
  // sums, so the same image; rt_stats.chunk_records = 0).  A buffer more than 4x larger than
  // this render needs (and over 256 MiB) is released first.
  bool use_csum = mode == RT_MODE_FUSED && env_int("RT_CSUM", 1) != 0;
  {
    const size_t need_b = 32 * (size_t)n_chunks;
    auto drop_csum = [&]() -> int {
      if (!st->csum) return RT_OK;
      HIP_OK(hipFree(st->csum));
      st->allocs.erase(std::find(st->allocs.begin(), st->allocs.end(), (void*)st->csum));
      st->csum = nullptr;
      st->csum_chunks = 0;
      return RT_OK;
    };
    if (st->csum && (!use_csum || (st->csum_chunks > 4 * (size_t)n_chunks &&
                                   32 * st->csum_chunks > ((size_t)256 << 20))))
      if ((rc = drop_csum())) return rc;
    if (use_csum && st->csum_chunks < n_chunks) {
      if ((rc = drop_csum())) return rc;
      size_t free_b = 0, total_b = 0;
      const size_t cap_b = (size_t)std::max(0, env_int("RT_CSUM_MAX_MB", 16384)) << 20;
      if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
      void* q = nullptr;
      if (need_b <= cap_b && need_b <= free_b / 2 && hipMalloc(&q, std::max<size_t>(need_b, 32)) == hipSuccess) {
        st->allocs.push_back(q);
        st->csum = (unsigned long long*)q;
        st->csum_chunks = n_chunks;
      } else {
        (void)hipGetLastError();  // a failed allocation is not sticky: pixel atomics instead
        use_csum = false;
      }
    }
  }

  hipStream_t stream = (hipStream_t)o.stream;
  if (!stream) {
    if (!st->own_stream) HIP_OK(hipStreamCreateWithFlags(&st->own_stream, hipStreamNonBlocking));
    stream = st->own_stream;
  }

  Params p{};
  p.sc = ds->d;
  if (tree == 2) {
    p.sc.nodes = ds->nodes2;
    p.sc.root = ds->root2;
    p.sc.n_nodes = ds->n_nodes2;
  } else if (tree == 5) {
    p.sc.nodes = ds->qnodes;
    p.sc.root = 0;  // item 0: the root node (trav_init)
    p.sc.n_nodes = (int32_t)std::min<size_t>(ds->qitems, 0x7FFFFFFF);  // 64-B items
  } else if (tree == 8) {
    p.sc.root = 0;  // BVH8 node 0 (trav_init)
  } else if (tree == 0) {
    p.sc.n_nodes = 0;  // records only (stage_nodes puts them at the start of the cache)
    p.sc.leafprims = ds->brute_pairs;
    p.sc.n_refs = (int32_t)brute_slots;  // even: whole pairs
    if (shade_tab && f_recs) {  // the shade table follows the pairs, in LDS as in HBM
      p.sc.shade_lds = (int32_t)(4 * brute_slots);
      p.sc.shade_n = ds->shade_n;
    }
  }
  for (int i = 0; i < 3; ++i) {
    p.p00r[i] = (float)(cd.pixel00[i] - cd.center[i]);
    p.du[i] = (float)cd.delta_u[i];
    p.dv[i] = (float)cd.delta_v[i];
    p.cc[i] = (float)cd.center[i];
    p.dku[i] = (float)cd.defocus_u[i];
    p.dkv[i] = (float)cd.defocus_v[i];
    p.bg[i] = (float)cd.background[i];
  }
  if (!(p.bg[0] >= 0.0f && p.bg[1] >= 0.0f && p.bg[2] >= 0.0f)) p.sc.merge_ok = 0;
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
  p.K2 = K2;
  p.S1 = S1;
  p.n1 = npix * cpp1;
  p.n_chunks = n_chunks;
  p.P = P;
  p.ss = ss;
  uint32_t g_ng = 1u;  // chunk-order groups of this rank
  {
    // chunk order (chunk_pixel): groups of `grows` of this rank's rows, so the paths in
    // flight start from a band of a few rows instead of the whole image (C5 -10 %,
    // C3 -5 %, C4 -3 %, C2 -1 % against image-wide pixel-fastest chunks; 1, 4 and 16
    // rows measured alike, profiles/r2_chunk_order_ab.jsonl)
    const int env_rows = env_int("RT_CHUNK_ROWS", -1);
    uint32_t grows = env_rows > 0 ? (uint32_t)env_rows : 4u;
    grows = std::max<uint32_t>(1u, std::min<uint32_t>(grows, std::max<uint32_t>(rows, 1u)));
    while (rows % grows) --grows;  // a divisor of the rank's row count
    const uint32_t gpix = std::max<uint32_t>(1u, grows * W);
    p.fd_gpix = make_fastdiv(gpix);
    p.fd_gchunks = make_fastdiv(gpix * cpp1);
    p.fd_gchunks2 = make_fastdiv(std::max<uint32_t>(1u, gpix * cpp2));
    g_ng = rows / grows;
  }
  // The order the sweep takes the row groups in (chunk_pixel, k_resolve; images do not
  // depend on it): RT_SWEEP = forward (image order, the default) or reverse.  A render's tail
  // is the paths still in flight when the chunk pool runs dry, so it depends on which rows
  // the sweep ends on: book2's costly bottom rows (fog, the box ground) end its forward sweep,
  // and its 2- / 8-GPU shares are 2.3 / 3.2 % faster reversed, while C5 and book1 are 1-6 %
  // slower (the sky ends their reverse sweep right after the metal dragon / the sphere field,
  // whose long specular paths are then still in flight); no probe of the rows' costs chose
  // between them reliably, DESIGN.md §8.  Feature-set kernels only (the record loop maps
  // chunks in one phase).  The group of sweep position q is (q ^ gflip) + gbase, compiled in
  // only with -DRT_SWEEP_ORDER: even that form, two kernel-argument words and two VALU ops
  // per chunk start, measured C4 +0.3 % and C5 +0.5 % in the default order at full size
  // (profiles/r6_sweep_table_cost_ab.jsonl; a table lookup the same).
#ifdef RT_SWEEP_ORDER
  p.gflip = p.gbase = 0u;
#endif
  {
    std::string v;
    if (tune_str("RT_SWEEP", &v) && v == "reverse") {
#ifdef RT_SWEEP_ORDER
      if (mode == RT_MODE_FUSED && ft_set != 0u && g_ng > 1 && npix > 0) {
        p.gflip = ~0u;  // (q ^ ~0) + ng = ng - 1 - q
        p.gbase = g_ng;
      }
#else
      return set_error(RT_ERR_UNSUPPORTED, "RT_SWEEP=reverse needs a library built with -DRT_SWEEP_ORDER");
#endif
    }
  }
  p.fd_width = make_fastdiv(W);
  p.fd_s = make_fastdiv((uint32_t)cd.spp_sqrt);
  // Scheduling rounds, measured on the full-size configs (tools/sched_sweep.py,
  // tools/sched_ab.sh, profiles/r1_sched_sweep*.jsonl, r2_sched_ab*.jsonl): trees read
  // through L1/L2 gain from bounded rounds so short rays do not idle behind long ones —
  // 8 steps for large trees (C5 +75 %, C4 +10 % over unbounded), 12 for small ones
  // (C3's 485 spheres: 7 % faster than 8); LDS-resident trees (C2) lose from any bound.
  // Kernels with long shading gain from waiting until enough lanes are ready: 32 for
  // the book2 and all-features sets (C4 -1.2 %), 16 for large trees otherwise (C5 -2 %).
  // Round 5, on the compressed BVH4 (cheaper node steps, 5 waves per SIMD): the mesh
  // scene is fastest at 5 steps and 32 ready lanes (C5 +4.6 % over 8 / 16 at 256 spp;
  // 64 ready lanes halves it), book2 unchanged at 8 / 32 (6 / 32 within 0.1 %), book1 at
  // 12 / 1 (profiles/r5_sched_sweep_q.jsonl) -- then 10 steps for book1: -0.7 % at full size
  // (r5_c3_step_ab.jsonl; 9 to 16 swept at 256 spp, r5_knob_sweeps_q.jsonl)
  const bool big_tree = s->h.nodes4.size() / 8 >= 1024;
  const bool long_shade = ft_set == FT_ALL || (ft_set & FT_NOISE);
  // (book2 at full size: 7 steps and 40 ready lanes -0.7 % against 8 / 32,
  // profiles/r5_c4_c5_knobs_full.jsonl)
  // (clamped where read, as every scheduling knob: a round without a traversal step would
  // never finish a traversal)
  // (round 6, with the mesh set's 256-chunk batches: 4 steps -0.5 % on C5's whole image, -0.4 /
  // -0.6 % on its 2- / 8-GPU shares against 5; 3 as 4 except the 8-GPU share, 2 +1.5 %; the
  // ready-lane bar 24 as 32, 16 +2.5 %, 40 +2 %; profiles/r6_c5_sched_sweep.jsonl)
  p.step_budget = std::max(1, env_int("RT_STEP_BUDGET", f_lds ? (1 << 30) : big_tree ? (long_shade ? 7 : 4) : 10));
  p.shade_min = (uint32_t)std::max(1, env_int("RT_SHADE_MIN", f_lds ? 1 : long_shade ? 40 : big_tree ? 32 : 1));
  // chunks per refill of a wave's batch (one returning atomic on the chunk
  // counter each): C2 grab sweep (profiles/r1_grab_sweep.jsonl) 64 -> 128:
  // -4 % at 1-2 ranks' shares; 256 for small chunks: -11 % on the 8-GPU share
  // Round 4, with the 64 partitioned counters below: batches of 32 chunks for the
  // LDS-resident scenes (C2 -1.7 % on the whole image, its 8-GPU share 5.13 ms against
  // 5.22 with 128; profiles/r4_share_probe_grab_v1.jsonl, r4_grab_ab.jsonl), while the
  // scenes that traverse a tree through L1/L2 keep 128 (32 measured C3 +3.7 %, C4 +2.2 %,
  // C5 +2 %: their waves refill more often and spread over more of the image)
  // (round 6: 16 for C2's record loop at any K: its whole image at K = 64 -0.4 % against 32
  // (64 +1 %, 128 +4 %), its 2- / 4-GPU shares -0.9 / -1.3 %, the 8-GPU share ±0;
  // profiles/r6_chunk_sweep.jsonl, r6_grab_sweep_c2_shares.jsonl)
  // (round 6: 256 for the mesh set at any K: C5 -1.0 % on the whole image, -0.5 % on its 2-GPU
  // share; 512 ±0, 1024 +5 %; book2 keeps 128: -0.4 % whole but +0.4 % on its 2-GPU share, and
  // book1 128: 64 +0.7 %, 256 +2 %; profiles/r6_grab_sweep.jsonl)
  const bool mesh_set = ft_set == (FT_SPHERE | FT_TRI | FT_METAL);
  p.grab_min = (uint32_t)std::max(1, env_int("RT_GRAB_MIN", f_lds ? (tree == 0 && ft_set == 0u ? 16 : 32) : (K <= 8u || mesh_set) ? 256 : 128));
  {  // drain splitting (k_fused's record-loop kernel): share when >= split_min samples are left
    const int sm = env_int("RT_SPLIT_MIN", 1);
    p.split_min = sm > 0 ? (uint32_t)sm : 0xFFFFFFFFu;  // 0: off (no lane has that many)
  }
  // partitioned chunk counters (rt_path.h grab_chunk): 64 partitions interleaved in
  // granules of 256 chunks; progress slices use one counter (their ranges are contiguous)
  p.parts_log2 = (uint32_t)std::min(6, std::max(0, env_int("RT_PARTS_LOG2", 6)));
  p.gran_log2 = (uint32_t)std::min(20, std::max(0, env_int("RT_GRAN_LOG2", 8)));
  p.wave_times = nullptr;
  p.recs_lds = f_recs ? 1u : 0u;
  p.seed = o.seed;
  p.ray_o = st->ray_o;
  p.ray_d = st->ray_d;
  p.hit = st->hit;
  p.path = st->path;
  p.pend = st->pend;
  p.pre = st->pre;

  p.stack = st->stack;
  p.queue[0] = st->queue[0];
  p.queue[1] = st->queue[1];
  p.ctr = st->ctr;
  p.accum = st->accum;
  p.csum = use_csum ? st->csum : nullptr;
  p.side = st->side;
  // |v| < 2^31 / ss: the ss-sample fixed-point sum of a pixel stays inside int64
  p.vlim = std::nextafter((float)(2147483648.0 / (double)std::max<uint32_t>(ss, 1u)), 0.0f);
  p.pflags = st->pflags;
  p.ostack = st->ostack;
  p.stack_cols = st->ostack_cols;

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
  std::vector<std::pair<int, int>> ev_ext, ev_shade, ev_fused;  // event index pairs
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
    HIP_OK(hipMemsetAsync(st->side, 0, 3 * (size_t)npix * sizeof(double), stream));
    HIP_OK(hipMemsetAsync(st->pflags, 0, (size_t)npix * sizeof(uint32_t), stream));
  }
  int iterations = 0;
  int n_ext = 0, n_sh = 0;
  // rt_progress: the fused render as `slices` launches over consecutive chunk
  // ranges, an event after each (the image does not depend on the split)
  const int slices = (mode == RT_MODE_FUSED && n_chunks > 0)
                         ? std::max(1, std::min(o.progress_slices, 1024))
                         : 1;
  if (slices > 1) p.parts_log2 = 0;
  while ((int)st->prog_events.size() < slices) {
    hipEvent_t e;
    HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    st->prog_events.push_back(e);
  }
  // rt_progress follows one render per scene: an rt_render call (slot 0) claims the
  // record when no other render holds it (rt_render_multi claims it for its shares)
  bool track = false;
  if (slot_id == 0) {
    std::lock_guard<std::mutex> lk(s->prog.mu);
    if (!s->prog.busy) {  // claimed: no return before prog_done below releases it
      s->prog.busy = 1;
      track = true;
    }
  }
  if (track) {
    std::lock_guard<std::mutex> lk(s->prog.mu);
    s->prog.total = (uint64_t)npix * ss;
    s->prog.done = 0;
    s->prog.device = o.device;
    s->prog.events.clear();
    s->prog.cum.clear();
    if (slices > 1)
      for (int sl = 0; sl < slices; ++sl) {
        s->prog.events.push_back((void*)st->prog_events[sl]);
        s->prog.cum.push_back((uint64_t)((double)s->prog.total *
                                         (double)((uint64_t)n_chunks * (sl + 1) / slices) /
                                         (double)n_chunks));
      }
    s->prog.busy = 1;
  }
  struct ProgressDone {  // every return path below ends the in-flight state
    Progress& p;
    bool track;
    bool ok = false;
    ~ProgressDone() {
      if (!track) return;
      std::lock_guard<std::mutex> lk(p.mu);
      if (ok) p.done = p.total;
      p.busy = 0;
    }
  } prog_done{s->prog, track};
  if (n_chunks > 0 && mode == RT_MODE_FUSED) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (prof) {
      if ((rc = next_event(&e0)) || (rc = next_event(&e1))) return rc;
      HIP_OK(hipEventRecord(e0, stream));
    }
    // debug: per-wave start/end clocks (100 MHz), segments and (RT_PHASES builds) phase
    // cycles -> binary file RT_WAVE_TIMES, kWaveRec u64 per wave
    std::string wt_file;
    const char* wt_path = tune_str("RT_WAVE_TIMES", &wt_file) ? wt_file.c_str() : nullptr;
    unsigned long long* wt = nullptr;
    const size_t n_waves = (size_t)fused_blocks * 4;
    if (wt_path && *wt_path) {
      HIP_OK(hipMalloc(&wt, kWaveRec * n_waves * sizeof(unsigned long long)));
      p.wave_times = wt;
    }
    void* args[] = {&p};
    for (int sl = 0; sl < slices; ++sl) {
      if (slices > 1) {  // chunks [n*sl/S, n*(sl+1)/S): the counter starts at the range
        p.n_chunks = (uint32_t)((uint64_t)n_chunks * (sl + 1) / slices);
        if (sl > 0)  // one partition (parts_log2 = 0 with slices): its counter is the head
          HIP_OK(hipMemsetD32Async((hipDeviceptr_t)&st->ctr->part[0],
                                   (int)((uint64_t)n_chunks * sl / slices), 1, stream));
      }
      HIP_OK(hipLaunchKernel(fused_kernel, dim3(fused_blocks), dim3(256), args, fused_lds, stream));
      HIP_OK(hipGetLastError());
      if (slices > 1) HIP_OK(hipEventRecord(st->prog_events[sl], stream));
    }
    p.n_chunks = n_chunks;
    if (wt) {
      std::vector<unsigned long long> h(kWaveRec * n_waves);
      HIP_OK(hipMemcpyAsync(h.data(), wt, h.size() * sizeof(h[0]), hipMemcpyDeviceToHost, stream));
      HIP_OK(hipStreamSynchronize(stream));
      HIP_OK(hipFree(wt));
      p.wave_times = nullptr;
      if (FILE* f = fopen(wt_path, "wb")) {
        fwrite(h.data(), sizeof(h[0]), h.size(), f);
        fclose(f);
      }
    }
    if (prof) {
      HIP_OK(hipEventRecord(e1, stream));
      ev_fused.push_back({ev_used - 2, ev_used - 1});
    }
    iterations = 1;
  } else if (n_chunks > 0) {
    hipLaunchKernelGGL(k_init, dim3((P + 255) / 256), dim3(256), 0, stream, p);
    HIP_OK(hipGetLastError());
    uint32_t n_est = std::min(P, n_chunks);
    const int kBatch = 4;
    while (n_est > 0) {
      for (int b = 0; b < kBatch; ++b) {
        if (iterations + 1 >= kMaxIt)
          return set_error(RT_ERR_UNSUPPORTED, "more than %d wavefront iterations", kMaxIt);
        const uint32_t ext_blocks = std::max<uint32_t>(
            1u, std::min<uint32_t>((n_est + 255) / 256, (uint32_t)st->resident_blocks));
        hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;
        if (prof) {
          if ((rc = next_event(&e0)) || (rc = next_event(&e1)) || (rc = next_event(&e2))) return rc;
          HIP_OK(hipEventRecord(e0, stream));
        }
        int it_arg = iterations;
        void* eargs[] = {&p, &it_arg};
        HIP_OK(hipLaunchKernel(extend_kernel, dim3(ext_blocks), dim3(256), eargs, 0, stream));
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
      uint32_t n_now[kXcd];
      HIP_OK(hipMemcpyAsync(n_now, &st->ctr->cnt[iterations % kMaxIt][0], sizeof n_now,
                            hipMemcpyDeviceToHost, stream));
      HIP_OK(hipStreamSynchronize(stream));
      n_est = 0;
      for (int x = 0; x < kXcd; ++x) n_est += n_now[x];
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
  if (gather && npix > 0)
    HIP_OK(hipMemcpyPeerAsync(gather->dst, gather->dst_device, dst, o.device,
                              3 * (size_t)npix * sizeof(float), stream));
  HIP_OK(hipStreamSynchronize(stream));
  prog_done.ok = true;
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
    stats->overflow_samples = hc.overflow;
    stats->extend_rays = hc.segments;
    stats->shade_rays = hc.segments;
    stats->ms_total = std::chrono::duration<double, std::milli>(t_end - t_start).count();
    stats->n_extend_launches = n_ext;
    stats->n_shade_launches = n_sh;
    stats->iterations = iterations;
    stats->rows = (int32_t)rows;
    stats->mode = mode;
    stats->path_slots = (int32_t)P;
    stats->kernel_features = mode == RT_MODE_FUSED ? (int32_t)ft_set : (int32_t)FT_ALL;
    stats->scene_features = (int32_t)feats;
    stats->tree_width = tree;
    stats->chunk_samples = (int32_t)K;
    stats->record_boxes = tree == 0 ? ds->brute_boxes : 0;
    stats->tuned = tuned;
    stats->chunk_records = p.csum ? 1 : 0;
    stats->lds_scene = mode == RT_MODE_FUSED ? (f_lds ? 1 : 0) : (lds_nodes ? 1 : 0);
    auto sum_ms = [&](const std::vector<std::pair<int, int>>& v, double* acc) -> int {
      for (auto& pr : v) {
        float ms = 0;
        HIP_OK(hipEventElapsedTime(&ms, st->events[pr.first], st->events[pr.second]));
        *acc += ms;
      }
      return RT_OK;
    };
    if (prof) {
      if ((rc = sum_ms(ev_ext, &stats->ms_extend)) || (rc = sum_ms(ev_shade, &stats->ms_shade)) ||
          (rc = sum_ms(ev_fused, &stats->ms_fused)))
        return rc;
    }
  }
  return RT_OK;
}

// rows of share i ([rows_per][W][3] at gather + i*rows_per*W*3) -> image rows r = i + n*k
__global__ __launch_bounds__(256) void k_deinterleave(const float* gather, float* out, uint32_t H,
                                                      uint32_t W, uint32_t n, uint32_t rows_per) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t row_floats = 3ull * W;
  if (i >= (uint64_t)H * row_floats) return;
  const uint32_t r = (uint32_t)(i / row_floats);
  const uint64_t x = i - (uint64_t)r * row_floats;
  out[i] = gather[((uint64_t)(r % n) * rows_per + r / n) * row_floats + x];
}

// rt_render_multi: share i (rows r % n == i, camera.go:119-122) on devices[i], one
// host thread and stream per share, each with its own render slot; the shares are
// peer-copied to devices[0] and de-interleaved there.
static int render_multi(rt_scene* scene, const rt_camera* cam, const rt_render_opts* opts,
                        const int32_t* devices, int32_t n, float* out_host, float* out_dev,
                        rt_stats* stats) {
  if (!scene || !cam || !devices || n <= 0)
    return set_error(RT_ERR_INVALID, "rt_render_multi: null argument or n <= 0");
  rt_render_opts o{};
  if (opts) o = *opts;
  if (o.nranks > 1 || o.rank != 0)
    return set_error(RT_ERR_INVALID, "rt_render_multi: shards the image itself (rank/nranks)");
  if (o.stream) return set_error(RT_ERR_INVALID, "rt_render_multi: one stream per share (opts.stream)");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return set_error(RT_ERR_DEVICE, "rt_render_multi: no HIP device available");
  for (int i = 0; i < n; ++i)
    if (devices[i] < 0 || devices[i] >= ndev)
      return set_error(RT_ERR_INVALID, "rt_render_multi: device %d of %d", devices[i], ndev);
  rt_camera_derived cd;
  int rc = rt_camera_derive(cam, &cd);
  if (rc) return rc;
  Scene* s = &scene->s;
  std::lock_guard<std::mutex> multi(s->multi_mu);
  const auto t0 = std::chrono::steady_clock::now();
  const uint32_t H = (uint32_t)cd.height, W = (uint32_t)cd.width, N = (uint32_t)n;
  const uint32_t rows_per = (H + N - 1) / N;
  const size_t gather_floats = (size_t)N * rows_per * W * 3, img_floats = (size_t)H * W * 3;
  const int d0 = devices[0];
  DeviceGuard dg;  // the caller's current device is restored on every return
  HIP_OK(hipSetDevice(d0));
  const size_t need = (gather_floats + img_floats) * sizeof(float);
  if (!s->multi_buf || s->multi_dev != d0 || s->multi_bytes < need) {
    if (s->multi_buf) {
      (void)hipSetDevice(s->multi_dev);
      (void)hipFree(s->multi_buf);
      s->multi_buf = nullptr;
      HIP_OK(hipSetDevice(d0));
    }
    HIP_OK(hipMalloc(&s->multi_buf, std::max<size_t>(need, 4)));
    s->multi_bytes = need;
    s->multi_dev = d0;
  }
  float* gbuf = (float*)s->multi_buf;
  float* img = out_dev ? out_dev : gbuf + gather_floats;
  // xGMI peer access both ways.  "Already enabled" is success; any other failure is
  // an error (the copies would silently fall back to staging through host memory).
  // Devices that report no peer path copy through the runtime's staged path.
  auto enable_peer = [](int from, int to) -> int {
    HIP_OK(hipSetDevice(from));
    const hipError_t e = hipDeviceEnablePeerAccess(to, 0);
    if (e == hipErrorPeerAccessAlreadyEnabled) {
      (void)hipGetLastError();  // clear the sticky "already enabled" status
      return RT_OK;
    }
    if (e != hipSuccess)
      return set_error(RT_ERR_DEVICE, "rt_render_multi: peer access %d -> %d: %s", from, to,
                       hipGetErrorString(e));
    return RT_OK;
  };
  for (int i = 1; i < n; ++i)
    if (devices[i] != d0) {
      int can_a = 0, can_b = 0;
      HIP_OK(hipDeviceCanAccessPeer(&can_a, devices[i], d0));
      HIP_OK(hipDeviceCanAccessPeer(&can_b, d0, devices[i]));
      if (can_a && (rc = enable_peer(devices[i], d0))) return rc;
      if (can_b && (rc = enable_peer(d0, devices[i]))) return rc;
    }
  HIP_OK(hipSetDevice(d0));
  // RCCL gather (RT_FLAG_GATHER_RCCL): communicators over the device list, cached
  const bool use_rccl = (o.flags & RT_FLAG_GATHER_RCCL) != 0;
  RcclGather* rg = nullptr;
  const size_t share_floats = (size_t)rows_per * W * 3;
  if (use_rccl) {
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < i; ++j)
        if (devices[i] == devices[j])
          return set_error(RT_ERR_INVALID, "rt_render_multi: RCCL gather needs distinct devices");
    if (!s->rccl) s->rccl = new RcclGather();
    rg = static_cast<RcclGather*>(s->rccl);
    if (rg->devs != std::vector<int>(devices, devices + n)) {
      rg->release();
      rg->devs.assign(devices, devices + n);
      rg->comms.assign(n, nullptr);
      const ncclResult_t r = ncclCommInitAll(rg->comms.data(), n, devices);
      if (r != ncclSuccess) {
        rg->comms.clear();
        rg->devs.clear();
        return set_error(RT_ERR_DEVICE, "rt_render_multi: ncclCommInitAll: %s", ncclGetErrorString(r));
      }
      rg->streams.assign(n, nullptr);
      rg->send.assign(n, nullptr);
      for (int i = 0; i < n; ++i) {
        HIP_OK(hipSetDevice(devices[i]));
        HIP_OK(hipStreamCreateWithFlags(&rg->streams[i], hipStreamNonBlocking));
      }
    }
    if (rg->send_floats < share_floats) {
      for (int i = 0; i < n; ++i) {
        HIP_OK(hipSetDevice(devices[i]));
        if (rg->send[i]) HIP_OK(hipFree(rg->send[i]));
        rg->send[i] = nullptr;
        HIP_OK(hipMalloc(&rg->send[i], std::max<size_t>(share_floats, 1) * sizeof(float)));
      }
      rg->send_floats = share_floats;
    }
    HIP_OK(hipSetDevice(d0));
  }
  // rt_progress: this call's shares are the tracked render unless another holds it.
  // Claimed only after every early return of the setup above; the guard is built in
  // the same statement sequence, so every return below releases it.
  bool track = false;
  {
    std::lock_guard<std::mutex> lk(s->prog.mu);
    if (!s->prog.busy) {
      track = true;
      s->prog.total = (uint64_t)H * W * cd.spp_sqrt * cd.spp_sqrt;
      s->prog.done = 0;
      s->prog.device = d0;
      s->prog.events.clear();  // no slice events: the shares add their samples when done
      s->prog.cum.clear();
      s->prog.busy = 1;
    }
  }
  struct ProgressDone {  // every return path below ends the tracked state
    Progress& p;
    bool track;
    bool ok = false;
    ~ProgressDone() {
      if (!track) return;
      std::lock_guard<std::mutex> lk(p.mu);
      if (ok) p.done = p.total;
      p.busy = 0;
    }
  } prog_done{s->prog, track};
  std::vector<rt_stats> st(n);
  std::vector<int> rcs(n, RT_OK);
  std::vector<std::string> errs(n);
  std::vector<std::thread> th;
  for (int i = 0; i < n; ++i)
    th.emplace_back([&, i] {
      rt_render_opts oi = o;
      oi.device = devices[i];
      oi.rank = i;
      oi.nranks = n;
      oi.progress_slices = 0;
      const Gather g = {gbuf + (size_t)i * rows_per * W * 3, d0};
      if (rg)  // the share's rows into its padded send buffer; the gather follows
        rcs[i] = render_impl(scene, cam, &oi, nullptr, rg->send[i], &st[i], 1 + i, nullptr);
      else
        rcs[i] = render_impl(scene, cam, &oi, nullptr, nullptr, &st[i], 1 + i, &g);
      if (rcs[i] != RT_OK) {
        errs[i] = rt_last_error();
      } else if (track) {  // rt_progress advances share by share
        std::lock_guard<std::mutex> lk(s->prog.mu);
        s->prog.done = std::min(s->prog.total, s->prog.done + st[i].samples);
      }
    });
  for (auto& t : th) t.join();
  for (int i = 0; i < n; ++i)
    if (rcs[i] != RT_OK) return set_error(rcs[i], "rt_render_multi share %d: %s", i, errs[i].c_str());
  if (rg && share_floats > 0) {
    // one collective: every share's [rows_per][W][3] tile to devices[0]'s gather buffer
    // (rank-major, the layout k_deinterleave reads); rows past a short share are padding
    ncclResult_t r = ncclGroupStart();
    for (int i = 0; r == ncclSuccess && i < n; ++i) {
      HIP_OK(hipSetDevice(devices[i]));
      r = ncclGather(rg->send[i], i == 0 ? (void*)gbuf : nullptr, share_floats, ncclFloat32, 0,
                     rg->comms[i], rg->streams[i]);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r == ncclSuccess) r = r2;
    if (r != ncclSuccess)
      return set_error(RT_ERR_DEVICE, "rt_render_multi: ncclGather: %s", ncclGetErrorString(r));
    for (int i = 0; i < n; ++i) {
      HIP_OK(hipSetDevice(devices[i]));
      HIP_OK(hipStreamSynchronize(rg->streams[i]));
    }
  }
  HIP_OK(hipSetDevice(d0));
  if (img_floats > 0) {
    hipLaunchKernelGGL(k_deinterleave, dim3((unsigned)((img_floats + 255) / 256)), dim3(256), 0,
                       (hipStream_t)0, gbuf, img, H, W, N, rows_per);
    HIP_OK(hipGetLastError());
    if (out_host)
      HIP_OK(hipMemcpy(out_host, img, img_floats * sizeof(float), hipMemcpyDeviceToHost));
  }
  HIP_OK(hipStreamSynchronize((hipStream_t)0));
  prog_done.ok = true;
  if (stats) {
    memset(stats, 0, sizeof *stats);
    *stats = st[0];
    stats->samples = stats->segments = stats->stack_pushes = stats->overflow_samples = 0;
    stats->extend_rays = stats->shade_rays = 0;
    stats->rows = 0;
    stats->ms_fused = stats->ms_extend = stats->ms_shade = 0;
    for (int i = 0; i < n; ++i) {
      stats->samples += st[i].samples;
      stats->segments += st[i].segments;
      stats->stack_pushes += st[i].stack_pushes;
      stats->overflow_samples += st[i].overflow_samples;
      stats->extend_rays += st[i].extend_rays;
      stats->shade_rays += st[i].shade_rays;
      stats->rows += st[i].rows;
      // the slowest share bounds the render
      stats->ms_fused = std::max(stats->ms_fused, st[i].ms_fused);
      stats->ms_extend = std::max(stats->ms_extend, st[i].ms_extend);
      stats->ms_shade = std::max(stats->ms_shade, st[i].ms_shade);
    }
    stats->ms_total =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return RT_OK;
}

}  // namespace rt

extern "C" {

int rt_render_multi(rt_scene* s, const rt_camera* cam, const rt_render_opts* opts,
                    const int32_t* devices, int32_t n, float* out_rgb, rt_stats* stats) {
  if (!out_rgb) return rt::set_error(RT_ERR_INVALID, "rt_render_multi: null output");
  return rt::render_multi(s, cam, opts, devices, n, out_rgb, nullptr, stats);
}

int rt_render_multi_device(rt_scene* s, const rt_camera* cam, const rt_render_opts* opts,
                           const int32_t* devices, int32_t n, float* out_rgb_device,
                           rt_stats* stats) {
  if (!out_rgb_device) return rt::set_error(RT_ERR_INVALID, "rt_render_multi_device: null output");
  return rt::render_multi(s, cam, opts, devices, n, nullptr, out_rgb_device, stats);
}


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

int rt_progress(const rt_scene* sc, uint64_t* done, uint64_t* total) {
  if (!sc || !done || !total) return rt::set_error(RT_ERR_INVALID, "rt_progress: null");
  rt::Progress& p = const_cast<rt_scene*>(sc)->s.prog;
  std::lock_guard<std::mutex> lk(p.mu);
  *total = p.total;
  *done = p.done;  // 0 while a render without slices is in flight; multi shares add theirs
  if (!p.busy || p.events.empty()) return RT_OK;
  if (hipSetDevice(p.device) != hipSuccess) return rt::set_error(RT_ERR_DEVICE, "rt_progress");
  for (size_t i = 0; i < p.events.size(); ++i) {  // slices complete in stream order
    if (hipEventQuery((hipEvent_t)p.events[i]) != hipSuccess) break;
    *done = p.cum[i];
  }
  return RT_OK;
}

int rt_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int rt_scene_export_qbvh(const rt_scene* sc, float* items, int32_t* n_items, float* nodes4,
                         int32_t* n_nodes4, uint32_t* root4) {
  if (!sc) return rt::set_error(RT_ERR_INVALID, "rt_scene_export_qbvh: null");
  const rt::HostScene& h = sc->s.h;
  std::vector<rt::F4> recs, qb;
  rt::build_leaf_records(h, recs);
  size_t n = 0;
  const int rc = rt::build_qbvh(h, recs, &qb, &n);
  if (rc != RT_OK) return rc;
  if (n_items) *n_items = (int32_t)n;
  if (n_nodes4) *n_nodes4 = (int32_t)(h.nodes4.size() / 8);
  if (root4) *root4 = h.root4;
  if (items && n) memcpy(items, qb.data(), n * 64);
  if (nodes4 && !h.nodes4.empty()) memcpy(nodes4, h.nodes4.data(), h.nodes4.size() * 16);
  return RT_OK;
}

}  // extern "C"
