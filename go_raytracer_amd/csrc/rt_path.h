// rt_path.h — per-path device logic shared by the wavefront and fused kernels:
// launch parameters, camera rays, closest-hit traversal, media, textures,
// light sampling and the shading core (one rayColor vertex, camera.go:293-331).
// The shading core is templated on where path state lives: HBM structure-of-
// arrays (wavefront kernels) or registers (fused persistent kernel).
#pragma once
#include "rt_kernels.h"

namespace rt {

constexpr int kLdsNodes = 384;   // 64-B slots staged in LDS per workgroup (24 KB): BVH nodes,
                                 // then the leaf records when both fit (LDS instantiation)
constexpr int kLdsWMax = 6;      // clamp-weight stack entries per lane kept in LDS (fused, max)
constexpr int kStack = 64;       // traversal stack entries per lane (LDS short stack + HBM overflow)
constexpr int kShortStack = 12;  // LDS entries per lane (column layout: [entry][thread])
constexpr int kShortStackMin = 6;  // smallest short stack of any kernel (fused lean set)
constexpr int kBruteMax = 48;      // scenes up to this many leaf entries skip the tree (fused)
constexpr int kMaxIt = 1 << 16;  // per-iteration counter slots (no per-iteration memsets)
constexpr int kXcd = 8;          // queue counters are sharded per XCD (blockIdx % 8)
constexpr int kMaxParts = 64;    // chunk-range partitions of the fused kernel (one counter each)
constexpr int kPartStride = 64;  // u32 between partition counters (256 B: own cache lines)

enum : uint32_t { F_PEND = 1u, F_PRE = 2u, F_NONFINITE = 4u };
// Path::flags above this bit: the sample count of the path's chunk (chunk_ids().count, set
// when the chunk starts), so the per-sample "last sample?" test needs no launch parameter
constexpr uint32_t kCountShift = 8;
// Path::flags bit 7 (kept by next_sample): the path runs samples split off another lane's
// chunk (k_fused's drain, split_samples); its sums go to the pixel with atomics, not to the
// chunk's record
constexpr uint32_t F_SPLIT = 0x80u;

#ifdef RT_NO_SPLIT_TREES
constexpr bool kSplitTrees = false;  // A/B builds: drain splitting in the record-loop kernel only
#else
constexpr bool kSplitTrees = true;
#endif
enum { OUT_DEAD = 0, OUT_ALIVE = 1, OUT_NEED_CHUNK = 2 };

struct Counters {
  unsigned long long segments;
  unsigned long long pushes;
  unsigned long long overflow;  // samples whose channel left the fixed-point range (add_sample)
  uint32_t chunk_head;
  uint32_t _pad[11];
  uint32_t part[kMaxParts * kPartStride];  // fused kernel: next position of partition p at [p * stride]
  uint32_t cnt[kMaxIt][kXcd];  // per-XCD queue lengths entering iteration i
};

// Division by a launch-invariant divisor: q = (t + ((n - t) >> s1)) >> s2 with
// t = mulhi(m, n) (round-up magic, exact for all 32-bit n and d >= 1; host side
// make_fastdiv in rt_render.hip; Hacker's Delight 10-8 with the add fix-up).
struct FastDiv {
  uint32_t m, s1, s2, d;
};
RT_D uint32_t fdiv(uint32_t n, const FastDiv& f) {
  const uint32_t t = __umulhi(f.m, n);
  return (t + ((n - t) >> f.s1)) >> f.s2;
}

struct Params {
  DevScene sc;
  FastDiv fd_width, fd_s;
  FastDiv fd_gchunks, fd_gpix;  // chunk order: groups of fd_gpix.d pixels x all sample blocks
  FastDiv fd_gchunks2;          // the tail phase's chunks per group (gpix x its blocks)
#ifdef RT_SWEEP_ORDER
  uint32_t gflip, gbase;        // group at sweep position q: (q ^ gflip) + gbase (0, 0: image
                                // order; ~0, groups: reversed, RT_SWEEP) -- and back (k_resolve)
#endif
  // camera (initialize camera.go:179-253, converted to fp32)
  float p00r[3], du[3], dv[3], cc[3], dku[3], dkv[3];  // p00r = pixel00 - center
  float bg[3];
  float recip_s, maxc;
  int s, defocus, max_depth;
  int width, rank, nranks;
  uint32_t npix;       // pixels of this rank
  uint32_t K;          // samples per chunk (first phase)
  uint32_t K2;         // samples per chunk of the tail phase (chunk ids >= n1)
  uint32_t S1;         // samples [0, S1) of every pixel in the first phase, [S1, ss) in the tail
  uint32_t n1;         // chunks of the first phase (npix * S1 / K)
  uint32_t n_chunks;
  uint32_t P;          // path slots (stack column count)
  uint32_t ss;         // s*s
  int step_budget;     // fused: traversal steps per scheduling round
  uint32_t shade_min;  // fused: lanes that must be waiting before a wave shades
  uint32_t grab_min;   // fused: chunks a wave takes per refill of its batch (>= 1)
  uint32_t parts_log2; // fused: the chunk range is split over 2^parts_log2 partitions ...
  uint32_t gran_log2;  // ... interleaved in granules of 2^gran_log2 chunks (grab_chunk)
  uint32_t split_min;  // fused drain: a lane with >= split_min samples left shares them (0: off)
  unsigned long long* wave_times;  // debug (RT_WAVE_TIMES): per wave {start, end, segments}
  uint32_t recs_lds;   // leaf records cached in LDS after the nodes (stage_nodes)
  uint64_t seed;
  // wavefront state (SoA, slot-indexed)
  F4* ray_o;   // origin | time
  F4* ray_d;   // direction | 0
  F4* hit;     // t, u, v, prim ref bits
  uint2* path; // chunk, packed(j:12 | vertex:8 | nstack:8 | flags:4)
  F4* pend;    // pending clamp-vertex weight (top of the weight stack)
  F4* pre;     // camera-side product of specular attenuations
  F4* stack;   // [vertex][slot] clamp-vertex weights spilled to HBM
  uint32_t* queue[2];  // each kXcd segments of P entries
  Counters* ctr;
  unsigned long long* accum;  // 3 planes x npix: per-sample fixed point 2^-32, summed exactly
  unsigned long long* csum;   // fused: per-chunk sums, 4 x u64 per chunk id (x, y, z, 0), each
                              // stored once by the lane that ran the chunk (SampleAcc::flush);
                              // k_resolve adds a pixel's chunks.  Null: atomics into accum
  double* side;               // 3 planes x npix: samples outside the fixed-point range (fp64)
  float vlim;                 // fixed-point range per sample: |v| < 2^31 / ss (no int64 wrap)
  uint32_t* pflags;           // per pixel NaN (bits 0-2) / +Inf (bits 3-5) / -Inf (bits 6-8)
  uint32_t* ostack;            // traversal-stack overflow [kStack - kShortStackMin][stack_cols]
  uint32_t stack_cols;         // = launched threads of the traversal kernel
  F4* trace;                  // debug path trace (3 F4 per vertex) or null
  uint32_t trace_gpix, trace_sample;
  int trace_cap;
};

RT_D uint32_t pack_path(uint32_t j, uint32_t k, uint32_t nst, uint32_t flags) {
  return (j & 0xFFFu) | ((k & 0xFFu) << 12) | ((nst & 0xFFu) << 20) | ((flags & 0xFu) << 28);
}

// address-space-typed loads and stores (see trace_world's note)
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) float lds_f32;
typedef __attribute__((address_space(1))) uint32_t glb_u32;
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4f lds_v4;
typedef __attribute__((address_space(1))) v4f glb_v4;
typedef float v2f __attribute__((ext_vector_type(2)));
// 16 B from a wave-uniform address through the scalar cache (s_load into SGPRs):
// for tables indexed by a loop counter or a broadcast index
RT_D F4 ld_cst(const F4* p) {
  typedef __attribute__((address_space(4))) const v4f cst_v4;
  const v4f v = *(const cst_v4*)p;
  return {v.x, v.y, v.z, v.w};
}
RT_D F4 ld_lds(const F4* p) {
  const v4f v = *(const lds_v4*)p;
  return {v.x, v.y, v.z, v.w};
}
RT_D F4 ld_glb(const F4* p) {
  const v4f v = *(const glb_v4*)p;
  return {v.x, v.y, v.z, v.w};
}
RT_D void st_lds(F4* p, F4 v) { *(lds_v4*)p = v4f{v.x, v.y, v.z, v.w}; }
// s_waitcnt vmcnt(0) (gfx9 encoding: expcnt/lgkmcnt left unconstrained).  Placed
// at the end of a RARE global-memory branch whose result merges with an LDS
// branch: without it the compiler's wait lands after the merge, on the common
// LDS path too, where it drains every outstanding store and atomic.
RT_D void wait_vm() { __builtin_amdgcn_s_waitcnt(0x0F70); }
RT_D void st_glb(F4* p, F4 v) { *(glb_v4*)p = v4f{v.x, v.y, v.z, v.w}; }

// m ? b : a, bitwise (v_bitop3_b32, truth table 0xD8 over (a, b, m)).  With m a sign mask
// this is a select in one full-rate instruction: hipcc turns the same C expression into
// v_cmp + v_cndmask, both of which issue at half rate or less on gfx950
// (profiles/r4_instr_rate.jsonl)
RT_D uint32_t pick_by(uint32_t a, uint32_t b, uint32_t m) { return __builtin_amdgcn_bitop3_b32(a, b, m, 0xD8); }
// a & ~m as one v_bitop3 (written as `a & ~m` with m a spread sign, LLVM turns it into a
// compare and a v_cndmask_b32_e32 on vcc, which issues at ~23 cycles per wave64 on gfx950
// whatever the occupancy: tools/instr_rate.hip, profiles/r6_instr_rate.jsonl)
RT_D uint32_t and_not(uint32_t a, uint32_t m) { return __builtin_amdgcn_bitop3_b32(a, m, 0u, 0x30); }
// all ones when x < 0 (sign bit set), else 0: -0 and negative NaNs count as negative
RT_D uint32_t neg_mask(float x) { return (uint32_t)((int32_t)__float_as_uint(x) >> 31); }
RT_D uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// Debug build (-DRT_PHASES, tools/phase_probe.py): shader-clock cycles each wave
// spends per phase of the fused loop, accumulated by lane 0 in LDS and written with
// the RT_WAVE_TIMES record.  Timing perturbs the kernel (s_memtime waits): use the
// shares, not the absolute cycles.
enum { PH_GRAB, PH_TRAV, PH_MEDIA, PH_SHADE, PH_TEX, PH_LIGHT, PH_TERM, PH_LOOP,
       PH_TRAV_LANES, PH_TRAV_ROUNDS, PH_SHADE_LANES, PH_SHADE_ROUNDS, PH_STEP_LANES,
       PH_STEP_WAVE, PH_QNODE_LANES, PH_QLEAF_LANES, PH_QMIXED, PH_QITERS,
       // compressed-BVH steps: lanes on the first active lane's item, distinct items per
       // iteration, and lanes on items of BFS levels 0-3 (item < 85) / 4-5 (item < 1365)
       PH_QSAME, PH_QUNIQ, PH_QTOP, PH_QMID, PH_N = 22 };
constexpr int kWaveRec = 4 + PH_N;  // {start, end, segments, pad, phases...} per wave
#ifdef RT_PHASES
__shared__ unsigned long long g_ph[4][PH_N];
RT_D unsigned long long ph_now() { return __builtin_readcyclecounter(); }
RT_D void ph_acc(int i, unsigned long long v) {  // first active lane (divergent code too)
  if (lane_id() == (uint32_t)(__ffsll((long long)__ballot(1)) - 1)) g_ph[threadIdx.x >> 6][i] += v;
}
#define PH_T(v) const unsigned long long v = ::rt::ph_now()
#define PH_ADD(i, v) ::rt::ph_acc(i, ::rt::ph_now() - (v))
#define PH_CNT(i, n) ::rt::ph_acc(i, (unsigned long long)(n))
// traversal steps: summed over the lanes, and the wave's maximum (loop trips)
RT_D void ph_steps(int n) {
  atomicAdd(&g_ph[threadIdx.x >> 6][PH_STEP_LANES], (unsigned long long)n);
  int m = n;
  for (int off = 32; off > 0; off >>= 1) m = max(m, __shfl_xor(m, off));
  ph_acc(PH_STEP_WAVE, (unsigned long long)m);
}
#else
#define PH_T(v)
#define PH_ADD(i, v)
#define PH_CNT(i, n)
#endif
RT_D uint32_t prefix_count(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
RT_D uint32_t wave_uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// chunk c -> (local pixel, global pixel, first sample).  The rank's pixels are
// taken in groups of G = fd_gpix.d consecutive pixels (G divides npix); a group's
// chunks are pixel-fastest over all its sample blocks, so a wave's consecutive
// chunks are adjacent pixels (coherent camera rays, different accumulators) and the
// chunks in flight cover only a few groups of the image (a small working set of the
// scene for the camera rays and their first bounces) instead of the whole image.
// G = npix is the image-wide pixel-fastest order.
struct Ids {
  uint32_t lpix, gpix, row, col, sample0, count;
};
typedef __attribute__((address_space(4))) const Params cst_params;
// The launch parameters re-read through the scalar cache where they are used: the asm
// barrier hides that the pointer is the kernel-argument segment's, so the compiler
// cannot hoist the loads to the kernel entry and hold the values in SGPRs across the
// whole loop (where they spill to VGPR lanes).
RT_D const cst_params* kparams() {
  const cst_params* p = (const cst_params*)__builtin_amdgcn_kernarg_segment_ptr();
  __asm__ volatile("" : "+s"(p));
  return p;
}
// Two phases (render_impl): chunk ids [0, n1) cover samples [0, S1) of every pixel in
// chunks of K, ids [n1, n_chunks) the rest in chunks of K2 <= K, both in row-group order.
// The partitioned grab hands out the first phase before the tail, so the render's last
// chunks are short (the tail that idles lanes) while most samples pay the per-chunk cost of
// the large K.  `sub` is the sample block in its phase's units.
// (the tail's parameters are read from the kernel-argument segment where used, kparams:
// held in SGPRs for the whole kernel they cost the mesh and book1 kernels ~45 SGPR spills)
RT_D uint32_t chunk_pixel(const Params& P, uint32_t chunk, uint32_t& sub) {
  const cst_params* kp = kparams();
  const uint32_t n1 = kp->n1;
  const bool tail = chunk >= n1;
  const uint32_t c = tail ? chunk - n1 : chunk;
  const FastDiv fg = tail ? FastDiv{kp->fd_gchunks2.m, kp->fd_gchunks2.s1, kp->fd_gchunks2.s2,
                                    kp->fd_gchunks2.d}
                          : P.fd_gchunks;
  const uint32_t qs = fdiv(c, fg);
  const uint32_t r = c - qs * fg.d;
#ifdef RT_SWEEP_ORDER  // (opt-in build: RT_SWEEP=reverse, DESIGN.md §8 "Sweep order")
  const uint32_t q = (qs ^ kp->gflip) + kp->gbase;  // the group at this sweep position
#else
  const uint32_t q = qs;
#endif
  sub = fdiv(r, P.fd_gpix);
  return q * P.fd_gpix.d + (r - sub * P.fd_gpix.d);
}
// ONE: a launch without a tail phase (S1 = ss), with the launch parameters held in SGPRs:
// the record-loop kernel, whose chunk starts lost 3 % to the tail mapping's kernel-argument
// loads (profiles/r4_tail_code_ab.jsonl); render_impl never gives it a tail
template <bool ONE = false>
RT_D Ids chunk_ids(const Params& P, uint32_t chunk) {
  Ids r;
  uint32_t sub;
  if (ONE) {
    const uint32_t q = fdiv(chunk, P.fd_gchunks);
    const uint32_t rr = chunk - q * P.fd_gchunks.d;
    sub = fdiv(rr, P.fd_gpix);
    r.lpix = q * P.fd_gpix.d + (rr - sub * P.fd_gpix.d);
    const uint32_t row_l = fdiv(r.lpix, P.fd_width);
    r.col = r.lpix - row_l * (uint32_t)P.width;
    r.row = row_l * (uint32_t)P.nranks + (uint32_t)P.rank;
    r.gpix = r.row * (uint32_t)P.width + r.col;
    r.sample0 = sub * P.K;
    r.count = min(P.K, P.ss - r.sample0);
    return r;
  }
  r.lpix = chunk_pixel(P, chunk, sub);
#ifdef RT_ABLATE_REVERSED  // timing ablation only (wrong images): the rank's pixels traced in reverse order
  const uint32_t lrev = (uint32_t)P.npix - 1u - r.lpix;
  uint32_t row_l = fdiv(lrev, P.fd_width);
  r.col = lrev - row_l * (uint32_t)P.width;
#else
  uint32_t row_l = fdiv(r.lpix, P.fd_width);
  r.col = r.lpix - row_l * (uint32_t)P.width;
#endif
  r.row = row_l * (uint32_t)P.nranks + (uint32_t)P.rank;
  r.gpix = r.row * (uint32_t)P.width + r.col;
  const cst_params* kp = kparams();
  const bool tail = chunk >= kp->n1;
  const uint32_t S1 = kp->S1, K2 = kp->K2;
  r.sample0 = tail ? S1 + sub * K2 : sub * P.K;
  r.count = tail ? min(K2, P.ss - r.sample0) : min(P.K, S1 - r.sample0);
  return r;
}

// The camera constants in LDS (every kernel that starts samples stages them once,
// stage_camera): read with broadcast ds_reads where a ray starts instead of held in
// SGPRs for the whole kernel (the fused kernels run out of SGPRs and spill them to
// VGPR lanes, one v_readlane per use).  [0] pixel00 - center | 1/s, [1] du | fd_s.m,
// [2] dv | fd_s shifts, [3] center | s, [4] defocus u | defocus flag, [5] defocus v.
__shared__ F4 g_cam[6];
// the dynamic LDS of the fused kernels (k_fused's lnodes: tree, records, shade table)
extern __shared__ F4 g_dyn_lds[];
// Kernels that read the camera from g_cam (round 2, against SGPR-resident constants): the
// book2 and mesh sets (C4 -3.6 %, C5 -2.3 %, fewer SGPR and VGPR spills); the C2 and C3
// kernels lost from it (their VGPR budget takes the loaded constants: C2 +26 %)
constexpr bool cam_lds(uint32_t ft) {
  return ft == (FT_SPHERE | FT_TRI | FT_METAL) ||
         ft == FT_SET_BOOK2;
}
// Where a kernel reads the camera constants: 1 = g_cam (book2 set), 2 = scalar loads from
// the kernel-argument segment where a ray starts (kparams: SGPRs live only there), 0 = the
// SGPRs the compiler holds P in for the whole kernel (A/B builds: -DRT_CAM_SGPR).  Against
// 0, mode 2 took C2's SGPR spills to VGPR lanes from 78 to 34 and C3's from 101 to 32: C2
// -1.9 / -4.6 %, C3 -2.1 / -2.5 % (two boxes); against 1, C5 -2.0 / -2.2 % but C4 +1.1 %
// (profiles/r3_cam_kernarg_ab.jsonl); images bit-identical.
constexpr int cam_mode(uint32_t ft) {
#ifdef RT_CAM_SGPR
  return cam_lds(ft) ? 1 : 0;
#else
  return ft == FT_SET_BOOK2 ? 1 : 2;
#endif
}
RT_D void stage_camera(const Params& P) {  // before a __syncthreads of every thread
  if (threadIdx.x == 0) {
    g_cam[0] = {P.p00r[0], P.p00r[1], P.p00r[2], P.recip_s};
    g_cam[1] = {P.du[0], P.du[1], P.du[2], bitsf(P.fd_s.m)};
    g_cam[2] = {P.dv[0], P.dv[1], P.dv[2], bitsf(P.fd_s.s1 | (P.fd_s.s2 << 8))};
    g_cam[3] = {P.cc[0], P.cc[1], P.cc[2], bitsf((uint32_t)P.s)};
    g_cam[4] = {P.dku[0], P.dku[1], P.dku[2], bitsf((uint32_t)P.defocus)};
    g_cam[5] = {P.dkv[0], P.dkv[1], P.dkv[2], 0.0f};
  }
}

// getRay camera.go:256-270 + sampleSquareStratified :277-282 + defocusDiskSample :285-290;
// r = rt_rng_draw(seed, gpix, sample, RT_STREAM_CAMERA), drawn by the caller.
// CAM: where the constants come from (cam_mode): P (0), g_cam (1) or the kernarg segment (2).
template <int CAM>
RT_D void camera_ray_r(const Params& P, const Ids& id, uint32_t sample, const rt_u32x4& r, f3& o,
                       f3& d, float& time) {
  F4 c0, c1, c2, c3;
  FastDiv fd_s;
  uint32_t s;
  bool defocus;
  if constexpr (CAM == 1) {
    c0 = ld_lds(&g_cam[0]), c1 = ld_lds(&g_cam[1]), c2 = ld_lds(&g_cam[2]), c3 = ld_lds(&g_cam[3]);
    const uint32_t sh = fbits(c2.w);
    s = fbits(c3.w);
    fd_s = {fbits(c1.w), sh & 0xFFu, sh >> 8, s};
    defocus = fbits(ld_lds(&g_cam[4]).w) != 0u;
  } else if constexpr (CAM == 2) {
    const cst_params* kp = kparams();
    c0 = {kp->p00r[0], kp->p00r[1], kp->p00r[2], kp->recip_s};
    c1 = {kp->du[0], kp->du[1], kp->du[2], 0.0f};
    c2 = {kp->dv[0], kp->dv[1], kp->dv[2], 0.0f};
    c3 = {kp->cc[0], kp->cc[1], kp->cc[2], 0.0f};
    fd_s = {kp->fd_s.m, kp->fd_s.s1, kp->fd_s.s2, kp->fd_s.d};
    s = (uint32_t)kp->s;
    defocus = kp->defocus != 0;
  } else {
    c0 = {P.p00r[0], P.p00r[1], P.p00r[2], P.recip_s};
    c1 = {P.du[0], P.du[1], P.du[2], 0.0f};
    c2 = {P.dv[0], P.dv[1], P.dv[2], 0.0f};
    c3 = {P.cc[0], P.cc[1], P.cc[2], 0.0f};
    fd_s = P.fd_s;
    s = (uint32_t)P.s;
    defocus = P.defocus != 0;
  }
  uint32_t si = fdiv(sample, fd_s), sj = sample - si * s;
  float px = (((float)sj + rt_unit_f(r.v[0])) * c0.w) - 0.5f;
  float py = (((float)si + rt_unit_f(r.v[1])) * c0.w) - 0.5f;
  float fx = (float)id.col + px, fy = (float)id.row + py;
  // pixelSample - rayOrigin rearranged as (pixel00 - center) + du*fx + dv*fy - disk:
  // the same vector without fp32 cancellation against large camera coordinates
  d = mk3(c0.x + c1.x * fx + c2.x * fy, c0.y + c1.y * fx + c2.y * fy, c0.z + c1.z * fx + c2.z * fy);
  o = mk3(c3.x, c3.y, c3.z);
  if (defocus) {
    F4 c4, c5;
    if constexpr (CAM == 1) {
      c4 = ld_lds(&g_cam[4]), c5 = ld_lds(&g_cam[5]);
    } else if constexpr (CAM == 2) {
      const cst_params* kp = kparams();
      c4 = {kp->dku[0], kp->dku[1], kp->dku[2], 0.0f};
      c5 = {kp->dkv[0], kp->dkv[1], kp->dkv[2], 0.0f};
    } else {
      c4 = {P.dku[0], P.dku[1], P.dku[2], 0.0f};
      c5 = {P.dkv[0], P.dkv[1], P.dkv[2], 0.0f};
    }
    // the disk's two uniforms are the halves of camera word [3] (rt_rng.h): no second
    // Philox call per defocused camera ray (C3, C5)
    f3 dk = uniform_disk(rt_unit16_hi_f(r.v[3]), rt_unit16_lo_f(r.v[3]));
    f3 off = mk3(c4.x, c4.y, c4.z) * dk.x + mk3(c5.x, c5.y, c5.z) * dk.y;
    o = o + off;
    d = d - off;
  }
  time = rt_unit_f(r.v[2]);
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
// LDS = true: the whole node array is staged in LDS (ds_read_b128); false: nodes
// come from HBM/L2 (global_load_dwordx4).  The two are separate instantiations:
// mixing both sources in one loop makes hipcc merge them into flat loads.
// The traversal stack lives in LDS (kShortStack entries per lane, one column
// per thread: conflict-free ds_read/write_b32) and overflows to HBM.
// Explicit address spaces: with generic pointers hipcc selects between the two
// bases and emits a flat load (slower, counts against both vmcnt and lgkmcnt).
struct TravStack {
  uint32_t* lds;     // &lds_stack[0][threadIdx.x], stride blockDim.x
  uint32_t* ovf;     // &ostack[slot], stride cols
  uint32_t cols;
  int nshort;        // LDS entries (a compile-time constant of each kernel)
#ifdef RT_COUNT_TRAV_OVF
  unsigned long long* dbg;  // debug builds: HBM overflow pushes, into Counters::pushes
#endif
  RT_D void push(int sp, uint32_t v) const {
    if (sp < nshort) {
      ((lds_u32*)lds)[sp * 256] = v;
    } else {
      ((glb_u32*)ovf)[(size_t)(sp - nshort) * cols] = v;
#ifdef RT_COUNT_TRAV_OVF
      if (dbg) atomicAdd(dbg, 1ull);
#endif
    }
  }
  RT_D uint32_t pop(int sp) const {
    uint32_t v;
    if (sp < nshort) {
      v = ((lds_u32*)lds)[sp * 256];
    } else {
      v = ((glb_u32*)ovf)[(size_t)(sp - nshort) * cols];
      wait_vm();
    }
    return v;
  }
};

// Resumable closest-hit traversal (replaces BVHNode.Hit bvh.go:69-82 +
// HittableList.Hit hittable.go:122-138 + AABB.Hit aabb.go:90-113).  One step =
// one inner node or one leaf; the fused kernel runs a bounded number of steps
// per scheduling round so a lane that finishes early does not idle until the
// wave's slowest ray is done (see k_fused).
constexpr uint32_t TRAV_DONE = 0xFFFFFFFFu;  // never a node or leaf code (host_bvh.cpp)
struct Trav {
  f3 inv;
  uint32_t cur;
  int sp;        // stack depth; entry sp-1 lives in `top`, entries below in TravStack
  uint32_t top;  // register copy of the top entry: a pop uses it at once and refills it
                 // from LDS in the background (the refill lands while the popped
                 // subtree is traversed), taking the LDS latency off the pop
  Hit best;
  // a triangle the last round's fp32 test rejected within its rounding error of an edge
  // (hit_tri_rec_m `near`), for tri_hit64 after trav_steps; PRIM_NONE: none.  Set only by the
  // round that ends on it, consumed before the next one (retest_near)
  uint32_t pend;
};
// the fp64 re-test of a round's near-edge rejection (hit_tri_rec_m): taken when it hits
// within the closest hit so far, as the fp32 test would have taken it.  Divergent and rare.
template <uint32_t FT>
RT_D void retest_near(const DevScene& sc, f3 o, f3 d, float tmin, Trav& tr) {
  if constexpr (HAS(FT_TRI)) {
    if (tr.pend != PRIM_NONE) {
      float t, u, v;
      if (tri_hit64(sc, tr.pend & 0x3FFFFFFFu, o, d, tmin, tr.best.t, t, u, v)) tr.best = {t, u, v, tr.pend};
    }
  }
}
// A new ray: the traversal state, and the spheres kept out of the BVH (radius >=
// kBigSphereR: the ground spheres of book1 and the mesh scene) tested first, in fp64, by
// every lane at once (a uniform loop over scalar-loaded records), so the BVH's sphere
// leaves are all small and tested in fp32 (hit_sphere_rec32) without a divergent fp64
// branch.  Their hit's v = -1 tells finish_hit that t is already fp64-solved.
template <uint32_t FT>
RT_D void trav_init(const DevScene& sc, f3 o, f3 d, float time, Trav& tr) {
  tr.inv = mk3(rcp(d.x), rcp(d.y), rcp(d.z));
  tr.cur = sc.root == PRIM_NONE ? TRAV_DONE : sc.root;
  tr.sp = 0;
  tr.top = 0;
  tr.best = {kInf, 0.0f, 0.0f, PRIM_NONE};
  if (HAS(FT_SPHERE))
    for (int i = 0; i < sc.n_big; ++i) {
      const F4* q = sc.big_recs + 4 * (size_t)__builtin_amdgcn_readfirstlane(i);
      const F4 rec[4] = {ld_cst(q), ld_cst(q + 1), ld_cst(q + 2), ld_cst(q + 3)};
      float t;
      if (hit_sphere_rec64(rec, o, d, time, 0.001f, tr.best.t, t))
        tr.best = {t, 0.0f, -1.0f, fbits(rec[0].w)};
    }
}

// LDS instantiation: lnodes holds the node array and, when recs_lds, the leaf
// records right after it (uniform flag: both load forms exist, one runs)
// one fp16 half of a 32-bit word as fp32 (an fma on it compiles to v_fma_mix_f32)
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
template <int H> RT_D float half_of(uint32_t w) { return (float)__builtin_bit_cast(h2v, w)[H]; }

// The compressed BVH4 node test (trav_steps QN): the four children's entry distances
// (inf: missed) and codes, sorted front to back
RT_D void qnode_children(const F4 v[4], f3 o, f3 inv, float tmin, float tmax, float tn[4],
                         uint32_t ch[4]) {
  // t = off * inv + (corner - o) * inv per plane (v_fma_mix_f32 on the fp16 offset).
  // Planes come as (lo 0|1, lo 2|3, hi 0|1, hi 2|3) per axis; the near pair is lo when
  // inv >= 0 and hi otherwise (a sign-mask select per word), so no min/max per axis.
  const float bx = (v[0].x - o.x) * inv.x, by = (v[0].y - o.y) * inv.y,
              bz = (v[0].z - o.z) * inv.z;
  const uint32_t info = fbits(v[0].w);
  const uint32_t base = info & 0x0FFFFFFFu, lmask = info >> 28;
  const uint32_t mx = neg_mask(inv.x), my = neg_mask(inv.y), mz = neg_mask(inv.z);
  const uint32_t nx[2] = {pick_by(fbits(v[1].x), fbits(v[1].z), mx), pick_by(fbits(v[1].y), fbits(v[1].w), mx)};
  const uint32_t fx[2] = {pick_by(fbits(v[1].z), fbits(v[1].x), mx), pick_by(fbits(v[1].w), fbits(v[1].y), mx)};
  const uint32_t ny[2] = {pick_by(fbits(v[2].x), fbits(v[2].z), my), pick_by(fbits(v[2].y), fbits(v[2].w), my)};
  const uint32_t fy[2] = {pick_by(fbits(v[2].z), fbits(v[2].x), my), pick_by(fbits(v[2].w), fbits(v[2].y), my)};
  const uint32_t nz[2] = {pick_by(fbits(v[3].x), fbits(v[3].z), mz), pick_by(fbits(v[3].y), fbits(v[3].w), mz)};
  const uint32_t fz[2] = {pick_by(fbits(v[3].z), fbits(v[3].x), mz), pick_by(fbits(v[3].w), fbits(v[3].y), mz)};
  auto child = [&](auto hk, int k) {
    constexpr int H = decltype(hk)::value;
    const int w = k >> 1;
    const float tx0 = fmaf(half_of<H>(nx[w]), inv.x, bx), tx1 = fmaf(half_of<H>(fx[w]), inv.x, bx);
    const float ty0 = fmaf(half_of<H>(ny[w]), inv.y, by), ty1 = fmaf(half_of<H>(fy[w]), inv.y, by);
    const float tz0 = fmaf(half_of<H>(nz[w]), inv.z, bz), tz1 = fmaf(half_of<H>(fz[w]), inv.z, bz);
    const float t0 = fmaxf(fmaxf(tx0, ty0), fmaxf(tz0, tmin));
    const float t1 = fminf(fminf(tx1, ty1), fminf(tz1, tmax));
    tn[k] = bitsf(pick_by(fbits(t0), 0x7F800000u, neg_mask(t1 * 1.00000024f - t0)));
    ch[k] = (base + (uint32_t)k) | (((lmask >> k) & 1u) << 31);
  };
  child(std::integral_constant<int, 0>{}, 0);
  child(std::integral_constant<int, 1>{}, 1);
  child(std::integral_constant<int, 0>{}, 2);
  child(std::integral_constant<int, 1>{}, 3);
  auto cx = [&](int a, int b) {  // as the 128-B path's network
    const uint32_t m = neg_mask(tn[b] - tn[a]);
    const uint32_t ta = fbits(tn[a]), tb = fbits(tn[b]);
    const uint32_t ca = ch[a], cb = ch[b];
    tn[a] = bitsf(pick_by(ta, tb, m));
    tn[b] = bitsf(pick_by(tb, ta, m));
    ch[a] = pick_by(ca, cb, m);
    ch[b] = pick_by(cb, ca, m);
  };
  cx(0, 1);
  cx(2, 3);
  cx(0, 2);
  cx(1, 3);
  cx(1, 2);
}

// The compressed BVH4's root tested where a ray starts (trav_init), from scalar loads: every
// lane reads the same 64-B item 0, so s_load_dwordx4 x 4 through the scalar cache instead of
// one of the ~8 vector-memory steps per segment (C5's traversal is bound by the vector-memory
// path), and the traversal begins at the nearest child with the others on the
// stack, exactly as the step would have left it (same qnode_children arithmetic: same image).
RT_D void trav_root_q(const TravStack& stack, f3 o, float tmin, Trav& tr) {
  if (tr.cur != 0u) return;  // item 0 is the root (render_impl, tree 5)
  const F4* rn = kparams()->sc.nodes;
  const F4 v[4] = {ld_cst(rn), ld_cst(rn + 1), ld_cst(rn + 2), ld_cst(rn + 3)};
  float tn[4];
  uint32_t ch[4];
  qnode_children(v, o, tr.inv, tmin, tr.best.t, tn, ch);
  if (tn[0] == kInf) {
    tr.cur = TRAV_DONE;
    return;
  }
  lds_u32* q = (lds_u32*)stack.lds;  // sp = 0: entries 0-2 are in the short stack
  int sp = 0;
  q[sp * 256] = ch[3];
  sp += tn[3] != kInf;
  q[sp * 256] = ch[2];
  sp += tn[2] != kInf;
  q[sp * 256] = ch[1];
  sp += tn[1] != kInf;
  tr.sp = sp;
  tr.cur = ch[0];
}

// QN: the compressed BVH4 (host_qbvh.cpp, rt_device.h "compressed BVH4 node"), 64-B
// items read through L1/L2; cur = item index, LEAF_BIT set for a single-prim leaf record
template <bool LDS, uint32_t FT, bool W4 = true, bool QN = false>
RT_D int trav_steps(const DevScene& sc, const F4* lnodes, bool recs_lds, const TravStack& stack,
                     f3 o, f3 d, float time, float tmin, Trav& tr, int budget) {
  uint32_t cur = tr.cur;
  int sp = tr.sp;
  uint32_t top = tr.top;
  // The register top is used with the BVH2 only (tiny LDS scenes, +1.2 % on C2):
  // with the BVH4 its extra store per push cost C3-C5 1-2 %.
  constexpr bool kTopReg = !W4;
  // push v: with kTopReg the old top goes down to the stack proper (entry sp-1)
  auto push = [&](uint32_t v) {
    if (kTopReg) {
      if (sp > 0) stack.push(sp - 1, top);
      top = v;
      ++sp;
    } else {
      stack.push(sp++, v);
    }
  };
  const f3 inv = tr.inv;
  // a near-edge rejection of this round, re-tested in fp64 after it (retest_near); a second
  // one ends the round before its step, which the next round repeats
  uint32_t pend = PRIM_NONE;
  int n = 0;
  for (; n < budget && cur != TRAV_DONE; ++n) {
    if constexpr (QN) {
      // One 64-B item per step, node or leaf record alike (4 x 16 B, issued together).
      const bool leaf = (cur & LEAF_BIT) != 0u;
#ifdef RT_PHASES
      {  // node / leaf steps of this iteration, and whether both kinds ran in it
        const unsigned long long ml = __ballot(leaf), mn = __ballot(!leaf);
        PH_CNT(PH_QLEAF_LANES, __popcll(ml));
        PH_CNT(PH_QNODE_LANES, __popcll(mn));
        PH_CNT(PH_QMIXED, (ml && mn) ? 1 : 0);
        PH_CNT(PH_QITERS, 1);
        const uint32_t item = cur & 0x0FFFFFFFu;
        const uint32_t first_item = __builtin_amdgcn_readfirstlane(item);
        PH_CNT(PH_QSAME, __popcll(__ballot(item == first_item)));
        PH_CNT(PH_QTOP, __popcll(__ballot(item < 85u)));
        PH_CNT(PH_QMID, __popcll(__ballot(item >= 85u && item < 1365u)));
        unsigned long long left = __ballot(1);
        uint32_t uniq = 0;
        while (left) {  // distinct items among the active lanes (debug build only)
          const uint32_t lead = (uint32_t)(__ffsll((long long)left) - 1);
          const uint32_t vi = __builtin_amdgcn_readlane(item, lead);
          left &= ~__ballot(item == vi);
          ++uniq;
        }
        PH_CNT(PH_QUNIQ, uniq);
      }
#endif
      const F4* it = (const F4*)((const char*)sc.nodes + ((cur & 0x0FFFFFFFu) << 6));
      F4 v[4];
      // (all four unconditionally: a leaf lane skipping the fourth when the scene has no
      // quads made hipcc wait for the first loads before the predicated one, C5 +1.9 %)
#ifdef RT_QTOP
      if ((cur & 0x0FFFFFFFu) < (uint32_t)RT_QTOP) {  // a top item: its LDS copy (k_fused)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = ld_lds(lnodes + 4 * (cur & 0x0FFFFFFFu) + e);
      } else
#endif
      {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = ld_glb(it + e);
      }
      if (!leaf) {
        float tn[4];
        uint32_t ch[4];
        qnode_children(v, o, inv, tmin, tr.best.t, tn, ch);
        if (tn[0] != kInf) {
          if (sp + 3 <= stack.nshort) {
            lds_u32* q = (lds_u32*)stack.lds;
            q[sp * 256] = ch[3];
            sp += tn[3] != kInf;
            q[sp * 256] = ch[2];
            sp += tn[2] != kInf;
            q[sp * 256] = ch[1];
            sp += tn[1] != kInf;
          } else {
            if (tn[3] != kInf && sp < kStack) push(ch[3]);
            if (tn[2] != kInf && sp < kStack) push(ch[2]);
            if (tn[1] != kInf && sp < kStack) push(ch[1]);
          }
          cur = ch[0];
          continue;
        }
      } else {
        float t, u, vv;
        uint32_t ref;
        bool near;
        const uint32_t rej = hit_record_m<FT>(v, o, d, inv.y, time, tmin, tr.best.t, t, u, vv, ref, near);
        tr.best.t = bitsf(pick_by(fbits(t), fbits(tr.best.t), rej));
        tr.best.u = bitsf(pick_by(fbits(u), fbits(tr.best.u), rej));
        tr.best.v = bitsf(pick_by(fbits(vv), fbits(tr.best.v), rej));
        tr.best.ref = pick_by(ref, tr.best.ref, rej);
        if (HAS(FT_TRI) && near) {
          if (pend != PRIM_NONE) {  // (rejected: nothing changed) this leaf again next round
            n = budget;
            continue;
          }
          pend = ref;
        }
      }
      if (sp == 0) cur = TRAV_DONE;
      else cur = stack.pop(--sp);
      continue;
    }
#ifndef RT_SPLIT_FETCH
    if (W4 && !LDS) {
      // One fetch per step for node and leaf lanes alike: the node (nodes + 8 cur,
      // 7 x 16 B) or the leaf's first record (leafprims + 4 first, 4 x 16 B), issued
      // together before either is used.  With the loads inside each branch, a wave
      // whose lanes are split between nodes and leaves waited for two dependent
      // memory round trips per step; here it waits for one (C3 -1.7 %, C4 -4.9 %,
      // C5 -2.8 %, profiles/r3_unified_fetch_ab.jsonl).
      // Node and leaf record share one allocation (rt_render.hip upload_scene): both are
      // addressed as 32-bit byte offsets from the node base (global_load with an SGPR
      // base).  A node's planes are fetched already ordered by the ray's direction signs:
      // the near x plane of the four children is lo.x (offset 0) when inv.x >= 0 and hi.x
      // (offset 16) when inv.x < 0, the far plane the other one, and likewise for y / z.
      // The slab test then needs no min/max per axis (v_min/v_max_f32 issue at half the
      // rate of v_sub/v_mul on gfx950, profiles/r4_instr_rate.jsonl): 16 min/max per node
      // instead of 40.  The same planes as min/max would pick, so the same t0, t1.
      const bool leaf = (cur & LEAF_BIT) != 0u;
      const uint32_t first = (cur >> 4) & 0x7FFFFFFu;
      const uint32_t rec0 = (uint32_t)((const char*)sc.leafprims - (const char*)sc.nodes);
      const uint32_t off = leaf ? rec0 + (first << 6) : cur << 7;
      const uint32_t nmask = leaf ? 0u : 16u;
      const uint32_t sx = (fbits(inv.x) >> 27) & nmask, sy = (fbits(inv.y) >> 27) & nmask;
      // (node: v[0] = the child codes, then near x, far x, near y; a leaf: its record)
      const char* nb = (const char*)sc.nodes;
      F4 v[7];
      v[0] = ld_glb((const F4*)(nb + off));
      v[1] = ld_glb((const F4*)(nb + (off + (16u + sx))));
      v[2] = ld_glb((const F4*)(nb + (off + (32u - sx))));
      v[3] = ld_glb((const F4*)(nb + (off + (48u + sy))));
      if (!leaf) {
        const uint32_t sz = (fbits(inv.z) >> 27) & 16u;
        v[4] = ld_glb((const F4*)(nb + (off + (64u - sy))));
        v[5] = ld_glb((const F4*)(nb + (off + (80u + sz))));
        v[6] = ld_glb((const F4*)(nb + (off + (96u - sz))));
        const float tmax = tr.best.t;
        float tn[4];
        uint32_t ch[4];
        const float Nx[4] = {v[1].x, v[1].y, v[1].z, v[1].w}, Fx[4] = {v[2].x, v[2].y, v[2].z, v[2].w};
        const float Ny[4] = {v[3].x, v[3].y, v[3].z, v[3].w}, Fy[4] = {v[4].x, v[4].y, v[4].z, v[4].w};
        const float Nz[4] = {v[5].x, v[5].y, v[5].z, v[5].w}, Fz[4] = {v[6].x, v[6].y, v[6].z, v[6].w};
        const uint32_t C[4] = {fbits(v[0].x), fbits(v[0].y), fbits(v[0].z), fbits(v[0].w)};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float tx0 = (Nx[k] - o.x) * inv.x, tx1 = (Fx[k] - o.x) * inv.x;
          const float ty0 = (Ny[k] - o.y) * inv.y, ty1 = (Fy[k] - o.y) * inv.y;
          const float tz0 = (Nz[k] - o.z) * inv.z, tz1 = (Fz[k] - o.z) * inv.z;
          const float t0 = fmaxf(fmaxf(tx0, ty0), fmaxf(tz0, tmin));
          const float t1 = fminf(fminf(tx1, ty1), fminf(tz1, tmax));
          // hit when t0 <= t1 * (1 + 2 ulp) (slab() semantics), i.e. when that difference
          // is not negative: tn = hit ? t0 : inf as a sign-mask select.  (An empty slot's
          // inverted infinite box gives t1 = -inf: no code check.  t0 = t1 = inf gives a
          // NaN difference with the sign clear: a "hit" at inf, as with the comparison.)
          tn[k] = bitsf(pick_by(fbits(t0), 0x7F800000u, neg_mask(t1 * 1.00000024f - t0)));
          ch[k] = C[k];
        }
        // compare-exchange as sign-mask selects: swap when tn[b] - tn[a] < 0, i.e. when
        // tn[b] < tn[a] (the difference of two distinct floats is never +-0; inf - inf
        // gives a NaN with the sign clear: no swap, like the comparison)
        auto cx = [&](int a, int b) {
          const uint32_t m = neg_mask(tn[b] - tn[a]);
          const uint32_t ta = fbits(tn[a]), tb = fbits(tn[b]);
          const uint32_t ca = ch[a], cb = ch[b];
          tn[a] = bitsf(pick_by(ta, tb, m));
          tn[b] = bitsf(pick_by(tb, ta, m));
          ch[a] = pick_by(ca, cb, m);
          ch[b] = pick_by(cb, ca, m);
        };
        cx(0, 1);
        cx(2, 3);
        cx(0, 2);
        cx(1, 3);
        cx(1, 2);
        if (tn[0] != kInf) {
#ifndef RT_PUSH_BRANCHED
          // The sorted hits are a prefix (tn[1] <= tn[2] <= tn[3], misses at inf): all three
          // candidates are written to consecutive LDS entries, farthest first, and the stack
          // pointer advances past the valid ones — no exec-mask branch per push when the
          // short stack has room (C3 -0.5 %, C4 -1.0 %, C5 -0.5 %, bit-identical,
          // profiles/r3_push_nobranch_ab.jsonl)
          if (!kTopReg && sp + 3 <= stack.nshort) {
            lds_u32* q = (lds_u32*)stack.lds;
            q[sp * 256] = ch[3];
            sp += tn[3] != kInf;
            q[sp * 256] = ch[2];
            sp += tn[2] != kInf;
            q[sp * 256] = ch[1];
            sp += tn[1] != kInf;
          } else
#endif
          {
            if (tn[3] != kInf && sp < kStack) push(ch[3]);
            if (tn[2] != kInf && sp < kStack) push(ch[2]);
            if (tn[1] != kInf && sp < kStack) push(ch[1]);
          }
          cur = ch[0];
          continue;
        }
      } else {
        const uint32_t count = (cur & 15u) + 1u;
        F4 rec[4] = {v[0], v[1], v[2], v[3]};
        uint32_t k = 0;
        for (;;) {
          float t, u, vv;
          uint32_t ref;
          bool near;
          const uint32_t rej = hit_record_m<FT>(rec, o, d, inv.y, time, tmin, tr.best.t, t, u, vv, ref, near);
          tr.best.t = bitsf(pick_by(fbits(t), fbits(tr.best.t), rej));
          tr.best.u = bitsf(pick_by(fbits(u), fbits(tr.best.u), rej));
          tr.best.v = bitsf(pick_by(fbits(vv), fbits(tr.best.v), rej));
          tr.best.ref = pick_by(ref, tr.best.ref, rej);
          if (HAS(FT_TRI) && near) {
            if (pend != PRIM_NONE) {  // the round ends before this prim (repeated next round)
              n = budget;
              break;
            }
            pend = ref;
          }
          ++k;
          if (k >= count) break;
          const F4* q = sc.leafprims + 4 * (size_t)(first + k);
          for (int e = 0; e < 4; ++e) rec[e] = ld_glb(q + e);
        }
        if (HAS(FT_TRI) && k < count) {
          cur = LEAF_BIT | ((first + k) << 4) | (count - k - 1u);
          continue;
        }
      }
      if (sp == 0) cur = TRAV_DONE;
      else cur = stack.pop(--sp);
      continue;
    }
#endif
    if (!W4 && !(cur & LEAF_BIT)) {
      // BVH2 node (tiny scenes, see render_impl): both child boxes, nearer first
      const F4* g = LDS ? lnodes + 4 * cur : sc.nodes + 4 * (size_t)cur;
      const F4 a0 = g[0], a1 = g[1], b0 = g[2], b1 = g[3];
      bool h0, h1;
      float t0, t1;
      slab(a0, a1, o, inv, tmin, tr.best.t, h0, t0);
      slab(b0, b1, o, inv, tmin, tr.best.t, h1, t1);
      const uint32_t c0 = fbits(a0.w), c1 = fbits(a1.w);
      if (h0 && h1) {
        const uint32_t nearc = t0 <= t1 ? c0 : c1, farc = t0 <= t1 ? c1 : c0;
        if (sp < kStack) push(farc);
        cur = nearc;
        continue;
      }
      if (h0 || h1) {
        cur = h0 ? c0 : c1;
        continue;
      }
    } else if (W4 && !(cur & LEAF_BIT)) {
      // BVH4 node: four slab tests, children ordered front to back; the
      // nearest is visited next, the others pushed farthest first
      const F4* g = LDS ? lnodes + 8 * cur : sc.nodes + 8 * (size_t)cur;
      const F4 cc = g[0], lx = g[1], hx = g[2], ly = g[3], hy = g[4], lz = g[5], hz = g[6];
      const float tmax = tr.best.t;
      float tn[4];
      uint32_t ch[4];
      const float Lx[4] = {lx.x, lx.y, lx.z, lx.w}, Hx[4] = {hx.x, hx.y, hx.z, hx.w};
      const float Ly[4] = {ly.x, ly.y, ly.z, ly.w}, Hy[4] = {hy.x, hy.y, hy.z, hy.w};
      const float Lz[4] = {lz.x, lz.y, lz.z, lz.w}, Hz[4] = {hz.x, hz.y, hz.z, hz.w};
      const uint32_t C[4] = {fbits(cc.x), fbits(cc.y), fbits(cc.z), fbits(cc.w)};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float tx0 = (Lx[k] - o.x) * inv.x, tx1 = (Hx[k] - o.x) * inv.x;
        const float ty0 = (Ly[k] - o.y) * inv.y, ty1 = (Hy[k] - o.y) * inv.y;
        const float tz0 = (Lz[k] - o.z) * inv.z, tz1 = (Hz[k] - o.z) * inv.z;
        const float t0 = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), tmin));
        const float t1 = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax));
        const bool h = t0 <= t1 * 1.00000024f && C[k] != CHILD_EMPTY;  // slab() semantics
        tn[k] = h ? t0 : kInf;
        ch[k] = C[k];
      }
      // sorting network (0,1)(2,3)(0,2)(1,3)(1,2): ascending entry distance
      auto cx = [&](int a, int b) {
        const bool sw = tn[b] < tn[a];
        const float ta = tn[a], tb = tn[b];
        const uint32_t ca = ch[a], cb = ch[b];
        tn[a] = sw ? tb : ta;
        tn[b] = sw ? ta : tb;
        ch[a] = sw ? cb : ca;
        ch[b] = sw ? ca : cb;
      };
      cx(0, 1);
      cx(2, 3);
      cx(0, 2);
      cx(1, 3);
      cx(1, 2);
      if (tn[0] != kInf) {
        if (tn[3] != kInf && sp < kStack) push(ch[3]);
        if (tn[2] != kInf && sp < kStack) push(ch[2]);
        if (tn[1] != kInf && sp < kStack) push(ch[1]);
        cur = ch[0];
        continue;
      }
    } else {
      uint32_t first = (cur >> 4) & 0x7FFFFFFu, count = (cur & 15u) + 1u;
      // leaf records are contiguous: no ref indirection, all four loads issue at once
      uint32_t k = 0;
      for (; k < count;) {
        const uint32_t ri = 4 * (first + k);
        F4 rec[4];
        if (LDS && recs_lds) {
          const F4* q = lnodes + (W4 ? 8 : 4) * sc.n_nodes + ri;
          for (int e = 0; e < 4; ++e) rec[e] = ld_lds(q + e);
        } else {
          const F4* q = sc.leafprims + ri;
          for (int e = 0; e < 4; ++e) rec[e] = ld_glb(q + e);
          if (LDS) wait_vm();  // LDS kernel whose records did not fit: keep the wait here
        }
        float t, u, v;
        uint32_t ref;
        bool near;
        const uint32_t rej = hit_record_m<FT>(rec, o, d, inv.y, time, tmin, tr.best.t, t, u, v, ref, near);
        tr.best.t = bitsf(pick_by(fbits(t), fbits(tr.best.t), rej));
        tr.best.u = bitsf(pick_by(fbits(u), fbits(tr.best.u), rej));
        tr.best.v = bitsf(pick_by(fbits(v), fbits(tr.best.v), rej));
        tr.best.ref = pick_by(ref, tr.best.ref, rej);
        if (HAS(FT_TRI) && near) {
          if (pend != PRIM_NONE) {  // the round ends before this prim (repeated next round)
            n = budget;
            break;
          }
          pend = ref;
        }
        ++k;
      }
      if (HAS(FT_TRI) && k < count) {  // the leaf's other prims first, next round
        cur = LEAF_BIT | ((first + k) << 4) | (count - k - 1u);
        continue;
      }
    }
    if (sp == 0) {
      cur = TRAV_DONE;
    } else if (kTopReg) {
      cur = top;
      if (--sp > 0) top = stack.pop(sp - 1);
    } else {
      cur = stack.pop(--sp);
    }
  }
  tr.cur = cur;
  tr.sp = sp;
  tr.top = top;
  tr.pend = pend;
  return n;
}

// ---- BVH8 (large scenes, host_bvh8.cpp layout, rt_device.h "BVH8 node") ----
// A child slot's traversal code from its meta byte: inner node child_base + rank, or
// a leaf code over recs8 (the same LEAF_BIT format as the BVH4's leaves).
RT_D uint32_t bvh8_code(uint32_t m, uint32_t child_base, uint32_t leaf_base) {
  return (m & 0x80u) ? child_base + (m & 7u)
                     : LEAF_BIT | ((leaf_base + (m & 31u)) << 4) | ((m >> 5) & 3u);
}
RT_D uint32_t bvh8_meta(uint32_t m0, uint32_t m1, uint32_t k) {
  return (uint32_t)((((unsigned long long)m1 << 32) | m0) >> (8u * k)) & 0xFFu;
}
// Resumable closest-hit traversal of the BVH8 (same contract as trav_steps).  A
// node step fetches one 128-B line per lane and tests eight children: each plane
// is t = (origin + q * 2^e - o) * inv, evaluated as fma(q, 2^e * inv, (origin - o)
// * inv) (2^e * inv is exact); the boxes carry one quantum of padding and the hit
// test 4 ulp of slack on the exit distance, which cover this form's rounding.
// The hit children's entry distances are sorted as keys (t0 bits with the slot in
// the low 3 bits: t0 >= tmin > 0, so the bits order like the floats) by a
// 19-comparator network of integer min/max; the nearest is visited next, the rest
// pushed farthest first.  Leaf steps fetch the record (64 B) only.
template <uint32_t FT>
RT_D int trav_steps8(const DevScene& sc, const TravStack& stack, f3 o, f3 d, float time,
                     float tmin, Trav& tr, int budget) {
  uint32_t cur = tr.cur;
  int sp = tr.sp;
  const f3 inv = tr.inv;
  const bool negx = inv.x < 0.0f, negy = inv.y < 0.0f, negz = inv.z < 0.0f;
  int n = 0;
  for (; n < budget && cur != TRAV_DONE; ++n) {
    const bool leaf = (cur & LEAF_BIT) != 0u;
    const uint32_t first = (cur >> 4) & 0x7FFFFFFu;
    const F4* g = leaf ? sc.recs8 + 4 * (size_t)first : sc.nodes8 + 8 * (size_t)cur;
    F4 v[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = ld_glb(g + e);
    if (!leaf) {
#pragma unroll
      for (int e = 4; e < 8; ++e) v[e] = ld_glb(g + e);
      const uint32_t ex = fbits(v[0].w);
      const float scx = bitsf((ex & 0xFFu) << 23) * inv.x;
      const float scy = bitsf(((ex >> 8) & 0xFFu) << 23) * inv.y;
      const float scz = bitsf(((ex >> 16) & 0xFFu) << 23) * inv.z;
      const float bx = (v[0].x - o.x) * inv.x, by = (v[0].y - o.y) * inv.y,
                  bz = (v[0].z - o.z) * inv.z;
      const uint32_t child_base = fbits(v[1].x), leaf_base = fbits(v[1].y);
      const uint32_t m0 = fbits(v[1].z), m1 = fbits(v[1].w);
      const uint32_t LX[4] = {fbits(v[2].x), fbits(v[2].y), fbits(v[2].z), fbits(v[2].w)};
      const uint32_t HX[4] = {fbits(v[3].x), fbits(v[3].y), fbits(v[3].z), fbits(v[3].w)};
      const uint32_t LY[4] = {fbits(v[4].x), fbits(v[4].y), fbits(v[4].z), fbits(v[4].w)};
      const uint32_t HY[4] = {fbits(v[5].x), fbits(v[5].y), fbits(v[5].z), fbits(v[5].w)};
      const uint32_t LZ[4] = {fbits(v[6].x), fbits(v[6].y), fbits(v[6].z), fbits(v[6].w)};
      const uint32_t HZ[4] = {fbits(v[7].x), fbits(v[7].y), fbits(v[7].z), fbits(v[7].w)};
      // entry / exit planes by the ray's direction signs, selected as whole words
      uint32_t NX[4], FX[4], NY[4], FY[4], NZ[4], FZ[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        NX[j] = negx ? HX[j] : LX[j];
        FX[j] = negx ? LX[j] : HX[j];
        NY[j] = negy ? HY[j] : LY[j];
        FY[j] = negy ? LY[j] : HY[j];
        NZ[j] = negz ? HZ[j] : LZ[j];
        FZ[j] = negz ? LZ[j] : HZ[j];
      }
      const float tmax = tr.best.t;
      uint32_t key[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int j = k >> 1, sh = (k & 1) * 16;
        auto q = [&](uint32_t w) { return (float)((w >> sh) & 0xFFFFu); };
        const float t0 = fmaxf(fmaxf(fmaf(q(NX[j]), scx, bx), fmaf(q(NY[j]), scy, by)),
                               fmaxf(fmaf(q(NZ[j]), scz, bz), tmin));
        const float t1 = fminf(fminf(fmaf(q(FX[j]), scx, bx), fmaf(q(FY[j]), scy, by)),
                               fminf(fmaf(q(FZ[j]), scz, bz), tmax));
        const uint32_t m = ((k < 4 ? m0 : m1) >> (8 * (k & 3))) & 0xFFu;
        const bool h = t0 <= t1 * 1.0000005f && m != 0xFFu;
        key[k] = h ? (fbits(t0) & ~7u) | (uint32_t)k : 0xFFFFFFFFu;
      }
      auto cx = [&](int a, int b) {
        const uint32_t lo = min(key[a], key[b]), hi = max(key[a], key[b]);
        key[a] = lo;
        key[b] = hi;
      };
      cx(0, 1), cx(2, 3), cx(4, 5), cx(6, 7);
      cx(0, 2), cx(1, 3), cx(4, 6), cx(5, 7);
      cx(1, 2), cx(5, 6);
      cx(0, 4), cx(1, 5), cx(2, 6), cx(3, 7);
      cx(2, 4), cx(3, 5);
      cx(1, 2), cx(3, 4), cx(5, 6);
      if (key[0] != 0xFFFFFFFFu) {
#pragma unroll
        for (int i = 7; i >= 1; --i)
          if (key[i] != 0xFFFFFFFFu && sp < kStack)
            stack.push(sp++, bvh8_code(bvh8_meta(m0, m1, key[i] & 7u), child_base, leaf_base));
        cur = bvh8_code(bvh8_meta(m0, m1, key[0] & 7u), child_base, leaf_base);
        continue;
      }
    } else {
      const uint32_t count = (cur & 15u) + 1u;
      F4 rec[4] = {v[0], v[1], v[2], v[3]};
      for (uint32_t k = 0;;) {
        float t, u, vv;
        uint32_t ref;
        bool near;
        const uint32_t rej = hit_record_m<FT>(rec, o, d, inv.y, time, tmin, tr.best.t, t, u, vv, ref, near);
        tr.best.t = bitsf(pick_by(fbits(t), fbits(tr.best.t), rej));
        tr.best.u = bitsf(pick_by(fbits(u), fbits(tr.best.u), rej));
        tr.best.v = bitsf(pick_by(fbits(vv), fbits(tr.best.v), rej));
        tr.best.ref = pick_by(ref, tr.best.ref, rej);
        // (opt-in BVH8 kernels: the near-edge fp64 re-test applied at once, not deferred)
        if (HAS(FT_TRI) && near && tri_hit64(sc, ref & 0x3FFFFFFFu, o, d, tmin, tr.best.t, t, u, vv))
          tr.best = {t, u, vv, ref};
        if (++k >= count) break;
        const F4* q = sc.recs8 + 4 * (size_t)(first + k);
        for (int e = 0; e < 4; ++e) rec[e] = ld_glb(q + e);
      }
    }
    if (sp == 0) cur = TRAV_DONE;
    else cur = stack.pop(--sp);
  }
  tr.cur = cur;
  tr.sp = sp;
  return n;
}

// Tiny scenes: every leaf record, in order, from the LDS cache (or through the
// scalar cache).  All lanes test the same record at the same time (a broadcast
// read, no divergence, no stack), which on 64-wide SIMDs beats a divergent BVH
// walk when the scene has a few dozen prims (C2: 18 quads).  Closest hit over all
// records = BVHNode.Hit's result (hittable.go:122-138; quad.go Hit per record).
// The small feature sets hold quads only, so the loop is the quad test alone,
// two records at a time in packed fp32 (v_pk_fma_f32: one issue, two records)
// from the pair layout (rt_device.h), branch-free: the loop keeps the closest t
// and its record index; the winner's (alpha, beta) and ref are recomputed once
// after the loop with the same fma sequence, so they equal the loop's values.
// The record loop is VALU-issue bound (C2: ~55 % of the kernel), so every
// instruction per record counts: 11 packed/rcp ops + 5 checks + 2 selects
// (18 VALU per record test, was 36 with one record at a time and early exits).
RT_D v2f pfma(v2f a, v2f b, v2f c) { return __builtin_elementwise_fma(a, b, c); }
// 0 <= a <= 1 && 0 <= b <= 1 as one unsigned max + compare: non-negative floats
// order like their bits, and negatives / NaN have the sign or exponent bits set
// above 1.0f's.  (-0.0f is rejected where the reference accepts it: exactly
// zero alpha with a negative sign; measure zero, within the parity tolerance.)
RT_D bool unit_ab(float a, float b) {
  return max(__float_as_uint(a), __float_as_uint(b)) <= 0x3F800000u;
}
// The record tests' acceptance as a sign mask (all ones = reject), from differences whose
// sign bit says the same as each comparison: |den| - 1e-8, t - tmin, best - t (>= 0 when
// the comparison holds; equal values give +0) and unit_ab_rej.  Then the closest-hit update
// is two v_bitop3 selects instead of v_cmp / v_cndmask (half rate and slower on gfx950,
// profiles/r4_instr_rate.jsonl): same choices.
RT_D uint32_t rec_reject(float den, float t, float tmin, float best, float a, float b) {
  const uint32_t ab = unit_ab_rej(a, b);
  const uint32_t any = __builtin_amdgcn_bitop3_b32(__float_as_uint(fabsf(den) - 1e-8f),
                                                   __float_as_uint(t - tmin),
                                                   __float_as_uint(best - t), 0xFE) | ab;
  return (uint32_t)((int32_t)any >> 31);
}
// the same without the denominator test (axis-aligned records: the inverse of the axis
// direction component is NaN when |d_a| < 1e-8; a NaN t makes alpha and beta NaN, whose
// bits exceed 1.0f's in either sign, so the alpha/beta term rejects it as t >= tmin did)
RT_D uint32_t rec_reject_t(float t, float tmin, float best, float a, float b) {
  const uint32_t ab = unit_ab_rej(a, b);
  const uint32_t any = __builtin_amdgcn_bitop3_b32(__float_as_uint(t - tmin),
                                                   __float_as_uint(best - t), ab, 0xFE);
  return (uint32_t)((int32_t)any >> 31);
}
// one record pair's loop fields (7 x 16 B) from the LDS cache or the scalar cache
template <bool SMEM>
RT_D void load_pair(const DevScene& sc, const F4* lrec, int p, v4f r[7]) {
  if (SMEM) {
    typedef __attribute__((address_space(4))) const v4f cst_v4;
    const cst_v4* q = (const cst_v4*)sc.leafprims + 8 * __builtin_amdgcn_readfirstlane(p);
#pragma unroll
    for (int e = 0; e < 7; ++e) r[e] = q[e];
  } else {
    const lds_v4* q = (const lds_v4*)lrec + 8 * p;
#pragma unroll
    for (int e = 0; e < 7; ++e) r[e] = q[e];
  }
}
// component I of Q, A, B for both records (floats 8-13, 14-19, 20-25 of the pair)
template <int I> RT_D v2f pair_q(const v4f* r) { return I == 0 ? r[2].xy : I == 1 ? r[2].zw : r[3].xy; }
template <int I> RT_D v2f pair_a(const v4f* r) { return I == 0 ? r[3].zw : I == 1 ? r[4].xy : r[4].zw; }
template <int I> RT_D v2f pair_b(const v4f* r) { return I == 0 ? r[5].xy : I == 1 ? r[5].zw : r[6].xy; }
// Axis-aligned pairs (unit normal +-e_AX, A_AX = B_AX = 0; grouped by the host after
// the general pairs).  With n = +-e_AX the general test's n.d is +-d_AX and n.o is
// +-o_AX, and the zero components of n, A and B add exact zeros, so t = (D' - o_AX)
// * rcp(d_AX) with D' = D / n_AX (stored by the host) and alpha, beta over the two
// in-plane axes are the general test's values bit for bit: 10 packed ops per pair
// instead of 20, and one rcp per ray and axis instead of two per pair.
template <int AX, bool SMEM>
RT_D void brute_axis(const DevScene& sc, const F4* lrec, int p0, int p1, const v2f* O,
                     const v2f* Dv, float tmin, float& best, uint32_t& bk) {
  constexpr int B0 = AX == 0 ? 1 : 0, B1 = AX == 2 ? 1 : 2;  // in-plane axes, ascending
  const float da = Dv[AX].x;
  // |n.d| < 1e-8: no hit (NaN), as a sign-mask select (a compare and v_cndmask_b32_e32 on
  // vcc cost ~23 cycles, and_not above)
  const float ia = bitsf(pick_by(fbits(rcp(da)), 0x7FC00000u, neg_mask(fabsf(da) - 1e-8f)));
  const v2f inv = {ia, ia};
  for (int p = p0; p < p1; ++p) {
    v4f r[7];
    load_pair<SMEM>(sc, lrec, p, r);
    const uint32_t k0 = __float_as_uint(r[6].z), k1 = __float_as_uint(r[6].w);
    const v2f t = (r[1].zw - O[AX]) * inv;
    const v2f pb = pfma(Dv[B0], t, O[B0]) - pair_q<B0>(r);
    const v2f pc = pfma(Dv[B1], t, O[B1]) - pair_q<B1>(r);
    const v2f a = pfma(pc, pair_a<B1>(r), pb * pair_a<B0>(r));
    const v2f b = pfma(pc, pair_b<B1>(r), pb * pair_b<B0>(r));
    const uint32_t m0 = rec_reject_t(t.x, tmin, best, a.x, b.x);
    best = bitsf(pick_by(fbits(t.x), fbits(best), m0));
    bk = pick_by(k0, bk, m0);
    const uint32_t m1 = rec_reject_t(t.y, tmin, best, a.y, b.y);
    best = bitsf(pick_by(fbits(t.y), fbits(best), m1));
    bk = pick_by(k1, bk, m1);
  }
}
// A mixed pair: record 2p axis-aligned on A0, record 2p+1 on A1 (A0 < A1; the odd records of
// two axis groups, host-paired; one pair per scene at most).  Each half runs brute_axis's
// arithmetic on its own axis in scalar form -- the same operations on the same operands
// (a packed op is two IEEE fp32 ops), so the same t, alpha, beta bit for bit -- reading the
// ray's components from o and d directly: a packed form gathered {o[A0], o[A1]}, ... into
// ten new registers, which spilled three VGPRs of the record-loop kernel.
template <int I> RT_D float comp(f3 v) { return I == 0 ? v.x : I == 1 ? v.y : v.z; }
template <int A, int H>
RT_D void brute_half(const v4f* r, f3 o, f3 d, float tmin, float& best, uint32_t& bk) {
  constexpr int B0 = A == 0 ? 1 : 0, B1 = A == 2 ? 1 : 2;  // in-plane axes, ascending
  const float da = comp<A>(d);
  // |n.d| < 1e-8: no hit (NaN), as a sign-mask select (a compare and v_cndmask_b32_e32 on
  // vcc cost ~23 cycles, and_not above)
  const float ia = bitsf(pick_by(fbits(rcp(da)), 0x7FC00000u, neg_mask(fabsf(da) - 1e-8f)));
  const float t = ((H ? r[1].w : r[1].z) - comp<A>(o)) * ia;
  const float pb = fmaf(comp<B0>(d), t, comp<B0>(o)) - (H ? pair_q<B0>(r).y : pair_q<B0>(r).x);
  const float pc = fmaf(comp<B1>(d), t, comp<B1>(o)) - (H ? pair_q<B1>(r).y : pair_q<B1>(r).x);
  const float a = fmaf(pc, H ? pair_a<B1>(r).y : pair_a<B1>(r).x, pb * (H ? pair_a<B0>(r).y : pair_a<B0>(r).x));
  const float b = fmaf(pc, H ? pair_b<B1>(r).y : pair_b<B1>(r).x, pb * (H ? pair_b<B0>(r).y : pair_b<B0>(r).x));
  const uint32_t m = rec_reject_t(t, tmin, best, a, b);
  best = bitsf(pick_by(fbits(t), fbits(best), m));
  bk = pick_by(__float_as_uint(H ? r[6].w : r[6].z), bk, m);
}
template <int A0, int A1, bool SMEM>
RT_D void brute_mixed(const DevScene& sc, const F4* lrec, int p, f3 o, f3 d, float tmin,
                      float& best, uint32_t& bk) {
  v4f r[7];
  load_pair<SMEM>(sc, lrec, p, r);
  brute_half<A0, 0>(r, o, d, tmin, best, bk);
  brute_half<A1, 1>(r, o, d, tmin, best, bk);
}
// Pairs parallel to axis AX (host-grouped): n_AX = 0 and A_AX = 0 exactly and B has only
// its AX component (NewBox's side faces after RotateY: v is the vertical edge).  Each
// dropped term of the general test is an exact zero, so den, num, alpha and beta are the
// general test's values (up to the sign of an exact zero): 15 packed ops per pair instead
// of 20.  (r: n.x 0, n.y 1, n.z 2 | Q 2-3 | A 3-4 | B 5-6, as pair_q/a/b)
template <int I> RT_D v2f pair_n(const v4f* r) { return I == 0 ? r[0].xy : I == 1 ? r[0].zw : r[1].xy; }
template <int AX, bool SMEM>
RT_D void brute_vert(const DevScene& sc, const F4* lrec, int p0, int p1, const v2f* O,
                     const v2f* Dv, float tmin, float& best, uint32_t& bk) {
  constexpr int B0 = AX == 0 ? 1 : 0, B1 = AX == 2 ? 1 : 2;  // the other axes, ascending
  for (int p = p0; p < p1; ++p) {
    v4f r[7];
    load_pair<SMEM>(sc, lrec, p, r);
    const uint32_t k0 = __float_as_uint(r[6].z), k1 = __float_as_uint(r[6].w);
    const v2f D = r[1].zw;
    const v2f den = pfma(pair_n<B1>(r), Dv[B1], pair_n<B0>(r) * Dv[B0]);
    const v2f num = D - pfma(pair_n<B1>(r), O[B1], pair_n<B0>(r) * O[B0]);
    const v2f t = num * v2f{rcp(den.x), rcp(den.y)};
    const v2f pa = pfma(Dv[AX], t, O[AX]) - pair_q<AX>(r);
    const v2f p0v = pfma(Dv[B0], t, O[B0]) - pair_q<B0>(r);
    const v2f p1v = pfma(Dv[B1], t, O[B1]) - pair_q<B1>(r);
    const v2f a = pfma(p1v, pair_a<B1>(r), p0v * pair_a<B0>(r));
    const v2f b = pa * pair_b<AX>(r);
    const uint32_t m0 = rec_reject(den.x, t.x, tmin, best, a.x, b.x);
    best = bitsf(pick_by(fbits(t.x), fbits(best), m0));
    bk = pick_by(k0, bk, m0);
    const uint32_t m1 = rec_reject(den.y, t.y, tmin, best, a.y, b.y);
    best = bitsf(pick_by(fbits(t.y), fbits(best), m1));
    bk = pick_by(k1, bk, m1);
  }
}
// Boxes rotated about y (host-detected: six records forming a box, rt_render.hip), two per
// descriptor pair: C.x | C.z | ax/|ax|^2 | az/|az|^2 (x, z) | y range | face slots.  In the
// box's frame (x' = (p - C).ax/|ax|^2, z' likewise, y unchanged) the faces are the planes
// x' = 0 / 1, y = ylo / yhi, z' = 0 / 1, and each face's quad test is t = (k - o'_a) / d'_a:
// the reference's own arithmetic in rotateY.Hit's object frame (transformation.go:94-107,
// objects.go:102-118).  The closest face with t in [tmin, best] is the entering one when
// t_near >= tmin, else the leaving one: one slab test instead of six record tests.  The
// winner is recorded as a box code (pair, half, leaving) and resolved to its face record
// after the loop (box_face).
constexpr uint32_t kBoxCode = 0x40000000u;
template <bool SMEM>
RT_D void brute_box(const DevScene& sc, const F4* lrec, int p0, int p1, const v2f* O,
                    const v2f* Dv, float iy1, float tmin, float& best, uint32_t& bk) {
  const v2f iy = {iy1, iy1};
  for (int p = p0; p < p1; ++p) {
    v4f r[4];
    if (SMEM) {
      typedef __attribute__((address_space(4))) const v4f cst_v4;
      const cst_v4* q = (const cst_v4*)sc.leafprims + 8 * __builtin_amdgcn_readfirstlane(p);
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = q[e];
    } else {
      const lds_v4* q = (const lds_v4*)lrec + 8 * p;
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = q[e];
    }
    const v2f ex = O[0] - r[0].xy, ez = O[2] - r[0].zw;
    const v2f lx = pfma(ez, r[1].zw, ex * r[1].xy), lz = pfma(ez, r[2].zw, ex * r[2].xy);
    const v2f vx = pfma(Dv[2], r[1].zw, Dv[0] * r[1].xy), vz = pfma(Dv[2], r[2].zw, Dv[0] * r[2].xy);
    const v2f ix = {rcp(vx.x), rcp(vx.y)}, iz = {rcp(vz.x), rcp(vz.y)};
    const v2f tx0 = -lx * ix, tx1 = pfma(-lx, ix, ix);
    const v2f tz0 = -lz * iz, tz1 = pfma(-lz, iz, iz);
    const v2f ty0 = (r[3].xy - O[1]) * iy, ty1 = (r[3].zw - O[1]) * iy;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float ax0 = h ? tx0.y : tx0.x, ax1 = h ? tx1.y : tx1.x;
      const float ay0 = h ? ty0.y : ty0.x, ay1 = h ? ty1.y : ty1.x;
      const float az0 = h ? tz0.y : tz0.x, az1 = h ? tz1.y : tz1.x;
      const float tn = fmaxf(fmaxf(fminf(ax0, ax1), fminf(ay0, ay1)), fminf(az0, az1));
      const float tf = fminf(fminf(fmaxf(ax0, ax1), fmaxf(ay0, ay1)), fmaxf(az0, az1));
      // enter = tn >= tmin; t = enter ? tn : tf; accept = tn <= tf && t >= tmin && t <= best,
      // all as sign masks and v_bitop3 selects (rec_reject)
      const uint32_t leave = neg_mask(tn - tmin);
      const float t = bitsf(pick_by(fbits(tn), fbits(tf), leave));
      const uint32_t rej = (uint32_t)((int32_t)__builtin_amdgcn_bitop3_b32(
                               fbits(tf - tn), fbits(t - tmin), fbits(best - t), 0xFE) >> 31);
      best = bitsf(pick_by(fbits(t), fbits(best), rej));
      bk = pick_by(kBoxCode | ((uint32_t)p << 2) | ((uint32_t)h << 1) | (leave & 1u), bk, rej);
    }
  }
}
// the face record slot of a box code: the plane (of the entering or leaving three) whose
// t is the loop's winning t, recomputed with the loop's operations
template <bool SMEM>
RT_D uint32_t box_face(const DevScene& sc, const F4* lrec, uint32_t code, f3 o, f3 d, float iy,
                       float best) {
  const uint32_t base = 32u * ((code & ~kBoxCode) >> 2) + ((code >> 1) & 1u);
  float f[8];  // C.x, C.z, a.x, a.z, b.x, b.z, ylo, yhi (then the six face slots)
  if (SMEM) {
    const float* g = (const float*)sc.leafprims + base;
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = *(const __attribute__((address_space(1))) float*)(g + 2 * e);
  } else {
    const lds_f32* l = (const lds_f32*)lrec + base;
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = l[2 * e];
  }
  const float ex = o.x - f[0], ez = o.z - f[1];
  const float lx = fmaf(ez, f[3], ex * f[2]), lz = fmaf(ez, f[5], ex * f[4]);
  const float ix = rcp(fmaf(d.z, f[3], d.x * f[2])), iz = rcp(fmaf(d.z, f[5], d.x * f[4]));
  const float t[6] = {-lx * ix, fmaf(-lx, ix, ix), (f[6] - o.y) * iy, (f[7] - o.y) * iy,
                      -lz * iz, fmaf(-lz, iz, iz)};
  // Entering plane of slab a: the smaller t (ties: the lo plane); leaving: the larger.  The
  // face is the first slab whose plane t is nearest the winning t.  As sign-mask selects and
  // ONE load of the face slot: written with dynamic indices (t[2a + side], f[8 + face]) hipcc
  // loaded all 14 fields and chained ~60 v_cmp / v_cndmask, about 100 VALU on every shading
  // round of the record-loop kernel (a wave almost always has a lane whose hit is a box).
  const uint32_t flip = (code & 1u) ? 0xFFFFFFFFu : 0u;  // leaving: take the larger
  uint32_t slot = 0u;
  float err = kInf;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const uint32_t m = neg_mask(t[2 * a + 1] - t[2 * a]) ^ flip;  // all ones: the hi plane
    // (fminf: a NaN distance reads as inf, so it never replaces, as with e < err)
    const float e = fminf(fabsf(bitsf(pick_by(fbits(t[2 * a]), fbits(t[2 * a + 1]), m)) - best), kInf);
    const uint32_t nearer = neg_mask(e - err);  // e < err
    slot = pick_by(slot, 2u * (uint32_t)a + (m & 1u), nearer);
    err = bitsf(pick_by(fbits(err), fbits(e), nearer));
  }
  if (SMEM)
    return *(const __attribute__((address_space(1))) uint32_t*)((const float*)sc.leafprims + base +
                                                                 2 * (8 + slot));
  return ((const lds_u32*)lrec)[base + 2 * (8 + slot)];
}
template <uint32_t FT, bool SMEM>
RT_D void trav_brute(const DevScene& sc, const F4* lrec, f3 o, f3 d, float time, float tmin,
                     Trav& tr) {
  static_assert(!HAS(FT_SPHERE | FT_TRI), "record loop: quad-only feature sets");
  // the group bounds re-read from the kernel-argument segment on every call (kparams): held
  // in SGPRs across the kernel's loop they were spilled to VGPR lanes, ~15 v_readlane per
  // segment in the loops' prologues
  const cst_params* kp = kparams();
  const int nax = kp->sc.brute_ax[0], nay = kp->sc.brute_ax[1], naz = kp->sc.brute_ax[2];
  const int nvy = kp->sc.brute_vt[1];  // y-parallel pairs only (RotateY is the only rotation)
  // general pairs first, then the y-parallel and the axis-aligned groups
  const int ng = kp->sc.brute_ng;
  const v2f ox = {o.x, o.x}, oy = {o.y, o.y}, oz = {o.z, o.z};
  const v2f dx = {d.x, d.x}, dy = {d.y, d.y}, dz = {d.z, d.z};
  float best = tr.best.t;
  uint32_t bk = 0xFFFFFFFFu;
  for (int p = 0; p < ng; ++p) {
    v4f r[7];
    load_pair<SMEM>(sc, lrec, p, r);
    // record indices 2p, 2p+1 as stored data: the select takes them from a VGPR
    // (a loop-counter SGPR would need a v_mov first: one constant-bus read per op)
    const uint32_t k0 = __float_as_uint(r[6].z), k1 = __float_as_uint(r[6].w);
    const v2f nx = r[0].xy, ny = r[0].zw, nz = r[1].xy, D = r[1].zw;
    const v2f den = pfma(nz, dz, pfma(ny, dy, nx * dx));
    const v2f num = D - pfma(nz, oz, pfma(ny, oy, nx * ox));
    const v2f t = num * v2f{rcp(den.x), rcp(den.y)};
    const v2f px = pfma(dx, t, ox) - r[2].xy;
    const v2f py = pfma(dy, t, oy) - r[2].zw;
    const v2f pz = pfma(dz, t, oz) - r[3].xy;
    const v2f a = pfma(pz, r[4].zw, pfma(py, r[4].xy, px * r[3].zw));
    const v2f b = pfma(pz, r[6].xy, pfma(py, r[5].zw, px * r[5].xy));
    const uint32_t m0 = rec_reject(den.x, t.x, tmin, best, a.x, b.x);
    best = bitsf(pick_by(fbits(t.x), fbits(best), m0));
    bk = pick_by(k0, bk, m0);
    const uint32_t m1 = rec_reject(den.y, t.y, tmin, best, a.y, b.y);
    best = bitsf(pick_by(fbits(t.y), fbits(best), m1));
    bk = pick_by(k1, bk, m1);
  }
  const v2f O[3] = {ox, oy, oz}, Dv[3] = {dx, dy, dz};
  const int q = ng + nvy;
  brute_vert<1, SMEM>(sc, lrec, ng, q, O, Dv, tmin, best, bk);
  brute_axis<0, SMEM>(sc, lrec, q, q + nax, O, Dv, tmin, best, bk);
  brute_axis<1, SMEM>(sc, lrec, q + nax, q + nax + nay, O, Dv, tmin, best, bk);
  brute_axis<2, SMEM>(sc, lrec, q + nax + nay, q + nax + nay + naz, O, Dv, tmin, best, bk);
  const int qm = q + nax + nay + naz, mx = kp->sc.brute_mx;  // the mixed pair (0 or 1)
  if (mx == (1 | (2 << 2))) brute_mixed<0, 1, SMEM>(sc, lrec, qm, o, d, tmin, best, bk);
  else if (mx == (1 | (3 << 2))) brute_mixed<0, 2, SMEM>(sc, lrec, qm, o, d, tmin, best, bk);
  else if (mx == (2 | (3 << 2))) brute_mixed<1, 2, SMEM>(sc, lrec, qm, o, d, tmin, best, bk);
  const int qb = qm + (mx != 0 ? 1 : 0);
  const float iy = rcp(d.y);
  brute_box<SMEM>(sc, lrec, qb, qb + kp->sc.brute_box, O, Dv, iy, tmin, best, bk);
  if (bk != 0xFFFFFFFFu) {
    if (bk & kBoxCode) bk = box_face<SMEM>(sc, lrec, bk, o, d, iy, best);
    // the winner's fields (pair bk/2, half bk&1): Q at floats 8/10/12, A at
    // 14/16/18, B at 20/22/24, ref at 28 (+ half)
    const uint32_t base = 32u * (bk >> 1) + (bk & 1u);
    float f[10];
    if (SMEM) {
      const float* g = (const float*)sc.leafprims + base + 8;
#pragma unroll
      for (int e = 0; e < 10; ++e)
        f[e] = *(const __attribute__((address_space(1))) float*)(g + 2 * e + (e == 9 ? 2 : 0));
    } else {
      const lds_f32* l = (const lds_f32*)lrec + base + 8;
#pragma unroll
      for (int e = 0; e < 10; ++e) f[e] = l[2 * e + (e == 9 ? 2 : 0)];
    }
    const float px = fmaf(d.x, best, o.x) - f[0];
    const float py = fmaf(d.y, best, o.y) - f[1];
    const float pz = fmaf(d.z, best, o.z) - f[2];
    tr.best.t = best;
    tr.best.u = fmaf(pz, f[5], fmaf(py, f[4], px * f[3]));
    tr.best.v = fmaf(pz, f[8], fmaf(py, f[7], px * f[6]));
    tr.best.ref = __float_as_uint(f[9]);
  }
  tr.cur = TRAV_DONE;
}

// the whole traversal at once (wavefront extend kernel)
template <bool LDS, uint32_t FT>
RT_D void trace_world(const DevScene& sc, const F4* lnodes, bool recs_lds, const TravStack& stack,
                      f3 o, f3 d, float time, float tmin, Hit& best) {
  Trav tr;
  trav_init<FT>(sc, o, d, time, tr);
  do {  // a near-edge rejection ends a round early (retest_near)
    trav_steps<LDS, FT>(sc, lnodes, recs_lds, stack, o, d, time, tmin, tr, 0x7FFFFFFF);
    retest_near<FT>(sc, o, d, tmin, tr);
  } while (tr.cur != TRAV_DONE);
  best = tr.best;
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
// Interval arithmetic in fp64: the reference searches (t1 + 1e-4, inf) with
// |t1| up to ~1e4 (book2 fog, R = 5000), below fp32 resolution.
// `spare`: rt_spare24 of the call that generated this ray, the scene's last draw
// index (rt_rng.h), so the outermost medium needs no Philox call of its own.
RT_D void trace_media(const Params& P, f3 o, f3 d, float time, float tmin, uint32_t gpix,
                      uint32_t sample, uint32_t vertex, uint32_t spare, Hit& best) {
  const DevScene& sc = P.sc;
  rt_u32x4 r = {{0, 0, 0, 0}};
  int cached_group = -1;
  const float ray_len = length(d);
  for (int mi = 0; mi < sc.n_media; ++mi) {
    // the medium record and its boundary through the scalar cache (a uniform index: no
    // vector-memory load, and no s_waitcnt vmcnt on the traversal's outstanding loads)
    static_assert(sizeof(DevMedium) == 32, "DevMedium: two 16-B scalar loads");
    const F4* mr = (const F4*)(sc.media + __builtin_amdgcn_readfirstlane(mi));
    const F4 ma = ld_cst(mr), mb = ld_cst(mr + 1);
    DevMedium m;
    m.bfirst = fbits(ma.x);
    m.bcount = fbits(ma.y);
    m.neg_inv_density = ma.z;
    m.phase_mat = (int32_t)fbits(ma.w);
    m.draw_base = (int32_t)fbits(mb.x);
    m.mult = (int32_t)fbits(mb.y);
    // The free-flight distance first (its draws are a pure function of the path's
    // counters, rt_rng.h, so drawing them before the boundary test changes nothing).
    // The medium's hit lies at max(t1, tmin) + hd / |d| > hd / |d|: when that is already
    // past the closest hit, the medium cannot be the closest hit and its fp64 boundary
    // roots are not needed -- book2's R = 5000 fog (mean free path 10^4) skips them on
    // most segments.  Same result as computing them (tm < best.t fails either way).
    float hd = kInf;
    for (int k = 0; k < m.mult; ++k) {
      int draw = m.draw_base + k;
      float u;
      if (draw == sc.medium_draws - 1) {
        u = rt_unit_f(spare);
      } else {
        int group = 1 + (draw >> 2);
        if (group != cached_group) {
          r = rt_rng_draw(P.seed, gpix, sample, RT_STREAM(vertex, group));
          cached_group = group;
        }
        u = rt_unit_f(r.v[draw & 3]);
      }
      hd = fminf(hd, m.neg_inv_density * logf(u));
    }
    const float hd_t = hd / ray_len;  // the same quotient as tm's below
#ifndef RT_NO_MEDIA_SKIP
    if (!(hd_t < best.t)) continue;
#endif
    double t1, t2;
    typedef __attribute__((address_space(4))) const uint32_t cst_u32;
    const uint32_t b0 = m.bcount == 1 ? *(const cst_u32*)(sc.medium_refs + m.bfirst) : PRIM_NONE;
    if ((b0 >> 30) == PRIM_SPHERE && b0 != PRIM_NONE) {
      // a sphere boundary (book2's fog and glass-ball interior): one quadratic gives
      // both boundary.Hit calls of medium.go:33-42 — t1 = the smaller root (always
      // inside (-inf, inf)), t2 = the larger one if it exceeds t1 + 1e-4
      double r0, r1;
      const uint32_t bi = b0 & 0x3FFFFFFFu;
      if (!sphere_roots_cm(ld_cst(sc.sph_cr + bi), ld_cst(sc.sph_mv + bi), o, d, time, r0, r1))
        continue;
      t1 = r0;
      if (!(t1 + 0.0001 < r1 && r1 < (double)kInf)) continue;
      t2 = r1;
    } else {
      if (!boundary_hit(sc, m, o, d, time, -(double)kInf, (double)kInf, t1)) continue;
      if (!boundary_hit(sc, m, o, d, time, t1 + 0.0001, (double)kInf, t2)) continue;
    }
    t1 = fmax(t1, (double)tmin);
    if (t1 >= t2) continue;
    t1 = fmax(0.0, t1);
    double inside = (t2 - t1) * (double)ray_len;
    if ((double)hd > inside) continue;
    float tm = (float)(t1 + (double)hd_t);
    if (tm < best.t) {
      best.t = tm;
      best.u = 0.0f;
      best.v = 0.0f;
      best.ref = prim_ref(PRIM_MEDIUM, (uint32_t)mi);
    }
  }
}

// ---------------------------------------------------------------- shading --
// Texture.Value texture.go:10-125 (checker chains resolved iteratively)
// Perlin tables of perlin 0 in LDS (kernels with FT_NOISE stage them at start,
// stage_perlin): ranvec as float4 and the three byte permutations, the same layout
// as DevPerlin.  The noise evaluation is 7 octaves x 8 lattice corners of dependent
// table reads (book2's marble sphere, C4): from HBM/L2 they were latency-bound (C4
// -23 % with texture evaluation ablated).  One code path serves both copies: the
// tables are reached through a generic pointer (LDS for perlin 0, global for the
// others), so the hardware routes each flat load (a second, address-space-specific
// copy of the noise code doubled the kernel's spills).
__shared__ DevPerlin g_perlin;

// before the kernel's first __syncthreads (stage_nodes), every thread of the block
RT_D void stage_perlin(const DevScene& sc) {
  if (sc.n_perlins <= 0) return;
  const F4* src = (const F4*)sc.perlins;
  F4* dst = (F4*)&g_perlin;
  for (int i = threadIdx.x; i < (int)(sizeof(DevPerlin) / 16); i += blockDim.x) dst[i] = src[i];
}

// PL: const DevPerlin* (global or LDS, the all-features kernel: flat loads) or
// LdsPerlin (table 0 in LDS, the feature-set kernels: ds_read, 3 % faster on C4
// than flat loads and fewer spills)
typedef __attribute__((address_space(3))) const DevPerlin* LdsPerlin;
template <typename PL>
RT_D float perlin_noise(PL pl, f3 p) {  // perlin.go:34-54
  float fx = floorf(p.x), fy = floorf(p.y), fz = floorf(p.z);
  float u = p.x - fx, v = p.y - fy, w = p.z - fz;
  int i = (int)fx, j = (int)fy, k = (int)fz;
  float uu = u * u * (3 - 2 * u), vv = v * v * (3 - 2 * v), ww = w * w * (3 - 2 * w);
  const int pi[2] = {pl->perm[0][i & 255], pl->perm[0][(i + 1) & 255]},
            pj[2] = {pl->perm[1][j & 255], pl->perm[1][(j + 1) & 255]},
            pk[2] = {pl->perm[2][k & 255], pl->perm[2][(k + 1) & 255]};
  // the corner weights i*uu + (1-i)*(1-uu) of perlin.go:49-51 for i = 0, 1: since uu is in
  // [0, 1], 0*uu + (1-uu) and uu + 0*(1-uu) are exactly 1-uu and uu (hipcc kept the 0*x
  // terms, which it may not drop for a NaN x: 12 fma per noise call, 84 per turbulence)
  const float wx[2] = {1 - uu, uu}, wy[2] = {1 - vv, vv}, wz[2] = {1 - ww, ww};
  float accum = 0.0f;
  for (int di = 0; di < 2; ++di)
    for (int dj = 0; dj < 2; ++dj)
      for (int dk = 0; dk < 2; ++dk) {
        const int gi = pi[di] ^ pj[dj] ^ pk[dk];
        const F4 g = {pl->ranvec[gi].x, pl->ranvec[gi].y, pl->ranvec[gi].z, 0.0f};
        f3 wt = mk3(u - (float)di, v - (float)dj, w - (float)dk);
        accum += wx[di] * wy[dj] * wz[dk] * dot(xyz(g), wt);
      }
  return accum;
}
template <typename PL>
RT_D float perlin_turb(PL pl, f3 p, int depth) {  // perlin.go:57-69
  float accum = 0.0f, weight = 1.0f;
#pragma unroll 1  // unrolled, the scheduler hoists every octave's table reads
  for (int i = 0; i < depth; ++i) {
    accum += weight * perlin_noise(pl, p);
    weight *= 0.5f;
    p = p * 2.0f;
  }
  return fabsf(accum);
}

template <uint32_t FT>
RT_D f3 tex_value(const DevScene& sc, int tex, float u, float v, f3 p) {
#ifdef ABL_NO_TEX
  return xyz(sc.texs[tex].color);  // ablation build (timing only)
#endif
  for (int guard = 0; guard < 64; ++guard) {
    const DevTexture T = sc.texs[tex];
    if (!HAS(FT_CHECKER | FT_IMAGE | FT_NOISE) || T.kind == RT_TEX_SOLID) return xyz(T.color);
    if (HAS(FT_CHECKER) && T.kind == RT_TEX_CHECKER) {  // texture.go:50-60
      float inv = T.color.w;
      int x = (int)floorf(inv * p.x), y = (int)floorf(inv * p.y), z = (int)floorf(inv * p.z);
      tex = ((x + y + z) % 2 == 0) ? T.a : T.b;
      continue;
    }
#ifdef ABL_NO_IMAGE
    if (HAS(FT_IMAGE) && T.kind == RT_TEX_IMAGE) return xyz(T.color);  // ablation build (timing only)
#endif
#ifdef ABL_NO_NOISE
    if (HAS(FT_NOISE) && T.kind == RT_TEX_NOISE) return xyz(T.color);  // ablation build (timing only)
#endif
    if (HAS(FT_IMAGE) && (!HAS(FT_NOISE) || T.kind == RT_TEX_IMAGE)) {  // texture.go:70-86 + PixelData imageLoader.go:52-62
      const DevImage im = sc.images[T.a];
      if (im.h <= 0) return mk3(0, 1, 1);
      // fmod(u, 1) is u - trunc(u) exactly (no rounding for any finite u; inf and NaN give
      // NaN either way), without the library fmodf's loop and selects
      float uu = fabsf(u - truncf(u));
      float vv = 1.0f - fabsf(v - truncf(v));
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
    if (!HAS(FT_NOISE)) return mk3(0, 0, 0);
    // noise, texture.go:112-125 (perlin 0 from its LDS copy when staged)
    const float scale = T.color.w;
    float s;
    auto eval = [&](auto pl) {
      if (T.variant == RT_NOISE_MARBLE) return 0.5f * (1.0f + sinf(scale * p.z + 10.0f * perlin_turb(pl, p, 7)));
      if (T.variant == RT_NOISE_TURBULENT) return perlin_turb(pl, p, 7);
      return 0.5f * (1.0f + perlin_noise(pl, p * scale));
    };
    if constexpr (FT == FT_ALL)
      s = eval((T.a == 0 && sc.n_perlins > 0) ? (const DevPerlin*)&g_perlin : sc.perlins + T.a);
    else
      s = eval((LdsPerlin)&g_perlin);  // table 0 (render_impl picks FT_ALL otherwise)
    return mk3(s, s, s);
  }
  return mk3(0, 0, 0);
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

// light PdfValue: sphere objects.go:52-62, quad :152-160, triangle :356-367
template <uint32_t FT>
RT_D float prim_pdf(const DevScene& sc, uint32_t ref, int li, f3 origin, f3 dir) {
  uint32_t type = ref >> 30, idx = ref & 0x3FFFFFFFu;
  if (HAS(FT_SPHERE) && type == PRIM_SPHERE) {
    float t;
    if (!hit_sphere(sc, idx, origin, dir, 0.0f, 0.0001f, kInf, t)) return 0.0f;
    const F4 cr = sc.sph_cr[idx];
    f3 oc = xyz(cr) - origin;
    float dist2 = dot(oc, oc);
    float cmax = fsqrt(1.0f - cr.w * cr.w * rcp(dist2));
    return rcp(2.0f * kPi * (1.0f - cmax));
  }
  float t, u, v, area;
  f3 n;
  uint32_t miss = 0u;  // quad lights: the reject mask of the branch-free test
  if (!HAS(FT_TRI) || type == PRIM_QUAD) {
    // the light's leaf-record copy (uniform index: scalar loads) and the traversal's quad test
    F4 rec[4];
    if (FT != FT_ALL) {
#ifdef RT_LIGHTS_SGPR
      const F4* lr = sc.light_recs + 8 * (size_t)__builtin_amdgcn_readfirstlane(li);
#else
      const F4* lr = kparams()->sc.light_recs + 8 * (size_t)__builtin_amdgcn_readfirstlane(li);
#endif
      rec[0] = ld_cst(lr), rec[1] = ld_cst(lr + 1), rec[2] = ld_cst(lr + 2), rec[3] = ld_cst(lr + 3);
    } else {
      const F4* lr = sc.light_recs + 8 * (size_t)li;
      rec[0] = lr[0], rec[1] = lr[1], rec[2] = lr[2], rec[3] = lr[3];
    }
    miss = hit_quad_rec_m(rec, origin, dir, 0.001f, kInf, t, u, v);
    n = xyz(rec[1]);
    area = rec[2].w;
  } else {
    if (!hit_tri(sc, idx, origin, dir, 0.001f, kInf, t, u, v)) return 0.0f;
    n = tri_normal(sc, idx, u, v);
    area = sc.tri[3 * (size_t)idx + 1].w;
  }
  // dist2 / (cosine * area) with dist2 = t^2 |dir|^2, cosine = |dir.n| / |dir|; +0 on a
  // miss (the mask clears every bit of whatever the missed test's t gave)
  const float dd = dot(dir, dir);
  return bitsf(and_not(fbits((t * t * dd) * fsqrt(dd) * rcp(fabsf(dot(dir, n)) * area)), miss));
}

// HittableList.PdfValue hittable.go:89-97 over the flattened light table
// (the light table's size and address re-read from the kernel-argument segment, kparams:
// held in SGPRs across the fused loop they were spilled to VGPR lanes, one v_readlane each
// per scattering vertex)
template <uint32_t FT>
RT_D float lights_pdf(const DevScene& sc, f3 origin, f3 dir) {
  float sum = 0.0f;
#ifdef RT_LIGHTS_SGPR  // (A/B builds: the light table's fields as the compiler holds them)
  const int n_lights = sc.n_lights;
  const DevLight* lights = sc.lights;
#else
  const cst_params* kp = kparams();
  const int n_lights = kp->sc.n_lights;
  const DevLight* lights = kp->sc.lights;
#endif
  for (int i = 0; i < n_lights; ++i) {  // uniform loop: the table entry is a scalar load
    const F4 e = FT != FT_ALL ? ld_cst((const F4*)lights + __builtin_amdgcn_readfirstlane(i))
                              : ((const F4*)lights)[i];
    const uint32_t ref = fbits(e.x);
    if (ref == PRIM_NONE) continue;
    sum += e.z * prim_pdf<FT>(sc, ref, i, origin, dir);
  }
  return sum;
}

// HittableList.Random hittable.go:98-103 + sphere/quad/Triangle.Random
template <uint32_t FT>
RT_D f3 lights_random(const DevScene& sc, f3 origin, const rt_u32x4& r) {
  const float s0 = rt_unit_f(r.v[2]), s1 = rt_unit_f(r.v[3]);
#ifdef RT_LIGHTS_SGPR
  const int n_lights = sc.n_lights;
  const DevLight* lights = sc.lights;
  const F4* light_recs = sc.light_recs;
#else
  const cst_params* kp = kparams();  // (as lights_pdf)
  const int n_lights = kp->sc.n_lights;
  const DevLight* lights = kp->sc.lights;
  const F4* light_recs = kp->sc.light_recs;
#endif
  int lo = 0, hi = n_lights - 1;
  if (n_lights <= 0) return mk3(rt_unit_f(r.v[1]), s0, s1);  // vec.Random()
  const uint32_t u24 = rt_u24(r.v[1]);
  while (lo < hi) {  // last entry with lo24 <= u24
    int mid = (lo + hi + 1) >> 1;
    if (lights[mid].lo24 <= u24) lo = mid;
    else hi = mid - 1;
  }
  const uint32_t ref =
      FT != FT_ALL && n_lights == 1 ? fbits(ld_cst((const F4*)lights).x) : lights[lo].ref;
  if (ref == PRIM_NONE) return mk3(rt_unit_f(r.v[1]), s0, s1);
  uint32_t type = ref >> 30, idx = ref & 0x3FFFFFFFu;
  if (HAS(FT_SPHERE) && type == PRIM_SPHERE) {  // sphere.Random + randomToSphere objects.go:63-80
    const F4 cr = sc.sph_cr[idx];
    f3 dir = xyz(cr) - origin;
    float dist2 = dot(dir, dir);
    Onb b = make_onb(dir);
    float z = 1.0f + s1 * (fsqrt(1.0f - cr.w * cr.w * rcp(dist2)) - 1.0f);
    float tt = fsqrt(1.0f - z * z);  // phi = 2*pi*s0
    return onb_transform(b, mk3(cos2pi(s0) * tt, sin2pi(s0) * tt, z));
  }
  if (!HAS(FT_TRI) || type == PRIM_QUAD) {  // quad.Random objects.go:161-165
    // the light record's Q, u, v; one light: a uniform index, so scalar loads
    F4 Q, U, V;
    if (FT != FT_ALL && n_lights == 1) {
      const F4* lr = light_recs + 4;
      Q = ld_cst(lr), U = ld_cst(lr + 1), V = ld_cst(lr + 2);
    } else {
      const F4* lr = light_recs + 8 * (size_t)lo + 4;
      Q = lr[0], U = lr[1], V = lr[2];
    }
    return (xyz(Q) + xyz(U) * s0 + xyz(V) * s1) - origin;
  }
  // Triangle.Random objects.go:369-385 (non-uniform barycentrics kept)
  const F4* tr = sc.tri + 3 * (size_t)idx;
  float r1 = s0, r2 = s1 * (1.0f - r1);
  f3 v0 = xyz(tr[0]), v1 = v0 + xyz(tr[1]), v2 = v0 + xyz(tr[2]);
  f3 p = v0 * (1.0f - r1 - r2) + v1 * r1 + v2 * r2;
  return p - origin;
}

// ---------------------------------------------------------- pixel sums -----
// pixelColor += rayColor(...) (camera.go:97-101) for every sample, in fixed point:
// each sample's channel becomes floor(v * 2^32) and the pixel sums are int64, so
// the sum is exact and independent of how samples are grouped into chunks, which
// lane or kernel renders them, and how rows are split over ranks (bitwise the same
// image for any chunk size, schedule, strategy and GPU count).  |v| < vlim = 2^31/ss
// keeps the ss-sample sum inside int64; a finite sample outside that range (never
// in the BASELINE scenes) is added in fp64 to a side plane and counted
// (Counters::overflow, rt_stats.overflow_samples); NaN and +-Inf set pixel flags
// with the reference's sum semantics (NaN, or +Inf and -Inf, give NaN).
RT_D uint32_t local_pixel(const Params& P, uint32_t chunk) {
  uint32_t sub;
  return chunk_pixel(P, chunk, sub);
}
// floor(v * 2^32) for |v| < 2^31: the integer part in the high word, the fraction
// in the low.  v - floor(v) is exact except for v in (-2^-24, 0), where it rounds
// to 1.0f; the fraction is capped at 1 - 2^-24 so its conversion stays in range
// (those samples count as -2^-24: error below 2^-24, still a fixed function of v,
// so the sums stay order-independent); * 2^32 only moves the exponent.
RT_D unsigned long long to_fixed(float v) {
  const float hi = floorf(v);
  const uint32_t lo = (uint32_t)(fminf(v - hi, 0x1.fffffep-1f) * 4294967296.0f);
  return ((unsigned long long)(uint32_t)(int32_t)hi << 32) | lo;
}
// a sample with a channel outside the fixed-point range or non-finite (rare): every
// channel goes straight to the pixel (fixed-point channels included: the integer sum
// does not care where it is added)
// (the buffers' addresses re-read from the kernel-argument segment: held across the fused
// loop for these rare branches they cost the record-loop kernel spilled VGPRs)
RT_D void add_sample_rare(const Params& P, uint32_t lp, float x, float y, float z) {
  const cst_params* kp = kparams();
  const float c[3] = {x, y, z};
  for (int ch = 0; ch < 3; ++ch) {
    const float v = c[ch];
    if (fabsf(v) < kp->vlim) {
      atomicAdd(&kp->accum[(size_t)ch * kp->npix + lp], to_fixed(v));
    } else if (isnan(v)) {
      atomicOr(&kp->pflags[lp], 1u << ch);
    } else if (isinf(v)) {
      atomicOr(&kp->pflags[lp], (v > 0.0f ? 8u : 64u) << ch);
    } else {
      atomicAdd(&kp->side[(size_t)ch * kp->npix + lp], (double)v);
      atomicAdd(&kp->ctr->overflow, 1ull);
    }
  }
}
typedef __attribute__((address_space(3))) unsigned long long lds_u64;
// Per-lane chunk sums: the fused kernel keeps them in an LDS column (3 x u64 per
// lane, [channel][thread]; ds_add_u64, no registers held across the path) and
// flushes them to the pixel with one global atomic per channel when the chunk
// ends; the wavefront kernels (lds == null) add every sample to the pixel.
struct SampleAcc {
  unsigned long long* lds;  // &lacc[0][threadIdx.x], stride 256, or null
  RT_D void add(const Params& P, uint32_t chunk, f3 L) const {
    const bool fixed = fabsf(L.x) < P.vlim && fabsf(L.y) < P.vlim && fabsf(L.z) < P.vlim;
    if (!fixed) {
      add_sample_rare(P, local_pixel(P, chunk), L.x, L.y, L.z);
      return;
    }
    const unsigned long long fx = to_fixed(L.x), fy = to_fixed(L.y), fz = to_fixed(L.z);
    if (lds) {
#ifdef RT_ABLATE_ACC  // timing ablation only (wrong images): no per-sample LDS adds
      if (fx == 0x1234567ull) __atomic_fetch_add((lds_u64*)lds, fx, __ATOMIC_RELAXED);
      return;
#endif
      __atomic_fetch_add((lds_u64*)lds, fx, __ATOMIC_RELAXED);
      __atomic_fetch_add((lds_u64*)lds + 256, fy, __ATOMIC_RELAXED);
      __atomic_fetch_add((lds_u64*)lds + 512, fz, __ATOMIC_RELAXED);
    } else {
      const uint32_t lp = local_pixel(P, chunk);
      atomicAdd(&P.accum[lp], fx);
      atomicAdd(&P.accum[(size_t)P.npix + lp], fy);
      atomicAdd(&P.accum[2 * (size_t)P.npix + lp], fz);
    }
  }
  RT_D void flush(const Params& P, uint32_t chunk, bool split = false) const {
    if (!lds) return;
    if (P.csum && !split) {
      // the chunk's own 32-B record, two plain 16-B stores.  A pixel atomic is performed
      // beyond L2 and completes late, and every later s_waitcnt vmcnt of the wave (the
      // traversal's node loads, the shading's) waited for it: C3 -4.4 %, C2 -2.5 %, C4
      // -1.5 % without them (profiles/r4_flush_*); stores retire at L2
      typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
      typedef __attribute__((address_space(1))) u64x2 glb_u64x2;
      const unsigned long long s0 = ((lds_u64*)lds)[0], s1 = ((lds_u64*)lds)[256],
                               s2 = ((lds_u64*)lds)[512];
      ((lds_u64*)lds)[0] = 0ull;
      ((lds_u64*)lds)[256] = 0ull;
      ((lds_u64*)lds)[512] = 0ull;
      glb_u64x2* rec = (glb_u64x2*)(P.csum + 4 * (size_t)chunk);
      rec[0] = u64x2{s0, s1};
      rec[1] = u64x2{s2, 0ull};
      return;
    }
    const uint32_t lp = local_pixel(P, chunk);
    const cst_params* kp = kparams();  // (as add_sample_rare: a rare branch)
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      lds_u64* q = (lds_u64*)lds + ch * 256;
      const unsigned long long s = *q;
      *q = 0ull;
#ifdef RT_ABLATE_FLUSH  // timing ablation only (wrong images): no global pixel atomics
      if (s == 0x1234567ull)
#else
      if (s)
#endif
#ifdef RT_ABLATE_STFLUSH  // timing ablation only (wrong images): plain stores, not atomics
        kp->accum[(size_t)ch * kp->npix + lp] = s;
#else
        atomicAdd(&kp->accum[(size_t)ch * kp->npix + lp], s);
#endif
    }
  }
};

// ------------------------------------------------------------- path state --
// One path.  In the fused kernel every field lives in registers; in the
// wavefront kernels ray/key fields are loaded from SoA and pend/pre/acc are
// touched in HBM only when a vertex needs them (SOA = true).
struct Path {
  f3 o, d;
  float time;
  uint32_t chunk, j, k, nst, flags;
  uint32_t gpix, s0;  // global pixel and first sample of the chunk (chunk_ids, cached)
  uint32_t spare;     // rt_spare24 of the call that generated the ray (trace_media)
  f3 pend, pre;
  uint32_t segs;    // world.Hit calls of this lane (statistics)
  uint32_t pushes;  // clamp weights stored (statistics, RT_COUNT_PUSHES builds only)
};

template <bool SOA>
RT_D f3 get_pend(const Params& P, uint32_t slot, const Path& s) {
  return SOA ? xyz(P.pend[slot]) : s.pend;
}
template <bool SOA>
RT_D void set_pend(const Params& P, uint32_t slot, Path& s, f3 v) {
  if (SOA) P.pend[slot] = {v.x, v.y, v.z, 0.0f};
  else s.pend = v;
}
template <bool SOA>
RT_D f3 get_pre(const Params& P, uint32_t slot, const Path& s) {
  return SOA ? xyz(P.pre[slot]) : s.pre;
}
template <bool SOA>
RT_D void set_pre(const Params& P, uint32_t slot, Path& s, f3 v) {
  if (SOA) P.pre[slot] = {v.x, v.y, v.z, 0.0f};
  else s.pre = v;
}

// Clamp-weight stack: entries below nlds in an LDS column (fused kernel, one
// per thread), the rest in HBM [entry - nlds][slot].  LDS keeps the common
// shallow pushes off the vector-memory counter (a store holds vmcnt for
// hundreds of cycles and every later load waits behind it).
struct WStack {
  float* lds;  // &lds_w[0][0][threadIdx.x]: [channel][entry][thread] planes, 12 B per entry
  int nlds;
  RT_D void put(const Params& P, uint32_t slot, uint32_t k, F4 v) const {
    if ((int)k < nlds) {
      lds_f32* q = (lds_f32*)lds + k * 256;
      q[0] = v.x;
      q[nlds * 256] = v.y;
      q[2 * nlds * 256] = v.z;
    } else {
      st_glb(hbm_entry(P, slot, k), v);
    }
  }
  // entry k (the top) *= w: a dominated clamp vertex merged into it (shade_core);
  // returns the new entry
  RT_D f3 mul(const Params& P, uint32_t slot, uint32_t k, f3 w) const {
    f3 r;
    if ((int)k < nlds) {
      lds_f32* q = (lds_f32*)lds + k * 256;
      r = mk3(q[0] * w.x, q[nlds * 256] * w.y, q[2 * nlds * 256] * w.z);
      q[0] = r.x;
      q[nlds * 256] = r.y;
      q[2 * nlds * 256] = r.z;
    } else {
      F4* e = hbm_entry(P, slot, k);
      const F4 v = ld_glb(e);
      r = mk3(v.x * w.x, v.y * w.y, v.z * w.z);
      st_glb(e, {r.x, r.y, r.z, 0.0f});
    }
    return r;
  }
  // HBM entries: [entry][slot] (a wave's lanes at one depth coalesce) or, with
  // WSTACK_SLOT_MAJOR, [slot][entry] (one lane's pushes share cache lines)
  // the entry's address, with the stack base and column count re-read from the
  // kernel-argument segment (kparams): these rare HBM branches otherwise kept a 64-bit base
  // live across the fused loop (2 spilled VGPRs in the record-loop kernel)
  RT_D F4* hbm_entry(const Params& P, uint32_t slot, uint32_t k) const {
    const cst_params* kp = kparams();
#ifdef WSTACK_SLOT_MAJOR
    return kp->stack + ((size_t)slot * (kp->max_depth + 1) + (k - nlds));
#else
    return kp->stack + ((size_t)(k - nlds) * kp->P + slot);
#endif
  }
  RT_D size_t hbm_index(const Params& P, uint32_t slot, uint32_t k) const {
#ifdef WSTACK_SLOT_MAJOR
    return (size_t)slot * (P.max_depth + 1) + (k - nlds);
#else
    return (size_t)(k - nlds) * P.P + slot;
#endif
  }
  // The backward clamp fold (camera.go:328-330) as one scale.  A clamp only scales its
  // vector, by s_k = min(1, M / I(w_k (.) v_k+1)) with I the channel sum, so the folded
  // value is (prod s_k) times the plain product P_0 = w_0 (.) ... (.) w_n (.) L, and the
  // scales telescope: prod s_k = min(1, min_k M / I(P_k)) over the suffix products
  // P_k = w_k (.) ... (.) L.  So the walk from the last weight back multiplies and
  // keeps the largest channel sum; one scale by M / max I at the end (if max I > M)
  // replaces a compare, reciprocal and select per clamp vertex.  Same value as the
  // step-by-step clamps up to fp32 rounding (weights and radiance are non-negative).
  // `v` is pend (.) L with maxI = I(v) on entry; entries nst-1 .. 0: HBM ones (rare)
  // one by one, then the LDS ones, unrolled.
  RT_D void fold_max(const Params& P, uint32_t slot, uint32_t nst, f3& v, float& maxI) const {
    int k = (int)nst - 1;
#ifndef RT_FOLD_ONE_LOAD
    // HBM entries two at a time: both loads in flight before the products need them
    for (; k - 1 >= nlds; k -= 2) {
      const F4 a = ld_glb(hbm_entry(P, slot, (uint32_t)k));
      const F4 b = ld_glb(hbm_entry(P, slot, (uint32_t)(k - 1)));
      v = xyz(a) * v;
      maxI = fmaxf(maxI, v.x + v.y + v.z);
      v = xyz(b) * v;
      maxI = fmaxf(maxI, v.x + v.y + v.z);
    }
#endif
    for (; k >= nlds; --k) {
      v = xyz(ld_glb(hbm_entry(P, slot, (uint32_t)k))) * v;
      maxI = fmaxf(maxI, v.x + v.y + v.z);
    }
    if (nlds > 0 && nst > 0) {
      const lds_f32* q = (const lds_f32*)lds;
      f3 e[kLdsWMax];
#pragma unroll
      for (int i = 0; i < kLdsWMax; ++i)
        if (i < nlds)  // entries >= nst are garbage, unused
          e[i] = mk3(q[i * 256], q[(nlds + i) * 256], q[(2 * nlds + i) * 256]);
#pragma unroll
      for (int i = kLdsWMax - 1; i >= 0; --i)
        if (i < nlds && i < (int)nst) {
          v = e[i] * v;
          maxI = fmaxf(maxI, v.x + v.y + v.z);
        }
    }
  }
  // the step-by-step fold (A/B builds: -DRT_FOLD_STEPWISE)
  RT_D f3 fold(const Params& P, uint32_t slot, uint32_t nst, f3 L) const {
    for (int k = (int)nst - 1; k >= nlds; --k)
      L = clamp_contribution(xyz(ld_glb(hbm_entry(P, slot, (uint32_t)k))) * L, P.maxc);
    if (nlds > 0 && nst > 0) {
      const lds_f32* q = (const lds_f32*)lds;
      f3 e[kLdsWMax];
#pragma unroll
      for (int i = 0; i < kLdsWMax; ++i)
        if (i < nlds)  // entries >= nst are garbage, unused
          e[i] = mk3(q[i * 256], q[(nlds + i) * 256], q[(2 * nlds + i) * 256]);
#pragma unroll
      for (int i = kLdsWMax - 1; i >= 0; --i)
        if (i < nlds && i < (int)nst) L = clamp_contribution(e[i] * L, P.maxc);
    }
    return L;
  }
};

template <bool SOA>
RT_D void store_ray(const Params& P, uint32_t slot, const Path& s) {
  if (SOA) {
    P.ray_o[slot] = {s.o.x, s.o.y, s.o.z, s.time};
    P.ray_d[slot] = {s.d.x, s.d.y, s.d.z, bitsf(s.spare)};
    P.path[slot] = make_uint2(s.chunk, pack_path(s.j, s.k, s.nst, s.flags));
  }
}

RT_D void load_path(const Params& P, uint32_t slot, Path& s) {
  const F4 ro = P.ray_o[slot], rd = P.ray_d[slot];
  const uint2 ps = P.path[slot];
  s.o = xyz(ro);
  s.time = ro.w;
  s.d = xyz(rd);
  s.spare = fbits(rd.w);
  s.chunk = ps.x;
  const Ids id = chunk_ids(P, s.chunk);
  s.gpix = id.gpix;
  s.s0 = id.sample0;
  s.j = ps.y & 0xFFFu;
  s.k = (ps.y >> 12) & 0xFFu;
  s.nst = (ps.y >> 20) & 0xFFu;
  s.flags = (ps.y >> 28) | (id.count << kCountShift);
}

// the next sample of the same chunk, its camera draw already made: the path
// state (pixel ids cached in s) is reset for sample j
template <bool SOA, int CAM = 0>
RT_D void next_sample(const Params& P, uint32_t slot, Path& s, uint32_t j, const rt_u32x4& r) {
  Ids id;
  id.gpix = s.gpix;
  id.row = fdiv(s.gpix, P.fd_width);
  id.col = s.gpix - id.row * (uint32_t)P.width;
  camera_ray_r<CAM>(P, id, s.s0 + j, r, s.o, s.d, s.time);
  s.spare = rt_spare24(r);
  s.j = j;
  s.k = 0;
  s.nst = 0;
  s.flags &= ~(F_SPLIT - 1u);  // the chunk's sample count and F_SPLIT stay
  store_ray<SOA>(P, slot, s);
}

// camera ray for sample j of `chunk` (path state reset)
template <bool SOA, int CAM = 0, bool ONE = false>
RT_D void start_sample(const Params& P, uint32_t slot, Path& s, uint32_t chunk, uint32_t j) {
  Ids id = chunk_ids<ONE>(P, chunk);
  const rt_u32x4 r = rt_rng_draw(P.seed, id.gpix, id.sample0 + j, RT_STREAM_CAMERA);
  camera_ray_r<CAM>(P, id, id.sample0 + j, r, s.o, s.d, s.time);
  s.spare = rt_spare24(r);
  s.chunk = chunk;
  s.gpix = id.gpix;
  s.s0 = id.sample0;
  s.j = j;
  s.k = 0;
  s.nst = 0;
  s.flags = id.count << kCountShift;
  store_ray<SOA>(P, slot, s);
}

// One vertex of rayColor (camera.go:293-331) given its closest hit.
// Returns OUT_ALIVE (continue with s.o/s.d), or OUT_NEED_CHUNK (chunk flushed).
template <bool SOA, uint32_t FT>
RT_D int shade_core(const Params& P, uint32_t slot, Path& s, const Hit& h, const WStack& ws,
                    const SampleAcc& sa) {
  const DevScene& sc = P.sc;
  const f3 o = s.o, d = s.d;
  const float time = s.time;
  const uint32_t ref = h.ref;
  f3 lterm = mk3(0, 0, 0);
  bool term = false;
  rt_u32x4 rcam;  // camera draw of the next sample, when this vertex made it
  bool have_rcam = false;
  f3 p = mk3(0, 0, 0), n = mk3(0, 0, 0);
  float u = h.u, v = h.v;
  bool ff = true;
  DevMaterial M;
  bool scat = false;
  // lean record-loop kernel: the quad's normal, material kind and solid colour from the
  // shade table in LDS (rt_render.hip), no global loads
  bool ltab = false;
  f3 lcol = mk3(0, 0, 0);
  // The hit point goes back onto the surface it was found on.  r.At(t) in fp32 carries
  // the rounding of t along the ray (~|p - o| * 2^-22: up to ~1e-4 off the surface for the
  // long rays of the 555- and 1000-unit scenes), and from a point that far on the wrong
  // side a next ray leaving at a grazing angle re-hits the same quad or sphere at t >=
  // 0.001 -- a vertex the fp64 reference (point on the surface to ~1e-13) never makes.
  // That self-hit was 98 % of C2's and ~40 % of C4's forked samples
  // (tools/fork_census.py).  Quads: projected onto their plane, p - n (n.p - D), exact for
  // axis-aligned quads (every term is an exact zero or a Sterbenz difference, so p lands
  // ON the plane and the next test's t is exactly 0).  Spheres: onto the sphere, and then
  // `eta` (4x the rounding left) to the side the next ray leaves on (below).
  float eta = 0.0f;
  if (ref != PRIM_NONE) {
    const float t = h.t;
    p = o + d * t;  // r.At(t)
    const uint32_t type = ref >> 30, idx = ref & 0x3FFFFFFFu;
    f3 nout;
    int mat;
    if (HAS(FT_SPHERE) && type == PRIM_SPHERE) {
      const F4 cr = sc.sph_cr[idx], mv = sc.sph_mv[idx];
      f3 cc = xyz(cr) + xyz(mv) * time;
      // p moved along the unit normal by r - |p - c|, that offset from r^2 - |p - c|^2
      // formed in fp64 (the sphere test's centre; every fp32 square is exact there), so the
      // point is on the sphere to its coordinates' rounding, ~2^-24 sum|p_i n_i|, even for
      // the R=1000 ground where p - c cancels in fp32.  eta, 4x that bound, then puts it
      // on the right side (below).  nout = (p - c) / r objects.go:102 (a negative radius
      // keeps its inward normal).
      {
        const double cx = (double)cr.x + (double)time * (double)mv.x;
        const double cy = (double)cr.y + (double)time * (double)mv.y;
        const double cz = (double)cr.z + (double)time * (double)mv.z;
        const double ex = (double)p.x - cx, ey = (double)p.y - cy, ez = (double)p.z - cz;
        const double rr = (double)cr.w;
        const float dn = (float)(rr * rr - (ex * ex + ey * ey + ez * ez));  // (r - |e|)(r + |e|)
        const f3 e = p - cc;
        const float le = length(e);
        const f3 nu = e * rcp(le);
        p = p + nu * (dn * rcp(fabsf(cr.w) + le));
        nout = cr.w < 0.0f ? -nu : nu;
        eta = 0x1p-22f * (fabsf(p.x * nu.x) + fabsf(p.y * nu.y) + fabsf(p.z * nu.z));
      }
      mat = (int)fbits(mv.w);
      ff = dot(d, nout) < 0;  // setFaceNormal hittable.go:27-34
      n = ff ? nout : -nout;
      if (HAS(FT_IMAGE) && sc.mats[mat]._pad != 0.0f) {  // texture reads u,v: calculateSphereUV objects.go:44-50
        const F2 rs = sc.sph_uv[idx];
        f3 no = mk3(rs.x * nout.x - rs.y * nout.z, nout.y, rs.y * nout.x + rs.x * nout.z);
        float theta = acosf(-no.y);
        float phi = atan2f(-no.z, no.x) + kPi;
        u = phi * (0.5f * kInvPi);
        v = theta * kInvPi;
      }
    } else if (FT == 0u && sc.shade_lds >= 0) {
      const F4* tab = g_dyn_lds + sc.shade_lds + 2 * idx;
      const F4 a = ld_lds(tab), b = ld_lds(tab + 1);
      lcol = xyz(b);
      nout = xyz(a);
#ifndef RT_NO_LEAN_SNAP  // (A/B builds: the record-loop kernel without the projection)
      p = p - nout * (dot(nout, p) - b.w);  // onto the plane n.p = D (b.w, rt_render.hip)
#endif
      mat = (int)fbits(a.w);  // the material KIND here
      ltab = true;
      ff = dot(d, nout) < 0;
      n = ff ? nout : -nout;
    } else if (!HAS(FT_TRI | FT_MEDIA) || type == PRIM_QUAD) {
      const F4* q = sc.quad + 5 * (size_t)idx;
      nout = xyz(q[3]);
      p = p - nout * (dot(nout, p) - q[0].w);  // onto the plane n.p = D
      mat = (int)fbits(q[2].w);
      ff = dot(d, nout) < 0;
      n = ff ? nout : -nout;
      if (HAS(FT_BOX) && u < 0.0f) {
        // a box leaf's face (hit_box_rec): quad.Hit's alpha, beta (objects.go:186-187) at
        // this p, computed only when the material reads them (image textures)
        if (HAS(FT_IMAGE) && sc.mats[mat]._pad != 0.0f) {
          const f3 pp = p - xyz(q[0]), w = xyz(q[4]);
          u = dot(w, cross(pp, xyz(q[2])));
          v = dot(w, cross(xyz(q[1]), pp));
        } else {
          u = v = 0.0f;
        }
      }
    } else if (HAS(FT_TRI) && (!HAS(FT_MEDIA) || type == PRIM_TRI)) {
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
      mat = sc.media[idx].phase_mat;
      n = mk3(1, 0, 0);
      ff = true;
      u = v = 0.0f;
    }
    if (ltab)
      M.kind = mat;
    else
      M = sc.mats[mat];
    scat = M.kind != RT_MAT_DIFFUSE_LIGHT;
  }
  // ONE Philox call per vertex for the whole wave: a scattering vertex draws its
  // own numbers; a path ending here (miss or light) draws the camera numbers of
  // the chunk's next sample (otherwise two divergent calls per iteration):
  // C2 +3 %, C3 +2 %.  The all-features kernel (3 waves/SIMD, register-bound)
  // keeps the two draws in their branches (merged there: C4 -3 %).
  constexpr bool kMergeDraws = FT != FT_ALL;
  rt_u32x4 r;
  if (kMergeDraws)
    r = rt_rng_draw(P.seed, s.gpix, s.s0 + s.j + (scat ? 0u : 1u),
                    scat ? RT_STREAM(s.k, 0) : RT_STREAM_CAMERA);
  if (!scat) {
    if (ref == PRIM_NONE)
      lterm = mk3(P.bg[0], P.bg[1], P.bg[2]);  // camera.go:300-302
    else  // Emitted materials.go:150-155; Scatter false
      lterm = ff ? (ltab ? lcol : tex_value<FT>(sc, M.tex, u, v, p)) : mk3(0, 0, 0);
    term = true;
    if (kMergeDraws) {
      rcam = r;
      have_rcam = true;
    }
  } else {
    if (!kMergeDraws) r = rt_rng_draw(P.seed, s.gpix, s.s0 + s.j, RT_STREAM(s.k, 0));
    {
      f3 ndir;
      bool clamp_vertex = false;
      f3 weight;
      if (HAS(FT_METAL) && M.kind == RT_MAT_METAL) {  // materials.go:70-79
        f3 refl = unit(reflect(d, n));
        ndir = refl + uniform_sphere(rt_unit_f(r.v[2]), rt_unit_f(r.v[3])) * M.param;
        weight = xyz(M.albedo);
      } else if (HAS(FT_DIEL) && M.kind == RT_MAT_DIELECTRIC) {  // materials.go:94-130
        float ior = M.param;
        float ri = ff ? rcp(ior) : ior;
        f3 ud = unit(d);
        float cs = fminf(dot(-ud, n), 1.0f);
        float sn = fsqrt(1.0f - cs * cs);
        bool cannot = ri * sn > 1.0f;
        bool refl = cannot;
        if (!cannot) {
          float r0 = (1.0f - ior) * rcp(1.0f + ior);
          r0 = r0 * r0;
          // Schlick's (1 - cos)^5 (materials.go:132-136, math.Pow) as three multiplies: the
          // library powf is ~40 instructions with its special-case selects; the product is
          // within a few ulp of it for the base in [0, 1]
          const float x = 1.0f - cs, x2 = x * x;
          float refl_p = r0 + (1.0f - r0) * (x2 * x2 * x);
          refl = refl_p > rt_unit_f(r.v[0]);
        }
        ndir = refl ? reflect(ud, n) : refract(ud, n, ri);
        weight = mk3(1, 1, 1);
      } else {  // lambertian materials.go:45-57 / isotropic :157-177 + mixture pdf.go:58-74
        const bool iso = HAS(FT_MEDIA) && M.kind == RT_MAT_ISOTROPIC;
        PH_T(t_tex);
        f3 att = ltab ? lcol : tex_value<FT>(sc, M.tex, u, v, p);
        PH_ADD(PH_TEX, t_tex);
        PH_T(t_light);
        Onb b;
        if (!iso) b = make_onb_unit(n);
        if (rt_unit_f(r.v[0]) < 0.5f) {
          ndir = lights_random<FT>(sc, p, r);
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
          bsdf_pdf = fmaxf(0.0f, dot(ud, b.w) * kInvPi);  // 1 ulp of /pi, no division sequence
          float ct = dot(n, ud);
          spdf = fmaxf(0.0f, ct * kInvPi);  // (kInvPi > 0: zero exactly when ct < 0)
        }
#ifdef ABL_NO_LIGHTPDF
        float pdf = 0.5f * 0.01f + 0.5f * bsdf_pdf;  // ablation build (timing only)
#else
        float pdf = 0.5f * lights_pdf<FT>(sc, p, ndir) + 0.5f * bsdf_pdf;
#endif
        PH_ADD(PH_LIGHT, t_light);
        // pdf >= 1e-30 when every light entry is a prim (sc.pdf_floor): a direction below
        // the surface (spdf = 0) whose light pdf test just misses the light's edge in fp32
        // (pdf = 0) weighs 0, not 0 * inf = NaN (camera.go:321-328 divides by the mixture
        // pdf; one sample in ~1e9 of C2 met this).  Any pdf > 1e-30 is untouched.  An empty
        // lights list's pdf is 0 by the reference's rules (hittable.go:89-103): its 0/0 NaNs
        // are the reference's own and stay (floor 0, test_world_without_lights_list).
        weight = (att * spdf) * rcp(fmaxf(pdf, sc.pdf_floor));
        clamp_vertex = true;
      }
      // vertex bookkeeping (H1: the clamp is folded backwards at termination)
      if (clamp_vertex) {
        if (s.flags & F_PEND) {
          const f3 pv = get_pend<SOA>(P, slot, s);
#ifndef RT_NO_WEIGHT_MERGE
          // Dominated clamp vertices are merged, not pushed.  The fold needs
          // max_k I(P_k) over the suffix products P_k = w_k (.) P_k+1 (WStack::fold_max);
          // with 0 <= w_k <= 1 in every channel, I(P_k) <= I(P_k+1) whatever follows,
          // so vertex k never sets the scale and only its product matters: w_k is
          // multiplied into the entry below instead of taking a stack entry (the
          // bottom entry is still pushed: merging it into the camera-side prefix
          // `pre`, which the book2 kernel keeps in scratch, cost more than it saved).
          // Same folded value up to fp32 rounding; paths through the water orb and
          // the fog (book2, up to 40 isotropic vertices) keep most of their stack in LDS.
          // Needs P_k+1 >= 0 in every channel: scenes with a negative colour, albedo or
          // background (sc.merge_ok = 0) push every vertex, which the fold handles exactly
          // for any sign.
          // (the flag is re-read from the kernel-argument segment here, kparams(): held in
          // an SGPR across the loop it added SGPR spills)
          const bool merge = kparams()->sc.merge_ok && s.nst > 0 && pv.x >= 0.0f && pv.y >= 0.0f &&
                             pv.z >= 0.0f && pv.x <= 1.0f && pv.y <= 1.0f && pv.z <= 1.0f;
#else
          const bool merge = false;
#endif
          if (merge) {
            f3 top = ws.mul(P, slot, s.nst - 1, pv);
            // Kernels with media also cascade: the merged top may itself now be
            // dominated by the new clamp vertex (0 <= top <= 1), so it folds into the
            // entry below, and so on.  Book2's HBM pushes: 309 M -> 126 M (merge) ->
            // 19 M (cascade) at 400 x 400 x 1024; C4 -1.7 %, while the lean and mesh
            // kernels, whose stacks stay shallow, lost 0.6-1.4 % to the loop
            // (profiles/r3_weight_cascade_ab.jsonl).
            if (HAS(FT_MEDIA))
              while (s.nst >= 2 && top.x >= 0.0f && top.y >= 0.0f && top.z >= 0.0f &&
                     top.x <= 1.0f && top.y <= 1.0f && top.z <= 1.0f) {
                top = ws.mul(P, slot, s.nst - 2, top);
                --s.nst;
              }
          } else {
            ws.put(P, slot, s.nst, {pv.x, pv.y, pv.z, 0.0f});
            ++s.nst;
#ifdef RT_COUNT_PUSHES
            ++s.pushes;  // a per-lane counter costs the fused kernels a VGPR: opt-in
#elif defined(RT_COUNT_HBM_PUSHES)
            if ((int)s.nst > ws.nlds) ++s.pushes;  // pushes that went to HBM (debug builds)
#endif
          }
        }
        set_pend<SOA>(P, slot, s, weight);
        s.flags |= F_PEND;
      } else if (s.flags & F_PEND) {
        set_pend<SOA>(P, slot, s, get_pend<SOA>(P, slot, s) * weight);
      } else {
        f3 w = (s.flags & F_PRE) ? get_pre<SOA>(P, slot, s) : mk3(1, 1, 1);
        set_pre<SOA>(P, slot, s, w * weight);
        s.flags |= F_PRE;
      }
      if (!finite3(weight)) s.flags |= F_NONFINITE;
      ++s.k;
      if ((int)s.k > P.max_depth) {  // rayColor(depth-1 < 0) == black, camera.go:294-296
        term = true;
        lterm = mk3(0, 0, 0);
      } else {
        // spheres: the new origin eta off the surface on the side the ray leaves to, so
        // the fp64 sphere test (exact for this fp32 point) sees it where the reference's
        // point is: outside for a ray leaving outward (no root ahead), inside for one
        // refracted or fuzz-reflected inward (the far root only).  eta = 0 elsewhere.
        if (HAS(FT_SPHERE)) p = p + n * copysignf(eta, dot(ndir, n));
        s.o = p;
        s.d = ndir;
        s.spare = rt_spare24(r);
        store_ray<SOA>(P, slot, s);
        return OUT_ALIVE;
      }
    }
  }
  // ---- termination: backward clamp fold (camera.go:316, :328-330)
  PH_T(t_term);
  f3 L = lterm;
  const bool zero = lterm.x == 0.0f && lterm.y == 0.0f && lterm.z == 0.0f;
  if (!(zero && !(s.flags & F_NONFINITE))) {
#ifdef RT_FOLD_STEPWISE
    if (s.flags & F_PEND) L = clamp_contribution(get_pend<SOA>(P, slot, s) * L, P.maxc);
    L = ws.fold(P, slot, s.nst, L);
#elif !defined(ABL_NO_FOLD)  // (ABL_NO_FOLD: ablation build, timing only)
    float maxI = 0.0f;  // no clamp vertex: no scale
    if (s.flags & F_PEND) {
      L = get_pend<SOA>(P, slot, s) * L;
      maxI = L.x + L.y + L.z;
      ws.fold_max(P, slot, s.nst, L, maxI);
    }
    // min(1, M / maxI) as one v_min: no compare and three v_cndmask_b32_e32 (and_not); the
    // scale is exactly 1 whenever M * rcp(maxI) >= 1 (maxI below M by more than an ulp)
    L = L * fminf(1.0f, P.maxc * rcp(maxI));
#endif
    if (s.flags & F_PRE) L = get_pre<SOA>(P, slot, s) * L;
  } else {
    L = mk3(0, 0, 0);
  }
#ifdef RT_NAN_DEBUG
  if (isnan(L.x) || isnan(L.y) || isnan(L.z)) printf("NAN gpix %u sample %u\n", s.gpix, s.s0 + s.j);
#endif
  sa.add(P, s.chunk, L);
  const uint32_t count = s.flags >> kCountShift;  // chunk_ids().count, or a drain split's
  if (s.j + 1 < count) {
    if (!have_rcam)  // a miss, or the depth limit: the camera draw is made here
      rcam = rt_rng_draw(P.seed, s.gpix, s.s0 + s.j + 1, RT_STREAM_CAMERA);
    next_sample<SOA, cam_mode(FT)>(P, slot, s, s.j + 1, rcam);
    PH_ADD(PH_TERM, t_term);
    return OUT_ALIVE;
  }
  sa.flush(P, s.chunk, (FT == 0u || kSplitTrees) && (s.flags & F_SPLIT));
  PH_ADD(PH_TERM, t_term);
  return OUT_NEED_CHUNK;
}

// the n-th (from 0) set bit of m, n < popcount(m)
RT_D uint32_t nth_set_bit(unsigned long long m, uint32_t n) {
  uint32_t pos = 0u;
#pragma unroll
  for (uint32_t w = 32u; w > 0u; w >>= 1) {
    const uint32_t lo = (uint32_t)__popcll(m & ((1ull << w) - 1ull));
    if (n >= lo) {
      n -= lo;
      m >>= w;
      pos += w;
    }
  }
  return pos;
}

// Drain of the fused kernel (every chunk handed out, wave-uniform call): the k-th lane
// without work takes the upper half of the samples left in the k-th lane that has at least
// P.split_min left after its current one.  Samples are keyed by (pixel, sample) and summed
// exactly, so who traces them does not change the image; the taker's sums go to the pixel
// with atomics (F_SPLIT), the giver's chunk record covers the samples it kept.  A taker gets
// the giver's chunk in `c`, its samples [j0, n0) of it (j0 >= 1), for start_sample.  A giver
// may be a taker or have given before: the count it passes on is its current one.
RT_D void split_samples(const Params& P, Path& s, bool has, uint32_t& c, uint32_t& j0,
                        uint32_t& n0) {
  const uint32_t cnt = s.flags >> kCountShift;
  const uint32_t left = has ? cnt - 1u - s.j : 0u;
  const bool giver = left >= kparams()->split_min;
  const unsigned long long need = __ballot(!has && c == 0xFFFFFFFFu), give = __ballot(giver);
  if (!need || !give) return;
  const uint32_t n_need = (uint32_t)__popcll(need), n_give = (uint32_t)__popcll(give);
  const bool needs = ((need >> lane_id()) & 1ull) != 0ull;
  const uint32_t rank = prefix_count(needs ? need : give);
  const bool taker = needs && rank < n_give;
  const uint32_t keep = cnt - ((left + 1u) >> 1);  // the giver's new sample count
  const uint32_t src = taker ? nth_set_bit(give, rank) : lane_id();
  const uint32_t t_chunk = __shfl(s.chunk, (int)src), t_keep = __shfl(keep, (int)src),
                 t_cnt = __shfl(cnt, (int)src);
  if (giver && rank < n_need) s.flags = (s.flags & ((1u << kCountShift) - 1u)) | (keep << kCountShift);
  if (taker) {
    c = t_chunk;
    j0 = t_keep;
    n0 = t_cnt;
  }
}

// Wave-batched work distribution over partitioned counters.  The chunk range is split
// into NP = 2^parts_log2 partitions, interleaved in granules of G = 2^gran_log2 chunks
// (granule j belongs to partition j % NP), each with its own counter of positions
// (Counters::part, 256 B apart).  Every partition therefore sweeps the image in the same
// order as one counter would (the row-group locality of chunk_pixel is kept), while the
// returning atomics are spread over NP addresses: one address saturates near 88
// returning atomics per µs on MI355X, which is what forced large batches (and the long
// tail they leave when the range runs out) on a single counter.  A wave starts on
// partition (wave id % NP); when its partition is used up it probes every counter with
// one load per lane and moves to the next one with work left.  Partitions whose atomic
// came back exhausted are remembered (`dead`), so the search ends after at most NP + 1
// atomics even on stale probes.  Lanes that need a chunk take consecutive positions from
// the wave's batch; the batch is refilled with ONE returning atomic per >= grab_min
// positions.  parts_log2 = 0 is the single counter (progress slices use it).
struct WaveBatch {
  uint32_t next, end;   // wave-uniform: positions [next, end) of partition `part`
  uint32_t part;        // the wave's partition; kMaxParts once every partition is used up
  unsigned long long dead;  // partitions known exhausted
};
RT_D uint32_t part_end(const Params& P, uint32_t p) {
  const uint32_t gl = P.gran_log2, lg = P.parts_log2;
  const uint32_t granules = (P.n_chunks + (1u << gl) - 1u) >> gl;
  return granules > p ? (((granules - p - 1u) >> lg) + 1u) << gl : 0u;
}
RT_D uint32_t part_chunk(const Params& P, uint32_t p, uint32_t pos) {
  const uint32_t gl = P.gran_log2;
  return ((((pos >> gl) << P.parts_log2) + p) << gl) | (pos & ((1u << gl) - 1u));
}
RT_D WaveBatch batch_init(const Params& P) {
  // wave-uniform (readfirstlane): the batch lives in SGPRs, not in VGPRs of every lane
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  return {0u, 0u, wave & ((1u << P.parts_log2) - 1u), 0ull};
}
RT_D uint32_t grab_chunk(const Params& P, WaveBatch& b, bool need) {
  const unsigned long long m = __ballot(need);
  if (!m) return 0xFFFFFFFFu;
  const uint32_t n = (uint32_t)__popcll(m);
  const uint32_t r = prefix_count(m);
  const uint32_t avail = b.end - b.next;
  // per lane only the chunk id: positions are mapped with the (uniform) partition of
  // the batch they come from, so no per-lane partition or position stays live
  uint32_t c = r < avail && b.part < (uint32_t)kMaxParts ? part_chunk(P, b.part, b.next + r)
                                                         : 0xFFFFFFFFu;
  if (n <= avail) {
    b.next = __builtin_amdgcn_readfirstlane(b.next + n);
  } else {
    const uint32_t leader = (uint32_t)(__ffsll((long long)m) - 1);
    const uint32_t np = 1u << P.parts_log2;
    uint32_t g = 0u, gend = 0u;
    // a wave-uniform loop: each pass either takes a batch, finds every partition used
    // up, or marks one more partition dead (at most NP + 1 passes)
    while (b.part < (uint32_t)kMaxParts) {
      const uint32_t endp = part_end(P, b.part);
      const uint32_t want = max(P.grab_min, n - avail);
      uint32_t v = 0u;
      if (lane_id() == leader) v = atomicAdd(&P.ctr->part[b.part * kPartStride], want);
      g = __builtin_amdgcn_readlane(v, leader);
      if (g < endp) {
        gend = min(g + want, endp);
        break;
      }
      b.dead |= 1ull << b.part;
      // probe: lane i reads partition i's counter (stale values only read low)
      const uint32_t li = lane_id();
      bool left = false;
      if (li < np)
        left = __hip_atomic_load(&P.ctr->part[li * kPartStride], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT) < part_end(P, li);
      const unsigned long long live = __ballot(left) & ~b.dead;
      if (!live) {
        b.part = (uint32_t)kMaxParts;
        break;
      }
      // the next live partition after this one, cyclically
      const uint32_t sh = b.part + 1u;
      const unsigned long long rot = sh >= 64u ? live : ((live >> sh) | (live << (64u - sh)));
      b.part = __builtin_amdgcn_readfirstlane((sh + (uint32_t)(__ffsll((long long)rot) - 1)) & 63u);
    }
    const uint32_t take = r - avail;  // this lane's offset in the new batch (r >= avail)
    if (r >= avail)
      c = b.part < (uint32_t)kMaxParts && g + take < gend ? part_chunk(P, b.part, g + take)
                                                          : 0xFFFFFFFFu;
    b.next = __builtin_amdgcn_readfirstlane(min(g + (n - avail), gend));
    b.end = __builtin_amdgcn_readfirstlane(gend);
  }
  if (!need) return 0xFFFFFFFFu;
  return c < P.n_chunks ? c : 0xFFFFFFFFu;
}

}  // namespace rt
