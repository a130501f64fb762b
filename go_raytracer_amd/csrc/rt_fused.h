// rt_fused.h — the fused persistent kernel k_fused and the device helpers it shares with
// the wavefront kernels (stage_nodes, finish_hit).  A header so that kernel instantiations
// can be compiled in their own translation units with their own code-generation flags
// (rt_fused_sets.hip: the scheduler strategy per kernel); rt_render.hip holds the rest.
#pragma once
#include "rt_path.h"

namespace rt {

// the whole node array (W F4 per node) -> LDS (only used when it fits in
// kLdsNodes 64-B slots), then the leaf records when they fit too
RT_D bool stage_nodes(const Params& P, F4* lnodes, int W) {
  const int nl = min(P.sc.n_nodes, 4 * kLdsNodes / W);
  for (int i = threadIdx.x; i < W * nl; i += blockDim.x) lnodes[i] = P.sc.nodes[i];
  const bool recs = P.recs_lds != 0u;
  if (recs) {
    // + the lean set's shade table after the record pairs (rt_render.hip)
    const int n = 4 * P.sc.n_refs + (P.sc.shade_lds >= 0 ? P.sc.shade_n : 0);
    for (int i = threadIdx.x; i < n; i += blockDim.x) lnodes[W * nl + i] = P.sc.leafprims[i];
  }
  __syncthreads();
  return recs;
}

RT_D void record_trace(const Params& P, const Path& s, const Hit& best) {
  if (s.gpix == P.trace_gpix && s.s0 + s.j == P.trace_sample && (int)s.k < P.trace_cap) {
    P.trace[3 * s.k + 0] = {s.o.x, s.o.y, s.o.z, s.time};
    P.trace[3 * s.k + 1] = {s.d.x, s.d.y, s.d.z, (float)s.k};
    P.trace[3 * s.k + 2] = {best.t, best.u, best.v, bitsf(best.ref)};
  }
}

// media + debug trace on top of the world closest hit, camera.go:300
template <uint32_t FT>
RT_D void finish_hit(const Params& P, const Path& s, Hit& best) {
#ifndef RT_NO_TRI_REFINE
  if (HAS(FT_TRI) && best.ref != PRIM_NONE && (best.ref >> 30) == PRIM_TRI)
    refine_tri_hit(P.sc, best.ref & 0x3FFFFFFFu, s.o, s.d, best.t, best.u, best.v);
#endif
#ifdef RT_SPHERE32_LEAVES
  // a BVH sphere leaf won (fp32 test): its t in fp64 (v = -1: a big sphere, fp64 already)
  if (HAS(FT_SPHERE) && best.ref != PRIM_NONE && (best.ref >> 30) == PRIM_SPHERE && best.v >= 0.0f)
    refine_sphere_hit(P.sc, best.ref & 0x3FFFFFFFu, s.o, s.d, s.time, best.t);
#endif
#ifdef ABL_NO_MEDIA
  if (false)
#else
  if (HAS(FT_MEDIA) && P.sc.n_media > 0)
#endif
    trace_media(P, s.o, s.d, s.time, 0.001f, s.gpix, s.s0 + s.j, s.k, s.spare, best);
  if (P.trace) record_trace(P, s, best);
}

// ----------------------------------------------------------------- fused ---
// FT = compiled-in scene features (rt_device.h), chosen per scene by pick_fused.
// Waves per SIMD by feature set: the lean sets fit more waves in the register
// file (VGPRs <= 512 / waves) and in LDS (24 KB static + the scene cache).
#ifndef MESH_WAVES
#define MESH_WAVES 4
#endif
#ifndef TRI_WAVES
#define TRI_WAVES 4
#endif
#ifndef TRI_QWAVES
// the {sphere, triangle, metal} set (C5) on the compressed BVH4 at 5 waves per SIMD (round
// 5): that kernel needs 113 VGPRs at 4, and 5 waves (96 VGPRs, 1 spilled with the default
// scheduler; 13 LDS stack entries, TRI_QSHORT, so five blocks fit the CU's LDS) measured C5 -3.8 %
// (profiles/r5_c4_c5_isolation_ab.jsonl); round 2's 5-wave try of the 128-B-node kernel
// spilled 32 VGPRs in the traversal loop and lost 24 %
#define TRI_QWAVES 5
#endif
// RT_QTOP=N (experiment): the compressed BVH4's first N items (BFS order: the root and its
// top levels, which nearly every ray visits) staged in dynamic LDS at kernel start and read
// from there, off the vector-memory return path that bounds C5; one LDS stack entry fewer
// so five blocks still fit
#ifdef RT_QTOP
#ifndef TRI_QSHORT
#define TRI_QSHORT 12
#endif
#ifndef MESH_QSHORT
#define MESH_QSHORT 12
#endif
#endif
#ifndef TRI_QSHORT
// 13 LDS traversal-stack entries fill five blocks' LDS (5 x 31,776 B of 160 KiB): C5 -1.5 %,
// C3 -0.3 % against 12, 10 +4.5 % (profiles/r5_qshort_ab.jsonl)
#define TRI_QSHORT 13
#endif
#ifndef MESH_QWAVES
// book1's set (C3) on the compressed BVH4 at 5 waves too (96 VGPRs, 1 spilled with the default
// scheduler, 13 LDS stack entries): C3 -1.2 % with the ILP scheduler's 26 spills
// (profiles/r5_waves5_ab.jsonl), -5.5 % more without them; book2's set at 5 waves lost 3 %
// (31 spilled), it stays at 4
#define MESH_QWAVES 5
#endif
#ifndef MESH_QSHORT
#define MESH_QSHORT 13
#endif
#ifndef FT_TEX_WAVES
#define FT_TEX_WAVES 4
#endif
#ifndef BRUTE_WAVES
#define BRUTE_WAVES 6
#endif
// The record-loop kernels (TREE 0) need no traversal stack: kBruteWaves.
constexpr int kBruteWaves = BRUTE_WAVES;
constexpr int fused_waves(uint32_t ft, int tree = 4) {
  return (tree == 0 && ft == 0u) ? kBruteWaves  // 7 measured within noise of 6, 8 -3 %
         : ft == 0u ? 6
         : ft == FT_MEDIA ? 4
         : ft == (FT_SPHERE | FT_TRI | FT_METAL) ? (tree == 5 ? TRI_QWAVES : TRI_WAVES)
         : ft == (FT_SPHERE | FT_TRI | FT_METAL | FT_DIEL | FT_CHECKER) ? (tree == 5 ? MESH_QWAVES : MESH_WAVES)
         : ft == FT_SET_BOOK2 ? FT_TEX_WAVES
                                                                                  : 3;
}
// LDS clamp-weight entries (12 B each): 6 (C2 +1 %, C3 +2.5 % over 3-4), 4 for the
// mesh set, whose specular paths rarely push weights (C5 -1.5 % with 6), and 4 for
// the lean set's tree kernels (their stack + sums must fit 6 waves/SIMD)
#ifndef MESH_WLDS
#define MESH_WLDS 4
#endif
#ifndef MESH_SHORT
#define MESH_SHORT 16  // C5's 1M-triangle tree: -1.3 % against 12 (r2_mesh_short_ab.jsonl)
#endif
#ifndef TRI_SHORT
#define TRI_SHORT MESH_SHORT  // the {sphere, triangle, metal} set (C5)
#endif
#ifndef TRI_WLDS
#define TRI_WLDS MESH_WLDS
#endif
#ifndef TEX_SHORT
// book2's set: 10 traversal-stack and 5 weight entries fill its 4-wave LDS budget with the
// staged perlin tables (C4 -0.8 % against 13 x 4, +2 % at 7 x 6 on the compressed BVH4,
// profiles/r5_c4_stack_split_ab.jsonl; round 3 on the 128-B nodes: 16 x 3 / 18 x 2 / 21 x 1
// +0.6 to +1.7 % against 13 x 4, r3_tex_stack_ab.jsonl)
#define TEX_SHORT 10
#endif
#ifndef TEX_WLDS
#define TEX_WLDS 5
#endif
#ifndef ALL_WLDS
#define ALL_WLDS 4  // 6 pushed the C3-size trees out of the 3-wave LDS budget
#endif
#ifndef BRUTE_WLDS
#define BRUTE_WLDS kLdsWMax
#endif
constexpr int fused_wlds(uint32_t ft, int tree = 4) {
  return ft == (FT_SPHERE | FT_TRI | FT_METAL | FT_DIEL | FT_CHECKER) ? MESH_WLDS
         : ft == (FT_SPHERE | FT_TRI | FT_METAL)                    ? TRI_WLDS
         : (ft == 0u && tree != 0)                                  ? 4
         : (ft == 0u && tree == 0)                                  ? BRUTE_WLDS
         : ft == FT_ALL                                             ? ALL_WLDS
         : ft == FT_SET_BOOK2 ? TEX_WLDS
                                                                    : kLdsWMax;
}
// short traversal stack: none for the record loop, 6 entries for the lean set
// (tiny trees; its LDS budget at 6 waves/SIMD), 12 elsewhere; deeper ones in HBM
constexpr int fused_short(uint32_t ft, int tree = 4) {
  return tree == 0                                                    ? 0
         : ft == 0u                                                   ? kShortStackMin
         : ft == (FT_SPHERE | FT_TRI | FT_METAL | FT_DIEL | FT_CHECKER) ? (tree == 5 ? MESH_QSHORT : MESH_SHORT)
         : ft == (FT_SPHERE | FT_TRI | FT_METAL)                      ? (tree == 5 ? TRI_QSHORT : TRI_SHORT)
         : ft == FT_SET_BOOK2 ? TEX_SHORT
                                                                      : kShortStack;
}
// + 24 B per lane of chunk sums (SampleAcc) + the perlin tables of noise kernels
constexpr unsigned fused_static_lds(uint32_t ft, int tree = 4) {
  return (unsigned)(fused_short(ft, tree) * 4 + fused_wlds(ft, tree) * 12 + 24) * 256u +
         ((ft & FT_NOISE) ? 256u * 16u + 768u : 0u);
}
__shared__ unsigned long long g_tstart[4];  // per wave: k_fused's start time (RT_WAVE_TIMES)
#ifdef RT_DRAIN_TIMES
__shared__ unsigned long long g_tdrain[4];  // debug builds: when the wave's grab came back empty
__shared__ unsigned long long g_dinfo[4][3];  // ... and then: samples left, busy lanes, segments
#endif
// TREE: 4 = BVH4, 5 = compressed BVH4 (64-B nodes, global only), 2 = BVH2, 0 = no tree
// (every record tested, tiny scenes)
template <bool LDS, uint32_t FT, int TREE>
__global__ __launch_bounds__(256, fused_waves(FT, TREE)) void k_fused(Params P) {
  extern __shared__ F4 lnodes[];  // LDS scene cache, sized at launch (scene_lds_bytes)
  __shared__ uint32_t lstack[(fused_short(FT, TREE) > 0 ? fused_short(FT, TREE) : 1) * 256];
  __shared__ float lw[3 * fused_wlds(FT, TREE) * 256];
  __shared__ unsigned long long lacc[3 * 256];  // per-lane chunk sums (SampleAcc)
  for (int ch = 0; ch < 3; ++ch) lacc[ch * 256 + threadIdx.x] = 0ull;
  if constexpr (HAS(FT_NOISE)) stage_perlin(P.sc);  // before stage_nodes' barrier
  if constexpr (cam_mode(FT) == 1) stage_camera(P);
  const bool recs_lds = LDS && TREE != 8 && stage_nodes(P, lnodes, TREE == 4 ? 8 : 4);
#ifdef RT_QTOP
  if constexpr (TREE == 5) {  // the top items into the dynamic LDS (sized at launch)
    const uint32_t nq = 4u * (uint32_t)min(RT_QTOP, P.sc.n_nodes);
    for (uint32_t i = threadIdx.x; i < nq; i += blockDim.x) st_lds(&lnodes[i], ld_glb(P.sc.nodes + i));
  }
#endif
  if (!LDS) __syncthreads();  // staged tables visible to every wave (stage_nodes ends with one)
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;  // weight-stack column
  const TravStack ts = {&lstack[threadIdx.x], P.ostack + slot, P.stack_cols, fused_short(FT, TREE)
#ifdef RT_COUNT_TRAV_OVF
                        , &P.ctr->pushes
#endif
  };
  const WStack ws = {&lw[threadIdx.x], fused_wlds(FT, TREE)};
  const SampleAcc sa = {&lacc[threadIdx.x]};
  Path s;
  s.pushes = 0;
  if constexpr ((FT == 0u && TREE == 0) || kSplitTrees) {  // read by split_samples before a lane's first chunk
    s.chunk = s.j = 0u;
    s.flags = 0u;
  }
#ifdef RT_WAVE_SEGS
  uint32_t wave_segs = 0;  // segments shaded by this wave (wave-uniform: no VGPR)
#else
  s.segs = 0;
#endif
  Trav tr;
  tr.cur = TRAV_DONE;
  bool has = false;
  WaveBatch b = batch_init(P);
  // debug (RT_WAVE_TIMES): the wave's start time parks in LDS (a register held across the
  // loop for this was the record-loop kernel's one spilled VGPR)
  // (the record-loop kernel keeps the wave's index in an SGPR: threadIdx.x >> 6 kept to the
  // end took its one spilled VGPR; the compressed-BVH kernels spill two more VGPRs that way)
  const uint32_t wave_in_group = (FT == 0u && TREE == 0) ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)
                                                         : threadIdx.x >> 6;
  if (P.wave_times && lane_id() == 0u) g_tstart[wave_in_group] = wall_clock64();
#ifdef RT_DRAIN_TIMES
  if (lane_id() == 0u) g_tdrain[wave_in_group] = 0ull;
#endif
  // Scheduling round: lanes without work take a chunk; traversing lanes run up
  // to step_budget traversal steps; lanes whose traversal is done are shaded
  // together once at least shade_min of them wait (or nothing else traverses),
  // so traversal divergence costs idle lanes only until the next round.
#ifdef RT_PHASES
  if (threadIdx.x < 4 * PH_N) (&g_ph[0][0])[threadIdx.x] = 0ull;
  __syncthreads();
#endif
  PH_T(t_loop);
  for (;;) {
    PH_T(t_grab);
    uint32_t c = grab_chunk(P, b, !has), j0 = 0u, n0 = 0u;
    // lanes share samples in the drain (split_samples; RT_NO_SPLIT_TREES: the record-loop
    // kernel only)
    constexpr bool kSplit = (FT == 0u && TREE == 0) || kSplitTrees;
    if constexpr (kSplit)
      if (b.part >= (uint32_t)kMaxParts) split_samples(P, s, has, c, j0, n0);
    if (c != 0xFFFFFFFFu) {
      start_sample<false, cam_mode(FT), FT == 0u && TREE == 0>(P, slot, s, c, j0);
      if constexpr (kSplit)
        if (j0) s.flags = F_SPLIT | (n0 << kCountShift);
      trav_init<FT>(P.sc, s.o, s.d, s.time, tr);
#ifdef RT_QROOT  // (opt-in: +2-4 % on C3-C5)
      if constexpr (TREE == 5) trav_root_q(ts, s.o, 0.001f, tr);
#endif
      has = true;
    }
    PH_ADD(PH_GRAB, t_grab);
#ifdef RT_DRAIN_TIMES
    if (b.part >= (uint32_t)kMaxParts && __builtin_amdgcn_readfirstlane((uint32_t)(g_tdrain[wave_in_group] != 0ull)) == 0u) {
      uint32_t rem = has ? (s.flags >> kCountShift) - s.j : 0u, act = has ? 1u : 0u;
#ifndef RT_WAVE_SEGS
      uint32_t sg = s.segs;
#else
      uint32_t sg = 0u;
#endif
      for (int off = 32; off > 0; off >>= 1) {
        rem += __shfl_xor(rem, off);
        act += __shfl_xor(act, off);
        sg += __shfl_xor(sg, off);
      }
      if (lane_id() == 0u) {
        g_tdrain[wave_in_group] = wall_clock64();
        g_dinfo[wave_in_group][0] = rem;
        g_dinfo[wave_in_group][1] = act;
        g_dinfo[wave_in_group][2] = sg;
      }
    }
#endif
    if (!__any(has)) break;
    PH_T(t_trav);
    if (has && tr.cur != TRAV_DONE)
    {
      PH_CNT(PH_TRAV_LANES, __popcll(__ballot(1)));
      PH_CNT(PH_TRAV_ROUNDS, 1);
      if constexpr (TREE == 0)
        trav_brute<FT, !LDS>(P.sc, lnodes, s.o, s.d, s.time, 0.001f, tr);
      else if constexpr (TREE == 8)
      {
        const int nsteps = trav_steps8<FT>(P.sc, ts, s.o, s.d, s.time, 0.001f, tr, P.step_budget);
#ifdef RT_PHASES
        ph_steps(nsteps);
#endif
        (void)nsteps;
      }
      else
      {
        // TREE 5: the compressed BVH4 (64-B items, host_qbvh.cpp), read through L1/L2
        const int nsteps = trav_steps<LDS, FT, TREE == 4 || TREE == 5, TREE == 5>(
            P.sc, lnodes, recs_lds, ts, s.o, s.d, s.time, 0.001f, tr, P.step_budget);
        retest_near<FT>(P.sc, s.o, s.d, 0.001f, tr);
#ifdef RT_PHASES
        ph_steps(nsteps);
#endif
        (void)nsteps;
      }
    }
    PH_ADD(PH_TRAV, t_trav);
    const bool ready = has && tr.cur == TRAV_DONE;
    const uint32_t n_ready = (uint32_t)__popcll(__ballot(ready));
    const bool busy = __any(has && !ready);
    if (n_ready >= P.shade_min || !busy) {
#ifdef RT_WAVE_SEGS
      wave_segs += n_ready;
#endif

      if (ready) {
        PH_CNT(PH_SHADE_LANES, n_ready);
        PH_CNT(PH_SHADE_ROUNDS, 1);
        PH_T(t_media);
        Hit best = tr.best;
        finish_hit<FT>(P, s, best);
        PH_ADD(PH_MEDIA, t_media);
#ifndef RT_WAVE_SEGS
        ++s.segs;
#endif
        PH_T(t_shade);
        if (shade_core<false, FT>(P, slot, s, best, ws, sa) == OUT_NEED_CHUNK) has = false;
        else {
          trav_init<FT>(P.sc, s.o, s.d, s.time, tr);
#ifdef RT_QROOT  // (opt-in: +2-4 % on C3-C5)
          if constexpr (TREE == 5) trav_root_q(ts, s.o, 0.001f, tr);
#endif
        }
        PH_ADD(PH_SHADE, t_shade);
      }
    }
  }
  PH_ADD(PH_LOOP, t_loop);
#ifdef RT_WAVE_SEGS
  const uint32_t segs = wave_segs;
#else
  uint32_t segs = s.segs;
  for (int off = 32; off > 0; off >>= 1) segs += __shfl_xor(segs, off);
#endif
  uint32_t pushes = s.pushes;
  for (int off = 32; off > 0; off >>= 1) pushes += __shfl_xor(pushes, off);
  if (lane_id() == 0) {
    atomicAdd(&P.ctr->segments, (unsigned long long)segs);
    atomicAdd(&P.ctr->pushes, (unsigned long long)pushes);
    if (P.wave_times) {
      const size_t w = (size_t)blockIdx.x * 4 + wave_in_group;
      unsigned long long* rec = P.wave_times + kWaveRec * w;
      rec[0] = g_tstart[wave_in_group];
      rec[1] = wall_clock64();
      rec[2] = segs;
#ifdef RT_DRAIN_TIMES
      rec[3] = g_tdrain[wave_in_group];
#else
      rec[3] = 0ull;
#endif
#ifdef RT_PHASES
      for (int i = 0; i < PH_N; ++i) rec[4 + i] = g_ph[wave_in_group][i];
#else
      for (int i = 0; i < PH_N; ++i) rec[4 + i] = 0ull;
#ifdef RT_DRAIN_TIMES
      for (int i = 0; i < 3; ++i) rec[4 + i] = g_dinfo[wave_in_group][i];
#endif
#endif
    }
  }
}

// The kernels compiled in rt_fused_sets.hip instead of rt_render.hip, with LLVM's
// iterative-ILP machine scheduler (Makefile): the C5 mesh set and the C3 sphere set
// (C5 -0.6 / -1.0 %, C3 -0.8 %, images bit-identical; the same strategy costs the C2 kernel
// 3.5 %, profiles/r3_sched_strategy_ab.jsonl, r3_split_ilp_ab.jsonl).  X(LDS, FT, TREE).
// The compressed-BVH kernels (TREE 5) are not in this list: at 5 waves per SIMD the ILP
// scheduler spilled 6 / 26 VGPRs in them against 1 / 2 with the default one, and the default
// one renders C3 5.5 % and C5 0.3 % faster (bit-identical, profiles/r5_q_sched_ab.jsonl).
// (book2's compressed-BVH kernel with the ILP scheduler: C4 +0.7 %, r5_book2_sched_ab.jsonl)
#define RT_FUSED_ILP_KERNELS(X)                                             \
  X(true, (FT_SPHERE | FT_TRI | FT_METAL), 4)                               \
  X(false, (FT_SPHERE | FT_TRI | FT_METAL), 4)                              \
  X(true, (FT_SPHERE | FT_TRI | FT_METAL | FT_DIEL | FT_CHECKER), 4)        \
  X(false, (FT_SPHERE | FT_TRI | FT_METAL | FT_DIEL | FT_CHECKER), 4)

}  // namespace rt
