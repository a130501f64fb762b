/*
 * rt_rng.h — the counter-based random stream shared by the HIP path tracer and
 * the CPU oracle.  Part of the parity contract, not of the algorithm under test.
 *
 * The reference draws every random number from Go's process-global, unseeded
 * math/rand (camera.go:268,278-279; pdf.go:70; objects.go:71-72,162,372-373;
 * medium.go:47; materials.go:112; vec.go:28,178-179), so its renders are not
 * reproducible.  Here every draw is a pure function of
 *     (seed, global pixel index, sample index, path vertex, group, lane)
 * computed with Philox4x32-10 (Salmon et al., SC'11; Random123 constants).
 * Both implementations therefore consume identical uniforms no matter in which
 * order, on which rank, or in which wavefront slot a path is processed.
 *
 * Uniforms are 24-bit: u = (x >> 8) * 2^-24 in [0, 1 - 2^-24], exactly
 * representable in float and double, so the fp32 device path and the fp64
 * oracle start every path from bit-identical random numbers.
 *
 * Dimension map (one Philox call = 4 lanes):
 *   camera  group 0: [0] jitter x (inner stratum s_j)  [1] jitter y (outer s_i)
 *                    [2] ray time
 *                    [3] defocus disk (only when DefocusAngle > 0): its high and low
 *                        16 bits as two 16-bit uniforms (rt_unit16_hi / _lo), so a
 *                        defocused camera ray needs no second Philox call (round 4;
 *                        round 3 drew them from a camera group-1 call)
 *   vertex k group 0: [0] coin (mixture pdf pdf.go:70 / dielectric materials.go:112)
 *                     [1] light pick (hittable.go:102 rand.Intn) — 24-bit integer
 *                     [2],[3] direction sample (cosine, light, sphere, fuzz)
 *   vertex k group 1+g: medium free-flight draws 4g..4g+3 (medium.go:47), except
 *                     the scene's LAST free-flight draw index (medium_draws - 1),
 *                     which takes the spare bits below
 *   spare bits: every call above uses only the high 24 bits of a word, so the low
 *   bytes of words [0],[1],[2] of the call that generated a segment's ray (the
 *   camera group-0 call of its sample, or group 0 of the vertex that scattered it)
 *   form one more independent 24-bit uniform, rt_spare24(); it is that segment's
 *   last free-flight draw.  A scene whose only (or outermost, last-added) medium is
 *   crossed by every segment (book2's fog) then needs no group-1 call at all.
 */
#ifndef RT_RNG_H
#define RT_RNG_H

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define RT_RNG_FN __host__ __device__ __forceinline__
#else
#define RT_RNG_FN static inline
#endif

#define RT_PHILOX_M0 0xD2511F53u
#define RT_PHILOX_M1 0xCD9E8D57u
#define RT_PHILOX_W0 0x9E3779B9u
#define RT_PHILOX_W1 0xBB67AE85u

/* stream ids */
#define RT_STREAM_CAMERA 0xFFFFFFF0u
#define RT_STREAM(vertex, group) ((((uint32_t)(vertex)) << 4) | (uint32_t)(group))

typedef struct {
  uint32_t v[4];
} rt_u32x4;

RT_RNG_FN rt_u32x4 rt_philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                    uint32_t k0, uint32_t k1) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(RT_RNG_ROLLED)
  /* ten rounds straight-line (the compiler kept a loop of three): C3 -0.5 %, C4 -0.5 %,
     C5 -0.4 %, C2 +-0, same words (profiles/r3_rng_unroll_ab.jsonl) */
#pragma unroll
#endif
#ifndef RT_PHILOX_ROUNDS
#define RT_PHILOX_ROUNDS 10 /* other values: timing ablations only (not the parity stream) */
#endif
  for (int r = 0; r < RT_PHILOX_ROUNDS; ++r) {
    if (r) {
      k0 += RT_PHILOX_W0;
      k1 += RT_PHILOX_W1;
    }
    uint64_t p0 = (uint64_t)RT_PHILOX_M0 * (uint64_t)c0;
    uint64_t p1 = (uint64_t)RT_PHILOX_M1 * (uint64_t)c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
#if defined(__HIP_DEVICE_COMPILE__) && !defined(RT_RNG_XOR2)
    /* gfx950 v_bitop3_b32 (truth table 0x96 = a ^ b ^ c): one instruction per
       three-way xor where hipcc emits two v_xor_b32; the same words */
    uint32_t n0 = __builtin_amdgcn_bitop3_b32(hi1, c1, k0, 0x96);
    uint32_t n2 = __builtin_amdgcn_bitop3_b32(hi0, c3, k1, 0x96);
#else
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
#endif
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  rt_u32x4 out;
  out.v[0] = c0;
  out.v[1] = c1;
  out.v[2] = c2;
  out.v[3] = c3;
  return out;
}

/* Four raw 32-bit draws for (pixel, sample, stream). */
RT_RNG_FN rt_u32x4 rt_rng_draw(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t stream) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#if defined(__HIP_DEVICE_COMPILE__) && !defined(RT_RNG_HOIST_KEYS)
  /* an empty asm that "changes" the key: the compiler cannot hoist the 18 round keys out
     of the fused kernels' main loops, where they sat in SGPRs for the whole kernel and
     pushed other values out to VGPR lanes; recomputing them is 18 scalar adds a call
     (C2 -1.5 %, C3 -0.7 %, C4 -0.5 %: profiles/r3_rng_keys_ab.jsonl) */
  __asm__ volatile("" : "+s"(k0), "+s"(k1));
#endif
  return rt_philox4x32_10(pixel, sample, stream, 0u, k0, k1);
}

RT_RNG_FN uint32_t rt_u24(uint32_t x) { return x >> 8; }

/* the 24 spare bits of a call (see the dimension map), as a word whose high 24 bits
   hold them: rt_unit_f / rt_unit_d of it is the spare uniform */
RT_RNG_FN uint32_t rt_spare24(rt_u32x4 r) {
  return ((r.v[0] & 0xFFu) << 24) | ((r.v[1] & 0xFFu) << 16) | ((r.v[2] & 0xFFu) << 8);
}

RT_RNG_FN float rt_unit_f(uint32_t x) { return (float)(x >> 8) * 5.9604644775390625e-08f; }

RT_RNG_FN double rt_unit_d(uint32_t x) { return (double)(x >> 8) * 5.9604644775390625e-08; }

/* 16-bit uniforms from the two halves of a word (the defocus disk, camera word [3]):
   exact in float and double, in [0, 1 - 2^-16] */
RT_RNG_FN float rt_unit16_hi_f(uint32_t x) { return (float)(x >> 16) * 1.52587890625e-05f; }
RT_RNG_FN float rt_unit16_lo_f(uint32_t x) { return (float)(x & 0xFFFFu) * 1.52587890625e-05f; }
RT_RNG_FN double rt_unit16_hi_d(uint32_t x) { return (double)(x >> 16) * 1.52587890625e-05; }
RT_RNG_FN double rt_unit16_lo_d(uint32_t x) { return (double)(x & 0xFFFFu) * 1.52587890625e-05; }

/* rand.Intn(n) replacement: exact integer map of the 24-bit uniform to [0, n). */
RT_RNG_FN uint32_t rt_pick(uint32_t x, uint32_t n) {
  return (uint32_t)(((uint64_t)(x >> 8) * (uint64_t)n) >> 24);
}

/* residual 24-bit uniform left after rt_pick (used for nested light lists) */
RT_RNG_FN uint32_t rt_pick_residual(uint32_t x, uint32_t n) {
  return (uint32_t)((((uint64_t)(x >> 8) * (uint64_t)n) & 0xFFFFFFu) << 8);
}

#endif /* RT_RNG_H */
