// Issue cost of the integer and fp ops the path tracer's RNG and traversal use (dev tool):
// hipcc --offload-arch=gfx950 -O3 tools/instr_rate.hip -o /tmp/instr_rate && /tmp/instr_rate
// Each kernel runs 8 independent chains of one instruction per lane for ITERS iterations (the
// loop unrolled 8x: 64 instructions per 3 SALU of loop control); the result is SIMD cycles
// per wave-instruction at 1, 2 and 4 waves per SIMD, from the launch's wall time at the
// shader clock measured in the kernel (one block per CU: see run()).
#include <hip/hip_runtime.h>
#pragma clang diagnostic ignored "-Wunused-value"
#pragma clang diagnostic ignored "-Wunused-result"
#include <stdio.h>
#include <stdint.h>

#define ITERS 4096  // x 8 independent chains per iteration, 8 x unrolled (below)

// In-kernel timing of wave 0 of block 0: s_memtime counts shader cycles
// (MI355X_MICROARCH.md constants table), s_memrealtime a constant 100 MHz.  The SIMD's issue
// cost is the wave's elapsed shader cycles over the instructions issued by the waves sharing
// its SIMD (every wave runs the same stream, all resident at once), so neither the clock
// frequency nor the launch overhead enters it; the clock itself is reported beside it.
__device__ unsigned long long g_tim[2];
#define T_BEGIN                                                                           \
  const unsigned long long _c0 = __builtin_amdgcn_s_memtime(),                            \
                           _r0 = __builtin_amdgcn_s_memrealtime();                \
  _Pragma("unroll 8")
#define T_END                                                                             \
  if (blockIdx.x == 0 && threadIdx.x == 0) {                                              \
    g_tim[0] = __builtin_amdgcn_s_memtime() - _c0;                                        \
    g_tim[1] = __builtin_amdgcn_s_memrealtime() - _r0;                                    \
  }

#define BODY8(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)

__global__ void k_mad_u64(uint32_t* out, uint32_t seed) {
  uint64_t a[8];
  uint32_t m = 0xD2511F53u ^ seed;
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) { uint64_t cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(a[i]), "=s"(cc) : "v"((uint32_t)a[i]), "s"(m)); }
    BODY8(OP)
#undef OP
  } T_END
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= (uint32_t)a[i] ^ (uint32_t)(a[i] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mul_hi(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  uint32_t m = 0xD2511F53u ^ seed;
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_mul_hi_u32 %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "s"(m));
    BODY8(OP)
#undef OP
  } T_END
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mul_lo(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  uint32_t m = 0xD2511F53u ^ seed;
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "s"(m));
    BODY8(OP)
#undef OP
  } T_END
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mul_u24(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  uint32_t m = 0x511F53u ^ seed;
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_mul_u32_u24 %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "s"(m));
    BODY8(OP)
#undef OP
  } T_END
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_xor(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  uint32_t m = 0xD2511F53u ^ seed;
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_xor_b32 %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "s"(m));
    BODY8(OP)
#undef OP
  } T_END
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fma(uint32_t* out, uint32_t seed) {
  float a[8];
  float m = 1.0000001f + (float)seed;
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_fma_f32 %0, %1, %2, %1" : "=v"(a[i]) : "v"(a[i]), "s"(m));
    BODY8(OP)
#undef OP
  } T_END
  float s = 0;
  for (int i = 0; i < 8; ++i) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = __float_as_uint(s);
}
typedef float v2f __attribute__((ext_vector_type(2)));
__global__ void k_pk_fma(uint32_t* out, uint32_t seed) {
  v2f a[8];
  v2f m = {1.0000001f + (float)seed, 1.0000002f};
  for (int i = 0; i < 8; ++i) a[i] = v2f{(float)threadIdx.x, (float)i};
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_pk_fma_f32 %0, %1, %2, %1" : "=v"(a[i]) : "v"(a[i]), "v"(m));
    BODY8(OP)
#undef OP
  } T_END
  float s = 0;
  for (int i = 0; i < 8; ++i) s += a[i].x + a[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = __float_as_uint(s);
}
__global__ void k_fma64(uint32_t* out, uint32_t seed) {
  double a[8];
  double m = 1.0000001 + (double)seed;
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_fma_f64 %0, %1, %2, %1" : "=v"(a[i]) : "v"(a[i]), "v"(m));
    BODY8(OP)
#undef OP
  } T_END
  double s = 0;
  for (int i = 0; i < 8; ++i) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}
__global__ void k_rcp(uint32_t* out, uint32_t seed) {
  float a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i + 1 + seed;
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_rcp_f32 %0, %1" : "=v"(a[i]) : "v"(a[i]));
    BODY8(OP)
#undef OP
  } T_END
  float s = 0;
  for (int i = 0; i < 8; ++i) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = __float_as_uint(s);
}
__global__ void k_cvt_f64(uint32_t* out, uint32_t seed) {
  double a[8];
  float f[8];
  for (int i = 0; i < 8; ++i) f[i] = threadIdx.x * 7 + i + 1 + seed;
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(a[i]) : "v"(f[i]));
    BODY8(OP)
#undef OP
  } T_END
  double s = 0;
  for (int i = 0; i < 8; ++i) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}

// generic: 8 independent chains of one VOP2/VOP3 op "OP dst, dst, s"
#define K_BIN(NAME, ASM, T)                                                              \
  __global__ void NAME(uint32_t* out, uint32_t seed) {                                    \
    T a[8];                                                                              \
    T m = (T)(1.0000001f + (float)seed);                                                 \
    for (int i = 0; i < 8; ++i) a[i] = (T)(threadIdx.x * 7 + i);                         \
    T_BEGIN for (int it = 0; it < ITERS; ++it) {                                                 \
      OPS_##NAME                                                                         \
    } T_END                                                                                    \
    T s = 0;                                                                             \
    for (int i = 0; i < 8; ++i) s += a[i];                                               \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;                            \
  }
#define CH(ASM, i) asm volatile(ASM : "+v"(a[i]) : "v"(m));
#define CH8(ASM) CH(ASM, 0) CH(ASM, 1) CH(ASM, 2) CH(ASM, 3) CH(ASM, 4) CH(ASM, 5) CH(ASM, 6) CH(ASM, 7)
#define OPS_k_add_f32 CH8("v_add_f32 %0, %0, %1")
#define OPS_k_mul_f32 CH8("v_mul_f32 %0, %0, %1")
#define OPS_k_max_f32 CH8("v_max_f32 %0, %0, %1")
#define OPS_k_min3_f32 CH8("v_min3_f32 %0, %0, %1, %0")
#define OPS_k_add_u32 CH8("v_add_u32 %0, %0, %1")
#define OPS_k_and_b32 CH8("v_and_b32 %0, %0, %1")
#define OPS_k_lshr_b32 CH8("v_lshrrev_b32 %0, 3, %0")
#define OPS_k_mov_b32 CH8("v_mov_b32 %0, %1")
#define OPS_k_cndmask CH8("v_cndmask_b32 %0, %0, %1, vcc")
#define OPS_k_bitop3 CH8("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96")
#define OPS_k_cvt_f32_u32 CH8("v_cvt_f32_u32 %0, %0")
#define OPS_k_sqrt_f32 CH8("v_sqrt_f32 %0, %0")
#define OPS_k_cmp_f32 CH8("v_cmp_lt_f32 vcc, %0, %1")
K_BIN(k_add_f32, 0, float)
K_BIN(k_mul_f32, 0, float)
K_BIN(k_max_f32, 0, float)
K_BIN(k_min3_f32, 0, float)
K_BIN(k_add_u32, 0, uint32_t)
K_BIN(k_and_b32, 0, uint32_t)
K_BIN(k_lshr_b32, 0, uint32_t)
K_BIN(k_mov_b32, 0, uint32_t)
K_BIN(k_cndmask, 0, uint32_t)
K_BIN(k_bitop3, 0, uint32_t)
K_BIN(k_cvt_f32_u32, 0, uint32_t)
K_BIN(k_sqrt_f32, 0, float)
K_BIN(k_cmp_f32, 0, float)

// selects: the mask set by a compare before the loop (vcc, or an SGPR pair through VOP3)
__global__ void k_cndmask_vcc(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  uint32_t m = 0x12345u ^ seed;
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" ::"v"(threadIdx.x) : "vcc");
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(m) : "vcc");
    BODY8(OP)
#undef OP
  } T_END
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_cndmask_sgpr(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  uint32_t m = 0x12345u ^ seed;
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  unsigned long long msk;
  asm volatile("v_cmp_gt_u32 %0, 32, %1" : "=s"(msk) : "v"(threadIdx.x));
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(m), "s"(msk));
    BODY8(OP)
#undef OP
  } T_END
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// the same select as VOP3 (e64) naming vcc, and VOP2 after a scalar write of vcc: is the
// ~23-cycle cost of v_cndmask_b32_e32 the encoding or the implicit vcc read?
__global__ void k_cndmask_e64_vcc(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  uint32_t m = 0x12345u ^ seed;
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" ::"v"(threadIdx.x) : "vcc");
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(m) : "vcc");
    BODY8(OP)
#undef OP
  } T_END
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_cndmask_vcc_salu(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  uint32_t m = 0x12345u ^ seed;
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  asm volatile("s_mov_b64 vcc, 0x5555" ::: "vcc");
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(m) : "vcc");
    BODY8(OP)
#undef OP
  } T_END
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// one VOP2 select on vcc after three independent adds (how a compiled kernel meets them)
__global__ void k_cndmask_mixed(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  float f[8];
  uint32_t m = 0x12345u ^ seed;
  for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * 7 + i; f[i] = (float)i; }
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" ::"v"(threadIdx.x) : "vcc");
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_add_f32 %0, %0, %0\n\tv_add_f32 %0, %0, %0\n\tv_add_f32 %0, %0, %0\n\t" \
                           "v_cndmask_b32 %1, %1, %2, vcc" : "+v"(f[i]), "+v"(a[i]) : "v"(m) : "vcc");
    BODY8(OP)
#undef OP
  } T_END
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i] ^ __float_as_uint(f[i]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// VOP2 select right after the VALU compare that writes vcc (the compiler's pattern), and after
// an SALU write of vcc (s_and_b64 vcc, s, vcc: the compiler's pattern for a select under a
// branch condition)
__global__ void k_cmp_cndmask(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  uint32_t m = 0x12345u ^ seed;
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\ts_nop 1\n\tv_cndmask_b32 %0, %0, %1, vcc" \
                           : "+v"(a[i]) : "v"(m) : "vcc");
    BODY8(OP)
#undef OP
  } T_END
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_sand_cndmask(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  uint32_t m = 0x12345u ^ seed;
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  unsigned long long msk;
  asm volatile("v_cmp_gt_u32 %0, 32, %1" : "=s"(msk) : "v"(threadIdx.x));
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("s_and_b64 vcc, %2, exec\n\tv_cndmask_b32 %0, %0, %1, vcc" \
                           : "+v"(a[i]) : "v"(m), "s"(msk) : "vcc", "scc");
    BODY8(OP)
#undef OP
  } T_END
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// v_add_f32 as ONE asm statement of 64 instructions per loop trip: the compiler puts an
// s_nop 0 between consecutive asm statements (it cannot see their hazards), so the 8-per-
// statement kernels above issue 9 instructions per 8 adds; here 1 per 64
#define ADD8 "v_add_f32 %0, %0, %8\n\t""v_add_f32 %1, %1, %8\n\t""v_add_f32 %2, %2, %8\n\t""v_add_f32 %3, %3, %8\n\t""v_add_f32 %4, %4, %8\n\t""v_add_f32 %5, %5, %8\n\t""v_add_f32 %6, %6, %8\n\t""v_add_f32 %7, %7, %8\n\t"
__global__ void k_add_f32_asm64(uint32_t* out, uint32_t seed) {
  float a[8];
  float m = 1.0000001f + (float)seed;
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  T_BEGIN for (int it = 0; it < ITERS; it += 8) {
    asm volatile(ADD8 ADD8 ADD8 ADD8 ADD8 ADD8 ADD8 ADD8
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                   "+v"(a[6]), "+v"(a[7])
                 : "v"(m));
  } T_END
  float s = 0;
  for (int i = 0; i < 8; ++i) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = __float_as_uint(s);
}

// compiler-generated selects: x = c ? y : x with c from a float compare each iteration
__global__ void k_select_cc(uint32_t* out, uint32_t seed) {
  float a[8], b[8];
  for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * 7 + i; b[i] = (float)(seed + i); }
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float t = b[i] * 1.0001f;
      a[i] = t < a[i] ? t : a[i];
      b[i] = t;
    }
  } T_END
  float s = 0;
  for (int i = 0; i < 8; ++i) s += a[i] + b[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = __float_as_uint(s);
}

#define CHS(ASM, i) asm volatile(ASM : "+v"(a[i]) : "s"(m));
#define CHS8(ASM) CHS(ASM, 0) CHS(ASM, 1) CHS(ASM, 2) CHS(ASM, 3) CHS(ASM, 4) CHS(ASM, 5) CHS(ASM, 6) CHS(ASM, 7)
#define K_BINS(NAME, ASM, T)                                                             \
  __global__ void NAME(uint32_t* out, uint32_t seed) {                                    \
    T a[8];                                                                              \
    T m = (T)(1.0000001f + (float)seed);                                                 \
    for (int i = 0; i < 8; ++i) a[i] = (T)(threadIdx.x * 7 + i);                         \
    T_BEGIN for (int it = 0; it < ITERS; ++it) { CHS8(ASM) } T_END                                     \
    T s = 0;                                                                             \
    for (int i = 0; i < 8; ++i) s += a[i];                                               \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;                            \
  }
K_BINS(k_xor_vs, "v_xor_b32_e64 %0, %0, %1", uint32_t)
#define OPS_k_xor_vv CH8("v_xor_b32 %0, %0, %1")
K_BIN(k_xor_vv, 0, uint32_t)
K_BINS(k_max_vs, "v_max_f32_e64 %0, %0, %1", float)
K_BINS(k_add_vs, "v_add_f32_e64 %0, %0, %1", float)
K_BINS(k_and_vs, "v_and_b32_e64 %0, %0, %1", uint32_t)
#define OPS_k_sub_f32 CH8("v_sub_f32 %0, %0, %1")
K_BIN(k_sub_f32, 0, float)
#define OPS_k_max3_f32 CH8("v_max3_f32 %0, %0, %1, %0")
K_BIN(k_max3_f32, 0, float)
#define OPS_k_max_u32 CH8("v_max_u32 %0, %0, %1")
K_BIN(k_max_u32, 0, uint32_t)
#define OPS_k_or_b32 CH8("v_or_b32 %0, %0, %1")
K_BIN(k_or_b32, 0, uint32_t)
#define OPS_k_lshl_add_u64 CH8("v_lshl_add_u64 %0, %0, 2, %1")

#define OPS_k_lshl_add_u64 CH8("v_lshl_add_u64 %0, %0, 2, %1")
__global__ void k_lshl_add_u64(uint32_t* out, uint32_t seed) {
  uint64_t a[8];
  uint64_t m = 0x12345ull ^ seed;
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_lshl_add_u64 %0, %0, 2, %1" : "+v"(a[i]) : "v"(m));
    BODY8(OP)
#undef OP
  } T_END
  uint64_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}
__global__ void k_mov_b64(uint32_t* out, uint32_t seed) {
  uint64_t a[8];
  uint64_t m = 0x12345ull ^ seed;
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_mov_b64 %0, %1" : "=v"(a[i]) : "v"(m + i));
    BODY8(OP)
#undef OP
  } T_END
  uint64_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}
__global__ void k_readlane(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i + seed;
  uint32_t acc = 0;
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) { uint32_t r; asm volatile("v_readlane_b32 %0, %1, 3" : "=s"(r) : "v"(a[i])); acc += r; }
    BODY8(OP)
#undef OP
  } T_END
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
__global__ void k_writelane(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  uint32_t sv = seed;
  T_BEGIN for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_writelane_b32 %0, %1, 5" : "+v"(a[i]) : "s"(sv));
    BODY8(OP)
#undef OP
  } T_END
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
#define OPS_k_cmp_eq_u32 CH8("v_cmp_eq_u32 vcc, %0, %1")
K_BIN(k_cmp_eq_u32, 0, uint32_t)
#define OPS_k_floor_f32 CH8("v_floor_f32 %0, %0")
K_BIN(k_floor_f32, 0, float)
#define OPS_k_cvt_u32_f32 CH8("v_cvt_u32_f32 %0, %0")
K_BIN(k_cvt_u32_f32, 0, uint32_t)
#define OPS_k_mbcnt CH8("v_mbcnt_lo_u32_b32 %0, -1, %0")
K_BIN(k_mbcnt, 0, uint32_t)
#define OPS_k_sub_u32 CH8("v_sub_u32 %0, %0, %1")
K_BIN(k_sub_u32, 0, uint32_t)
#define OPS_k_fmac_f32 CH8("v_fmac_f32 %0, %0, %1")
K_BIN(k_fmac_f32, 0, float)
#define OPS_k_pk_add_f32 CH8("v_pk_add_f32 %0, %0, %1")

typedef void (*K)(uint32_t*, uint32_t);

static void run(const char* name, K k, uint32_t* d) {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  // ONE block per CU (96 KiB of dynamic LDS each: two never fit the CU's 160 KiB), of w waves
  // per SIMD (64 x 4 x w threads): every SIMD then runs exactly w waves, so the kernel's
  // time is w x the per-wave instruction count at the SIMD's issue rate.  (Round 4's version
  // launched cus x w blocks of 256 threads and let the dispatcher place them: an uneven
  // placement puts w + 1 waves on some SIMDs and inflates every rate by up to ~20 %.)
  const size_t lds = 96 * 1024;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  for (int waves_per_simd : {1, 2, 4}) {
    const int threads = 256 * waves_per_simd;
    hipLaunchKernelGGL(k, dim3(cus), dim3(threads), lds, 0, d, 1u);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(cus), dim3(threads), lds, 0, d, 1u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    if (hipGetLastError() != hipSuccess) {
      printf("{\"instr\": \"%s\", \"error\": \"launch\"}\n", name);
      continue;
    }
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long tim[2] = {0, 0};
    hipMemcpyFromSymbol(tim, HIP_SYMBOL(g_tim), sizeof(tim));
    const double insts_per_simd = (double)waves_per_simd * ITERS * 8;  // one launch
    const double ghz = tim[1] ? (double)tim[0] / (double)tim[1] * 0.1 : 0.0;  // 100 MHz realtime
    // SIMD cycles per wave-instruction: the launch's wall time at the measured shader clock
    // (one wave's s_memtime / s_memrealtime ratio; the oldest wave of a SIMD issues first,
    // so its own elapsed cycles are not the SIMD's rate)
    const double cyc = ms * 1e-3 / 5.0 * ghz * 1e9;
    printf("{\"instr\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_wave_instr\": %.3f, "
           "\"cycles_per_wave_instr_at_2p4\": %.3f, \"oldest_wave_cycles_per_instr\": %.3f, "
           "\"shader_ghz\": %.3f}\n",
           name, waves_per_simd, cyc / insts_per_simd, ms * 1e-3 / 5.0 * 2.4e9 / insts_per_simd,
           (double)tim[0] / ((double)ITERS * 8), ghz);
  }
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 256 * 2048 * sizeof(uint32_t));  // cus x 1024 threads
  run("v_mad_u64_u32", k_mad_u64, d);
  run("v_mul_hi_u32", k_mul_hi, d);
  run("v_mul_lo_u32", k_mul_lo, d);
  run("v_mul_u32_u24", k_mul_u24, d);
  run("v_xor_b32", k_xor, d);
  run("v_fma_f32", k_fma, d);
  run("v_pk_fma_f32", k_pk_fma, d);
  run("v_fma_f64", k_fma64, d);
  run("v_rcp_f32", k_rcp, d);
  run("v_cvt_f64_f32", k_cvt_f64, d);
  run("v_add_f32", k_add_f32, d);
  run("v_add_f32 (64 per asm statement, no s_nop)", k_add_f32_asm64, d);
  run("v_mul_f32", k_mul_f32, d);
  run("v_max_f32", k_max_f32, d);
  run("v_min3_f32", k_min3_f32, d);
  run("v_add_u32", k_add_u32, d);
  run("v_and_b32", k_and_b32, d);
  run("v_lshrrev_b32", k_lshr_b32, d);
  run("v_mov_b32", k_mov_b32, d);
  run("v_cndmask_b32", k_cndmask, d);
  run("v_bitop3_b32", k_bitop3, d);
  run("v_cvt_f32_u32", k_cvt_f32_u32, d);
  run("v_sqrt_f32", k_sqrt_f32, d);
  run("v_cmp_lt_f32", k_cmp_f32, d);
  run("v_cndmask_b32 (vcc set once)", k_cndmask_vcc, d);
  run("v_cndmask_b32_e64 (sgpr mask)", k_cndmask_sgpr, d);
  run("v_cndmask_b32_e64 (vcc mask)", k_cndmask_e64_vcc, d);
  run("v_cndmask_b32 (vcc written by s_mov)", k_cndmask_vcc_salu, d);
  run("3 v_add_f32 + 1 v_cndmask_b32 (vcc): per 4 instructions", k_cndmask_mixed, d);
  run("v_cmp_gt_u32 vcc + s_nop 1 + v_cndmask_b32 (vcc): per pair", k_cmp_cndmask, d);
  run("s_and_b64 vcc + v_cndmask_b32 (vcc): per pair", k_sand_cndmask, d);
  run("compiled select: mul + cmp + cndmask per element", k_select_cc, d);
  run("v_xor_b32_e64 (sgpr operand)", k_xor_vs, d);
  run("v_xor_b32 (vgpr operands)", k_xor_vv, d);
  run("v_max_f32_e64 (sgpr operand)", k_max_vs, d);
  run("v_add_f32_e64 (sgpr operand)", k_add_vs, d);
  run("v_and_b32_e64 (sgpr operand)", k_and_vs, d);
  run("v_sub_f32", k_sub_f32, d);
  run("v_max3_f32", k_max3_f32, d);
  run("v_max_u32", k_max_u32, d);
  run("v_or_b32", k_or_b32, d);
  run("v_lshl_add_u64", k_lshl_add_u64, d);
  run("v_mov_b64", k_mov_b64, d);
  run("v_readlane_b32", k_readlane, d);
  run("v_writelane_b32", k_writelane, d);
  run("v_cmp_eq_u32", k_cmp_eq_u32, d);
  run("v_floor_f32", k_floor_f32, d);
  run("v_cvt_u32_f32", k_cvt_u32_f32, d);
  run("v_mbcnt_lo_u32_b32", k_mbcnt, d);
  run("v_sub_u32", k_sub_u32, d);
  run("v_fmac_f32", k_fmac_f32, d);
  hipFree(d);
  return 0;
}
