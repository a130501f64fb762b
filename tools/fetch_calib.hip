// fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE for the traversal's access
// pattern (dev tool).  The guide's gfx950 correction (FETCH_SIZE x 2) is established for
// wide coalesced streaming reads; the fused kernel instead gathers, per lane, one
// 128-B BVH node (7-8 x 16-B loads) or one 64-B leaf record at a divergent address.
// Each kernel here reads a KNOWN number of distinct lines exactly once, so FETCH_SIZE
// per launch can be compared with the true bytes:
//   k_stream  : coalesced 16 B per lane, consecutive (the guide's calibration shape)
//   k_gather8 : per lane 8 x 16 B from a distinct 128-B line (a BVH4 node fetch)
//   k_gather4 : per lane 4 x 16 B from a distinct 64-B half line (a leaf record fetch)
//   k_gather4s: per lane the FIRST 4 x 16 B of a distinct 128-B line (nothing else of the
//               line is read): same time as k_gather8 means 128-B fetch granularity
// Lines are visited in a scrambled order (an odd multiplier mod 2^k is a bijection), so
// every line is fetched once and neighbours are not fetched together.
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o /tmp/fetch_calib
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE -- /tmp/fetch_calib
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                  \
      return 1;                                                               \
    }                                                                         \
  } while (0)

__global__ void k_stream(const float4* __restrict__ src, float* out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 v = src[i];
  out[i] = v.x + v.y + v.z + v.w;
}

// lane i reads the line (i * mult) mod nlines, `per` consecutive float4 of it
template <int PER>
__global__ void k_gather(const float4* __restrict__ src, float* out, uint32_t n, uint32_t mask,
                         uint32_t mult) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t line = (i * mult) & mask;
  const float4* p = src + (size_t)line * PER;
  float s = 0.0f;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const float4 v = p[e];
    s += v.x + v.y + v.z + v.w;
  }
  out[i] = s;
}

// lane i reads the first 64 B of line (i * mult) mod nlines
__global__ void k_gather4s(const float4* __restrict__ src, float* out, uint32_t n, uint32_t mask,
                           uint32_t mult) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4* p = src + (size_t)((i * mult) & mask) * 8;
  float s = 0.0f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float4 v = p[e];
    s += v.x + v.y + v.z + v.w;
  }
  out[i] = s;
}

int main() {
  const uint32_t lines128 = 1u << 25;  // 32 M lines of 128 B = 4 GiB
  const size_t bytes = (size_t)lines128 * 128;
  float4* src = nullptr;
  float* out = nullptr;
  CHECK(hipMalloc(&src, bytes));
  CHECK(hipMalloc(&out, ((size_t)1 << 27) * sizeof(float)));
  CHECK(hipMemset(src, 0, bytes));
  CHECK(hipDeviceSynchronize());
  const uint32_t mult = 2654435761u;  // odd: a bijection on [0, 2^k)
  const uint32_t ns = 1u << 27, n8 = 1u << 24, n4 = 1u << 24;
  for (int rep = 0; rep < 3; ++rep) {
    // 1) stream: 2 GiB read once, coalesced (16 B per lane)
    hipLaunchKernelGGL(k_stream, dim3(ns / 256), dim3(256), 0, 0, src, out, ns);
    // 2) 16 M lanes, one distinct 128-B line each: 2 GiB
    hipLaunchKernelGGL(k_gather<8>, dim3(n8 / 256), dim3(256), 0, 0, src, out, n8, lines128 - 1,
                       mult);
    // 3) 16 M lanes, one distinct 64-B half line each: 1 GiB (of 2^26 half lines)
    hipLaunchKernelGGL(k_gather<4>, dim3(n4 / 256), dim3(256), 0, 0, src, out, n4,
                       2 * lines128 - 1, mult);
    // 4) 16 M lanes, the first half of a distinct 128-B line each: 1 GiB used
    hipLaunchKernelGGL(k_gather4s, dim3(n4 / 256), dim3(256), 0, 0, src, out, n4, lines128 - 1,
                       mult);
  }
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  printf("{\"k_stream\": %zu, \"k_gather8\": %zu, \"k_gather4\": %zu, \"k_gather4s\": %zu}\n",
         (size_t)ns * 16, (size_t)n8 * 128, (size_t)n4 * 64, (size_t)n4 * 64);
  return 0;
}
