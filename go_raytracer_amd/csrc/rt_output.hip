// rt_output.hip — on-device output path.
//
// The reference writes its image as PPM P3 text: the header of camera.go:160 and
// one "r g b\n" line per pixel from vec.PrintColor (vec/color.go:23-46: NaN -> 0,
// sqrt gamma, clamp to [0, 0.99999], x256 truncated).  Here the quantisation and
// the text are produced by HIP kernels from the image already in HBM, so a
// 2 M-pixel frame never round-trips through host formatting:
//
//   k_ppm_tiles  : per 1024-pixel tile, quantise and sum the line lengths
//   k_ppm_offsets: one block scans the tile sums (exclusive, int64)
//   k_ppm_write  : quantise again (cheaper than storing it), block-scan the line
//                  lengths, assemble the tile's text in LDS, copy it out with
//                  dword stores (byte head/tail around the unaligned base)
//
// Bytes per pixel: 12 read + 6-12 written (the text); the kernels are HBM-bound
// byte work and run in microseconds at 2 M pixels.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "rt_abi.h"

namespace rt {
int set_error(int code, const char* fmt, ...);
}
using rt::set_error;

namespace {

constexpr int kThreads = 256;
constexpr int kPxPerThread = 4;
constexpr int kTile = kThreads * kPxPerThread;  // pixels per tile
constexpr int kMaxLine = 12;                    // "255 255 255\n"

// PrintColor's component (color.go:23-46) computed exactly: floor(256*sqrt(v))
// clamped to 255 is the largest q with q*q <= 65536*v (v is a float, so 65536*v
// and q*q are exact in fp64); a correctly rounded sqrt cannot cross a q/256
// boundary that the exact root does not (|sqrt(v) - q/256| >= 2^-25 q/256 for a
// float v != q^2/65536), so this equals the host's int(sqrt(double(v))*256).
__device__ __forceinline__ uint32_t quant(float v) {
  if (!(v > 0.0f)) return 0;  // NaN and v <= 0
  if (v >= 1.0f) return 255;  // sqrt(v) >= 1 > 0.99999
  const double x = 65536.0 * (double)v;
  int q = (int)sqrt(x);
  if ((double)(q + 1) * (q + 1) <= x) ++q;
  if ((double)q * q > x) --q;
  return q > 255 ? 255u : (uint32_t)q;
}

__device__ __forceinline__ int ndig(uint32_t q) { return q < 10 ? 1 : (q < 100 ? 2 : 3); }

struct Px {
  uint32_t c[3];
  int len;
};

__device__ __forceinline__ Px pixel(const float* __restrict__ rgb, int64_t i) {
  Px p;
  p.c[0] = quant(rgb[3 * i]);
  p.c[1] = quant(rgb[3 * i + 1]);
  p.c[2] = quant(rgb[3 * i + 2]);
  p.len = ndig(p.c[0]) + ndig(p.c[1]) + ndig(p.c[2]) + 3;
  return p;
}

// exclusive block scan of one int per thread (4 waves of 64)
__device__ __forceinline__ int block_scan(int v, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
  for (int off = 1; off < 64; off <<= 1) {
    int y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int base = 0, all = 0;
  for (int k = 0; k < kThreads / 64; ++k) {
    if (k < w) base += wsum[k];
    all += wsum[k];
  }
  *total = all;
  return base + x - v;
}

__global__ __launch_bounds__(kThreads) void k_ppm_tiles(const float* __restrict__ rgb, int64_t n,
                                                        int64_t* __restrict__ tile_sums) {
  __shared__ int wsum[kThreads / 64];
  const int64_t first = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kPxPerThread;
  int len = 0;
  for (int k = 0; k < kPxPerThread; ++k)
    if (first + k < n) len += pixel(rgb, first + k).len;
  int total;
  block_scan(len, wsum, &total);
  if (threadIdx.x == 0) tile_sums[blockIdx.x] = total;
}

// one block: tile_sums -> exclusive offsets in place; *grand = the sum
__global__ __launch_bounds__(1024) void k_ppm_offsets(int64_t* __restrict__ tile_sums, int ntiles,
                                                      int64_t* __restrict__ grand) {
  __shared__ int64_t part[1024];
  const int per = (ntiles + 1023) / 1024;
  const int b = threadIdx.x * per;
  int64_t s = 0;
  for (int k = 0; k < per && b + k < ntiles; ++k) s += tile_sums[b + k];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele over 1024 partial sums
    int64_t y = threadIdx.x >= (unsigned)off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += y;
    __syncthreads();
  }
  int64_t run = part[threadIdx.x] - s;
  for (int k = 0; k < per && b + k < ntiles; ++k) {
    int64_t v = tile_sums[b + k];
    tile_sums[b + k] = run;
    run += v;
  }
  if (threadIdx.x == 1023) *grand = part[1023];
}

__global__ __launch_bounds__(kThreads) void k_ppm_write(const float* __restrict__ rgb, int64_t n,
                                                        const int64_t* __restrict__ tile_off,
                                                        int64_t header, char* __restrict__ out,
                                                        int64_t cap) {
  __shared__ int wsum[kThreads / 64];
  __shared__ char text[kTile * kMaxLine];
  const int64_t first = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kPxPerThread;
  Px px[kPxPerThread];
  int len = 0;
  for (int k = 0; k < kPxPerThread; ++k) {
    if (first + k < n) {
      px[k] = pixel(rgb, first + k);
      len += px[k].len;
    } else {
      px[k].len = 0;
    }
  }
  int total;
  int pos = block_scan(len, wsum, &total);
  for (int k = 0; k < kPxPerThread; ++k) {
    if (!px[k].len) continue;
    for (int ch = 0; ch < 3; ++ch) {
      uint32_t q = px[k].c[ch];
      if (q >= 100) text[pos++] = (char)('0' + q / 100);
      if (q >= 10) text[pos++] = (char)('0' + (q / 10) % 10);
      text[pos++] = (char)('0' + q % 10);
      text[pos++] = ch < 2 ? ' ' : '\n';
    }
  }
  __syncthreads();
  // copy text[0, total) to out[base, base + total): byte head up to a 4-byte
  // boundary of out, dword body, byte tail
  const int64_t base = header + tile_off[blockIdx.x];
  const int mis = (int)((4 - ((uintptr_t)(out + base) & 3)) & 3);
  const int head = mis < total ? mis : total;
  const int body = (total - head) & ~3;
  if ((int)threadIdx.x < head && base + threadIdx.x < cap) out[base + threadIdx.x] = text[threadIdx.x];
  uint32_t* o32 = (uint32_t*)(out + base + head);
  for (int i = threadIdx.x; i < body / 4; i += kThreads) {
    const int t = head + 4 * i;
    if (base + t + 4 > cap) break;
    o32[i] = (uint32_t)(uint8_t)text[t] | (uint32_t)(uint8_t)text[t + 1] << 8 |
             (uint32_t)(uint8_t)text[t + 2] << 16 | (uint32_t)(uint8_t)text[t + 3] << 24;
  }
  const int tail0 = head + body;
  const int t = tail0 + threadIdx.x;
  if (t < total && base + t < cap) out[base + t] = text[t];
}

__global__ __launch_bounds__(kThreads) void k_quantize(const float* __restrict__ rgb, int64_t n3,
                                                       uint8_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n3;
       i += (int64_t)gridDim.x * kThreads)
    out[i] = (uint8_t)quant(rgb[i]);
}

// grow-only per-device scratch for tile sums (+1 slot for the grand total)
struct Scratch {
  std::mutex mu;
  std::vector<void*> buf;
  std::vector<size_t> cap;
};
Scratch g_scratch;

int scratch(int device, size_t bytes, void** out) {
  std::lock_guard<std::mutex> lk(g_scratch.mu);
  if ((int)g_scratch.buf.size() <= device) {
    g_scratch.buf.resize(device + 1, nullptr);
    g_scratch.cap.resize(device + 1, 0);
  }
  if (g_scratch.cap[device] < bytes) {
    if (g_scratch.buf[device]) (void)hipFree(g_scratch.buf[device]);
    g_scratch.buf[device] = nullptr;
    g_scratch.cap[device] = 0;
    if (hipMalloc(&g_scratch.buf[device], bytes) != hipSuccess)
      return set_error(RT_ERR_OOM, "rt_format_ppm_device: scratch of %zu bytes", bytes);
    g_scratch.cap[device] = bytes;
  }
  *out = g_scratch.buf[device];
  return RT_OK;
}

#define HIP_OK(expr)                                                                    \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      return set_error(RT_ERR_DEVICE, "%s failed: %s", #expr, hipGetErrorString(_e));   \
  } while (0)

}  // namespace

extern "C" {

int rt_quantize_device(const float* rgb_dev, int64_t n_pixels, uint8_t* out_dev, int device,
                       void* stream) {
  if (n_pixels < 0 || (n_pixels > 0 && (!rgb_dev || !out_dev)))
    return set_error(RT_ERR_INVALID, "rt_quantize_device: bad args");
  if (n_pixels == 0) return RT_OK;
  HIP_OK(hipSetDevice(device));
  hipStream_t s = (hipStream_t)stream;
  const int64_t n3 = 3 * n_pixels;
  const int blocks = (int)std::min<int64_t>((n3 + kThreads - 1) / kThreads, 65536);
  hipLaunchKernelGGL(k_quantize, dim3(blocks), dim3(kThreads), 0, s, rgb_dev, n3, out_dev);
  HIP_OK(hipGetLastError());
  HIP_OK(hipStreamSynchronize(s));
  return RT_OK;
}

int64_t rt_format_ppm_device(const float* rgb_dev, int w, int h, char* out_dev, int64_t cap,
                             int device, void* stream) {
  if (w < 0 || h < 0 || (w * (int64_t)h > 0 && !rgb_dev) || (out_dev && cap < 0))
    return set_error(RT_ERR_INVALID, "rt_format_ppm_device: bad args");
  char hdr[64];
  const int hlen = snprintf(hdr, sizeof hdr, "P3\n%d %d\n255\n", w, h);  // camera.go:160
  const int64_t n = (int64_t)w * h;
  const int64_t ntiles = (n + kTile - 1) / kTile;
  if (ntiles > (int64_t)1024 * 65536)
    return set_error(RT_ERR_INVALID, "rt_format_ppm_device: %lld pixels", (long long)n);
  HIP_OK(hipSetDevice(device));
  hipStream_t s = (hipStream_t)stream;
  int64_t body = 0;
  if (n > 0) {
    void* scr = nullptr;
    int rc = scratch(device, (size_t)(ntiles + 1) * sizeof(int64_t), &scr);
    if (rc) return rc;
    int64_t* tiles = (int64_t*)scr;
    int64_t* grand = tiles + ntiles;
    hipLaunchKernelGGL(k_ppm_tiles, dim3((unsigned)ntiles), dim3(kThreads), 0, s, rgb_dev, n,
                       tiles);
    hipLaunchKernelGGL(k_ppm_offsets, dim3(1), dim3(1024), 0, s, tiles, (int)ntiles, grand);
    HIP_OK(hipGetLastError());
    if (out_dev) {
      if (cap >= hlen) HIP_OK(hipMemcpyAsync(out_dev, hdr, hlen, hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL(k_ppm_write, dim3((unsigned)ntiles), dim3(kThreads), 0, s, rgb_dev, n,
                         tiles, (int64_t)hlen, out_dev, cap);
      HIP_OK(hipGetLastError());
    }
    HIP_OK(hipMemcpyAsync(&body, grand, sizeof body, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
  } else if (out_dev && cap >= hlen) {
    HIP_OK(hipMemcpyAsync(out_dev, hdr, hlen, hipMemcpyHostToDevice, s));
    HIP_OK(hipStreamSynchronize(s));
  }
  const int64_t total = hlen + body;
  if (out_dev && total > cap) return set_error(RT_ERR_INVALID, "rt_format_ppm_device: buffer too small");
  return total;
}

}  // extern "C"
