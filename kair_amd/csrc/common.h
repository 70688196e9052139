// Shared device helpers for the KAIR MI355X (gfx950 / CDNA4) kernels.
// Wave64 everywhere; bf16 storage is the compiler's __bf16 (RNE conversions via v_cvt_pk_bf16_f32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kair_hip.h"

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) short short4v;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define KAIR_DEV __device__ __forceinline__
#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

// ---------------------------------------------------------------------------------------------
// error plumbing for the C-ABI: every entry point returns 0 or a negative code and leaves a
// thread-local message behind (kair_last_error()).
// ---------------------------------------------------------------------------------------------
int kair_set_error(int code, const char* fmt, ...);

#define KAIR_CHECK_ARG(cond, ...)                                                  \
  do {                                                                             \
    if (!(cond)) return kair_set_error(KAIR_ERR_ARG, __VA_ARGS__);                 \
  } while (0)

#define KAIR_CHECK_LAUNCH()                                                        \
  do {                                                                             \
    hipError_t e__ = hipGetLastError();                                            \
    if (e__ != hipSuccess)                                                         \
      return kair_set_error(KAIR_ERR_HIP, "%s: %s", __func__, hipGetErrorString(e__)); \
  } while (0)

template <typename T> KAIR_DEV float to_f(T v) { return (float)v; }
template <typename T> KAIR_DEV T from_f(float v) { return (T)v; }

KAIR_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
KAIR_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

KAIR_DEV float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
KAIR_DEV float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// Swin window <-> token row map (network_swinir.py:33-62 + torch.roll at :250/:270):
// GEMM row m enumerates tokens window-major (b, wy, wx, r, c); the token it reads / writes lives at
// ((wy*ws + r + shift) % H, (wx*ws + c + shift) % W) of image b.
struct WinMap {
  int H, W, ws, shift;  // ws == 0 => identity map
};
// 32-bit form (row counts < 2^31) for per-tile address setup in the GEMM mainloops
KAIR_DEV int win_to_token32(int m, const WinMap& w) {
  if (w.ws == 0) return m;
  const int ws2 = w.ws * w.ws;
  const int nWw = w.W / w.ws, nW = (w.H / w.ws) * nWw;
  const int win = m / ws2;
  const int t = m - win * ws2;
  const int b = win / nW;
  const int wi = win - b * nW;
  const int wy = wi / nWw, wx = wi - wy * nWw;
  const int ty = t / w.ws;
  int y = wy * w.ws + ty + w.shift;
  int x = wx * w.ws + (t - ty * w.ws) + w.shift;
  if (y >= w.H) y -= w.H;
  if (x >= w.W) x -= w.W;
  return (b * w.H + y) * w.W + x;
}
// inverse of win_to_token: window-order row of token t
KAIR_DEV long token_to_win(long t, const WinMap& w) {
  if (w.ws == 0) return t;
  const long hw = (long)w.H * w.W;
  const long b = t / hw;
  const int p = (int)(t - b * hw);
  int y = p / w.W, x = p - (p / w.W) * w.W;
  y -= w.shift; if (y < 0) y += w.H;
  x -= w.shift; if (x < 0) x += w.W;
  const int nWw = w.W / w.ws, nW = (w.H / w.ws) * nWw;
  const int wy = y / w.ws, wx = x / w.ws;
  return ((b * nW + wy * nWw + wx) * w.ws + (y - wy * w.ws)) * w.ws + (x - wx * w.ws);
}
KAIR_DEV long win_to_token(long m, const WinMap& w) {
  if (w.ws == 0) return m;
  const int ws2 = w.ws * w.ws;
  const int nWw = w.W / w.ws, nW = (w.H / w.ws) * nWw;
  const long win = m / ws2;
  const int t = (int)(m - win * ws2);
  const long b = win / nW;
  const int wi = (int)(win - b * nW);
  const int wy = wi / nWw, wx = wi - wy * nWw;
  int y = wy * w.ws + t / w.ws + w.shift;
  int x = wx * w.ws + t % w.ws + w.shift;
  if (y >= w.H) y -= w.H;
  if (x >= w.W) x -= w.W;
  return (b * w.H + y) * (long)w.W + x;
}

// Deterministic sum over `nparts` partial planes for 64 consecutive outputs per 1024-thread block:
// thread (tx, ty) sums planes ty, ty+16, ... at plane offset `off`, then the 16 phases are added in
// fixed order.  Returns the total in threads with ty == 0 (others get 0).
KAIR_DEV float split_sum16(const float* __restrict__ part, long nparts, long plane, long off, bool valid) {
  __shared__ float red[16][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  float s0 = 0.f, s1 = 0.f;
  if (valid) {
    long i = ty;
    for (; i + 16 < nparts; i += 32) {
      s0 += part[i * plane + off];
      s1 += part[(i + 16) * plane + off];
    }
    if (i < nparts) s0 += part[i * plane + off];
  }
  red[ty][tx] = s0 + s1;
  __syncthreads();
  float s = 0.f;
  if (ty == 0) {
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][tx];
  }
  return s;
}
