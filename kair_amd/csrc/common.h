// Shared device helpers for the KAIR MI355X (gfx950 / CDNA4) kernels.
// Wave64 everywhere; bf16 storage is the compiler's __bf16 (RNE conversions via v_cvt_pk_bf16_f32).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

#include "kair_hip.h"

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) short short4v;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef _Float16 f16;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
// 8-wide vector of a 16-bit element type (bf16 / fp16)
template <typename T> struct V8;
template <> struct V8<__bf16> { typedef bf16x8 t; };
template <> struct V8<_Float16> { typedef f16x8 t; };
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

// Perf-investigation ablation bits (store-dropping / compute-skipping switches read from KAIR_*_DBG
// environment variables) exist only in a library built with -DKAIR_DEBUG_ABLATIONS=1
// (python -m kair_amd.build --debug-ablations).  The release library reads no environment variable:
// kair_dbg_env() is 0 and every KAIR_DBG(...) test is a compile-time false, so the kernels carry no
// ablation code at all.
#ifndef KAIR_DEBUG_ABLATIONS
#define KAIR_DEBUG_ABLATIONS 0
#endif
#define KAIR_DBG(x) (KAIR_DEBUG_ABLATIONS && (x))
int kair_dbg_env(const char* name);

// Every libkair launch: KAIR_LAUNCH(kernel, grid, block, lds, stream, args...).  Outside a kernel timing window
// (kair_ktime_begin, bench.py) a plain launch; inside one, hipExtLaunchKernel with the slot's event pair, which the
// runtime stamps with the dispatch packet's start / end -- the kernel duration rocprofv3 --kernel-trace reports.
bool kair_ktime_take(const void* fn, hipStream_t s, hipEvent_t* e0, hipEvent_t* e1);
#define KAIR_LAUNCH(k, grid, block, lds, stream, ...)                                                        \
  do {                                                                                                      \
    hipEvent_t kt_e0_, kt_e1_;                                                                              \
    if (kair_ktime_take(reinterpret_cast<const void*>(k), (stream), &kt_e0_, &kt_e1_))                     \
      hipExtLaunchKernelGGL(k, (grid), (block), (lds), (stream), kt_e0_, kt_e1_, 0, __VA_ARGS__);            \
    else                                                                                                    \
      k<<<(grid), (block), (lds), (stream)>>>(__VA_ARGS__);                                                 \
  } while (0)

// An fp32 value the compiler may not fuse into the fp16 conversion after it: a pair split hi = f16(w), lo = f16(w - hi)
// of a product w = a b (b not a power of two) otherwise becomes hi = v_fma_mix(a, b) -- the exact product rounded once
// to fp16 -- beside a second, fp32-rounded conversion for the stored hi: at double-rounding points (~2^-13 of the
// values) the stored hi and the lo computed against the other one disagree by one hi ulp.  ("fp contract(off)" and
// __fmul_rn do not stop this fusion.)
KAIR_DEV float opaque(float w) {
  asm volatile("" : "+v"(w));
  return w;
}

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

// Sum over each aligned group of 16 lanes with DPP lane moves only (no LDS permute): quad
// butterflies (quad_perm [1,0,3,2], [2,3,0,1]) then row_half_mirror and row_mirror, which pair
// the quads and then the half-rows of a 16-lane DPP row.  Every lane of the group gets the sum.
template <int CTRL> KAIR_DEV float dpp_movc(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
KAIR_DEV float dpp_sum16(float v) {
  v += dpp_movc<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_movc<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_movc<0x141>(v);   // row_half_mirror
  v += dpp_movc<0x140>(v);   // row_mirror
  return v;
}

// Buffer-resource global access: a wave-uniform descriptor (SGPRs) + a 32-bit per-lane byte offset +
// a wave-uniform byte offset, so a persistent kernel keeps one VGPR per access stream instead of a
// 64-bit address; accesses past the resource's size are dropped (loads return 0).
typedef __amdgpu_buffer_rsrc_t BufRsrc;
KAIR_DEV BufRsrc buf_rsrc(const void* p, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)(bytes > 0x7fffffffL ? 0x7fffffffL : bytes),
                                           0x00020000);
}
typedef __attribute__((ext_vector_type(4))) unsigned buf_u32x4;
KAIR_DEV float4 buf_ld4(BufRsrc r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0));
}
// Stores fold the uniform offset into the lane offset and pass soffset = 0: ROCm 7.2's hazard
// recognizer treats a > 8-byte buffer store with an SGPR soffset as free of the "store data VGPRs
// overwritten by the next VALU instruction" hazard and inserts no wait state, but gfx950 has it --
// measured: the first data dword of some lanes of buffer_store_dwordx4 replaced by the value a
// following v_and_b32 wrote into that VGPR (tests/test_mlp_fused_gpu.py).  With soffset 0 the
// recognizer pads the store.
KAIR_DEV void buf_st4(BufRsrc r, unsigned voff, unsigned soff, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(buf_u32x4, v), r, (int)(voff + soff), 0, 0);
}
KAIR_DEV void buf_st16(BufRsrc r, unsigned voff, unsigned soff, uint4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(buf_u32x4, v), r, (int)(voff + soff), 0, 0);
}
KAIR_DEV void buf_st1(BufRsrc r, unsigned voff, unsigned soff, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)(voff + soff), 0, 0);
}

// erf(a) to ~1 ulp (minimax polynomials of the two ranges |a| <= 0.927734375 and beyond, max error 0.964 ulp
// against math.erf over [-6, 6] with an exact exp; __expf adds < 1 ulp), branch-free: ~20 VALU against the ~70
// of the library erff's inlined form -- the GELU epilogues of the fc1 GEMMs evaluate it per output element
KAIR_DEV float erf_f32(float a) {
  const float t = fabsf(a), s = a * a;
  float p = -5.96761703e-4f;
  p = fmaf(p, s, 4.99119423e-3f);
  p = fmaf(p, s, -2.67681349e-2f);
  p = fmaf(p, s, 1.12819925e-1f);
  p = fmaf(p, s, -3.76125336e-1f);
  p = fmaf(p, s, 1.28379166e-1f);
  p = fmaf(p, a, a);
  float r = fmaf(-1.72853470e-5f, t, 3.83197126e-4f);
  const float u = fmaf(-3.88396438e-3f, t, 2.42546219e-2f);
  r = fmaf(r, s, u);
  r = fmaf(r, t, -1.06777877e-1f);
  r = fmaf(r, t, -6.34846687e-1f);
  r = fmaf(r, t, -1.28717512e-1f);
  r = fmaf(r, t, -t);
  r = copysignf(1.0f - __expf(r), a);
  return t > 0.927734375f ? r : p;
}
KAIR_DEV float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_f32(x * 0.70710678118654752f)); }
KAIR_DEV float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + erf_f32(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// Fast integer division for 0 <= n < 2^24 (row / column indices): float reciprocal + one
// correction step (exact there).  Runtime-divisor integer division costs ~30-40 VALU on CDNA;
// this is ~6.
struct FDiv {
  int d;
  float r;
};
inline FDiv make_fdiv(int d) { return FDiv{d, d > 0 ? 1.0f / (float)d : 0.f}; }
KAIR_DEV int fdiv(int n, const FDiv& f) {
  int q = (int)((float)n * f.r);
  const int rem = n - q * f.d;
  if (rem < 0) --q;
  else if (rem >= f.d) ++q;
  return q;
}

// Fast erf (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7 absolute): ~12 VALU with one rcp and
// one exp, against ~30 for erff.  Used only on bf16-compute epilogues, where the output rounding
// (2^-9 relative) dominates; the fp32 parity path keeps erff.  The reciprocal is the hardware
// v_rcp_f32 (1 ulp): __frcp_rn compiles to the 8-instruction correctly-rounded division sequence.
KAIR_DEV float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.3275911f * ax);
  float y = 1.061405429f;
  y = fmaf(y, t, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  y = 1.0f - y * t * __expf(-ax * ax);
  return copysignf(y, x);
}
// GELU and GELU' of the same x sharing one rcp and one exp (gelu_fast / gelu_grad_fast maths)
KAIR_DEV void gelu_pair_fast(float x, float& y, float& dy) {
  const float z = x * 0.70710678118654752f, az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.3275911f * az);
  float p = 1.061405429f;
  p = fmaf(p, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = __expf(-az * az);   // = exp(-x^2 / 2)
  const float cdf = 0.5f * (1.0f + copysignf(1.0f - p * t * e, z));
  y = x * cdf;
  dy = cdf + x * 0.39894228040143268f * e;
}
// Two elements at once: the polynomial / products as packed fp32 (v_pk_fma_f32 / v_pk_mul_f32,
// two lanes' worth per instruction); rcp and exp stay per element.
typedef float f32x2 __attribute__((ext_vector_type(2)));
KAIR_DEV void gelu_pair_fast2(f32x2 x, f32x2& y, f32x2& dy) {
  const f32x2 z = x * 0.70710678118654752f;
  const f32x2 az = {fabsf(z.x), fabsf(z.y)};
  const f32x2 den = az * 0.3275911f + 1.0f;
  const f32x2 t = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  f32x2 p = t * 1.061405429f - 1.453152027f;
  p = p * t + 1.421413741f;
  p = p * t - 0.284496736f;
  p = p * t + 0.254829592f;
  const f32x2 sq = -(az * az);
  const f32x2 e = {__expf(sq.x), __expf(sq.y)};
  const f32x2 q = 1.0f - p * t * e;
  const f32x2 cdf = 0.5f * (1.0f + (f32x2){copysignf(q.x, z.x), copysignf(q.y, z.y)});
  y = x * cdf;
  dy = cdf + x * 0.39894228040143268f * e;
}
// erf_f32 / GELU / GELU' of two elements at once: both polynomials as packed fp32 (v_pk_fma_f32 / v_pk_mul_f32,
// two elements per instruction); exp, compares and selects stay per element.  The same arithmetic as erf_f32,
// gelu_erf and gelu_erf_grad, element for element
KAIR_DEV f32x2 erf_f32x2(f32x2 a) {
  const f32x2 t = {fabsf(a.x), fabsf(a.y)}, s = a * a;
  f32x2 p = {-5.96761703e-4f, -5.96761703e-4f};
  p = __builtin_elementwise_fma(p, s, (f32x2){4.99119423e-3f, 4.99119423e-3f});
  p = __builtin_elementwise_fma(p, s, (f32x2){-2.67681349e-2f, -2.67681349e-2f});
  p = __builtin_elementwise_fma(p, s, (f32x2){1.12819925e-1f, 1.12819925e-1f});
  p = __builtin_elementwise_fma(p, s, (f32x2){-3.76125336e-1f, -3.76125336e-1f});
  p = __builtin_elementwise_fma(p, s, (f32x2){1.28379166e-1f, 1.28379166e-1f});
  p = __builtin_elementwise_fma(p, a, a);
  f32x2 r = __builtin_elementwise_fma((f32x2){-1.72853470e-5f, -1.72853470e-5f}, t, (f32x2){3.83197126e-4f, 3.83197126e-4f});
  const f32x2 u = __builtin_elementwise_fma((f32x2){-3.88396438e-3f, -3.88396438e-3f}, t, (f32x2){2.42546219e-2f, 2.42546219e-2f});
  r = __builtin_elementwise_fma(r, s, u);
  r = __builtin_elementwise_fma(r, t, (f32x2){-1.06777877e-1f, -1.06777877e-1f});
  r = __builtin_elementwise_fma(r, t, (f32x2){-6.34846687e-1f, -6.34846687e-1f});
  r = __builtin_elementwise_fma(r, t, (f32x2){-1.28717512e-1f, -1.28717512e-1f});
  r = __builtin_elementwise_fma(r, t, -t);
  const f32x2 q = {copysignf(1.0f - __expf(r.x), a.x), copysignf(1.0f - __expf(r.y), a.y)};
  return (f32x2){t.x > 0.927734375f ? q.x : p.x, t.y > 0.927734375f ? q.y : p.y};
}
KAIR_DEV void gelu_erf_pair2(f32x2 x, f32x2& y, f32x2& dy) {
  const f32x2 cdf = 0.5f * (1.0f + erf_f32x2(x * 0.70710678118654752f));
  y = x * cdf;
  const f32x2 e = {__expf(-0.5f * x.x * x.x), __expf(-0.5f * x.y * x.y)};
  dy = __builtin_elementwise_fma(x * 0.39894228040143268f, e, cdf);
}
KAIR_DEV float gelu_fast(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }
KAIR_DEV float gelu_grad_fast(float x) {
  const float cdf = 0.5f * (1.0f + erf_fast(x * 0.70710678118654752f));
  return cdf + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}

// Swin window <-> token row map (network_swinir.py:33-62 + torch.roll at :250/:270):
// GEMM row m enumerates tokens window-major (b, wy, wx, r, c); the token it reads / writes lives at
// ((wy*ws + r + shift) % H, (wx*ws + c + shift) % W) of image b.  Indices < 2^24 (checked at the
// C-ABI entry points that take a window map).
struct WinMap {
  int H, W, ws, shift;  // ws == 0 => identity map
  FDiv dws2, dnW, dnWw, dws, dW, dHW;
};
inline WinMap make_winmap(int H, int W, int ws, int shift) {
  WinMap w{H, W, ws, shift, {}, {}, {}, {}, {}, {}};
  if (ws > 0) {
    const int nWw = W / ws, nW = (H / ws) * nWw;
    w.dws2 = make_fdiv(ws * ws);
    w.dnW = make_fdiv(nW);
    w.dnWw = make_fdiv(nWw);
    w.dws = make_fdiv(ws);
    w.dW = make_fdiv(W);
    w.dHW = make_fdiv(H * W);
  }
  return w;
}
constexpr long KAIR_MAX_MAPPED_ROWS = 1L << 24;

KAIR_DEV int win_to_token32(int m, const WinMap& w) {
  if (w.ws == 0) return m;
  const int win = fdiv(m, w.dws2);
  const int t = m - win * w.dws2.d;
  const int b = fdiv(win, w.dnW);
  const int wi = win - b * w.dnW.d;
  const int wy = fdiv(wi, w.dnWw), wx = wi - wy * w.dnWw.d;
  const int ty = fdiv(t, w.dws);
  int y = wy * w.ws + ty + w.shift;
  int x = wx * w.ws + (t - ty * w.ws) + w.shift;
  if (y >= w.H) y -= w.H;
  if (x >= w.W) x -= w.W;
  return (b * w.H + y) * w.W + x;
}
KAIR_DEV long win_to_token(long m, const WinMap& w) { return w.ws == 0 ? m : (long)win_to_token32((int)m, w); }

// inverse of win_to_token: window-order row of token t
KAIR_DEV long token_to_win(long tl, const WinMap& w) {
  if (w.ws == 0) return tl;
  const int t = (int)tl;
  const int b = fdiv(t, w.dHW);
  const int p = t - b * w.dHW.d;
  int y = fdiv(p, w.dW), x = p - y * w.W;
  y -= w.shift; if (y < 0) y += w.H;
  x -= w.shift; if (x < 0) x += w.W;
  const int wy = fdiv(y, w.dws), wx = fdiv(x, w.dws);
  return (((long)b * w.dnW.d + wy * w.dnWw.d + wx) * w.ws + (y - wy * w.ws)) * w.ws + (x - wx * w.ws);
}

// Deterministic sum over `nparts` partial planes for 64 consecutive outputs per 1024-thread block:
// thread (tx, ty) sums planes ty, ty+16, ... at plane offset `off`, then the 16 phases are added in
// fixed order.  Returns the total in threads with ty == 0 (others get 0).
KAIR_DEV float split_sum16(const float* __restrict__ part, long nparts, long plane, long off, bool valid) {
  __shared__ float red[16][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  float s0 = 0.f, s1 = 0.f;
  if (valid) {
    // 8 loads in flight (clamped, so the last partial batch issues them together too), summed
    // alternately into s0 / s1 in part order
    for (long i = ty; i < nparts; i += 128) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(i + 16 * u < nparts ? i + 16 * u : nparts - 1) * plane + off];
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        if (i + 16 * u < nparts) s0 += v[u];
        if (i + 16 * (u + 1) < nparts) s1 += v[u + 1];
      }
    }
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

// grouped weight-gradient finalize (kair_wgrad_grouped): one job per linear layer, partial planes
// [splits][Np][Kt] summed in fixed order and scattered to the reference layout (elementwise.hip)
constexpr int KAIR_WG_MAX = 24;
struct FinJob {
  const float* part; float* grad; float* bias;
  kair_wmap mp;
  int ones_col, Kt;
  long plane, blk0;                            // plane = Np * Kt; blk0 = first block of this job
};
struct FinGroup {
  FinJob j[KAIR_WG_MAX];
  int njobs, splits;
  long nblocks;
};
int kair_launch_finalize_grouped(const FinGroup& g, hipStream_t s);

// fp16-pair (fp32x3) window attention (attn_x3.hip): windows per backward wave, and the bias-table partial sum
// shared with window_attn.hip
long kair_attn_x3_wpg(long nWin, int nh);
int kair_attn_dtable_sum(const float* ws, long ngroups, int nh, float* dtable, int accumulate, hipStream_t s);

// split-fp16 GEMMs (gemm_x3.hip), reached through kair_gemm_nt / kair_gemm_tn with compute KAIR_COMPUTE_X3,
// and the operand validation they share with gemm.hip
int kair_check_operand(const kair_operand* o, const char* what);
int kair_gemm_nt_x3(const kair_operand* A, const kair_operand* B, const kair_epilogue* E, long M, int N, int K,
                    void* stream);
int kair_gemm_tn_x3(const kair_operand* A, const kair_operand* B, float* ws, int splits, long M, int N, int K,
                    void* stream);
