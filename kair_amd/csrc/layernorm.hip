// LayerNorm over the channel dim of token matrices (nn.LayerNorm(C), eps 1e-5:
// network_swinir.py:199,205,520,725).  One wave per token row; C <= 256 fits 4 values per lane.
// The forward can write its output straight into Swin window order (the gather that
// torch.roll + window_partition perform in network_swinir.py:250-256), so the QKV GEMM reads a
// plain row-major operand.  Backward accumulates into the fp32 residual-stream gradient and
// produces deterministic per-block partial sums for dgamma / dbeta.
#include "common.h"

namespace {

constexpr int MAXV = 4;  // C <= 256

template <typename T>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, long ldx, T* __restrict__ y, long ldy,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      float* __restrict__ mean_out, float* __restrict__ rstd_out, long M,
                                                      int C, float eps, WinMap wm) {
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long nw = (long)gridDim.x * 4;
  for (long r = wave; r < M; r += nw) {       // r = output row (window order if wm.ws > 0)
    const long t = win_to_token(r, wm);         // token row
    float v[MAXV];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = lane + 64 * i;
      v[i] = c < C ? x[t * ldx + c] : 0.f;
      s += v[i];
    }
    const float mu = wave_sum(s) / C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = lane + 64 * i;
      const float d = c < C ? v[i] - mu : 0.f;
      q += d * d;
    }
    const float rs = rsqrtf(wave_sum(q) / C + eps);
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = lane + 64 * i;
      if (c < C) y[r * ldy + c] = (T)((v[i] - mu) * rs * gamma[c] + beta[c]);
      else if (c < ldy) y[r * ldy + c] = (T)0.f;
    }
    if (lane == 0) {
      mean_out[t] = mu;
      rstd_out[t] = rs;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ x, long ldx, const T* __restrict__ dy,
                                                      long ldy, const float* __restrict__ gamma,
                                                      const float* __restrict__ mean, const float* __restrict__ rstd,
                                                      float* dx, long ld_dx, int dx_acc, float* __restrict__ part,
                                                      long M, int C, WinMap wm) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long wave = (long)blockIdx.x * 4 + w;
  const long nw = (long)gridDim.x * 4;
  float dg[MAXV] = {0.f, 0.f, 0.f, 0.f}, db[MAXV] = {0.f, 0.f, 0.f, 0.f};
  float g[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    g[i] = c < C ? gamma[c] : 0.f;
  }
  for (long r = wave; r < M; r += nw) {
    const long t = win_to_token(r, wm);
    const float mu = mean[t], rs = rstd[t];
    float xh[MAXV], gy[MAXV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = lane + 64 * i;
      if (c < C) {
        const float d = (float)dy[r * ldy + c];
        xh[i] = (x[t * ldx + c] - mu) * rs;
        gy[i] = d * g[i];
        dg[i] += d * xh[i];
        db[i] += d;
      } else {
        xh[i] = 0.f;
        gy[i] = 0.f;
      }
      s1 += gy[i];
      s2 += gy[i] * xh[i];
    }
    s1 = wave_sum(s1) / C;
    s2 = wave_sum(s2) / C;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = lane + 64 * i;
      if (c < C) {
        const float d = rs * (gy[i] - s1 - xh[i] * s2);
        float* o = dx + t * ld_dx + c;
        *o = dx_acc ? *o + d : d;
      }
    }
  }
  // block-level reduction of dgamma/dbeta partials (deterministic order)
  __shared__ float red[2][4][256];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    red[0][w][c] = dg[i];
    red[1][w][c] = db[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    part[(long)blockIdx.x * 2 * C + c] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
    part[(long)blockIdx.x * 2 * C + C + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
  }
}

// 64 columns per block, 4 row-phases per column, fixed summation order (deterministic)
__global__ __launch_bounds__(256) void ln_param_reduce(const float* __restrict__ part, int nb, int C, float* dgamma,
                                                       float* dbeta, int acc) {
  __shared__ float red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  float s = 0.f;
  if (c < 2 * C)
    for (int b = ty; b < nb; b += 4) s += part[(long)b * 2 * C + c];
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && c < 2 * C) {
    s = red[0][tx] + red[1][tx] + red[2][tx] + red[3][tx];
    float* o = c < C ? dgamma + c : dbeta + (c - C);
    *o = acc ? *o + s : s;
  }
}

}  // namespace

constexpr int LN_BLOCKS = 512;

extern "C" int kair_layernorm_fwd(const float* x, long ldx, void* y, int y_dtype, long ldy, const float* gamma,
                                  const float* beta, float* mean, float* rstd, long M, int C, float eps, int win_H,
                                  int win_W, int win_ws, int win_shift, void* stream) {
  KAIR_CHECK_ARG(x && y && gamma && beta && mean && rstd, "layernorm_fwd: null pointer");
  KAIR_CHECK_ARG(C > 0 && C <= 256 && ldx >= C && ldy >= C && M > 0, "layernorm_fwd: bad sizes");
  KAIR_CHECK_ARG(win_ws == 0 || (win_H % win_ws == 0 && win_W % win_ws == 0), "layernorm_fwd: window geometry");
  const WinMap wm{win_H, win_W, win_ws, win_shift};
  long nb = (M + 3) / 4;
  if (nb > 8192) nb = 8192;
  hipStream_t s = (hipStream_t)stream;
  if (y_dtype == KAIR_BF16)
    hipLaunchKernelGGL(ln_fwd_kernel<bf16>, dim3((unsigned)nb), dim3(256), 0, s, x, ldx, (bf16*)y, ldy, gamma, beta,
                       mean, rstd, M, C, eps, wm);
  else
    hipLaunchKernelGGL(ln_fwd_kernel<float>, dim3((unsigned)nb), dim3(256), 0, s, x, ldx, (float*)y, ldy, gamma, beta,
                       mean, rstd, M, C, eps, wm);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_layernorm_bwd(const float* x, long ldx, const void* dy, int dy_dtype, long ldy, const float* gamma,
                                  const float* mean, const float* rstd, float* dx_acc, long ld_dx, int dx_accumulate,
                                  float* dgamma, float* dbeta, int dparam_accumulate, float* ws, long M, int C,
                                  int win_H, int win_W, int win_ws, int win_shift, void* stream) {
  KAIR_CHECK_ARG(x && dy && gamma && mean && rstd && dx_acc && dgamma && dbeta && ws, "layernorm_bwd: null pointer");
  KAIR_CHECK_ARG(C > 0 && C <= 256 && M > 0, "layernorm_bwd: bad sizes");
  const WinMap wm{win_H, win_W, win_ws, win_shift};
  hipStream_t s = (hipStream_t)stream;
  long nb = (M + 3) / 4;
  if (nb > LN_BLOCKS) nb = LN_BLOCKS;
  if (dy_dtype == KAIR_BF16)
    hipLaunchKernelGGL(ln_bwd_kernel<bf16>, dim3((unsigned)nb), dim3(256), 0, s, x, ldx, (const bf16*)dy, ldy, gamma,
                       mean, rstd, dx_acc, ld_dx, dx_accumulate, ws, M, C, wm);
  else
    hipLaunchKernelGGL(ln_bwd_kernel<float>, dim3((unsigned)nb), dim3(256), 0, s, x, ldx, (const float*)dy, ldy, gamma,
                       mean, rstd, dx_acc, ld_dx, dx_accumulate, ws, M, C, wm);
  KAIR_CHECK_LAUNCH();
  hipLaunchKernelGGL(ln_param_reduce, dim3((2 * C + 63) / 64), dim3(256), 0, s, ws, (int)nb, C, dgamma, dbeta,
                     dparam_accumulate);
  KAIR_CHECK_LAUNCH();
  return 0;
}
