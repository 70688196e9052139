// BatchNorm2d over NHWC rows (+ fused ReLU / LeakyReLU) for the DnCNN conv stack:
// nn.BatchNorm2d(momentum 0.9, eps 1e-4, affine) of basicblock.conv mode 'B' (basicblock.py:69),
// train mode = batch statistics over (N, H, W) with the running-stat update
// running = (1 - momentum) * running + momentum * stat (unbiased variance for running_var),
// eval mode = running statistics.
//
// Statistics are two-pass (mean, then sum of squared deviations) with deterministic fixed-order
// reductions: per-block column partials (rows split over blocks, 16 row phases per column inside
// a block), then one final block per 64 columns.
#include "common.h"

namespace {

constexpr int BN_NB = 512;   // partial blocks (rows are split over them)

// partial[b][c] (and partial2[b][c]) over rows [b*rpb, (b+1)*rpb):
//   MODE 0: sum z            MODE 1: sum (z - mean)^2
//   MODE 2: sum dr, sum dr * xhat with dr = da * act'(a)
template <int MODE, typename TA>
__global__ __launch_bounds__(1024) void bn_partial(const float* __restrict__ z, long ldz, const TA* __restrict__ a, long lda,
                                                   const float* __restrict__ da, long ldda, long M, int C, long rpb,
                                                   const float* __restrict__ mean, const float* __restrict__ rstd, int act,
                                                   float slope, float* __restrict__ part, float* __restrict__ part2) {
  __shared__ float red[2][16][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + tx;
  const long r0 = (long)blockIdx.x * rpb;
  long r1 = r0 + rpb;
  if (r1 > M) r1 = M;
  float s = 0.f, s2 = 0.f;
  if (c < C) {
    const float mu = MODE >= 1 ? mean[c] : 0.f;
    const float rs = MODE == 2 ? rstd[c] : 0.f;
    for (long r = r0 + ty; r < r1; r += 16) {
      const float zv = z[r * ldz + c];
      if constexpr (MODE == 0) {
        s += zv;
      } else if constexpr (MODE == 1) {
        const float d = zv - mu;
        s += d * d;
      } else {
        float g = da[r * ldda + c];
        if (act) {
          const float av = (float)a[r * lda + c];
          g = av > 0.f ? g : (act == 2 ? g * slope : 0.f);
        }
        s += g;
        s2 += g * (zv - mu) * rs;
      }
    }
  }
  red[0][ty][tx] = s;
  red[1][ty][tx] = s2;
  __syncthreads();
  if (ty == 0 && c < C) {
    float t = 0.f, t2 = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      t += red[0][k][tx];
      t2 += red[1][k][tx];
    }
    part[(long)blockIdx.x * C + c] = t;
    if (MODE == 2) part2[(long)blockIdx.x * C + c] = t2;
  }
}

// final reductions (one 1024-thread block per 64 columns, fixed order)
//   MODE 0: mean = sum / M
//   MODE 1: var = sum / M -> rstd; running-stat update
//   MODE 2: dbeta (+)= sum dr, dgamma (+)= sum dr*xhat; keep the two means for the apply pass
template <int MODE>
__global__ __launch_bounds__(1024) void bn_final(const float* __restrict__ part, const float* __restrict__ part2, int nb,
                                                 int C, long M, float eps, float momentum, float* mean, float* rstd,
                                                 float* running_mean, float* running_var, float* dgamma, float* dbeta,
                                                 int acc, float* stash) {
  __shared__ float red[2][16][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  float s = 0.f, s2 = 0.f;
  if (c < C) {
    int b = ty;
    for (; b + 3 * 16 < nb; b += 4 * 16) {   // 4 partials (x2 in MODE 2) in flight, same summation order
      float v[4], w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[u] = part[(long)(b + 16 * u) * C + c];
        w[u] = MODE == 2 ? part2[(long)(b + 16 * u) * C + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s += v[u];
        if (MODE == 2) s2 += w[u];
      }
    }
    for (; b < nb; b += 16) {
      s += part[(long)b * C + c];
      if (MODE == 2) s2 += part2[(long)b * C + c];
    }
  }
  red[0][ty][tx] = s;
  red[1][ty][tx] = s2;
  __syncthreads();
  if (ty != 0 || c >= C) return;
  float t = 0.f, t2 = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    t += red[0][k][tx];
    t2 += red[1][k][tx];
  }
  if constexpr (MODE == 0) {
    mean[c] = t / (float)M;
  } else if constexpr (MODE == 1) {
    const float var = t / (float)M;
    rstd[c] = rsqrtf(var + eps);
    if (running_mean) {
      running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean[c];
      const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
      running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
    }
  } else {
    dbeta[c] = acc ? dbeta[c] + t : t;
    dgamma[c] = acc ? dgamma[c] + t2 : t2;
    stash[c] = t / (float)M;
    stash[C + c] = t2 / (float)M;
  }
}

// a = act(gamma * (z - mean) * rstd + beta), eval mode reads running stats
template <typename TO>
__global__ void bn_apply_fwd(const float* __restrict__ z, long ldz, TO* __restrict__ out, long ldo, long M, int C,
                             const float* __restrict__ gamma, const float* __restrict__ beta, const float* __restrict__ mean,
                             const float* __restrict__ rstd, const float* __restrict__ rvar, float eps, int act, float slope) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C) return;
  const long r = i / C;
  const int c = (int)(i - r * C);
  const float rs = rvar ? rsqrtf(rvar[c] + eps) : rstd[c];
  float v = gamma[c] * (z[r * ldz + c] - mean[c]) * rs + beta[c];
  if (act == 1) v = fmaxf(v, 0.f);
  else if (act == 2) v = v > 0.f ? v : v * slope;
  out[r * ldo + c] = (TO)v;
}

// dz = gamma * rstd * (dr - mean(dr) - xhat * mean(dr * xhat))
template <typename TA, typename TO>
__global__ void bn_apply_bwd(const float* __restrict__ z, long ldz, const TA* __restrict__ a, long lda,
                             const float* __restrict__ da, long ldda, TO* __restrict__ dz, long lddz, long M, int C,
                             const float* __restrict__ gamma, const float* __restrict__ mean, const float* __restrict__ rstd,
                             const float* __restrict__ stash, int act, float slope) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C) return;
  const long r = i / C;
  const int c = (int)(i - r * C);
  float g = da[r * ldda + c];
  if (act) {
    const float av = (float)a[r * lda + c];
    g = av > 0.f ? g : (act == 2 ? g * slope : 0.f);
  }
  const float rs = rstd[c];
  const float xh = (z[r * ldz + c] - mean[c]) * rs;
  dz[r * lddz + c] = (TO)(gamma[c] * rs * (g - stash[c] - xh * stash[C + c]));
}

inline unsigned nblk(long n, int bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

extern "C" long kair_bn_ws(int C) { return 2L * BN_NB * C + 2L * C; }

extern "C" int kair_bn_fwd(const float* z, long ldz, void* out, int out_dtype, long ldo, long M, int C, const float* gamma,
                           const float* beta, float* running_mean, float* running_var, float momentum, float eps,
                           int training, float* mean, float* rstd, int act, float slope, float* ws, void* stream) {
  KAIR_CHECK_ARG(z && out && gamma && beta && M > 0 && C > 0 && ldz >= C && ldo >= C, "bn_fwd: bad args");
  KAIR_CHECK_ARG(training ? (mean && rstd && ws) : (running_mean && running_var), "bn_fwd: missing statistics buffers");
  hipStream_t s = (hipStream_t)stream;
  const float* mu = mean;
  const float* rv = nullptr;
  if (training) {
    const long rpb = (M + BN_NB - 1) / BN_NB;
    const dim3 gp(BN_NB, (C + 63) / 64), bp(1024), gf((C + 63) / 64);
    KAIR_LAUNCH((bn_partial<0, float>), gp, bp, 0, s, z, ldz, nullptr, 0, nullptr, 0, M, C, rpb, nullptr, nullptr, 0,
                       0.f, ws, nullptr);
    KAIR_CHECK_LAUNCH();
    KAIR_LAUNCH(bn_final<0>, gf, bp, 0, s, ws, nullptr, BN_NB, C, M, eps, momentum, mean, rstd, nullptr, nullptr,
                       nullptr, nullptr, 0, nullptr);
    KAIR_CHECK_LAUNCH();
    KAIR_LAUNCH((bn_partial<1, float>), gp, bp, 0, s, z, ldz, nullptr, 0, nullptr, 0, M, C, rpb, mean, nullptr, 0,
                       0.f, ws, nullptr);
    KAIR_CHECK_LAUNCH();
    KAIR_LAUNCH(bn_final<1>, gf, bp, 0, s, ws, nullptr, BN_NB, C, M, eps, momentum, mean, rstd, running_mean,
                       running_var, nullptr, nullptr, 0, nullptr);
    KAIR_CHECK_LAUNCH();
  } else {
    mu = running_mean;
    rv = running_var;
  }
  const long n = M * C;
  if (out_dtype == KAIR_BF16)
    KAIR_LAUNCH(bn_apply_fwd<bf16>, dim3(nblk(n, 256)), dim3(256), 0, s, z, ldz, (bf16*)out, ldo, M, C, gamma, beta,
                       mu, rstd, rv, eps, act, slope);
  else
    KAIR_LAUNCH(bn_apply_fwd<float>, dim3(nblk(n, 256)), dim3(256), 0, s, z, ldz, (float*)out, ldo, M, C, gamma, beta,
                       mu, rstd, rv, eps, act, slope);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_bn_bwd(const float* z, long ldz, const void* a, int a_dtype, long lda, const float* da, long ldda,
                           void* dz, int dz_dtype, long lddz, long M, int C, const float* gamma, const float* mean,
                           const float* rstd, int act, float slope, float* dgamma, float* dbeta, int accumulate, float* ws,
                           void* stream) {
  KAIR_CHECK_ARG(z && da && dz && gamma && mean && rstd && dgamma && dbeta && ws && M > 0 && C > 0, "bn_bwd: bad args");
  KAIR_CHECK_ARG(!act || a, "bn_bwd: activation gate needs the post-activation tensor");
  hipStream_t s = (hipStream_t)stream;
  const long rpb = (M + BN_NB - 1) / BN_NB;
  const dim3 gp(BN_NB, (C + 63) / 64), bp(1024), gf((C + 63) / 64);
  float* part = ws;
  float* part2 = ws + (long)BN_NB * C;
  float* stash = ws + 2L * BN_NB * C;
  if (a_dtype == KAIR_BF16)
    KAIR_LAUNCH((bn_partial<2, bf16>), gp, bp, 0, s, z, ldz, (const bf16*)a, lda, da, ldda, M, C, rpb, mean, rstd,
                       act, slope, part, part2);
  else
    KAIR_LAUNCH((bn_partial<2, float>), gp, bp, 0, s, z, ldz, (const float*)a, lda, da, ldda, M, C, rpb, mean, rstd,
                       act, slope, part, part2);
  KAIR_CHECK_LAUNCH();
  KAIR_LAUNCH(bn_final<2>, gf, bp, 0, s, part, part2, BN_NB, C, M, 0.f, 0.f, nullptr, nullptr, nullptr, nullptr,
                     dgamma, dbeta, accumulate, stash);
  KAIR_CHECK_LAUNCH();
  const long n = M * C;
  const dim3 ga(nblk(n, 256)), ba(256);
  if (a_dtype == KAIR_BF16) {
    if (dz_dtype == KAIR_BF16)
      KAIR_LAUNCH((bn_apply_bwd<bf16, bf16>), ga, ba, 0, s, z, ldz, (const bf16*)a, lda, da, ldda, (bf16*)dz, lddz, M, C,
                         gamma, mean, rstd, stash, act, slope);
    else
      KAIR_LAUNCH((bn_apply_bwd<bf16, float>), ga, ba, 0, s, z, ldz, (const bf16*)a, lda, da, ldda, (float*)dz, lddz, M,
                         C, gamma, mean, rstd, stash, act, slope);
  } else {
    if (dz_dtype == KAIR_BF16)
      KAIR_LAUNCH((bn_apply_bwd<float, bf16>), ga, ba, 0, s, z, ldz, (const float*)a, lda, da, ldda, (bf16*)dz, lddz, M,
                         C, gamma, mean, rstd, stash, act, slope);
    else
      KAIR_LAUNCH((bn_apply_bwd<float, float>), ga, ba, 0, s, z, ldz, (const float*)a, lda, da, ldda, (float*)dz, lddz,
                         M, C, gamma, mean, rstd, stash, act, slope);
  }
  KAIR_CHECK_LAUNCH();
  return 0;
}
