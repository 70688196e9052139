// USRNet on gfx950 (CDNA4): 2-D DFTs of the HR grid, the closed-form data step (DataNet) forward
// and backward, and the small kernels around them (HyPaNet MLP, nearest upsample, input packing,
// deterministic reductions).
//
// Reference: /root/reference/models/network_usrnet_v1.py — splits :33-45, p2o :48-69,
// upsample :72-82, DataNet.forward :183-194, HyPaNet :204-216, USRNet.forward :245-262.
//
// Layout.  A complex plane set [planes = B*C][H][W] lives TRANSPOSED in HBM: T[plane][v][u]
// (v = column, u = row), float2.  Three passes per 2-D transform:
//   rows  (kair_usr_fft_rows)  : R consecutive image rows per CTA -> DFT along v in LDS -> every
//                                column line gets an R-element segment (R*8 contiguous bytes);
//   cols  (kair_usr_fft_cols)  : sf whole column lines per CTA, v = g + q*W/sf (q < sf), so every
//                                alias group {(u' + p*H/sf, g + q*W/sf)} of the `splits` block
//                                mean is CTA-local -> DFT along u -> closed form -> inverse DFT
//                                along u -> lines written back;
//   irows (kair_usr_ifft_rows) : R-row segments -> inverse DFT along v -> real part * scale.
// Line DFTs are Stockham autosort (radix 4/2/3, any N = 2^a 3^b <= 2048) ping-ponging between two
// LDS buffers; twiddles come from a per-CTA LDS table computed in double precision.
//
// DataNet maths (per batch element b; B = FB, C = conj(FB), w = mean_alias |FB|^2, d = 1/(w+a)):
//   FR = FBFy + a * F(x),  FX = (FR - C * T(S(B*FR)) * d) / a,  z = Re(F^-1(FX))
// where S = mean over the sf^2 aliases and T = tile back (repeat).  The map is self-adjoint, so
//   dL/dx = Re(F^-1(G - C * T(S(B*G)) * d))                 (G = F(dL/dz))
//   dL/da = (1/N) Re sum conj(G) * Z,  Z = ( C*T(S(B*FR))*d^2 - (FBFy - C*T(S(B*FBFy))*d)/a ) / a
// (derivation in DESIGN.md; FR of the forward is saved for the second line).
#include <math.h>

#include "common.h"

namespace {

// ------------------------------------------------------------------------------------------
// Stockham line DFTs in LDS
// ------------------------------------------------------------------------------------------
struct FftPlan {
  int n;    // line length
  int nst;  // stages
  int enc;  // 2 bits per stage: 0 -> radix 2, 1 -> radix 3, 2 -> radix 4
};

KAIR_DEV float2 cmul(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
KAIR_DEV float2 cmulc(float2 a, float2 b) { return make_float2(a.x * b.x + a.y * b.y, a.x * b.y - a.y * b.x); }  // conj(a)*b
KAIR_DEV float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
KAIR_DEV float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
KAIR_DEV float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
KAIR_DEV float2 mul_i(float2 a) { return make_float2(-a.y, a.x); }       // i * a
KAIR_DEV float2 mul_negi(float2 a) { return make_float2(a.y, -a.x); }    // -i * a

// tw[k] = exp(-2 pi i k / n)
KAIR_DEV void build_twiddles(float2* tw, int n) {
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    double s, c;
    sincospi(-2.0 * (double)k / (double)n, &s, &c);
    tw[k] = make_float2((float)c, (float)s);
  }
}

template <int R, bool INV>
KAIR_DEV void dft_small(float2 (&v)[R]) {
  if constexpr (R == 2) {
    const float2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
  } else if constexpr (R == 3) {
    const float h = 0.86602540378443865f;
    const float2 t1 = cadd(v[1], v[2]), t2 = csub(v[1], v[2]);
    const float2 m = make_float2(v[0].x - 0.5f * t1.x, v[0].y - 0.5f * t1.y);
    const float2 r = cscale(mul_i(t2), h);   // i*(sqrt3/2)*(a1 - a2)
    v[0] = cadd(v[0], t1);
    if (INV) { v[1] = cadd(m, r); v[2] = csub(m, r); }
    else { v[1] = csub(m, r); v[2] = cadd(m, r); }
  } else {
    const float2 s02 = cadd(v[0], v[2]), d02 = csub(v[0], v[2]);
    const float2 s13 = cadd(v[1], v[3]), d13 = csub(v[1], v[3]);
    const float2 r = INV ? mul_i(d13) : mul_negi(d13);
    v[0] = cadd(s02, s13);
    v[2] = csub(s02, s13);
    v[1] = cadd(d02, r);
    v[3] = csub(d02, r);
  }
}

// one radix-R Stockham stage over nl lines (length n, LDS line stride ls): src -> dst
template <int R, bool INV>
KAIR_DEV void fft_stage(const float2* __restrict__ src, float2* __restrict__ dst, int nl, int n, int ls, int Ns,
                        const float2* __restrict__ tw) {
  const int nb = n / R;
  const int tstep = n / (Ns * R);
  const FDiv dnb{nb, 1.0f / (float)nb}, dns{Ns, 1.0f / (float)Ns};
  const int total = nl * nb;
  for (int i = threadIdx.x; i < total; i += blockDim.x) {
    const int l = fdiv(i, dnb), j = i - l * nb;
    const int q = fdiv(j, dns), k = j - q * Ns;
    const float2* s = src + l * ls;
    float2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = s[j + r * nb];
#pragma unroll
    for (int r = 1; r < R; ++r) {
      float2 w = tw[r * k * tstep];
      if (INV) w.y = -w.y;
      v[r] = cmul(v[r], w);
    }
    dft_small<R, INV>(v);
    float2* d = dst + l * ls + q * Ns * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) d[r * Ns] = v[r];
  }
}

// full DFT of nl lines; returns the buffer holding the result (a or b).  Ends with a barrier.
template <bool INV>
KAIR_DEV float2* fft_lines(float2* a, float2* b, int nl, int ls, const FftPlan& p, const float2* tw) {
  int Ns = 1;
  for (int s = 0; s < p.nst; ++s) {
    const int code = (p.enc >> (2 * s)) & 3;
    if (code == 2) { fft_stage<4, INV>(a, b, nl, p.n, ls, Ns, tw); Ns *= 4; }
    else if (code == 0) { fft_stage<2, INV>(a, b, nl, p.n, ls, Ns, tw); Ns *= 2; }
    else { fft_stage<3, INV>(a, b, nl, p.n, ls, Ns, tw); Ns *= 3; }
    __syncthreads();
    float2* t = a;
    a = b;
    b = t;
  }
  return a;
}

// ------------------------------------------------------------------------------------------
// pass 1: rows, forward, real source -> transposed complex
// ------------------------------------------------------------------------------------------
struct RowSrc {
  const float* p;
  int mode;   // KAIR_USR_SRC_*
  int C;      // planes per batch element
  long ld;    // NHWC pixel stride
  int kh, kw; // PSF
  int sf;     // zero-upsample factor
};

KAIR_DEV float row_src(const RowSrc& s, int plane, int y, int v, int H, int W) {
  switch (s.mode) {
    case KAIR_USR_SRC_NCHW:
      return s.p[((long)plane * H + y) * W + v];
    case KAIR_USR_SRC_PSF: {   // otf[y][v] = psf[(y + kh/2) % H][(v + kw/2) % W] (zero outside the PSF)
      int ky = y + s.kh / 2, kx = v + s.kw / 2;
      if (ky >= H) ky -= H;
      if (kx >= W) kx -= W;
      return (ky < s.kh && kx < s.kw) ? s.p[((long)plane * s.kh + ky) * s.kw + kx] : 0.f;
    }
    case KAIR_USR_SRC_ZUP: {
      if ((y % s.sf) || (v % s.sf)) return 0.f;
      const int h = H / s.sf, w = W / s.sf;
      return s.p[((long)plane * h + y / s.sf) * w + v / s.sf];
    }
    default: {  // NHWC
      const int b = plane / s.C, c = plane - b * s.C;
      return s.p[(((long)b * H + y) * W + v) * s.ld + c];
    }
  }
}

__global__ __launch_bounds__(256) void fft_rows_fwd_kernel(RowSrc src, float2* __restrict__ T, int H, int W, int R,
                                                           FftPlan pw) {
  extern __shared__ float2 sm[];
  const int ls = W + 1;
  float2* tw = sm;
  float2* a = sm + W;
  float2* b = a + R * ls;
  const int plane = blockIdx.y, y0 = blockIdx.x * R;
  build_twiddles(tw, W);
  const FDiv dW{W, 1.0f / (float)W}, dR{R, 1.0f / (float)R};
  for (int i = threadIdx.x; i < R * W; i += blockDim.x) {
    const int r = fdiv(i, dW), v = i - r * W;
    a[r * ls + v] = make_float2(row_src(src, plane, y0 + r, v, H, W), 0.f);
  }
  __syncthreads();
  const float2* res = fft_lines<false>(a, b, R, ls, pw, tw);
  for (int i = threadIdx.x; i < R * W; i += blockDim.x) {
    const int v = fdiv(i, dR), r = i - v * R;
    T[((long)plane * W + v) * H + y0 + r] = res[r * ls + v];
  }
}

// ------------------------------------------------------------------------------------------
// pass 2: columns + closed form
// ------------------------------------------------------------------------------------------
struct ColArgs {
  const float2* T;      // in  [planes][W][H]
  float2* Tout;         // out [planes][W][H] (may alias T; NULL: skip the inverse DFT, bwd only)
  const float2* FB;     // [B][W][H]
  const float2* FBFy;   // [planes][W][H]
  float2* FR;           // fwd: saved if non-null; bwd: read
  float* invW;          // [B][W/sf][H/sf]
  const float* alpha;   // alpha of batch b at alpha[b * astride]
  int astride;
  float* part;          // bwd: [planes][W/sf] partial dL/dalpha
  int C, H, W, sf;
};

__global__ __launch_bounds__(256) void fft_cols_kernel(ColArgs A, int mode, FftPlan ph) {
  extern __shared__ float2 sm[];
  __shared__ float red[4];
  const int H = A.H, ls = H + 1, sf = A.sf, Wg = A.W / sf, Hg = H / sf;
  float2* tw = sm;
  float2* a = sm + H;
  float2* b = a + sf * ls;
  const int plane = blockIdx.y, g = blockIdx.x;
  const int bb = plane / A.C;
  build_twiddles(tw, H);
  const FDiv dH{H, 1.0f / (float)H};
  for (int i = threadIdx.x; i < sf * H; i += blockDim.x) {
    const int q = fdiv(i, dH), u = i - q * H;
    a[q * ls + u] = A.T[((long)plane * A.W + g + q * Wg) * H + u];
  }
  __syncthreads();
  float2* F = fft_lines<false>(a, b, sf, ls, ph, tw);
  float2* S = (F == a) ? b : a;
  const float inv_n = 1.0f / (float)(sf * sf);
  auto lidx = [&](int q, int u) { return ((long)plane * A.W + g + q * Wg) * H + u; };
  auto bidx = [&](int q, int u) { return ((long)bb * A.W + g + q * Wg) * H + u; };

  if (mode == KAIR_USR_COL_FB) {
    for (int up = threadIdx.x; up < Hg; up += blockDim.x) {
      float s = 0.f;
      for (int q = 0; q < sf; ++q)
        for (int p = 0; p < sf; ++p) {
          const float2 f = F[q * ls + up + p * Hg];
          s += f.x * f.x + f.y * f.y;
        }
      A.invW[((long)bb * Wg + g) * Hg + up] = s * inv_n;
    }
    for (int i = threadIdx.x; i < sf * H; i += blockDim.x) {
      const int q = fdiv(i, dH), u = i - q * H;
      A.Tout[lidx(q, u)] = F[q * ls + u];
    }
    return;
  }
  if (mode == KAIR_USR_COL_FBFY) {
    for (int i = threadIdx.x; i < sf * H; i += blockDim.x) {
      const int q = fdiv(i, dH), u = i - q * H;
      A.Tout[lidx(q, u)] = cmulc(A.FB[bidx(q, u)], F[q * ls + u]);
    }
    return;
  }
  const float al = A.alpha[(long)bb * A.astride];
  const float ial = 1.0f / al;
  if (mode == KAIR_USR_COL_DATA_FWD) {
    for (int up = threadIdx.x; up < Hg; up += blockDim.x) {
      const float d = 1.0f / (A.invW[((long)bb * Wg + g) * Hg + up] + al);
      float2 s = make_float2(0.f, 0.f);
      for (int q = 0; q < sf; ++q)
        for (int p = 0; p < sf; ++p) {
          const int u = up + p * Hg;
          const float2 fr = cadd(A.FBFy[lidx(q, u)], cscale(F[q * ls + u], al));
          if (A.FR) A.FR[lidx(q, u)] = fr;
          F[q * ls + u] = fr;
          s = cadd(s, cmul(A.FB[bidx(q, u)], fr));
        }
      s = cscale(s, inv_n * d);
      for (int q = 0; q < sf; ++q)
        for (int p = 0; p < sf; ++p) {
          const int u = up + p * Hg;
          const float2 fx = csub(F[q * ls + u], cmulc(A.FB[bidx(q, u)], s));
          F[q * ls + u] = cscale(fx, ial);
        }
    }
  } else {  // KAIR_USR_COL_DATA_BWD
    float acc = 0.f;
    for (int up = threadIdx.x; up < Hg; up += blockDim.x) {
      const float d = 1.0f / (A.invW[((long)bb * Wg + g) * Hg + up] + al);
      float2 sg = make_float2(0.f, 0.f), sr = sg, sy = sg;
      for (int q = 0; q < sf; ++q)
        for (int p = 0; p < sf; ++p) {
          const int u = up + p * Hg;
          const float2 fb = A.FB[bidx(q, u)];
          sg = cadd(sg, cmul(fb, F[q * ls + u]));
          sr = cadd(sr, cmul(fb, A.FR[lidx(q, u)]));
          sy = cadd(sy, cmul(fb, A.FBFy[lidx(q, u)]));
        }
      sg = cscale(sg, inv_n * d);
      sr = cscale(sr, inv_n * d * d);
      sy = cscale(sy, inv_n * d);
      for (int q = 0; q < sf; ++q)
        for (int p = 0; p < sf; ++p) {
          const int u = up + p * Hg;
          const float2 fb = A.FB[bidx(q, u)];
          const float2 G = F[q * ls + u];
          const float2 ly = cscale(csub(A.FBFy[lidx(q, u)], cmulc(fb, sy)), ial);
          const float2 Z = cscale(csub(cmulc(fb, sr), ly), ial);
          acc += G.x * Z.x + G.y * Z.y;
          F[q * ls + u] = csub(G, cmulc(fb, sg));
        }
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) A.part[(long)plane * Wg + g] = ((red[0] + red[1]) + red[2]) + red[3];
    if (!A.Tout) return;
  }
  __syncthreads();
  const float2* res = fft_lines<true>(F, S, sf, ls, ph, tw);
  for (int i = threadIdx.x; i < sf * H; i += blockDim.x) {
    const int q = fdiv(i, dH), u = i - q * H;
    A.Tout[lidx(q, u)] = res[q * ls + u];
  }
}

// ------------------------------------------------------------------------------------------
// pass 3: rows, inverse, transposed complex -> real
// ------------------------------------------------------------------------------------------
template <typename TO>
__global__ __launch_bounds__(256) void fft_rows_inv_kernel(const float2* __restrict__ T, TO* __restrict__ dst, int nhwc,
                                                           int C, long ld, float scale, int H, int W, int R, FftPlan pw) {
  extern __shared__ float2 sm[];
  const int ls = W + 1;
  float2* tw = sm;
  float2* a = sm + W;
  float2* b = a + R * ls;
  const int plane = blockIdx.y, y0 = blockIdx.x * R;
  build_twiddles(tw, W);
  const FDiv dW{W, 1.0f / (float)W}, dR{R, 1.0f / (float)R};
  for (int i = threadIdx.x; i < R * W; i += blockDim.x) {
    const int v = fdiv(i, dR), r = i - v * R;
    a[r * ls + v] = T[((long)plane * W + v) * H + y0 + r];
  }
  __syncthreads();
  const float2* res = fft_lines<true>(a, b, R, ls, pw, tw);
  const int bb = plane / C, c = plane - bb * C;
  for (int i = threadIdx.x; i < R * W; i += blockDim.x) {
    const int r = fdiv(i, dW), v = i - r * W;
    const float val = res[r * ls + v].x * scale;
    const int y = y0 + r;
    if (nhwc) dst[(((long)bb * H + y) * W + v) * ld + c] = (TO)val;
    else dst[((long)plane * H + y) * W + v] = (TO)val;
  }
}

// ------------------------------------------------------------------------------------------
// small kernels
// ------------------------------------------------------------------------------------------
// out[s * ostride] (+)= scale * sum_{j < seglen} ws[s * seglen + j]   (fixed order, one block/segment)
__global__ __launch_bounds__(256) void seg_sum_kernel(const float* __restrict__ ws, int seglen, float scale,
                                                      float* __restrict__ out, int ostride, int acc) {
  __shared__ float red[4];
  const int s = blockIdx.x;
  float v = 0.f;
  for (int j = threadIdx.x; j < seglen; j += 256) v += ws[(long)s * seglen + j];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t = (((red[0] + red[1]) + red[2]) + red[3]) * scale;
    float* o = out + (long)s * ostride;
    *o = acc ? *o + t : t;
  }
}

// ws[b * nchunk + chunk] = sum over the chunk's pixels of x[(b*HW + p) * ld + c]
__global__ __launch_bounds__(256) void chan_sum_partial_kernel(const float* __restrict__ x, long ld, int c, long HW,
                                                               int nchunk, float* __restrict__ ws) {
  __shared__ float red[4];
  const int chunk = blockIdx.x, b = blockIdx.y;
  const long per = (HW + nchunk - 1) / nchunk;
  const long p0 = chunk * per;
  long p1 = p0 + per;
  if (p1 > HW) p1 = HW;
  float v = 0.f;
  for (long p = p0 + threadIdx.x; p < p1; p += 256) v += x[((long)b * HW + p) * ld + c];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) ws[(long)b * nchunk + chunk] = ((red[0] + red[1]) + red[2]) + red[3];
}

// F.interpolate(x, scale_factor=sf, mode='nearest') of NCHW planes (network_usrnet_v1.py:252)
__global__ void upsample_nearest_kernel(const float* __restrict__ L, float* __restrict__ out, int h, int w, int sf,
                                        long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int W = w * sf, H = h * sf;
  const int x = (int)(i % W);
  const long py = i / W;
  const int y = (int)(py % H);
  const long plane = py / H;
  out[i] = L[(plane * h + y / sf) * w + x / sf];
}

// ResUNet input: torch.cat((x, beta.repeat(...)), 1) as NHWC rows of width ld (v1:261):
// channels [0, C) = x, C = beta[b], the rest 0
template <typename T>
__global__ void pack_input_kernel(const float* __restrict__ x, const float* __restrict__ beta, int bstride,
                                  T* __restrict__ out, int ld, int C, long HW, long npix) {
  const long pix = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= npix) return;
  const long b = pix / HW, p = pix - b * HW;
  for (int c = 0; c < ld; ++c) {
    float v = 0.f;
    if (c < C) v = x[(b * C + c) * HW + p];
    else if (c == C) v = beta[b * bstride];
    out[pix * ld + c] = (T)v;
  }
}

KAIR_DEV float softplus_t20(float x) { return x > 20.f ? x : log1pf(expf(x)); }   // nn.Softplus()
KAIR_DEV float softplus_grad(float x) { return x > 20.f ? 1.f : 1.f / (1.f + expf(-x)); }

// HyPaNet (v1:204-216): ab = softplus(W3 relu(W2 relu(W1 [sigma, sf] + b1) + b2) + b3) + 1e-6.
// One block; z1/z2/z3 of every batch element are kept in LDS.
struct HypaParams {
  const float *W1, *b1, *W2, *b2, *W3, *b3;
};

KAIR_DEV void hypa_forward_all(const float* sigma, float sf, const HypaParams& P, int hc, int no, int B, float* z1,
                               float* z2, float* z3) {
  for (int i = threadIdx.x; i < B * hc; i += blockDim.x) {
    const int b = i / hc, j = i - b * hc;
    z1[i] = P.W1[j * 2] * sigma[b] + P.W1[j * 2 + 1] * sf + P.b1[j];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < B * hc; i += blockDim.x) {
    const int b = i / hc, j = i - b * hc;
    float s = P.b2[j];
    for (int k = 0; k < hc; ++k) s += P.W2[j * hc + k] * fmaxf(z1[b * hc + k], 0.f);
    z2[i] = s;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < B * no; i += blockDim.x) {
    const int b = i / no, j = i - b * no;
    float s = P.b3[j];
    for (int k = 0; k < hc; ++k) s += P.W3[j * hc + k] * fmaxf(z2[b * hc + k], 0.f);
    z3[i] = s;
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void hypanet_fwd_kernel(const float* __restrict__ sigma, float sf, HypaParams P, int hc,
                                                          int no, int B, float* __restrict__ ab) {
  extern __shared__ float hs[];
  float *z1 = hs, *z2 = z1 + B * hc, *z3 = z2 + B * hc;
  hypa_forward_all(sigma, sf, P, hc, no, B, z1, z2, z3);
  for (int i = threadIdx.x; i < B * no; i += blockDim.x) ab[i] = softplus_t20(z3[i]) + 1e-6f;
}

struct HypaGrads {
  float *W1, *b1, *W2, *b2, *W3, *b3;
};

__global__ __launch_bounds__(256) void hypanet_bwd_kernel(const float* __restrict__ sigma, float sf, HypaParams P,
                                                          int hc, int no, int B, const float* __restrict__ gab,
                                                          HypaGrads Gp, int acc) {
  extern __shared__ float hs[];
  float *z1 = hs, *z2 = z1 + B * hc, *z3 = z2 + B * hc;
  float *g3 = z3 + B * no, *g2 = g3 + B * no, *g1 = g2 + B * hc;
  hypa_forward_all(sigma, sf, P, hc, no, B, z1, z2, z3);
  for (int i = threadIdx.x; i < B * no; i += blockDim.x) g3[i] = gab[i] * softplus_grad(z3[i]);
  __syncthreads();
  for (int i = threadIdx.x; i < B * hc; i += blockDim.x) {
    const int b = i / hc, k = i - b * hc;
    float s = 0.f;
    for (int j = 0; j < no; ++j) s += P.W3[j * hc + k] * g3[b * no + j];
    g2[i] = z2[i] > 0.f ? s : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < B * hc; i += blockDim.x) {
    const int b = i / hc, k = i - b * hc;
    float s = 0.f;
    for (int j = 0; j < hc; ++j) s += P.W2[j * hc + k] * g2[b * hc + j];
    g1[i] = z1[i] > 0.f ? s : 0.f;
  }
  __syncthreads();
  auto put = [&](float* o, float v) { *o = acc ? *o + v : v; };
  for (int i = threadIdx.x; i < no * hc; i += blockDim.x) {
    const int j = i / hc, k = i - j * hc;
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += g3[b * no + j] * fmaxf(z2[b * hc + k], 0.f);
    put(Gp.W3 + i, s);
  }
  for (int i = threadIdx.x; i < hc * hc; i += blockDim.x) {
    const int j = i / hc, k = i - j * hc;
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += g2[b * hc + j] * fmaxf(z1[b * hc + k], 0.f);
    put(Gp.W2 + i, s);
  }
  for (int i = threadIdx.x; i < hc * 2; i += blockDim.x) {
    const int j = i >> 1, k = i & 1;
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += g1[b * hc + j] * (k == 0 ? sigma[b] : sf);
    put(Gp.W1 + i, s);
  }
  for (int j = threadIdx.x; j < no; j += blockDim.x) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += g3[b * no + j];
    put(Gp.b3 + j, s);
  }
  for (int j = threadIdx.x; j < hc; j += blockDim.x) {
    float s2 = 0.f, s1 = 0.f;
    for (int b = 0; b < B; ++b) {
      s2 += g2[b * hc + j];
      s1 += g1[b * hc + j];
    }
    put(Gp.b2 + j, s2);
    put(Gp.b1 + j, s1);
  }
}

// ResUNet.forward's ReplicationPad2d to a multiple of 8 and crop (network_usrnet_v1.py:148-151, 164)
// and their adjoints, one element per thread:
//   REPLICATE  NHWC H x W -> Hp x Wp, edge pixels repeated (the padded U-Net input)
//   ZERO       NHWC H x W -> Hp x Wp, zeros outside (the crop's adjoint: the output gradient)
//   FOLD       NHWC Hp x Wp -> H x W, each pad pixel's value added to the edge pixel it copied
//              (the replicate pad's adjoint: the input gradient), fixed order
//   CROP_NCHW  planes Hp x Wp -> H x W (the U-Net output)
template <typename T>
__global__ __launch_bounds__(256) void usr_pad_kernel(const T* __restrict__ src, T* __restrict__ dst, int mode, int ldc,
                                                      int H, int W, int Hp, int Wp, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  if (mode == KAIR_USR_CROP_NCHW) {
    const long pl = i / ((long)H * W);
    const int r = (int)(i - pl * H * W), y = r / W, x = r - y * W;
    dst[i] = src[(pl * Hp + y) * Wp + x];
    return;
  }
  const int c = (int)(i % ldc);
  const long p = i / ldc;
  if (mode == KAIR_USR_PAD_FOLD) {
    const int x = (int)(p % W), y = (int)((p / W) % H);
    const long b = p / ((long)W * H);
    const int y1 = y == H - 1 ? Hp : y + 1, x1 = x == W - 1 ? Wp : x + 1;
    float s = 0.f;
    for (int yy = y; yy < y1; ++yy)
      for (int xx = x; xx < x1; ++xx) s += (float)src[((b * Hp + yy) * Wp + xx) * ldc + c];
    dst[i] = (T)s;
    return;
  }
  const int xp = (int)(p % Wp), yp = (int)((p / Wp) % Hp);
  const long b = p / ((long)Wp * Hp);
  if (mode == KAIR_USR_PAD_ZERO && (yp >= H || xp >= W)) {
    dst[i] = (T)0.f;
    return;
  }
  const int y = yp < H ? yp : H - 1, x = xp < W ? xp : W - 1;
  dst[i] = src[((b * H + y) * W + x) * ldc + c];
}

int make_plan(int n, FftPlan* p) {
  p->n = n;
  p->nst = 0;
  p->enc = 0;
  int m = n;
  auto push = [&](int code) { p->enc |= code << (2 * p->nst); ++p->nst; };
  while (m % 4 == 0 && p->nst < 15) { push(2); m /= 4; }
  while (m % 2 == 0 && p->nst < 15) { push(0); m /= 2; }
  while (m % 3 == 0 && p->nst < 15) { push(1); m /= 3; }
  if (m != 1) return kair_set_error(KAIR_ERR_ARG, "usr fft: length %d is not 2^a 3^b (<= 2048)", n);
  return 0;
}

int row_block(int H, int W) {
  int R = W <= 512 ? 8 : 4;
  while (R > 1 && H % R) R >>= 1;
  return R;
}

inline unsigned nblk(long n, int bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

// ============================================================================================
// C ABI
// ============================================================================================
extern "C" int kair_usr_fft_rows(const float* src, int src_mode, int C, long ld, int kh, int kw, int sf, void* T,
                                 int planes, int H, int W, void* stream) {
  KAIR_CHECK_ARG(src && T && planes > 0 && H > 1 && W > 1 && W <= 2048 && H <= 2048, "usr_fft_rows: bad args");
  KAIR_CHECK_ARG(src_mode >= KAIR_USR_SRC_NCHW && src_mode <= KAIR_USR_SRC_NHWC, "usr_fft_rows: bad source mode");
  KAIR_CHECK_ARG(src_mode != KAIR_USR_SRC_PSF || (kh > 0 && kw > 0 && kh <= H && kw <= W), "usr_fft_rows: PSF size");
  KAIR_CHECK_ARG(src_mode != KAIR_USR_SRC_ZUP || (sf > 0 && H % sf == 0 && W % sf == 0), "usr_fft_rows: zero-upsample");
  KAIR_CHECK_ARG(src_mode != KAIR_USR_SRC_NHWC || (C > 0 && ld >= C), "usr_fft_rows: NHWC geometry");
  FftPlan pw;
  if (int rc = make_plan(W, &pw)) return rc;
  const int R = row_block(H, W);
  RowSrc s{src, src_mode, C > 0 ? C : 1, ld, kh, kw, sf};
  const size_t lds = (size_t)(W + 2 * R * (W + 1)) * sizeof(float2);
  KAIR_LAUNCH(fft_rows_fwd_kernel, dim3(H / R, planes), dim3(256), lds, (hipStream_t)stream, s, (float2*)T, H, W, R,
                     pw);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_usr_fft_cols(int mode, const void* T, void* T_out, const void* FB, const void* FBFy, void* FR,
                                 float* invW, const float* alpha, int alpha_stride, float* part, int planes, int C, int H,
                                 int W, int sf, void* stream) {
  KAIR_CHECK_ARG(T && planes > 0 && C > 0 && planes % C == 0 && sf > 0 && H % sf == 0 && W % sf == 0 && H > 1 &&
                     H <= 2048, "usr_fft_cols: bad geometry");
  KAIR_CHECK_ARG(mode >= KAIR_USR_COL_FB && mode <= KAIR_USR_COL_DATA_BWD, "usr_fft_cols: bad mode");
  KAIR_CHECK_ARG(mode == KAIR_USR_COL_DATA_BWD || T_out, "usr_fft_cols: null output");
  KAIR_CHECK_ARG(mode == KAIR_USR_COL_FB ? invW != nullptr : FB != nullptr, "usr_fft_cols: FB / invW");
  KAIR_CHECK_ARG(mode < KAIR_USR_COL_DATA_FWD || (FBFy && invW && alpha), "usr_fft_cols: data-step operands");
  KAIR_CHECK_ARG(mode != KAIR_USR_COL_DATA_BWD || (FR && part), "usr_fft_cols: backward needs FR and part");
  FftPlan ph;
  if (int rc = make_plan(H, &ph)) return rc;
  ColArgs a{(const float2*)T, (float2*)T_out, (const float2*)FB, (const float2*)FBFy, (float2*)FR, invW, alpha,
            alpha_stride, part, C, H, W, sf};
  const size_t lds = (size_t)(H + 2 * sf * (H + 1)) * sizeof(float2);
  KAIR_CHECK_ARG(lds <= 150 * 1024, "usr_fft_cols: sf %d x H %d lines exceed LDS", sf, H);
  KAIR_LAUNCH(fft_cols_kernel, dim3(W / sf, planes), dim3(256), lds, (hipStream_t)stream, a, mode, ph);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_usr_ifft_rows(const void* T, void* dst, int nhwc, int dst_dtype, int C, long ld, float scale,
                                  int planes, int H, int W, void* stream) {
  KAIR_CHECK_ARG(T && dst && planes > 0 && H > 1 && W > 1 && W <= 2048, "usr_ifft_rows: bad args");
  KAIR_CHECK_ARG(!nhwc || (C > 0 && ld >= C && planes % C == 0), "usr_ifft_rows: NHWC geometry");
  KAIR_CHECK_ARG(nhwc || dst_dtype == KAIR_F32, "usr_ifft_rows: NCHW output is fp32");
  FftPlan pw;
  if (int rc = make_plan(W, &pw)) return rc;
  const int R = row_block(H, W);
  const size_t lds = (size_t)(W + 2 * R * (W + 1)) * sizeof(float2);
  hipStream_t s = (hipStream_t)stream;
  const int Cc = C > 0 ? C : 1;
  if (dst_dtype == KAIR_BF16)
    KAIR_LAUNCH(fft_rows_inv_kernel<bf16>, dim3(H / R, planes), dim3(256), lds, s, (const float2*)T, (bf16*)dst, nhwc,
                       Cc, ld, scale, H, W, R, pw);
  else
    KAIR_LAUNCH(fft_rows_inv_kernel<float>, dim3(H / R, planes), dim3(256), lds, s, (const float2*)T, (float*)dst,
                       nhwc, Cc, ld, scale, H, W, R, pw);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_usr_seg_sum(const float* ws, int seglen, int nseg, float scale, float* out, int ostride,
                                int accumulate, void* stream) {
  KAIR_CHECK_ARG(ws && out && seglen > 0 && nseg > 0, "usr_seg_sum: bad args");
  KAIR_LAUNCH(seg_sum_kernel, dim3(nseg), dim3(256), 0, (hipStream_t)stream, ws, seglen, scale, out, ostride,
                     accumulate);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_usr_chan_sum(const float* x, long ld, int c, long HW, int B, float* ws, float* out, int ostride,
                                 int accumulate, void* stream) {
  KAIR_CHECK_ARG(x && ws && out && ld > c && c >= 0 && HW > 0 && B > 0, "usr_chan_sum: bad args");
  const int nchunk = KAIR_USR_CHAN_CHUNKS;
  hipStream_t s = (hipStream_t)stream;
  KAIR_LAUNCH(chan_sum_partial_kernel, dim3(nchunk, B), dim3(256), 0, s, x, ld, c, HW, nchunk, ws);
  KAIR_CHECK_LAUNCH();
  KAIR_LAUNCH(seg_sum_kernel, dim3(B), dim3(256), 0, s, ws, nchunk, 1.0f, out, ostride, accumulate);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_usr_upsample_nearest(const float* L, float* out, int planes, int h, int w, int sf, void* stream) {
  KAIR_CHECK_ARG(L && out && planes > 0 && h > 0 && w > 0 && sf > 0, "usr_upsample_nearest: bad args");
  const long total = (long)planes * h * sf * w * sf;
  KAIR_LAUNCH(upsample_nearest_kernel, dim3(nblk(total, 256)), dim3(256), 0, (hipStream_t)stream, L, out, h, w, sf,
                     total);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_usr_pack_input(const float* x, const float* beta, int beta_stride, void* out, int dtype, int ld,
                                   int B, int C, long HW, void* stream) {
  KAIR_CHECK_ARG(x && beta && out && ld > C && B > 0 && C > 0 && HW > 0, "usr_pack_input: bad args");
  const long npix = (long)B * HW;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == KAIR_BF16)
    KAIR_LAUNCH(pack_input_kernel<bf16>, dim3(nblk(npix, 256)), dim3(256), 0, s, x, beta, beta_stride, (bf16*)out, ld,
                       C, HW, npix);
  else
    KAIR_LAUNCH(pack_input_kernel<float>, dim3(nblk(npix, 256)), dim3(256), 0, s, x, beta, beta_stride, (float*)out,
                       ld, C, HW, npix);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_usr_pad(const void* src, void* dst, int dtype, int mode, int ldc, int nb, int H, int W, int Hp, int Wp,
                            void* stream) {
  KAIR_CHECK_ARG(src && dst && src != dst && nb > 0 && H > 0 && W > 0 && Hp >= H && Wp >= W, "usr_pad: bad args");
  KAIR_CHECK_ARG(mode >= KAIR_USR_PAD_REPLICATE && mode <= KAIR_USR_CROP_NCHW, "usr_pad: bad mode");
  KAIR_CHECK_ARG(mode == KAIR_USR_CROP_NCHW || ldc > 0, "usr_pad: channel stride");
  KAIR_CHECK_ARG(dtype == KAIR_F32 || (dtype == KAIR_BF16 && mode <= KAIR_USR_PAD_ZERO), "usr_pad: fold / crop are fp32");
  const long npix = (mode == KAIR_USR_PAD_FOLD || mode == KAIR_USR_CROP_NCHW) ? (long)nb * H * W : (long)nb * Hp * Wp;
  const long total = mode == KAIR_USR_CROP_NCHW ? npix : npix * ldc;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == KAIR_BF16)
    KAIR_LAUNCH(usr_pad_kernel<bf16>, dim3(nblk(total, 256)), dim3(256), 0, s, (const bf16*)src, (bf16*)dst, mode, ldc,
                       H, W, Hp, Wp, total);
  else
    KAIR_LAUNCH(usr_pad_kernel<float>, dim3(nblk(total, 256)), dim3(256), 0, s, (const float*)src, (float*)dst, mode,
                       ldc, H, W, Hp, Wp, total);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_hypanet_fwd(const float* sigma, float sf, const float* W1, const float* b1, const float* W2,
                                const float* b2, const float* W3, const float* b3, int hc, int no, int B, float* ab,
                                void* stream) {
  KAIR_CHECK_ARG(sigma && W1 && b1 && W2 && b2 && W3 && b3 && ab && hc > 0 && no > 0 && B > 0, "hypanet_fwd: bad args");
  const size_t lds = (size_t)B * (2 * hc + no) * sizeof(float);
  KAIR_CHECK_ARG(lds <= 64 * 1024, "hypanet_fwd: batch too large for one block");
  HypaParams P{W1, b1, W2, b2, W3, b3};
  KAIR_LAUNCH(hypanet_fwd_kernel, dim3(1), dim3(256), lds, (hipStream_t)stream, sigma, sf, P, hc, no, B, ab);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_hypanet_bwd(const float* sigma, float sf, const float* W1, const float* b1, const float* W2,
                                const float* b2, const float* W3, const float* b3, int hc, int no, int B, const float* gab,
                                float* gW1, float* gb1, float* gW2, float* gb2, float* gW3, float* gb3, int accumulate,
                                void* stream) {
  KAIR_CHECK_ARG(sigma && W1 && b1 && W2 && b2 && W3 && b3 && gab && gW1 && gb1 && gW2 && gb2 && gW3 && gb3 && hc > 0 &&
                     no > 0 && B > 0, "hypanet_bwd: bad args");
  const size_t lds = (size_t)B * (4 * hc + 2 * no) * sizeof(float);
  KAIR_CHECK_ARG(lds <= 64 * 1024, "hypanet_bwd: batch too large for one block");
  HypaParams P{W1, b1, W2, b2, W3, b3};
  HypaGrads G{gW1, gb1, gW2, gb2, gW3, gb3};
  KAIR_LAUNCH(hypanet_bwd_kernel, dim3(1), dim3(256), lds, (hipStream_t)stream, sigma, sf, P, hc, no, B, gab, G,
                     accumulate);
  KAIR_CHECK_LAUNCH();
  return 0;
}
