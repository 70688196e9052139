// Training-patch synthesis on the MI355X: the per-sample work of
//   DatasetSR.__getitem__    data/dataset_sr.py:35-92   (modcrop'd H, MATLAB-bicubic x1/sf L of the
//                                                        whole image, aligned random crop, 8-way augment)
//   DatasetDnCNN.__getitem__ data/dataset_dncnn.py:50-75 (random crop, 8-way augment, L = H + sigma N)
// for a whole batch in one launch, reading an image pool resident in HBM (fp32 NCHW, [0, 1]).
//
// Augment modes (utils_image.augment_img, utils_image.py:387-405) are the 8 dihedral maps of a
// square n x n patch: out(i, j) = src(si, sj) with (p, q) = mode&1 ? (j, i) : (i, j),
// si = mode&2 ? n-1-p : p, sj = mode&4 ? n-1-q : q  (checked mode by mode against the numpy code).
// Bicubic: separable taps per output row / column (weights and symmetric-reflected source indices
// from calculate_weights_indices, utils_image.py:880-932, built on the host), summed rows-first then
// columns as imresize does (utils_image.py:938-1005).  AWGN: Philox-4x32-10 keyed by (seed, step),
// counter = element index, Box-Muller -- no bitwise pin to torch's CPU generator is possible (or
// meaningful); tests check the noise statistically.
#include "common.h"

namespace {

KAIR_DEV void aug_src(int mode, int i, int j, int n, int& si, int& sj) {
  int p = i, q = j;
  if (mode & 1) { p = j; q = i; }
  si = (mode & 2) ? n - 1 - p : p;
  sj = (mode & 4) ? n - 1 - q : q;
}

// one thread per output element: [0, nH) -> H patch elements, [nH, nH + nL) -> L patch elements
__global__ __launch_bounds__(256) void synth_sr_kernel(const float* __restrict__ pool, int C, int Hs, int Ws,
                                                       const int4* __restrict__ par, int B, int PS, int sf,
                                                       const float* __restrict__ wh, const int* __restrict__ ih,
                                                       const float* __restrict__ ww, const int* __restrict__ iw, int P,
                                                       float* __restrict__ outH, float* __restrict__ outL) {
  const int LS = PS / sf;
  const long nH = (long)B * C * PS * PS, nL = (long)B * C * LS * LS;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nH + nL) return;
  if (t < nH) {
    const int j = (int)(t % PS);
    long r = t / PS;
    const int i = (int)(r % PS);
    r /= PS;
    const int c = (int)(r % C), b = (int)(r / C);
    const int4 pr = par[b];   // x = image, y = rnd_h (LQ rows), z = rnd_w, w = mode
    int si, sj;
    aug_src(pr.w, i, j, PS, si, sj);
    outH[t] = pool[(((long)pr.x * C + c) * Hs + (long)pr.y * sf + si) * Ws + (long)pr.z * sf + sj];
    return;
  }
  const long u = t - nH;
  const int j = (int)(u % LS);
  long r = u / LS;
  const int i = (int)(r % LS);
  r /= LS;
  const int c = (int)(r % C), b = (int)(r / C);
  const int4 pr = par[b];
  int si, sj;
  aug_src(pr.w, i, j, LS, si, sj);
  const int gy = pr.y + si, gx = pr.z + sj;   // row / column of the whole-image L
  const float* img = pool + ((long)pr.x * C + c) * Hs * Ws;
  float acc = 0.f;
  for (int bq = 0; bq < P; ++bq) {
    const float wb = ww[gx * P + bq];
    const int x = iw[gx * P + bq];
    float col = 0.f;
    for (int a = 0; a < P; ++a) col = fmaf(wh[gy * P + a], img[(long)ih[gy * P + a] * Ws + x], col);
    acc = fmaf(wb, col, acc);
  }
  outL[u] = acc;
}

// Separable form, one workgroup per (sample, channel, band of L source rows): the vertical bicubic
// pass for the band's L-rows over the source-column window the horizontal taps touch is staged in
// LDS once, then every L pixel of the band is P horizontal taps over it -- LS*W*P + LS*LS*P MACs
// instead of LS*LS*P*P, with the same summation order as synth_sr_kernel (each vertical sum over a,
// then over bq), so the output is bitwise the same.  Bands split each sample's work over several
// workgroups (a 4-patch batch would otherwise run on 12 CUs); each also writes its share of the
// (augmented) H crop.  Outputs are addressed through the inverse augment map (dihedral: an
// involution up to the transpose), so a band writes exactly the L pixels whose source row it holds.
__global__ __launch_bounds__(256) void synth_sr_sep_kernel(const float* __restrict__ pool, int C, int Hs, int Ws,
                                                           const int4* __restrict__ par, int PS, int sf,
                                                           const float* __restrict__ wh, const int* __restrict__ ih,
                                                           const float* __restrict__ ww, const int* __restrict__ iw, int P,
                                                           int Wmax, int nband, float* __restrict__ outH,
                                                           float* __restrict__ outL) {
  extern __shared__ float sV[];   // [rows of the band][Wmax]
  __shared__ int sLo, sHi;
  const int tid = threadIdx.x;
  const int sc = blockIdx.x / nband, band = blockIdx.x - sc * nband;
  const int b = sc / C, c = sc - (sc / C) * C;
  const int4 pr = par[b];   // x = image, y = rnd_h (LQ rows), z = rnd_w, w = mode
  const int LS = PS / sf;
  const int rpb = (LS + nband - 1) / nband, r0 = band * rpb, r1 = min(LS, r0 + rpb), nr = r1 - r0;
  const float* img = pool + ((long)pr.x * C + c) * Hs * Ws;
  // this band's share of the H crop
  float* oH = outH + (long)(b * C + c) * PS * PS;
  const int hpb = (PS * PS + nband - 1) / nband, h0 = band * hpb, h1 = min(PS * PS, h0 + hpb);
  for (int t = h0 + tid; t < h1; t += 256) {
    const int i = t / PS, j = t - (t / PS) * PS;
    int si, sj;
    aug_src(pr.w, i, j, PS, si, sj);
    oH[t] = img[(long)(pr.y * sf + si) * Ws + pr.z * sf + sj];
  }
  if (nr <= 0) return;
  // source-column window of the horizontal taps of L columns pr.z .. pr.z + LS - 1
  if (tid == 0) { sLo = Ws; sHi = 0; }
  __syncthreads();
  int lo = Ws, hi = 0;
  for (int t = tid; t < LS * P; t += 256) {
    const int x = iw[(pr.z + t / P) * P + t - (t / P) * P];
    lo = min(lo, x);
    hi = max(hi, x + 1);
  }
  atomicMin(&sLo, lo);
  atomicMax(&sHi, hi);
  __syncthreads();
  lo = sLo;
  // W <= PS + P + 2 sf <= Wmax by the tap geometry (reflected indices fold inward); clamped anyway
  const int W = min(sHi - lo, Wmax);
  // vertical pass: V[r - r0][x - lo] = sum_a wh[gy][a] * img[ih[gy][a]][x], gy = pr.y + r
  for (int t = tid; t < nr * W; t += 256) {
    const int r = t / W, xo = t - (t / W) * W, gy = pr.y + r0 + r;
    float acc = 0.f;
    for (int a = 0; a < P; ++a) acc = fmaf(wh[gy * P + a], img[(long)ih[gy * P + a] * Ws + lo + xo], acc);
    sV[r * Wmax + xo] = acc;
  }
  __syncthreads();
  // horizontal pass for source rows si in [r0, r1); output pixel through the inverse augment map
  float* oL = outL + (long)(b * C + c) * LS * LS;
  for (int t = tid; t < nr * LS; t += 256) {
    const int si = r0 + t / LS, sj = t - (t / LS) * LS;
    const int p = (pr.w & 2) ? LS - 1 - si : si, q = (pr.w & 4) ? LS - 1 - sj : sj;
    const int i = (pr.w & 1) ? q : p, j = (pr.w & 1) ? p : q;
    const int gx = pr.z + sj;
    float acc = 0.f;
    for (int bq = 0; bq < P; ++bq) acc = fmaf(ww[gx * P + bq], sV[(si - r0) * Wmax + iw[gx * P + bq] - lo], acc);
    oL[i * LS + j] = acc;
  }
}

// Philox-4x32-10 (Salmon et al., SC'11)
KAIR_DEV uint4 philox(uint4 ctr, uint2 key) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * ctr.x;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * ctr.z;
    const unsigned h0 = (unsigned)(p0 >> 32), l0 = (unsigned)p0, h1 = (unsigned)(p1 >> 32), l1 = (unsigned)p1;
    ctr = make_uint4(h1 ^ ctr.y ^ key.x, l1, h0 ^ ctr.w ^ key.y, l0);
    key.x += 0x9E3779B9u;
    key.y += 0xBB67AE85u;
  }
  return ctr;
}

KAIR_DEV float normal_at(unsigned long long idx, unsigned long long seed, unsigned long long step) {
  const uint4 r = philox(make_uint4((unsigned)idx, (unsigned)(idx >> 32), (unsigned)step, (unsigned)(step >> 32)),
                         make_uint2((unsigned)seed, (unsigned)(seed >> 32)));
  const float u1 = ((r.x >> 8) + 1) * (1.0f / 16777216.0f);   // (0, 1]
  const float u2 = (r.y >> 8) * (1.0f / 16777216.0f);         // [0, 1)
  return sqrtf(-2.f * __logf(u1)) * __cosf(6.283185307179586f * u2);
}

// H = aug(crop(pool)); L = H + sigma * N(0, 1)   (sigma already divided by 255)
__global__ __launch_bounds__(256) void synth_dn_kernel(const float* __restrict__ pool, int C, int Hs, int Ws,
                                                       const int4* __restrict__ par, int B, int PS, float sigma,
                                                       unsigned long long seed, unsigned long long step,
                                                       float* __restrict__ outH, float* __restrict__ outL) {
  const long n = (long)B * C * PS * PS;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int j = (int)(t % PS);
  long r = t / PS;
  const int i = (int)(r % PS);
  r /= PS;
  const int c = (int)(r % C), b = (int)(r / C);
  const int4 pr = par[b];   // x = image, y = rnd_h, z = rnd_w, w = mode
  int si, sj;
  aug_src(pr.w, i, j, PS, si, sj);
  const float h = pool[(((long)pr.x * C + c) * Hs + pr.y + si) * Ws + pr.z + sj];
  outH[t] = h;
  outL[t] = h + sigma * normal_at((unsigned long long)t, seed, step);
}

long nblocks(long n) { return (n + 255) / 256; }

}  // namespace

extern "C" int kair_synth_sr(const float* pool, int C, int Hs, int Ws, const int* params, int B, int PS, int sf,
                             const float* wh, const int* ih, const float* ww, const int* iw, int P, float* outH,
                             float* outL, void* stream) {
  KAIR_CHECK_ARG(pool && params && wh && ih && ww && iw && outH && outL, "synth_sr: null pointer");
  KAIR_CHECK_ARG(C > 0 && Hs > 0 && Ws > 0 && B > 0 && sf > 0 && PS > 0 && PS % sf == 0 && P > 0,
                 "synth_sr: bad sizes (C %d, %dx%d, B %d, PS %d, sf %d, P %d)", C, Hs, Ws, B, PS, sf, P);
  KAIR_CHECK_ARG(PS <= Hs && PS <= Ws, "synth_sr: pool images smaller than the patch");
  // separable kernel when the staged vertical pass fits in LDS: the horizontal taps of LS L columns
  // span at most PS + 2P source columns (+ 2 sf of rounding slack)
  const int LS = PS / sf;
  const int Wmax = (PS + 2 * P + 2 * sf) < Ws ? (PS + 2 * P + 2 * sf) : Ws;
  // bands of L rows: ~2048 workgroups over the batch (B = 4: one L row per band)
  int nband = 2048 / (B * C);
  nband = nband < 1 ? 1 : (nband > LS ? LS : nband);
  const int rpb = (LS + nband - 1) / nband;
  const size_t lds = (size_t)rpb * Wmax * sizeof(float);
  if (lds <= 60 * 1024) {
    KAIR_LAUNCH(synth_sr_sep_kernel, dim3((unsigned)(B * C * nband)), dim3(256), lds, (hipStream_t)stream, pool, C,
                       Hs, Ws, (const int4*)params, PS, sf, wh, ih, ww, iw, P, Wmax, nband, outH, outL);
  } else {
    const long total = (long)B * C * PS * PS + (long)B * C * LS * LS;
    KAIR_LAUNCH(synth_sr_kernel, dim3((unsigned)nblocks(total)), dim3(256), 0, (hipStream_t)stream, pool, C, Hs, Ws,
                       (const int4*)params, B, PS, sf, wh, ih, ww, iw, P, outH, outL);
  }
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_synth_dn(const float* pool, int C, int Hs, int Ws, const int* params, int B, int PS, float sigma,
                             unsigned long long seed, unsigned long long step, float* outH, float* outL, void* stream) {
  KAIR_CHECK_ARG(pool && params && outH && outL, "synth_dn: null pointer");
  KAIR_CHECK_ARG(C > 0 && B > 0 && PS > 0 && PS <= Hs && PS <= Ws, "synth_dn: bad sizes");
  const long total = (long)B * C * PS * PS;
  KAIR_LAUNCH(synth_dn_kernel, dim3((unsigned)nblocks(total)), dim3(256), 0, (hipStream_t)stream, pool, C, Hs, Ws,
                     (const int4*)params, B, PS, sigma, seed, step, outH, outL);
  KAIR_CHECK_LAUNCH();
  return 0;
}
