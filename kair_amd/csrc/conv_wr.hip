// 3x3 convolution (stride 1, pad 1) for gfx950 with the weights streamed straight into registers:
// the RSTB convolutions of SwinIR (network_swinir.py:263-279 RSTB.conv, 3x3 180 -> 180 at the LQ size)
// and their input gradients, as an implicit GEMM  D[n][p] = sum_k W[n][k] X^T[k][p],  k = tap * C + c.
//
// Why not the LDS-ring halo kernel (gemm.hip conv3x3_halo_kernel): that one stages every 64-wide weight
// chunk through LDS for all eight waves of a 512-thread workgroup, so each chunk costs a workgroup
// barrier and an LDS-DMA round trip two chunks ahead; at two waves per SIMD both waves arrive at the
// barrier together and the chunk's LDS reads and DMA waits are exposed (measured: 22-25 % of the MFMA
// peak, 43 % of the wave cycles parked in s_waitcnt / s_barrier; profiles/r04_conv_micro.txt).
//
// Here one 256-thread workgroup per CU runs ONE wave per SIMD.  The input tile's halo lives in LDS for
// the whole tile (loaded once; with split activations BOTH the hi and the lo halves, 2 x 80 KB), and
// each wave owns 48 output channels of the tile: its weight fragments come from global memory (pack
// kind 15 / 16: 16x16x32 fragment order, one coalesced 1 KiB wave load per fragment) into a ring of
// registers three k-steps deep, its activation fragments from the halo one k-step ahead.  The k-loop
// has no barrier and no LDS traffic but the operand reads; each wave's only waits are its own loads.
//
//   split (fp32 image, kair_operand.a_split semantics): 3 products per k-step  hi.W_hi + hi.W_lo +
//          lo.W_hi  (lo = bf16(x - bf16(x)) formed while the halo is filled), 96-pixel tiles;
//   plain (bf16 image, e.g. the input gradient with flipped taps): 1 product, 144-pixel tiles.
// Epilogue per lane: 4 consecutive output channels of one pixel (bias, fp32 residual, fp32 / bf16
// rows).  The tile's own pixels can be copied out as bf16 rows (a_copy, + a ones column) for the
// weight gradient, as the halo kernel does.
#include "common.h"

namespace {

constexpr int WR_WAVES = 4;          // one per SIMD
constexpr int WR_NT = 64 * WR_WAVES;
// k-steps of weight fragments in flight: 3 where a k-step is 18+ MFMAs per wave, 9 for the narrow
// (RN = 1) forms whose k-step is 6-18 MFMAs (~100-300 cycles: three steps would not cover an L2 hit)
// (6 for the split N <= 64 form: 18 MFMAs per step, and the registers of 9 spill)
template <int RN, bool SPLIT> struct WrPD {
  static constexpr int PD = RN != 1 ? 3 : SPLIT ? 6 : 9, UNR = RN == 1 && !SPLIT ? 18 : 6;
};

struct ConvWrArgs {
  const void* x; long ldx;           // NHWC image rows: fp32 (split) or bf16
  const bf16* w;                     // kind 15 (split: [Np/16][KS][2][64][8]) or 16 ([Np/16][KS][64][8])
  const float* bias;                 // [>= N] or null
  const float* resid; long ldr;      // fp32 rows or null
  void* out; int odt; long ldo;
  bf16* acopy; long ldac; int acones;
  bf16* out_lo;                      // pair output: bf16(v - bf16(v)) at the same offsets (bf16 out only)
  int ps_r;                          // > 0: PixelShuffle(ps_r) sub-pixel-major output (n = (i r + j) nf + c)
  int act; float slope;              // KAIR_ACT_LEAKY: LeakyReLU(slope) before the store (no residual)
  const bf16* gate; long ldg;        // v *= (gate[m][n] > 0 ? 1 : slope): LeakyReLU' of a stored activation (rows)
  int psH, psW;                      // EM 2: the pre-shuffle grid (H / r, W / r) of the PixelUnshuffle store
  int B, H, W, C, N, flip;
  long tilesM;
  FDiv fc8, fhwd;                    // C / 8 and the halo row width (magic-number divisions)
};

// bf16 elements of one halo image: split -- two images (hi, lo) of 40,000 (96-pixel tiles); plain -- one
// of 80,000 (160,000 B: the whole LDS)
template <bool SPLIT> struct WrGeom {
  static constexpr int HALO = SPLIT ? 40000 : 80000;
};

// SPLIT with an fp32 image: lo formed in the halo fill; SPLIT with a bf16 image ("pair"): the image rows
// are [hi | lo] halves of C channels each (the split tail's activations), read into the two halos.
// RN: 16-wide output fragments per wave (1: N <= 64, 3: N <= 192, 4: N <= 256).  EM 1: PixelShuffle
// sub-pixel-major store (+ the lo plane of a bf16 pair output); EM 2: its inverse, PixelUnshuffle (an
// upsampling conv's input gradient into the previous conv's pre-shuffle rows).
template <typename TX, bool SPLIT, int BM, bool RESID, int RN, int EM>
__global__ __launch_bounds__(WR_NT, 1) void conv3x3_wr_kernel(const ConvWrArgs a) {
  constexpr bool PAIR = SPLIT && sizeof(TX) == 2;
  constexpr int RM = BM / 16;
  constexpr int HALO = WrGeom<SPLIT>::HALO;
  constexpr int NB = SPLIT ? 2 : 1;                         // weight fragments per (rn, k-step)
  __shared__ __attribute__((aligned(16))) bf16 sH[SPLIT ? 2 * HALO : HALO];
  bf16* const sLo = sH + (SPLIT ? HALO : 0);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int H = a.H, W = a.W, C = a.C;
  // CGP 2 (192-pixel tiles, plain): the channels in two halves, one halo pass each, accumulating
  constexpr int CGP = BM == 192 ? 2 : 1;
  static_assert(CGP == 1 || (!SPLIT && !RESID), "channel-half passes: plain image, no residual");
  const int CH = C / CGP;
  const int XW = W < BM ? W : BM, RPT = BM / XW, HWD = XW + 2, HR = RPT + 2, PS = CH + 8;
  const int c8n = CH / 8, halo_pieces = HR * HWD * c8n;
  const int cps = C / 32, cpsP = CH / 32, KSP = 9 * cpsP, KS = 9 * cps;   // k-steps of 32: per pass, all
  int pass = 0;
  // a pass's k-step sl -> the weight's k-step (k = tap * C + c)
  auto wstep = [&](int sl) { const int tap = sl / cpsP; return tap * cps + pass * cpsP + (sl - tap * cpsP); };
  int hb[RM];
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    const int p = i * 16 + fr;
    const int ry = p / XW, rx = p - (p / XW) * XW;
    hb[i] = ((ry + 1) * HWD + rx + 1) * PS + fq * 8;
  }
  // this wave's weight fragments: n blocks 3 w + rn, k-step s: one 1 KiB wave load per fragment
  const bf16* wb = a.w + ((long)(RN * wave) * KS * NB) * 512 + lane * 8;
  auto wfrag = [&](int rn, int s, int half) {
    return *(const bf16x8*)(wb + (((long)rn * KS + s) * NB + half) * 512);
  };
  float4 bias4[RN];
#pragma unroll
  for (int rn = 0; rn < RN; ++rn) {
    const int n = 16 * RN * wave + 16 * rn + 4 * fq;
    bias4[rn] = a.bias && n < a.N ? *(const float4*)(a.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  }

  constexpr int PD = WrPD<RN, SPLIT>::PD, UNR = WrPD<RN, SPLIT>::UNR;   // UNR: lcm(PD, 2); KS = 18 C / 64 is a multiple
  bf16x8 rb[PD][RN][NB];           // weight ring
  auto issue_w = [&](int slot, int s) {
#pragma unroll
    for (int rn = 0; rn < RN; ++rn)
#pragma unroll
      for (int h = 0; h < NB; ++h) rb[slot][rn][h] = wfrag(rn, s, h);
  };
  bf16x8 ra[2][RM][NB];            // activation fragments, one k-step ahead
  auto read_a = [&](int buf, int s) {
    const int tap = s / cpsP, c0 = (s - tap * cpsP) * 32;
    int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
    if (a.flip) { dy = -dy; dx = -dx; }
    const int off = (dy * HWD + dx) * PS + c0;
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      ra[buf][i][0] = *(const bf16x8*)(sH + hb[i] + off);
      if constexpr (SPLIT) ra[buf][i][1] = *(const bf16x8*)(sLo + hb[i] + off);
    }
  };

  const long tiles = a.tilesM;
  for (long t = blockIdx.x; t < tiles; t += gridDim.x) {
    const long p0 = t * BM;
    const int b = (int)(p0 / ((long)H * W));
    const int rem = (int)(p0 - (long)b * H * W);
    const int y0 = rem / W, x0 = rem - (rem / W) * W;
    f32x4 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int rn = 0; rn < RN; ++rn) acc[i][rn] = f32x4{0.f, 0.f, 0.f, 0.f};
    float4 ex[RESID ? RM : 1][RN];
    auto load_resid = [&]() {
      if constexpr (RESID) {
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int rn = 0; rn < RN; ++rn) {
            const long m = p0 + i * 16 + fr;
            const int n = 16 * RN * wave + 16 * rn + 4 * fq;
            ex[i][rn] = *(const float4*)(a.resid + m * a.ldr + (n < a.N ? n : 0));
          }
      }
    };
    for (pass = 0; pass < CGP; ++pass) {
    // the first k-steps' weights in flight under the halo fill
#pragma unroll
    for (int u = 0; u < PD; ++u) issue_w(u, wstep(u));
    __syncthreads();   // every wave is done with the previous tile's (or pass's) halo
    {
      // pieces per thread in one batch of loads (all issued, then landed, then written): the whole
      // halo at once where the registers allow it -- each batch is one exposed memory latency
      constexpr int HP = PAIR ? 5 : SPLIT ? 10 : (sizeof(TX) == 4 ? 12 : 16);
      const int per = (halo_pieces + WR_NT - 1) / WR_NT;
      for (int h0 = 0; h0 < per; h0 += HP) {
        uint4 v0[HP], v1[HP];
        bool okv[HP];
#pragma unroll
        for (int i = 0; i < HP; ++i) {
          const int idx = tid + WR_NT * (h0 + i);
          const int pix = fdiv(idx, a.fc8), c8 = idx - pix * c8n;
          const int hr = fdiv(pix, a.fhwd), hc = pix - hr * HWD;
          const int y = y0 - 1 + hr, x = x0 - 1 + hc;
          okv[i] = idx < halo_pieces && y >= 0 && y < H && x >= 0 && x < W;
          const long src = okv[i] ? ((long)(b * H + y) * W + x) * a.ldx + pass * CH + c8 * 8 : 0;
          if constexpr (sizeof(TX) == 4) {
            v0[i] = *(const uint4*)((const float*)a.x + src);
            v1[i] = *(const uint4*)((const float*)a.x + src + 4);
          } else {
            v0[i] = *(const uint4*)((const bf16*)a.x + src);
            if constexpr (PAIR) v1[i] = *(const uint4*)((const bf16*)a.x + src + C);
          }
        }
#pragma unroll
        for (int i = 0; i < HP; ++i) {
          const int idx = tid + WR_NT * (h0 + i);
          if (idx >= halo_pieces) continue;
          const int pix = fdiv(idx, a.fc8), c8 = idx - pix * c8n;
          uint4 qh, ql = make_uint4(0, 0, 0, 0);
          if constexpr (sizeof(TX) == 4) {
            const float4 u = __builtin_bit_cast(float4, v0[i]), v = __builtin_bit_cast(float4, v1[i]);
            const float f[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
            bf16x8 hh, ll;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              hh[e] = (bf16)f[e];
              if constexpr (SPLIT) ll[e] = (bf16)(f[e] - (float)hh[e]);
            }
            qh = __builtin_bit_cast(uint4, hh);
            if constexpr (SPLIT) ql = __builtin_bit_cast(uint4, ll);
          } else {
            qh = v0[i];
            if constexpr (PAIR) ql = v1[i];
          }
          if (!okv[i]) qh = ql = make_uint4(0, 0, 0, 0);
          *(uint4*)(sH + pix * PS + c8 * 8) = qh;
          if constexpr (SPLIT) *(uint4*)(sLo + pix * PS + c8 * 8) = ql;
          if (a.acopy) {   // the tile's own pixels: bf16 copy (+ ones column) for the weight gradient
            const int hr = fdiv(pix, a.fhwd), hc = pix - hr * HWD;
            if (hr >= 1 && hr <= RPT && hc >= 1 && hc <= XW) {
              uint4 qc = qh;
              const int oc = a.acones - c8 * 8;
              if ((unsigned)oc < 8u) {
                bf16x8 v8 = __builtin_bit_cast(bf16x8, qc);
                v8[oc] = (bf16)1.f;
                qc = __builtin_bit_cast(uint4, v8);
              }
              const long px = (long)(b * H + y0 + hr - 1) * W + x0 + hc - 1;
              *(uint4*)(a.acopy + px * a.ldac + c8 * 8) = qc;
            }
          }
        }
      }
    }
    __syncthreads();   // halo visible

    read_a(0, 0);
    // k-loop, unrolled by UNR (the weight ring is PD deep, the activation buffers 2): KSP % UNR == 0.
    // Every load is unconditional (the last steps re-read step KSP - 1): a load on only some paths makes
    // the compiler's wait at the merge the minimum over the paths (vmcnt / lgkmcnt 0 every step).
    auto step = [&](int u, int s, bool tail) {
      const int ab = u & 1, ws = u % PD;
      read_a(ab ^ 1, s + 1 < KSP ? s + 1 : KSP - 1);
      if (RESID && tail && u == UNR - 3) load_resid();
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int rn = 0; rn < RN; ++rn) {
          acc[i][rn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rb[ws][rn][0], ra[ab][i][0], acc[i][rn], 0, 0, 0);
          if constexpr (SPLIT) {
            acc[i][rn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rb[ws][rn][1], ra[ab][i][0], acc[i][rn], 0, 0, 0);
            acc[i][rn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rb[ws][rn][0], ra[ab][i][1], acc[i][rn], 0, 0, 0);
          }
        }
      issue_w(ws, wstep(s + PD < KSP ? s + PD : KSP - 1));
    };
    for (int s0 = 0; s0 < KSP - UNR; s0 += UNR) {
#pragma unroll
      for (int u = 0; u < UNR; ++u) step(u, s0 + u, false);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) step(u, KSP - UNR + u, CGP == 1 || pass == CGP - 1);
    }   // pass
    // epilogue: 4 consecutive channels of one pixel per lane
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int rn = 0; rn < RN; ++rn) {
        const long m = p0 + i * 16 + fr;
        const int n = 16 * RN * wave + 16 * rn + 4 * fq;
        if (n >= a.N) continue;
        const float4 bb = bias4[rn];
        float v[4] = {acc[i][rn][0] + bb.x, acc[i][rn][1] + bb.y, acc[i][rn][2] + bb.z, acc[i][rn][3] + bb.w};
        if constexpr (RESID) {
          v[0] += ex[i][rn].x; v[1] += ex[i][rn].y; v[2] += ex[i][rn].z; v[3] += ex[i][rn].w;
        }
        if (a.act == KAIR_ACT_LEAKY) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = v[q] > 0.f ? v[q] : v[q] * a.slope;
        }
        if (a.gate) {
          const bf16x4 gv = *(const bf16x4*)(a.gate + m * a.ldg + n);
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] *= (float)gv[q] > 0.f ? 1.f : a.slope;
        }
        long o = m * a.ldo + n;
        if constexpr (EM == 1) {   // sub-pixel-major columns: n = (i r + j) nf + c -> pixel (y r + i, x r + j)
          const int r = a.ps_r, nf = a.N / (r * r);
          const int bi = (int)(m / ((long)H * W)), pp = (int)(m - (long)bi * H * W), yy = pp / W, xx = pp - yy * W;
          const int sp = n / nf, cc = n - sp * nf, ii = sp / r, jj = sp - ii * r;
          o = (((long)bi * H * r + (long)yy * r + ii) * ((long)W * r) + (long)xx * r + jj) * a.ldo + cc;
        } else if constexpr (EM == 2) {   // pixel (y, x) -> pre-shuffle row (y / r, x / r), column (i r + j) N + n
          const int r = a.ps_r;
          const int bi = (int)(m / ((long)H * W)), pp = (int)(m - (long)bi * H * W), yy = pp / W, xx = pp - yy * W;
          const int yl = yy / r, xl = xx / r;
          o = (((long)bi * a.psH + yl) * a.psW + xl) * a.ldo + ((yy - yl * r) * r + (xx - xl * r)) * a.N + n;
        }
        if (a.odt == KAIR_BF16) {
          const bf16x4 hv = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          *(bf16x4*)((bf16*)a.out + o) = hv;
          if (a.out_lo)
            *(bf16x4*)(a.out_lo + o) = bf16x4{(bf16)(v[0] - (float)hv[0]), (bf16)(v[1] - (float)hv[1]),
                                              (bf16)(v[2] - (float)hv[2]), (bf16)(v[3] - (float)hv[3])};
        } else {
          *(float4*)((float*)a.out + o) = make_float4(v[0], v[1], v[2], v[3]);
        }
      }
  }
}

int wr_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}

// geometry of a BM-pixel tile: whole rows of width W <= BM, or BM-pixel pieces of wider rows
bool wr_geometry(int BM, int halo, long M, int H, int W, int C) {
  if (W <= 0 || H <= 0 || M <= 0) return false;
  if (W <= BM) {
    if (BM % W != 0 || H % (BM / W) != 0) return false;
  } else if (W % BM != 0) {
    return false;
  }
  const int XW = W < BM ? W : BM, RPT = BM / XW;
  return (long)(RPT + 2) * (XW + 2) * (C + 8) <= halo && M % BM == 0 && M % ((long)H * W) == 0;
}

}  // namespace

/* The tile (pixels) kair_conv3x3_wr uses for this shape, or 0 when the shape is not supported.  split:
 * two halos (split activations, fp32 image, or a bf16 [hi | lo] pair image of C channels per half). */
extern "C" int kair_conv3x3_wr_tile(int split, int B, int H, int W, int C, int N) {
  const long M = (long)B * H * W;
  if (C <= 0 || C > 256 || C % 64 != 0 || N <= 0 || N > 256 || N % 4 != 0) return 0;
  if (split && C > 192) return 0;
  if (!split && N > 192) return 0;
  // the largest tile that still gives >= 3/4 of a workgroup per CU, else the smallest that fits: at
  // B = 4 (M = 9,216) 48-pixel tiles put 192 workgroups on the chip instead of 96 / 64
  // plain C = 256 (the upsampling convs' input gradients): 192-pixel tiles in two channel-half passes
  // first (the 256-channel halo of a 96-pixel tile re-reads every input row three times)
  static const int cand_split[] = {96, 48}, cand_plain[] = {144, 96, 48}, cand_256[] = {192, 96, 48};
  const int* cand = split ? cand_split : C == 256 ? cand_256 : cand_plain;
  const int nc = split ? 2 : 3;
  const long want = 3L * wr_num_cus() / 4;
  int best = 0;
  for (int i = 0; i < nc; ++i) {
    const int bm = cand[i];
    if (!(split ? wr_geometry(bm, WrGeom<true>::HALO, M, H, W, C)
                : wr_geometry(bm, WrGeom<false>::HALO, M, H, W, bm == 192 ? C / 2 : C)))
      continue;
    // (only the N <= 64 input-gradient forms have the two-pass tile, and it pays only where a 96-pixel
    // tile is a single image row: W >= 96 -- at 48^2 it measured 68 -> 90 us)
    if (bm == 192 && (N > 64 || W < 96)) continue;
    best = bm;
    if (M / bm >= want) return bm;
  }
  return best;
}

#define KAIR_WR(TXV, SPV, BMV, RV, RNV, EMV) \
  KAIR_LAUNCH((conv3x3_wr_kernel<TXV, SPV, BMV, RV, RNV, EMV>), dim3(grid), dim3(WR_NT), 0, s, a)

extern "C" int kair_conv3x3_wr_ex(const void* x, int x_dtype, long ldx, int split, int flip, const void* w, int n_blocks,
                                  const float* bias, const float* resid, long ldr, void* out, int out_dtype, long ldo,
                                  void* out_lo, int ps_r, int act, float slope, const void* gate, long ldg, void* acopy,
                                  long ldac, int acones, int B, int H, int W, int C, int N, void* stream) {
  KAIR_CHECK_ARG(x && w && out && B > 0, "conv3x3_wr: null operand");
  KAIR_CHECK_ARG(x_dtype == KAIR_F32 || x_dtype == KAIR_BF16, "conv3x3_wr: image dtype");
  KAIR_CHECK_ARG(out_dtype == KAIR_F32 || out_dtype == KAIR_BF16, "conv3x3_wr: output dtype");
  const bool pair = split && x_dtype == KAIR_BF16;
  int BM = kair_conv3x3_wr_tile(split, B, H, W, C, N);
  KAIR_CHECK_ARG(BM > 0, "conv3x3_wr: unsupported geometry (B %d, H %d, W %d, C %d, N %d)", B, H, W, C, N);
  if (BM == 144 && resid) {   // the 144-pixel plain form has no residual instantiation (its registers spill)
    const long Mg = (long)B * H * W;
    BM = wr_geometry(96, WrGeom<false>::HALO, Mg, H, W, C) ? 96 : wr_geometry(48, WrGeom<false>::HALO, Mg, H, W, C) ? 48 : 0;
    KAIR_CHECK_ARG(BM > 0, "conv3x3_wr: no tile for a plain conv with a residual at this geometry");
  }
  const int RN = N > 192 ? 4 : N > 64 ? 3 : 1;
  KAIR_CHECK_ARG(n_blocks == 4 * RN, "conv3x3_wr: the packed weight needs %d output rows (%d blocks of 16), got %d blocks",
                 64 * RN, 4 * RN, n_blocks);
  KAIR_CHECK_ARG(ldx >= (pair ? 2 * C : C) && ldx % (x_dtype == KAIR_F32 ? 4 : 8) == 0 && ((uintptr_t)x & 15) == 0 &&
                     ((uintptr_t)w & 15) == 0,
                 "conv3x3_wr: image rows 16-byte aligned, ldx >= C (2 C for a [hi | lo] pair)");
  // ps_r > 0: PixelShuffle store of a split / pair conv; ps_r < 0: PixelUnshuffle(-ps_r) store of a plain one
  const int pr = ps_r < 0 ? -ps_r : ps_r;
  KAIR_CHECK_ARG(ps_r <= 0 || (N % (pr * pr) == 0 && (N / (pr * pr)) % 4 == 0 && !resid),
                 "conv3x3_wr: PixelShuffle output needs N %% r^2 == 0, N / r^2 %% 4 == 0 and no residual");
  KAIR_CHECK_ARG(ps_r >= 0 || (H % pr == 0 && W % pr == 0 && !resid && ldo >= (long)N * pr * pr),
                 "conv3x3_wr: PixelUnshuffle output needs H, W multiples of r, ldo >= N r^2, no residual");
  KAIR_CHECK_ARG(ldo >= (ps_r > 0 ? N / (pr * pr) : N) && ldo % 4 == 0 && ((uintptr_t)out & 15) == 0, "conv3x3_wr: output rows");
  KAIR_CHECK_ARG(!gate || (ps_r == 0 && !resid && ldg >= N && ldg % 4 == 0 && ((uintptr_t)gate & 7) == 0),
                 "conv3x3_wr: a gate needs a row output, no residual, 8-byte aligned bf16 rows");
  KAIR_CHECK_ARG(!out_lo || (out_dtype == KAIR_BF16 && ((uintptr_t)out_lo & 7) == 0), "conv3x3_wr: out_lo needs a bf16 output");
  KAIR_CHECK_ARG(!resid || (ldr >= N && ldr % 4 == 0 && ((uintptr_t)resid & 15) == 0), "conv3x3_wr: residual rows");
  KAIR_CHECK_ARG(!bias || ((uintptr_t)bias & 15) == 0, "conv3x3_wr: bias alignment");
  KAIR_CHECK_ARG(!acopy || (!pair && ldac >= C && ldac % 8 == 0 && ((uintptr_t)acopy & 15) == 0), "conv3x3_wr: a_copy rows");
  const long M = (long)B * H * W;
  KAIR_CHECK_ARG(M * (ldx > ldo ? ldx : ldo) * (ps_r ? ps_r * ps_r : 1) < (1L << 31), "conv3x3_wr: operands past 2^31 elements");
  ConvWrArgs a;
  a.x = x; a.ldx = ldx; a.w = (const bf16*)w; a.bias = bias; a.resid = resid; a.ldr = ldr;
  a.out = out; a.odt = out_dtype; a.ldo = ldo; a.acopy = (bf16*)acopy; a.ldac = ldac; a.acones = acopy ? acones : -1;
  a.out_lo = (bf16*)out_lo; a.ps_r = pr;
  a.gate = (const bf16*)gate; a.ldg = ldg;
  a.psH = pr ? H / pr : 0; a.psW = pr ? W / pr : 0;
  KAIR_CHECK_ARG(act == KAIR_ACT_NONE || (act == KAIR_ACT_LEAKY && !resid && !gate),
                 "conv3x3_wr: act none, or LeakyReLU without residual / gate");
  a.act = act; a.slope = slope;
  a.B = B; a.H = H; a.W = W; a.C = C; a.N = N; a.flip = flip;
  a.tilesM = M / BM;
  a.fc8 = make_fdiv(C / (BM == 192 ? 2 : 1) / 8);
  a.fhwd = make_fdiv((W < BM ? W : BM) + 2);
  const int ncu = wr_num_cus();
  const int grid = (int)(a.tilesM < ncu ? a.tilesM : ncu);
  hipStream_t s = (hipStream_t)stream;
  const bool rs = resid != nullptr;
#define KAIR_WR3(TXV, SPV, RV, RNV, EMV)                                                   \
  do {                                                                                     \
    if (BM == 48) KAIR_WR(TXV, SPV, 48, RV, RNV, EMV);                                     \
    else if (BM == 96) KAIR_WR(TXV, SPV, 96, RV, RNV, EMV);                                \
    else if constexpr (!SPV && !RV) KAIR_WR(TXV, SPV, 144, RV, RNV, EMV);                  \
  } while (0)
  if (pair) {   // the SwinIR x4 upsampling convs: [hi | lo] pair in, PixelShuffle [hi | lo] pair out
    KAIR_CHECK_ARG(RN == 4 && ps_r > 0 && !rs, "conv3x3_wr: the pair form is built for N in (192, 256] with a PixelShuffle store");
    KAIR_WR3(bf16, true, false, 4, 1);
  } else if (RN == 1 && !split) {   // the upsampling convs' input gradients (256 -> 64): unshuffled or gated rows
    KAIR_CHECK_ARG(x_dtype == KAIR_BF16 && ps_r <= 0 && !rs, "conv3x3_wr: the plain N <= 64 form takes a bf16 image");
    if (BM == 192) {
      KAIR_CHECK_ARG(!acopy, "conv3x3_wr: no a_copy with the two-pass tile");
      if (ps_r < 0) KAIR_WR(bf16, false, 192, false, 1, 2); else KAIR_WR(bf16, false, 192, false, 1, 0);
    } else if (ps_r < 0) KAIR_WR3(bf16, false, false, 1, 2); else KAIR_WR3(bf16, false, false, 1, 0);
  } else if (RN == 1) {   // conv_before_upsample (192 -> 64): split, row output (+ LeakyReLU, + lo plane)
    KAIR_CHECK_ARG(split && x_dtype == KAIR_F32 && ps_r == 0, "conv3x3_wr: the N <= 64 form takes an fp32 image, split, rows");
    if (rs) KAIR_WR3(float, true, true, 1, 0); else KAIR_WR3(float, true, false, 1, 0);
  } else {
    KAIR_CHECK_ARG(RN == 3 && ps_r == 0, "conv3x3_wr: N <= 192 row outputs for this form");
    if (split) {
      if (rs) KAIR_WR3(float, true, true, 3, 0); else KAIR_WR3(float, true, false, 3, 0);
    } else if (x_dtype == KAIR_F32) {
      if (rs) KAIR_WR3(float, false, true, 3, 0); else KAIR_WR3(float, false, false, 3, 0);
    } else {
      if (rs) KAIR_WR3(bf16, false, true, 3, 0); else KAIR_WR3(bf16, false, false, 3, 0);
    }
  }
#undef KAIR_WR3
#undef KAIR_WR
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_conv3x3_wr(const void* x, int x_dtype, long ldx, int split, int flip, const void* w, int n_blocks,
                               const float* bias, const float* resid, long ldr, void* out, int out_dtype, long ldo, void* acopy,
                               long ldac, int acones, int B, int H, int W, int C, int N, void* stream) {
  return kair_conv3x3_wr_ex(x, x_dtype, ldx, split, flip, w, n_blocks, bias, resid, ldr, out, out_dtype, ldo, nullptr, 0,
                            KAIR_ACT_NONE, 0.f, nullptr, 0, acopy, ldac, acones, B, H, W, C, N, stream);
}
