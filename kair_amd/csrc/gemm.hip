// Implicit-GEMM kernels for gfx950 (CDNA4): the contractions of nn.Linear and 3x3 nn.Conv2d on the
// KAIR hot path (forward, input gradient and weight gradient), with fused prologue address maps
// (Swin window partition + cyclic shift, im2col, head-blocked q/k/v) and fused epilogues
// (bias, GELU / LeakyReLU, residual add, PixelShuffle store, NCHW image store, act' gating).
//
//   kair_gemm_nt : C[m,n] = sum_k A[m,k] B[n,k]          (forward, dgrad)
//   kair_gemm_tn : P[s][n,k] = sum_{m in s} A[m,n] B[m,k]  (wgrad, split over m, deterministic)
//
// Tiles: 256 threads = 4 waves, BK = 32.  bf16 compute uses v_mfma_f32_16x16x32_bf16 (8 bf16 of K
// per lane, one ds_read_b128 per fragment); f32 compute uses v_mfma_f32_16x16x4_f32 (exact fp32,
// parity mode).  Operands are staged global -> registers -> LDS with the next K-tile's global
// loads issued before the current tile's MFMAs (register double buffering).
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace {

constexpr int BK = 32;
constexpr int NT = 256;

// ------------------------------------------------------------------------------------------
// operand chunk loader: 8 consecutive columns [k, k+8) of row m, returned as fp32
// ------------------------------------------------------------------------------------------
struct Op {
  const void* ptr;
  int dtype, mode;
  long ld;
  WinMap win;
  int imH, imW, imC, flip;
  int nh, hdp, tok;
  const float* rowscale;
  int rps;
  int ones_col;
  long M;  // total rows (QKVBLK part stride)
};

KAIR_DEV void load8(const Op& op, long m, int k, int K, float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = 0.f;
  if (m >= op.M || k >= K) return;
  long off;
  long srow = m;
  if (op.mode == KAIR_LD_ROWS) {
    srow = win_to_token(m, op.win);
    off = srow * op.ld + k;
  } else if (op.mode == KAIR_LD_IM2COL3) {
    const int tap = k / op.imC;
    const int c = k - tap * op.imC;
    int dy = tap / 3 - 1, dx = tap % 3 - 1;
    if (op.flip) { dy = -dy; dx = -dx; }
    const long hw = (long)op.imH * op.imW;
    const long b = m / hw;
    const int p = (int)(m - b * hw);
    const int y = p / op.imW + dy, x = p % op.imW + dx;
    if (y < 0 || y >= op.imH || x < 0 || x >= op.imW) {
      if (op.ones_col >= k && op.ones_col < k + 8) v[op.ones_col - k] = 1.f;
      return;
    }
    off = ((b * op.imH + y) * op.imW + x) * op.imC + c;
  } else {  // QKVBLK
    const int pw = op.nh * op.hdp;
    const int part = k / pw;
    const int r = k - part * pw;
    const int h = r / op.hdp, d = r - h * op.hdp;
    const long win = m / op.tok;
    const int t = (int)(m - win * op.tok);
    off = (long)part * op.M * pw + ((win * op.nh + h) * op.tok + t) * op.hdp + d;
  }
  if (op.dtype == KAIR_BF16) {
    const bf16x8 q = *(const bf16x8*)((const bf16*)op.ptr + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)q[j];
  } else {
    const float4 a = *(const float4*)((const float*)op.ptr + off);
    const float4 b = *(const float4*)((const float*)op.ptr + off + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  if (op.rowscale) {
    const float s = op.rowscale[srow / op.rps];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= s;
  }
  if (op.ones_col >= k && op.ones_col < k + 8) v[op.ones_col - k] = 1.f;
}

Op make_op(const kair_operand& o, long M) {
  Op op;
  op.ptr = o.ptr; op.dtype = o.dtype; op.mode = o.mode; op.ld = o.ld;
  op.win = WinMap{o.win_H, o.win_W, o.win_ws, o.win_shift};
  op.imH = o.im_H; op.imW = o.im_W; op.imC = o.im_C; op.flip = o.im_flip;
  op.nh = o.qkv_nh; op.hdp = o.qkv_hdp; op.tok = o.qkv_tok;
  op.rowscale = o.rowscale; op.rps = o.rows_per_scale > 0 ? o.rows_per_scale : 1;
  op.ones_col = o.ones_col;
  op.M = M;
  return op;
}

// ------------------------------------------------------------------------------------------
// epilogue
// ------------------------------------------------------------------------------------------
struct Epi {
  void* out; int odt, omode; long ldo;
  WinMap win;
  const float* bias;
  int act; float slope;
  void* pre; int pdt; long ldp;
  const float* resid; long ldr;
  const float* rowscale; int rps;
  const void* gate; int gdt; long ldg; int gkind;
  int r, psH, psW;
  int nh, hdp, tok;
  const float* mean; float range; int imgC, imgH, imgW;
  long M; int N;
};

KAIR_DEV void st(void* p, int dt, long off, float v) {
  if (dt == KAIR_BF16) ((bf16*)p)[off] = (bf16)v;
  else ((float*)p)[off] = v;
}
KAIR_DEV float ld1(const void* p, int dt, long off) {
  return dt == KAIR_BF16 ? (float)((const bf16*)p)[off] : ((const float*)p)[off];
}

KAIR_DEV void epi_store(const Epi& e, long m, int n, float v) {
  if (m >= e.M || n >= e.N) return;
  if (e.bias) v += e.bias[n];
  const float pre = v;
  if (e.act == KAIR_ACT_GELU) v = gelu_erf(v);
  else if (e.act == KAIR_ACT_LEAKY) v = v > 0.f ? v : v * e.slope;
  else if (e.act == KAIR_ACT_RELU) v = fmaxf(v, 0.f);
  if (e.omode == KAIR_OUT_ROWS) {
    const long row = win_to_token(m, e.win);
    if (e.gate) {
      const float g = ld1(e.gate, e.gdt, row * e.ldg + n);
      if (e.gkind == 1) v *= gelu_erf_grad(g);
      else if (e.gkind == 2) v *= (g > 0.f ? 1.f : e.slope);
      else v *= (g > 0.f ? 1.f : 0.f);
    }
    if (e.resid) {
      const float s = e.rowscale ? e.rowscale[row / e.rps] : 1.f;
      v = e.resid[row * e.ldr + n] + s * v;
    }
    st(e.out, e.odt, row * e.ldo + n, v);
    if (e.pre) st(e.pre, e.pdt, row * e.ldp + n, pre);
  } else if (e.omode == KAIR_OUT_QKVBLK) {
    const int pw = e.nh * e.hdp;
    const int part = n / pw, rr = n - part * pw;
    const int h = rr / e.hdp, d = rr - h * e.hdp;
    const long win = m / e.tok;
    const int t = (int)(m - win * e.tok);
    st(e.out, e.odt, (long)part * e.M * pw + ((win * e.nh + h) * e.tok + t) * e.hdp + d, v);
  } else if (e.omode == KAIR_OUT_PSHUF) {
    const int r = e.r, r2 = r * r;
    const int c = n / r2, ij = n - c * r2, i = ij / r, j = ij - i * r;
    const long hw = (long)e.psH * e.psW;
    const long b = m / hw;
    const int p = (int)(m - b * hw), y = p / e.psW, x = p - (p / e.psW) * e.psW;
    const long orow = (b * e.psH * r + (long)y * r + i) * ((long)e.psW * r) + (long)x * r + j;
    if (e.gate) {
      const float g = ld1(e.gate, e.gdt, orow * e.ldg + c);
      v *= (e.gkind == 2) ? (g > 0.f ? 1.f : e.slope) : (g > 0.f ? 1.f : 0.f);
    }
    st(e.out, e.odt, orow * e.ldo + c, v);
    if (e.pre) st(e.pre, e.pdt, orow * e.ldp + c, pre);
  } else if (e.omode == KAIR_OUT_PUNSHUF) {
    const int r = e.r;
    const long HW = (long)e.psH * r * e.psW * r;
    const long b = m / HW;
    const long p = m - b * HW;
    const int Y = (int)(p / (e.psW * r)), X = (int)(p - (long)Y * e.psW * r);
    const int y = Y / r, i = Y - y * r, x = X / r, j = X - x * r;
    const long orow = (b * e.psH + y) * e.psW + x;
    const int oc = n * r * r + i * r + j;
    if (e.gate) {
      const float g = ld1(e.gate, e.gdt, orow * e.ldg + oc);
      v *= (e.gkind == 2) ? (g > 0.f ? 1.f : e.slope) : (g > 0.f ? 1.f : 0.f);
    }
    st(e.out, e.odt, orow * e.ldo + oc, v);
  } else if (e.omode == KAIR_OUT_PSHUF_NCHW) {
    const int r = e.r, r2 = r * r;
    const int c = n / r2, ij = n - c * r2, i = ij / r, j = ij - i * r;
    if (c >= e.imgC) return;
    const long hw = (long)e.psH * e.psW;
    const long b = m / hw;
    const int p = (int)(m - b * hw), y = p / e.psW, x = p - (p / e.psW) * e.psW;
    v = v / e.range + (e.mean ? e.mean[c] : 0.f);
    ((float*)e.out)[((b * e.imgC + c) * e.psH * r + (long)y * r + i) * ((long)e.psW * r) + (long)x * r + j] = v;
  } else {  // NCHW image
    if (n >= e.imgC) return;
    const long hw = (long)e.imgH * e.imgW;
    const long b = m / hw;
    const long p = m - b * hw;
    v = v / e.range + (e.mean ? e.mean[n] : 0.f);
    ((float*)e.out)[(b * e.imgC + n) * hw + p] = v;
  }
}

Epi make_epi(const kair_epilogue& o, long M, int N) {
  Epi e;
  e.out = o.out; e.odt = o.out_dtype; e.omode = o.out_mode; e.ldo = o.ldo;
  e.win = WinMap{o.win_H, o.win_W, o.win_ws, o.win_shift};
  e.bias = o.bias; e.act = o.act; e.slope = o.slope;
  e.pre = o.out_pre; e.pdt = o.pre_dtype; e.ldp = o.ldp;
  e.resid = o.resid; e.ldr = o.ldr;
  e.rowscale = o.rowscale; e.rps = o.rows_per_scale > 0 ? o.rows_per_scale : 1;
  e.gate = o.gate; e.gdt = o.gate_dtype; e.ldg = o.ldg; e.gkind = o.gate_kind;
  e.r = o.ps_r; e.psH = o.ps_H; e.psW = o.ps_W;
  e.nh = o.qkv_nh; e.hdp = o.qkv_hdp; e.tok = o.qkv_tok;
  e.mean = o.img_mean; e.range = o.img_range; e.imgC = o.img_C; e.imgH = o.img_H; e.imgW = o.img_W;
  e.M = M; e.N = N;
  return e;
}

// bijective XCD-aware remap: logical tiles [x*q + min(x,r) ...] live on the same XCD group
KAIR_DEV int xcd_remap(int hw, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int x = hw % 8, pos = hw / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + pos;
}

// ------------------------------------------------------------------------------------------
// LDS tile helpers
// ------------------------------------------------------------------------------------------
template <typename CT> struct Lds;
template <> struct Lds<bf16> {
  static constexpr int LD = BK + 8;  // 80-byte rows: ds_read_b128 fragment reads conflict-free
};
template <> struct Lds<float> {
  static constexpr int LD = BK + 2;  // 136-byte rows
};

template <typename CT>
KAIR_DEV void lds_store8(CT* base, const float (&v)[8]) {
  if constexpr (sizeof(CT) == 2) {
    bf16x8 q;
#pragma unroll
    for (int j = 0; j < 8; ++j) q[j] = (bf16)v[j];
    *(bf16x8*)base = q;
  } else {
#pragma unroll
    for (int j = 0; j < 8; j += 2) *(float2*)(base + j) = make_float2(v[j], v[j + 1]);
  }
}

// ------------------------------------------------------------------------------------------
// NT kernel
// ------------------------------------------------------------------------------------------
template <typename CT, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(NT) void gemm_nt_kernel(Op A, Op B, Epi E, int K, int tilesN, int nwg) {
  constexpr int LD = Lds<CT>::LD;
  constexpr int TM = BM / WM, TN = BN / WN;  // per-wave tile
  constexpr int RM = TM / 16, RN = TN / 16;
  constexpr int CA = BM * BK / 8, CB = BN * BK / 8;  // 8-element chunks per tile
  constexpr int PA = (CA + NT - 1) / NT, PB = (CB + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) CT sA[BM * LD];
  __shared__ __attribute__((aligned(16))) CT sB[BN * LD];

  const int tile = xcd_remap(blockIdx.x, nwg);
  const int tm = tile / tilesN, tn = tile - tm * tilesN;
  const long m0 = (long)tm * BM;
  const int n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  float ra[PA][8], rb[PB][8];
  auto gload = [&](int k0) {
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int c = tid + p * NT;
      if (c < CA) load8(A, m0 + c / 4, k0 + (c & 3) * 8, K, ra[p]);
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int c = tid + p * NT;
      if (c < CB) load8(B, n0 + c / 4, k0 + (c & 3) * 8, K, rb[p]);
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int c = tid + p * NT;
      if (c < CA) lds_store8<CT>(sA + (c / 4) * LD + (c & 3) * 8, ra[p]);
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int c = tid + p * NT;
      if (c < CB) lds_store8<CT>(sB + (c / 4) * LD + (c & 3) * 8, rb[p]);
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (K + BK - 1) / BK;
  gload(0);
  for (int kt = 0; kt < nk; ++kt) {
    __syncthreads();
    sstore();
    __syncthreads();
    if (kt + 1 < nk) gload((kt + 1) * BK);
    const int fr = lane & 15, fq = lane >> 4;
    if constexpr (sizeof(CT) == 2) {
      bf16x8 af[RM], bfr[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) af[i] = *(const bf16x8*)(sA + (wm * TM + i * 16 + fr) * LD + fq * 8);
#pragma unroll
      for (int j = 0; j < RN; ++j) bfr[j] = *(const bf16x8*)(sB + (wn * TN + j * 16 + fr) * LD + fq * 8);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int s = 0; s < BK / 4; ++s) {
        float af[RM], bfr[RN];
#pragma unroll
        for (int i = 0; i < RM; ++i) af[i] = sA[(wm * TM + i * 16 + fr) * LD + s * 4 + fq];
#pragma unroll
        for (int j = 0; j < RN; ++j) bfr[j] = sB[(wn * TN + j * 16 + fr) * LD + s * 4 + fq];
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  // epilogue: 16x16 C/D map  col = lane&15, row = (lane>>4)*4 + r
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long m = m0 + wm * TM + i * 16 + (lane >> 4) * 4 + r;
        const int n = n0 + wn * TN + j * 16 + (lane & 15);
        epi_store(E, m, n, acc[i][j][r]);
      }
}

// ------------------------------------------------------------------------------------------
// TN kernel (weight gradient): P[s][n][k] = sum_{m in split s} A[m][n] * B[m][k]
// LDS holds both operands m-major ([32 m][BN], [32 m][BK]) exactly as loaded; bf16 fragments
// (8 consecutive m for one n) come from two ds_read_b64_tr_b16 transposed reads.
// ------------------------------------------------------------------------------------------
template <typename CT, int BN, int BKo>
__global__ __launch_bounds__(NT) void gemm_tn_kernel(Op A, Op B, float* ws, long M, int N, int K, long rows_per_split,
                                                     int tilesK) {
  constexpr int LDA = BN + 8, LDB = BKo + 8;  // m-major rows, padded
  constexpr int WN = 2, WK = 2;
  constexpr int TN_ = BN / WN, TK_ = BKo / WK;
  constexpr int RN = TN_ / 16, RK = TK_ / 16;
  constexpr int CA = BK * BN / 8, CB = BK * BKo / 8;
  constexpr int PA = (CA + NT - 1) / NT, PB = (CB + NT - 1) / NT;
  constexpr int CPA = BN / 8, CPB = BKo / 8;  // chunks per m-row
  __shared__ __attribute__((aligned(16))) CT sA[BK * LDA];
  __shared__ __attribute__((aligned(16))) CT sB[BK * LDB];

  const int tn = blockIdx.x / tilesK, tk = blockIdx.x - (blockIdx.x / tilesK) * tilesK;
  const int n0 = tn * BN, k0 = tk * BKo;
  const long mbeg = (long)blockIdx.y * rows_per_split;
  long mend = mbeg + rows_per_split;
  if (mend > M) mend = M;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave / WK, wk = wave % WK;

  float ra[PA][8], rb[PB][8];
  auto gload = [&](long mb) {
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int c = tid + p * NT;
      if (c < CA) {
        const long m = mb + c / CPA;
        if (m < mend) load8(A, m, n0 + (c % CPA) * 8, N, ra[p]);
        else
#pragma unroll
          for (int j = 0; j < 8; ++j) ra[p][j] = 0.f;
      }
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int c = tid + p * NT;
      if (c < CB) {
        const long m = mb + c / CPB;
        if (m < mend) load8(B, m, k0 + (c % CPB) * 8, K, rb[p]);
        else
#pragma unroll
          for (int j = 0; j < 8; ++j) rb[p][j] = 0.f;
      }
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int c = tid + p * NT;
      if (c < CA) lds_store8<CT>(sA + (c / CPA) * LDA + (c % CPA) * 8, ra[p]);
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int c = tid + p * NT;
      if (c < CB) lds_store8<CT>(sB + (c / CPB) * LDB + (c % CPB) * 8, rb[p]);
    }
  };

  f32x4 acc[RN][RK];
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int j = 0; j < RK; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  if (mbeg < mend) {
    gload(mbeg);
    for (long mb = mbeg; mb < mend; mb += BK) {
      __syncthreads();
      sstore();
      __syncthreads();
      if (mb + BK < mend) gload(mb + BK);
      if constexpr (sizeof(CT) == 2) {
        // lane 4q+p of 16-lane group g supplies row (8g + q [+4]) and columns c0 + 4p;
        // it receives column c0 + (lane&15) at rows 8g + 0..3 [4..7].
        const int q = (lane & 15) >> 2, p4 = (lane & 3) * 4, g8 = (lane >> 4) * 8;
        bf16x8 af[RN], bfr[RK];
#pragma unroll
        for (int i = 0; i < RN; ++i) {
          const CT* base = sA + (g8 + q) * LDA + wn * TN_ + i * 16 + p4;
          const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)(base));
          const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) short4v*)(base + 4 * LDA));
          short __attribute__((ext_vector_type(8))) s8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          af[i] = __builtin_bit_cast(bf16x8, s8);
        }
#pragma unroll
        for (int j = 0; j < RK; ++j) {
          const CT* base = sB + (g8 + q) * LDB + wk * TK_ + j * 16 + p4;
          const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)(base));
          const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) short4v*)(base + 4 * LDB));
          short __attribute__((ext_vector_type(8))) s8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          bfr[j] = __builtin_bit_cast(bf16x8, s8);
        }
#pragma unroll
        for (int i = 0; i < RN; ++i)
#pragma unroll
          for (int j = 0; j < RK; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      } else {
#pragma unroll
        for (int s = 0; s < BK / 4; ++s) {
          float af[RN], bfr[RK];
#pragma unroll
          for (int i = 0; i < RN; ++i) af[i] = sA[(s * 4 + fq) * LDA + wn * TN_ + i * 16 + fr];
#pragma unroll
          for (int j = 0; j < RK; ++j) bfr[j] = sB[(s * 4 + fq) * LDB + wk * TK_ + j * 16 + fr];
#pragma unroll
          for (int i = 0; i < RN; ++i)
#pragma unroll
            for (int j = 0; j < RK; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
      }
    }
  }
  float* P = ws + (long)blockIdx.y * N * K;
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int j = 0; j < RK; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * TN_ + i * 16 + fq * 4 + r;
        const int k = k0 + wk * TK_ + j * 16 + fr;
        if (n < N && k < K) P[(long)n * K + k] = acc[i][j][r];
      }
}

template <typename CT, int BM, int BN, int WM, int WN>
int launch_nt(const Op& A, const Op& B, const Epi& E, long M, int N, int K, hipStream_t s) {
  const long tilesM = (M + BM - 1) / BM;
  const int tilesN = (N + BN - 1) / BN;
  const long nwg = tilesM * tilesN;
  if (nwg > 0x7fffffff) return kair_set_error(KAIR_ERR_ARG, "gemm_nt: grid too large");
  hipLaunchKernelGGL((gemm_nt_kernel<CT, BM, BN, WM, WN>), dim3((unsigned)nwg), dim3(NT), 0, s, A, B, E, K, tilesN,
                     (int)nwg);
  KAIR_CHECK_LAUNCH();
  return 0;
}

template <typename CT>
int dispatch_nt(const Op& A, const Op& B, const Epi& E, long M, int N, int K, hipStream_t s) {
  if (N <= 16) return launch_nt<CT, 256, 16, 4, 1>(A, B, E, M, N, K, s);
  if (N <= 32) return launch_nt<CT, 256, 32, 4, 1>(A, B, E, M, N, K, s);
  if (N <= 64) return launch_nt<CT, 128, 64, 2, 2>(A, B, E, M, N, K, s);
  return launch_nt<CT, 128, 128, 2, 2>(A, B, E, M, N, K, s);
}

}  // namespace

// ============================================================================================
// C ABI
// ============================================================================================
static thread_local char g_err[512];

int kair_set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

extern "C" const char* kair_last_error(void) { return g_err; }

extern "C" int kair_device_arch(char* buf, int len) {
  hipDeviceProp_t p;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess)
    return kair_set_error(KAIR_ERR_HIP, "no HIP device");
  snprintf(buf, len, "%s", p.gcnArchName);
  return 0;
}

static int check_operand(const kair_operand* o, const char* what) {
  KAIR_CHECK_ARG(o && o->ptr, "%s: null operand", what);
  KAIR_CHECK_ARG(o->dtype == KAIR_F32 || o->dtype == KAIR_BF16, "%s: bad dtype", what);
  KAIR_CHECK_ARG(o->mode >= 0 && o->mode <= 2, "%s: bad mode", what);
  const int esz = o->dtype == KAIR_BF16 ? 2 : 4;
  KAIR_CHECK_ARG(((uintptr_t)o->ptr % 16) == 0, "%s: pointer not 16-byte aligned", what);
  if (o->mode == KAIR_LD_ROWS) KAIR_CHECK_ARG((o->ld * esz) % 16 == 0, "%s: row stride not 16-byte aligned", what);
  if (o->mode == KAIR_LD_IM2COL3) KAIR_CHECK_ARG(o->im_C % 8 == 0 && o->im_H > 0 && o->im_W > 0, "%s: im2col geometry", what);
  if (o->mode == KAIR_LD_QKVBLK) KAIR_CHECK_ARG(o->qkv_hdp % 8 == 0 && o->qkv_tok > 0 && o->qkv_nh > 0, "%s: qkv geometry", what);
  if (o->win_ws > 0)
    KAIR_CHECK_ARG(o->win_H % o->win_ws == 0 && o->win_W % o->win_ws == 0, "%s: window map geometry", what);
  return 0;
}

extern "C" int kair_gemm_nt(const kair_operand* A, const kair_operand* B, const kair_epilogue* E, long M, int N, int K,
                            int compute, void* stream) {
  int rc;
  if ((rc = check_operand(A, "gemm_nt A"))) return rc;
  if ((rc = check_operand(B, "gemm_nt B"))) return rc;
  KAIR_CHECK_ARG(E && E->out, "gemm_nt: null epilogue/out");
  KAIR_CHECK_ARG(M > 0 && N > 0 && K > 0 && K % 8 == 0, "gemm_nt: bad M/N/K (%ld,%d,%d), K%%8 must be 0", M, N, K);
  KAIR_CHECK_ARG(E->out_mode != KAIR_OUT_PSHUF || E->ps_r > 0, "gemm_nt: pixel shuffle r");
  const Op a = make_op(*A, M), b = make_op(*B, N);
  const Epi e = make_epi(*E, M, N);
  hipStream_t s = (hipStream_t)stream;
  if (compute == KAIR_BF16) return dispatch_nt<bf16>(a, b, e, M, N, K, s);
  if (compute == KAIR_F32) return dispatch_nt<float>(a, b, e, M, N, K, s);
  return kair_set_error(KAIR_ERR_ARG, "gemm_nt: bad compute type");
}

extern "C" int kair_wgrad_splits(long M, int N, int K) {
  const long tiles = (long)((N + 127) / 128) * ((K + 127) / 128);
  long s = 512 / (tiles > 0 ? tiles : 1);
  const long maxs = (M + 255) / 256;
  if (s > maxs) s = maxs;
  if (s < 1) s = 1;
  return (int)s;
}

extern "C" int kair_gemm_tn(const kair_operand* A, const kair_operand* B, float* ws, int splits, long M, int N, int K,
                            int compute, void* stream) {
  int rc;
  if ((rc = check_operand(A, "gemm_tn A"))) return rc;
  if ((rc = check_operand(B, "gemm_tn B"))) return rc;
  KAIR_CHECK_ARG(ws, "gemm_tn: null workspace");
  KAIR_CHECK_ARG(M > 0 && N > 0 && K > 0 && N % 8 == 0 && K % 8 == 0 && splits > 0, "gemm_tn: bad sizes");
  Op a = make_op(*A, M), b = make_op(*B, M);
  long rps = (M + splits - 1) / splits;
  rps = (rps + BK - 1) / BK * BK;
  hipStream_t s = (hipStream_t)stream;
  const bool small = (N <= 64 && K <= 64);
  if (small) {
    const int tilesN = (N + 63) / 64, tilesK = (K + 63) / 64;
    dim3 grid(tilesN * tilesK, splits);
    if (compute == KAIR_BF16)
      hipLaunchKernelGGL((gemm_tn_kernel<bf16, 64, 64>), grid, dim3(NT), 0, s, a, b, ws, M, N, K, rps, tilesK);
    else
      hipLaunchKernelGGL((gemm_tn_kernel<float, 64, 64>), grid, dim3(NT), 0, s, a, b, ws, M, N, K, rps, tilesK);
  } else {
    const int tilesN = (N + 127) / 128, tilesK = (K + 127) / 128;
    dim3 grid(tilesN * tilesK, splits);
    if (compute == KAIR_BF16)
      hipLaunchKernelGGL((gemm_tn_kernel<bf16, 128, 128>), grid, dim3(NT), 0, s, a, b, ws, M, N, K, rps, tilesK);
    else
      hipLaunchKernelGGL((gemm_tn_kernel<float, 128, 128>), grid, dim3(NT), 0, s, a, b, ws, M, N, K, rps, tilesK);
  }
  KAIR_CHECK_LAUNCH();
  return 0;
}
