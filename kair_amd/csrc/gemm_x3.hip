// The fp32 engine's contractions on the 16-bit matrix cores ("x3" arithmetic, KAIR_COMPUTE_X3): every
// operand x enters as an fp16 pair of x * 2^e (hi = f16(x 2^e), lo = f16(x 2^e - hi)) and every product as
// hi.hi + hi.lo + lo.hi (v_mfma_f32_16x16x32_f16, fp32 accumulation), the accumulator rescaled by 2^-(eA+eB).
// The pair carries 22 of fp32's 24 mantissa bits, so a product is exact to ~2^-21 -- the precision class of
// the fp32 reference (SwinIR classical x4 trains in fp32: models/model_plain.py:31-36 with no amp_enabled in
// options/swinir/train_swinir_sr_classical.json); the power-of-2 exponent keeps the operand inside fp16's
// range (weights 2^KAIR_X3_WEXP, activations 2^4, gradients 2^(log2 of the loss normalisation / loss weight) + 4;
// the activation / gradient exponents drop when the range guard fires, SwinIREngine.x3_backoff).
//
//   kair_gemm_nt_x3 : C[m,n] = sum_k A[m,k] B[n,k]            (nn.Linear / 3x3 nn.Conv2d forward + dgrad)
//   kair_gemm_tn_x3 : P[s][n,k] = sum_{m in s} A[m,n] B[m,k]   (their weight gradients, split over m)
//
// Operands: fp32 (split at the LDS commit, read from HBM once) or fp16 hi planes with their lo planes
// (kair_operand.lo_ptr).  LDS holds hi and lo planes of both operands; 32-deep k-steps (NT) / 32-row
// reduction steps (TN), double-buffered by register staging as the bf16 kernels (gemm.hip).
#include <string.h>

#include <type_traits>

#include "gemm_common.h"

namespace {

template <typename T> struct RawX3 { Raw<T> h, l; };

KAIR_DEV f32x4 mfma16(const f16x8& a, const f16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// the lo plane of an fp16 pair operand into LDS: masked rows 0, the ones column (hi 1.0) 0
KAIR_DEV void commit_lo_plane(f16* dst, const Raw<f16>& raw, const Pend& pd) {
  f16x8 q = __builtin_bit_cast(f16x8, raw.a);
  if (pd.scale == 0.f) q = f16x8{};
  if (pd.ones >= 0) q[pd.ones] = (f16)0.f;
  *(f16x8*)dst = q;
}

// commit one 8-column chunk of an x3 operand as its hi and lo planes (fp32: split with the operand's scale);
// an injected ones column reads 2^e (onev), the operand's own scale
template <typename T>
KAIR_DEV void commit_pair(f16* hi, f16* lo, const RawX3<T>& raw, const Pend& pd, float onev) {
  if constexpr (sizeof(T) == 4) {
    commit_chunk<f16, T>(hi, raw.h, pd, false, onev);
    commit_chunk<f16, T>(lo, raw.h, pd, true, onev);
  } else {
    commit_chunk<f16, T>(hi, raw.h, pd, false, onev);
    commit_lo_plane(lo, raw.l, pd);
  }
}

template <typename T>
KAIR_DEV f16x8 trfrag(const f16* base, int ld) {
  const short4v a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)base);
  const short4v b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)(base + 4 * ld));
  short __attribute__((ext_vector_type(8))) s8 = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(f16x8, s8);
}

// ------------------------------------------------------------------------------------------
// NT: 256 threads (2 x 2 waves), BM x BN output tile, k-steps of 32.  B is a split-packed weight: rows of
// 64-column chunks alternating hi / lo (pack kinds 9 / 17 / 18 / 19, fp16 destination).
// ------------------------------------------------------------------------------------------
// (visiting a 3x3 im2col's k-chunks channel-chunk-major -- the nine taps of a 32-channel chunk back to back -- left the
// 96^2 PixelUnshuffle input gradient at 548 us against 552 tap-major: not what bounds it; profiles/r06_im2col_order_ab.txt)
template <typename TA, int AM, int BM, int BN>
__global__ __launch_bounds__(NT, 2) void gemm_nt_x3_kernel(Op A, Op B, Epi E, int K, int tilesN, int nwg) {
  constexpr int BK = 32, LD = BK + 8;
  constexpr int WM = 2, WN = 2, TM = BM / WM, TN = BN / WN, RM = TM / 16, RN = TN / 16;
  constexpr int CPR = BK / 8;
  constexpr int CA = BM * CPR, CB = BN * CPR;
  constexpr int PA = (CA + NT - 1) / NT, PB = (CB + NT - 1) / NT;
  constexpr int PLANE = (BM + BN) * LD;    // A rows then B rows of one plane
  constexpr int STAGE = 2 * PLANE;         // hi plane, lo plane
  constexpr int EPI_LD = BN + 4;
  constexpr int LDS_MAIN = 2 * STAGE * 2, LDS_EPI = BM * EPI_LD * 4;
  constexpr int LDS_BYTES = LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI;
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  f16* lds = (f16*)smem;

  const int tile = xcd_remap(blockIdx.x, nwg);
  const int tm = tile / tilesN, tn = tile - tm * tilesN;
  const long m0 = (long)tm * BM;
  const int n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int KB = 2 * ((K + 63) / 64) * 64;   // packed row length of B

  RowState ra[PA], rb[PB];
#pragma unroll
  for (int p = 0; p < PA; ++p) {
    const int c = tid + p * NT;
    ra[p] = row_state<AM, TA>(A, c < CA ? m0 + c / CPR : A.M);
    ra[p].scale *= A.x3s;
  }
#pragma unroll
  for (int p = 0; p < PB; ++p) {
    const int c = tid + p * NT;
    rb[p] = row_state<AM_ROWS, f16>(B, c < CB ? (long)(n0 + c / CPR) : B.M);
  }
  RawX3<TA> va[PA];
  Raw<f16> vbh[PB], vbl[PB];
  Pend pa[PA], pb[PB], pbl[PB];
  auto gload = [&](int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int k = k0 + ((tid + p * NT) % CPR) * 8;
      issue_chunk<AM, TA>(A, ra[p], k, K, va[p].h, pa[p]);
      if constexpr (sizeof(TA) == 2) {
        Pend d;
        issue_chunk<AM, TA>(A, ra[p], k, K, va[p].l, d, A.lo_ptr);
      }
    }
    const int kb = (k0 >> 6) * 128 + (k0 & 63);   // hi chunk of k-step kt in the interleaved row; lo at + 64
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int k = kb + ((tid + p * NT) % CPR) * 8;
      issue_chunk<AM_ROWS, f16>(B, rb[p], k, KB, vbh[p], pb[p]);
      issue_chunk<AM_ROWS, f16>(B, rb[p], k + 64, KB, vbl[p], pbl[p]);
    }
  };
  auto sstore = [&](int st) {
    f16* s0 = lds + st * STAGE;
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int c = tid + p * NT;
      if (c < CA) {
        const int o = (c / CPR) * LD + (c % CPR) * 8;
        commit_pair<TA>(s0 + o, s0 + PLANE + o, va[p], pa[p], 1.f);
      }
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int c = tid + p * NT;
      if (c < CB) {
        const int o = BM * LD + (c / CPR) * LD + (c % CPR) * 8;
        commit_chunk<f16, f16>(s0 + o, vbh[p], pb[p]);
        commit_chunk<f16, f16>(s0 + PLANE + o, vbl[p], pbl[p]);
      }
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  const int nk = (K + BK - 1) / BK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const f16* sAh = lds + st * STAGE;
    const f16* sBh = sAh + BM * LD;
    const f16* sAl = sAh + PLANE;
    const f16* sBl = sAl + BM * LD;
    f16x8 ah[RM], al[RM], bh[RN], bl[RN];
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int o = (wm * TM + i * 16 + fr) * LD + fq * 8;
      ah[i] = *(const f16x8*)(sAh + o);
      al[i] = *(const f16x8*)(sAl + o);
    }
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int o = (wn * TN + j * 16 + fr) * LD + fq * 8;
      bh[j] = *(const f16x8*)(sBh + o);
      bl[j] = *(const f16x8*)(sBl + o);
    }
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        acc[i][j] = mfma16(ah[i], bh[j], acc[i][j]);
        acc[i][j] = mfma16(ah[i], bl[j], acc[i][j]);
        acc[i][j] = mfma16(al[i], bh[j], acc[i][j]);
      }
    if (kt + 1 < nk) sstore(st ^ 1);
    __syncthreads();
  }
  float* et = (float*)smem;
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) et[(wm * TM + i * 16 + fq * 4 + r) * EPI_LD + wn * TN + j * 16 + fr] = acc[i][j][r];
  __syncthreads();
  constexpr int CH = BM * BN / 8;
  for (int c = tid; c < CH; c += NT) {
    const int row = c / (BN / 8), col = (c % (BN / 8)) * 8;
    float v[8];
    const float4 a = *(const float4*)(et + row * EPI_LD + col);
    const float4 b = *(const float4*)(et + row * EPI_LD + col + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= E.acc_scale;
    epi_chunk(E, m0 + row, n0 + col, v);
  }
}

// ------------------------------------------------------------------------------------------
// TN: 256 threads (2 x 2 waves), BN x BKo tile of one split, 32 reduction rows per stage
// ------------------------------------------------------------------------------------------
template <typename TA, typename TB, int AMB, int BN, int BKo>
__global__ __launch_bounds__(NT, 2) void gemm_tn_x3_kernel(Op A, Op B, float* ws, long M, int N, int K, long rows_per_split,
                                                           int tilesK, float acc_scale) {
  constexpr int BMr = 32;
  constexpr int LDA = BN + 8, LDB = BKo + 8;
  constexpr int WN = 2, WK = 2;
  constexpr int TN_ = BN / WN, TK_ = BKo / WK;
  constexpr int RN = TN_ / 16, RK = TK_ / 16;
  constexpr int CPA = BN / 8, CPB = BKo / 8;
  constexpr int CA = BMr * CPA, CB = BMr * CPB;
  constexpr int PA = (CA + NT - 1) / NT, PB = (CB + NT - 1) / NT;
  constexpr int PL = BMr * (LDA + LDB);   // one plane (A rows, B rows)
  constexpr int STAGE = 2 * PL;           // hi plane, lo plane
  __shared__ __attribute__((aligned(16))) f16 lds[2 * STAGE];

  const int tn = blockIdx.x / tilesK, tk = blockIdx.x - (blockIdx.x / tilesK) * tilesK;
  const int n0 = tn * BN, k0 = tk * BKo;
  const long mbeg = (long)blockIdx.y * rows_per_split;
  long mend = mbeg + rows_per_split;
  if (mend > M) mend = M;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave / WK, wk = wave % WK;

  RawX3<TA> va[PA];
  RawX3<TB> vb[PB];
  Pend pa[PA], pb[PB];
  auto gload = [&](long mb) {
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int c = tid + p * NT;
      if (c < CA) {
        const long m = mb + c / CPA;
        RowState r = row_state<AM_ROWS, TA>(A, m < mend ? m : A.M);
        r.scale *= A.x3s;
        issue_chunk<AM_ROWS, TA>(A, r, n0 + (c % CPA) * 8, N, va[p].h, pa[p]);
        if constexpr (sizeof(TA) == 2) {
          Pend d;
          issue_chunk<AM_ROWS, TA>(A, r, n0 + (c % CPA) * 8, N, va[p].l, d, A.lo_ptr);
        }
      }
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int c = tid + p * NT;
      if (c < CB) {
        const long m = mb + c / CPB;
        RowState r = row_state<AMB, TB>(B, m < mend ? m : B.M);
        r.scale *= B.x3s;
        issue_chunk<AMB, TB>(B, r, k0 + (c % CPB) * 8, K, vb[p].h, pb[p]);
        if constexpr (sizeof(TB) == 2) {
          Pend d;
          issue_chunk<AMB, TB>(B, r, k0 + (c % CPB) * 8, K, vb[p].l, d, B.lo_ptr);
        }
      }
    }
  };
  const float onea = ldexpf(1.f, A.x3_exp), oneb = ldexpf(1.f, B.x3_exp);
  auto sstore = [&](int st) {
    f16* sAh = lds + st * STAGE;
    f16* sBh = sAh + BMr * LDA;
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int c = tid + p * NT;
      if (c < CA) {
        const int o = (c / CPA) * LDA + (c % CPA) * 8;
        commit_pair<TA>(sAh + o, sAh + PL + o, va[p], pa[p], onea);
      }
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int c = tid + p * NT;
      if (c < CB) {
        const int o = (c / CPB) * LDB + (c % CPB) * 8;
        commit_pair<TB>(sBh + o, sBh + PL + o, vb[p], pb[p], oneb);
      }
    }
  };

  f32x4 acc[RN][RK];
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int j = 0; j < RK; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nsteps = mbeg < mend ? (int)((mend - mbeg + BMr - 1) / BMr) : 0;
  if (nsteps > 0) {
    gload(mbeg);
    sstore(0);
    __syncthreads();
  }
  const int q = (lane & 15) >> 2, p4 = (lane & 3) * 4, g8 = (lane >> 4) * 8;
  for (int it = 0; it < nsteps; ++it) {
    const int st = it & 1;
    if (it + 1 < nsteps) gload(mbeg + (long)(it + 1) * BMr);
    const f16* sAh = lds + st * STAGE;
    const f16* sBh = sAh + BMr * LDA;
    const f16* sAl = sAh + PL;
    const f16* sBl = sBh + PL;
    f16x8 ah[RN], al[RN], bh[RK], bl[RK];
#pragma unroll
    for (int i = 0; i < RN; ++i) {
      const int o = (g8 + q) * LDA + wn * TN_ + i * 16 + p4;
      ah[i] = trfrag<f16>(sAh + o, LDA);
      al[i] = trfrag<f16>(sAl + o, LDA);
    }
#pragma unroll
    for (int j = 0; j < RK; ++j) {
      const int o = (g8 + q) * LDB + wk * TK_ + j * 16 + p4;
      bh[j] = trfrag<f16>(sBh + o, LDB);
      bl[j] = trfrag<f16>(sBl + o, LDB);
    }
#pragma unroll
    for (int i = 0; i < RN; ++i)
#pragma unroll
      for (int j = 0; j < RK; ++j) {
        acc[i][j] = mfma16(ah[i], bh[j], acc[i][j]);
        acc[i][j] = mfma16(ah[i], bl[j], acc[i][j]);
        acc[i][j] = mfma16(al[i], bh[j], acc[i][j]);
      }
    if (it + 1 < nsteps) sstore(st ^ 1);
    __syncthreads();
  }
  const int fr = lane & 15, fq = lane >> 4;
  float* P = ws + (long)blockIdx.y * N * K;
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int j = 0; j < RK; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * TN_ + i * 16 + fq * 4 + r;
        const int k = k0 + wk * TK_ + j * 16 + fr;
        if (n < N && k < K) P[(long)n * K + k] = acc[i][j][r] * acc_scale;
      }
}

// ------------------------------------------------------------------------------------------
// NT ring (x3): the streaming form of the NT product for the hot shapes (Swin linears, 192-channel 3x3
// convs).  512 threads, one CTA per CU, persistent over the 128 x 192 output tiles of ONE N-tile; every
// operand byte reaches LDS by LDS-DMA (global_load_lds_dwordx4) through an XR_NS-deep ring of 32-deep
// k-chunks that runs on across tile boundaries:
//   A chunk: 128 rows x 128 B -- fp32 (32 values, split into the fp16 pair at the fragment read, with the
//            operand's 2^e) or an fp16 pair (hi 32 | lo 32);
//   B chunk: 192 rows x 128 B -- the hi 32 | lo 32 of the split-packed weight row.
// 16-byte units of LDS row r sit at slot (unit ^ (r & 7)) (source-side XOR swizzle, the fragment reads
// are conflict-light).  8 waves as 4 (rows) x 2 (columns), wave tile 32 x 96; the MFMA operands are
// swapped (D = B A^T) so after a v_permlane16_swap of fragment pairs each lane owns 8 consecutive output
// columns of one row and finishes them with the shared 8-column epilogue.
// ------------------------------------------------------------------------------------------
constexpr int XR_BM = 128, XR_NB = 3, XR_ASTAGE = XR_BM * 128;   // B ring (L2-resident weights) depth; A stage 16 KiB
// the N-tile BN (64 / 128 / 192 / 256 columns) sets the B stage (BN x 128 B) and the A ring depth (HBM: the deeper
// ring, as deep as the 160 KiB allow: 5 stages up to BN = 192, 4 at 256)
template <int BN> struct XR {
  static constexpr int BSTAGE = BN * 128, NA = BN <= 192 ? 5 : 4, LDS = NA * XR_ASTAGE + XR_NB * BSTAGE + BN * 4;
  static constexpr int RN = BN / 32;    // 16-column fragments per wave (2 x 2 waves per group: BN / 2 columns each)
  static constexpr int BI = BN / 64;    // B DMA wave-instructions per wave per chunk
};

// XE_PSHUF / XE_PUNSHUF: fp32 stores in the PixelShuffle / PixelUnshuffle sub-pixel-major layouts (KAIR_OUT_PSHUF_SPM /
// KAIR_OUT_PUNSHUF_SPM: the upsampling convs' outputs and input gradients), bias only
enum { XE_ROWS_F32 = 0, XE_ROWS_PAIR = 1, XE_QKV = 2, XE_PSHUF = 3, XE_PUNSHUF = 4 };

// perf-investigation phase stamps of the NT ring (debug builds, KAIR_RING_DBG bit 8): CTAs 0..XS_CTAS-1, every
// wave, intervals 0..XS_IT-1, s_memtime at XS_N points (interval top, after the chunk wait, after the barrier +
// DMA issue, after the group's first phase, after its second); read with kair_debug_x3_stamps
constexpr int XS_CTAS = 4, XS_IT = 64, XS_N = 5;
__device__ unsigned long long g_x3_stamps[XS_CTAS * 8 * XS_IT * XS_N];
KAIR_DEV unsigned long long x3_now() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// fp32-rows epilogue activation / gate forms (compile-time: a run-time uniform test per element became a scalar
// branch per element, ~6.5 k cycles per tile epilogue)
enum { XA_NONE = 0, XA_GELU = 1, XA_GELU_X = 2, XA_LEAKY = 3 };   // GELU: pre = GELU'(x); GELU_X: pre = x
enum { XG_MUL = 4, XG_LEAKY = 2 };                                 // kair_epilogue.gate_kind 4 / 2

// Two wave groups in ping-pong (MI355X_MICROARCH "Two waves per SIMD"): waves 0-3 (group 0, one per SIMD) own
// rows 0-63 of the tile, waves 4-7 (group 1, the other wave of each SIMD) rows 64-127; each wave 32 rows x BN / 2
// columns.  Between two barriers (one per k-chunk t) group 0 reads chunk t's fragments then multiplies them, group 1
// multiplies chunk t-1 (fragments read in the previous interval) then reads chunk t's: while one wave of a SIMD
// waits on LDS, splits fp32 operands or runs its epilogue, its partner keeps the matrix pipe busy.  Chunk t's A
// part is issued NA - 1 intervals ahead (A ring of NA), its B part 2 ahead (B ring of 3, L2-resident weights); a
// wave waits for its own pieces of chunk t with a counted vmcnt (the DMA, epilogue loads and stores it issued
// after them) before the barrier that opens interval t.
template <typename TA, int AM, int EM, int EX, int ACT, int GK, int BN, int BM = XR_BM>
__global__ __launch_bounds__(512, 1) void gemm_nt_x3_ring(Op A, Op B, Epi E, int K, int tilesN, int tilesM, int m_base) {
  constexpr int NA = XR<BN>::NA, RN = XR<BN>::RN, NP = RN / 2, BI = XR<BN>::BI, BSTAGE = XR<BN>::BSTAGE, WC = BN / 2;
  // BM = 128 rows per tile (a wave multiplies 2 row fragments) or 64 (1: twice the tiles for small M -- the B = 4 per-GPU
  // shape of the 8-GPU run has 72 128-row tiles per N-tile for 256 CUs); RI row fragments / A DMA instructions per wave
  constexpr int RI = BM / 64, ASTAGE = BM * 128;
  static_assert(RI == 1 || RI == 2, "64- or 128-row tiles");
  // EX_LNB: + the row-sum exchange of partner waves ([4 row waves][2 column halves][32 rows][2]) and 8 wave flags
  constexpr int XLDS = EX == EX_LNB ? (4 * 2 * 32 * 2 + 8) * 4 : 0;
  // (64-row tiles keep the 5-stage A ring: 9 stages in the same LDS measured B = 4 348 -> 343, profiles/r06_nt_ring_depth_ab.txt)
  __shared__ __attribute__((aligned(16))) char smem[NA * ASTAGE + XR_NB * BSTAGE + BN * 4 + XLDS];
  char* const sA = smem;
  char* const sB = smem + NA * ASTAGE;
  float* const sBias = (float*)(sB + XR_NB * BSTAGE);   // the N-tile's bias (zeros without one), read by the epilogue
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wm = (wave >> 1) & 1, wn = wave & 1;
  const int fr = lane & 15, fq = lane >> 4, q8 = lane & 7;
  const int cta = xcd_remap(blockIdx.x, gridDim.x);
  const int nt = cta % tilesN, mstride = gridDim.x / tilesN, mt0 = cta / tilesN;
  if (mt0 >= tilesM) return;
  const int ntile = (tilesM - mt0 + mstride - 1) / mstride;
  const int nk = K / 32;
  const int total = ntile * nk;
  const int n0 = nt * BN;
  const f16* zero = (const f16*)g_kair_zero_line;

  // epilogue columns (fixed per CTA): after the permlane swap of fragment pair (2p, 2p + 1) a lane owns
  // columns c8[p] .. + 8 of fragment 2p + (fq & 1); their bias, and (QKV) the column part of the offset
  // SW: the 16-bit-output and shuffled forms re-lay fragment pair (2p, 2p + 1) with v_permlane16_swap so a lane owns
  // 8 consecutive columns (16-byte fp16-pair stores); the fp32-row form keeps the MFMA layout, a lane's 4 columns
  // 4 fq .. + 3 of each fragment (16-byte stores; a store instruction covers 64 contiguous bytes of 16 rows).  A
  // lane's 8 values are the two 4-column chunks at c8[p] and c8[p] + CB.
  constexpr bool SW = EM != XE_ROWS_F32;
  constexpr int CB = SW ? 4 : 16;   // the second chunk's column offset
  int c8[NP], oc[NP];
  long colo[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int n = SW ? n0 + wn * WC + (2 * p + (fq & 1)) * 16 + (fq >> 1) * 8 : n0 + wn * WC + 2 * p * 16 + 4 * fq;
    c8[p] = n;
    // this lane's slot (of 8) holding the ones column, or out of [0, 8)
    oc[p] = E.ones_col >= n + CB && E.ones_col < n + CB + 4 ? 4 + E.ones_col - n - CB
                                                            : (E.ones_col >= n && E.ones_col < n + 4 ? E.ones_col - n : -1);
    if constexpr (EM == XE_QKV) {
      const int pw = E.nh * E.hdp;
      const int part = fdiv(n, E.d_pw), rr = n - part * pw;
      const int h = fdiv(rr, E.d_hdp), d = rr - h * E.hdp;
      colo[p] = (long)part * E.M * pw + (long)h * E.tok * E.hdp + d;
    } else if constexpr (EM == XE_PSHUF) {   // column n = (i r + j) nf + c: sub-pixel (i, j) of the row's pixel
      const int nf = E.N / (E.r * E.r), sp = n / nf, c = n - sp * nf, i = sp / E.r, j = sp - i * E.r;
      colo[p] = ((long)i * E.psW * E.r + j) * E.ldo + c;
    } else {
      colo[p] = n;
    }
  }
  // (visible after the first barrier; EX_LNB: the LayerNorm weight over the real channels, zeros beyond)
  for (int i = tid; i < BN; i += 512) sBias[i] = E.bias && n0 + i < (EX == EX_LNB ? E.lnC : E.N) ? E.bias[n0 + i] : 0.f;
  if constexpr (EX == EX_LNB)
    if (tid < 8) ((int*)(sBias + BN + 4 * 2 * 32 * 2))[tid] = 0;
  // B loader: this lane's BI weight rows (fixed for the CTA), unit already swizzled
  const f16* bsrc[BI];
#pragma unroll
  for (int ii = 0; ii < BI; ++ii) {
    const int r = (wave * BI + ii) * 8 + (lane >> 3), u = q8 ^ (r & 7);
    bsrc[ii] = n0 + r < (int)B.M ? (const f16*)B.ptr + (long)(n0 + r) * B.ld + (u < 4 ? u * 8 : 64 + (u - 4) * 8) : nullptr;
  }
  // A loader: this lane's two rows of the tile being loaded
  long aoff[RI];
  int ay[RI], ax[RI], au[RI];
  bool aok[RI];
  auto load_rows = [&](int i) __attribute__((always_inline)) {
    const int mt = mt0 + i * mstride;
#pragma unroll
    for (int ii = 0; ii < RI; ++ii) {
      const int r = (wave * RI + ii) * 8 + (lane >> 3);
      const int m = m_base + mt * BM + r;
      au[ii] = q8 ^ (r & 7);
      aok[ii] = m < (int)A.M;
      const int mm = aok[ii] ? m : 0;
      if constexpr (AM == AM_ROWS) {
        aoff[ii] = (long)win_to_token32(mm, A.win) * A.ld;
      } else {
        const int hw = A.d_hw.d;
        const int b = fdiv(mm, A.d_hw), p = mm - b * hw;
        ay[ii] = fdiv(p, A.d_imW);
        ax[ii] = p - ay[ii] * A.imW;
        aoff[ii] = (long)b * (hw >> (2 * A.up_sh));
      }
    }
  };
  // issue cursors: A chunk (tile at, k-chunk ak, stage as_), B k-chunk bk in stage bs
  int at = 0, ak = 0, as_ = 0, bk = 0, bs = 0;
  // im2col: the current tap and channel offset (k = tap * C + c0, advanced per chunk: K = 9 C, C % 32 == 0) and
  // the lane's two source pixel rows for that tap (nullptr: outside the image / past M), recomputed per tap
  int a_tap = 0, a_c0 = 0;
  const float* arow[RI];
#pragma unroll
  for (int ii = 0; ii < RI; ++ii) arow[ii] = nullptr;
  auto set_tap = [&]() __attribute__((always_inline)) {
    int dy = a_tap / 3 - 1, dx = a_tap - (a_tap / 3) * 3 - 1;
    if (A.flip) { dy = -dy; dx = -dx; }
#pragma unroll
    for (int ii = 0; ii < RI; ++ii) {
      const int y = ay[ii] + dy, x = ax[ii] + dx;
      arow[ii] = aok[ii] && y >= 0 && y < A.imH && x >= 0 && x < A.imW
                     ? (const float*)A.ptr + (aoff[ii] + (long)(y >> A.up_sh) * (A.imW >> A.up_sh) + (x >> A.up_sh)) * A.ld +
                           au[ii] * 4
                     : nullptr;
    }
  };
  auto issue_a = [&]() __attribute__((always_inline)) {
    if (ak == 0) {
      load_rows(at);
      if constexpr (AM == AM_IM2COL) {
        a_tap = 0;
        a_c0 = 0;
        set_tap();
      }
    }
    const int k0 = ak * 32;
    char* st = sA + as_ * ASTAGE;
#pragma unroll
    for (int ii = 0; ii < RI; ++ii) {
      const void* src = zero;
      if constexpr (sizeof(TA) == 2) {
        const f16* pl = (const f16*)(au[ii] < 4 ? A.ptr : A.lo_ptr);
        if (aok[ii]) src = pl + aoff[ii] + k0 + (au[ii] & 3) * 8;
      } else if constexpr (AM == AM_ROWS) {
        if (aok[ii]) src = (const float*)A.ptr + aoff[ii] + k0 + au[ii] * 4;
      } else {
        if (arow[ii]) src = arow[ii] + a_c0;
      }
      if (!KAIR_DBG(E.dbg & 36)) glds16(src, st + (wave * RI + ii) * 1024);
    }
    if constexpr (AM == AM_IM2COL) {
      a_c0 += 32;
      if (a_c0 == A.imC) {
        a_c0 = 0;
        if (++a_tap < 9) set_tap();
      }
    }
    if (++ak == nk) { ak = 0; ++at; }
    if (++as_ == NA) as_ = 0;
  };
  auto issue_b = [&]() __attribute__((always_inline)) {
    const int k0 = bk * 32, kb = (k0 >> 6) * 128 + (k0 & 63);
    char* st = sB + bs * BSTAGE;
#pragma unroll
    for (int ii = 0; ii < BI; ++ii)
      if (!KAIR_DBG(E.dbg & 20)) glds16(bsrc[ii] ? (const void*)(bsrc[ii] + kb) : (const void*)zero, st + (wave * BI + ii) * 1024);
    if (++bk == nk) bk = 0;
    if (++bs == XR_NB) bs = 0;
  };
  // interval u issues A chunk u + NA - 1 and B chunk u + NB - 1 (when in range); the prologue runs the virtual
  // intervals -(NA - 1) .. -1.  nA / nB: the DMA instructions one interval issues.
  auto nA = [&](int u) __attribute__((always_inline)) { return u + NA - 1 >= 0 && u + NA - 1 < total ? RI : 0; };
  auto nB = [&](int u) __attribute__((always_inline)) { return u + XR_NB - 1 >= 0 && u + XR_NB - 1 < total ? BI : 0; };
  for (int u = -(NA - 1); u < 0; ++u) {
    if (nA(u)) issue_a();
    if (nB(u)) issue_b();
  }

  f32x4 acc[RI][RN];
#pragma unroll
  for (int i = 0; i < RI; ++i)
#pragma unroll
    for (int jn = 0; jn < RN; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};
  f16x8 ah[RI], al[RI], bh[RN], bl[RN];   // this wave's fragments of the chunk it multiplies next

  const float as = A.x3s;
  // chunk c's fragments from stages (c % NA, c % NB): A rows of this wave, B columns of this wave
  auto load_frags = [&](int sa, int sb) __attribute__((always_inline)) {
    if (KAIR_DBG(E.dbg & 64)) return;
    const char* stA = sA + sa * ASTAGE;
    const char* stB = sB + sb * BSTAGE;
#pragma unroll
    for (int i = 0; i < RI; ++i) {
      const int r = grp * (BM / 2) + wm * (BM / 4) + i * 16 + fr;
      const char* row = stA + r * 128;
      if constexpr (sizeof(TA) == 2) {
        ah[i] = *(const f16x8*)(row + ((fq ^ (r & 7)) << 4));
        al[i] = *(const f16x8*)(row + (((4 + fq) ^ (r & 7)) << 4));
      } else {
        const float4 x0 = *(const float4*)(row + (((2 * fq) ^ (r & 7)) << 4));
        const float4 x1 = *(const float4*)(row + (((2 * fq + 1) ^ (r & 7)) << 4));
        const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const float w = xv[c] * as;
          ah[i][c] = (f16)w;
          al[i][c] = (f16)(w - (float)ah[i][c]);
        }
      }
    }
#pragma unroll
    for (int jn = 0; jn < RN; ++jn) {
      const int n = wn * WC + jn * 16 + fr;
      const char* row = stB + n * 128;
      bh[jn] = *(const f16x8*)(row + ((fq ^ (n & 7)) << 4));
      bl[jn] = *(const f16x8*)(row + (((4 + fq) ^ (n & 7)) << 4));
    }
  };
  auto mfma_chunk = [&]() __attribute__((always_inline)) {
    if (KAIR_DBG(E.dbg & 2)) return;
#pragma unroll
    for (int i = 0; i < RI; ++i)
#pragma unroll
      for (int jn = 0; jn < RN; ++jn) {
        acc[i][jn] = mfma16(bh[jn], ah[i], acc[i][jn]);
        acc[i][jn] = mfma16(bl[jn], ah[i], acc[i][jn]);
        acc[i][jn] = mfma16(bh[jn], al[i], acc[i][jn]);
      }
  };
  // EX_LNB: the LayerNorm backward of the finished rows (network_swinir.py:199 / :205 norm1 / norm2 backward, as
  // kair_layernorm_bwd): dxn = the GEMM tile (the LayerNorm output's gradient), x / mean / rstd the LayerNorm's
  //   xh = (x - mu) rs,  gy = dxn gamma,  D += rs (gy - mean_c(gy) - xh mean_c(gy xh)),
  // then the optional fp16-pair copy of the finished D row (the next GEMMs' operand) and this row wave's dgamma /
  // dbeta partial sums (sum over its rows of dxn xh, dxn) -- one N-tile holds whole rows (N = 192 >= C).  A lane owns
  // 24 columns (3 chunk pairs, SW = false) of RI rows; the row sums go over the 4 lanes of a row (xor 16, 32) and the
  // partner wave that owns the other 96 columns, exchanged through LDS: each wave writes its sums and a per-tile flag,
  // then waits (s_sleep poll) for its partner's -- both run this epilogue in the same interval.  All loads issue
  // unconditionally (rows clamped), so the returned count is exact; stores as the rows / columns allow.
  auto ln_epilogue = [&](int ct, const int (&rowv)[RI], const bool (&okm)[RI], int nvm) __attribute__((always_inline)) -> int {
    float* const xch = sBias + BN;
    volatile int* const flg = (volatile int*)(xch + 4 * 2 * 32 * 2);
    const int rw = grp * 2 + wm, C = E.lnC;
    const long slot0 = ((long)(m_base / BM + mt0 + ct * mstride) * 4 + rw) * RI;
    long tr[RI];
    float mu[RI], rsd[RI];
#pragma unroll
    for (int i = 0; i < RI; ++i) {
      tr[i] = okm[i] ? rowv[i] : 0;   // (clamped: every load issues)
      mu[i] = E.lnmu[tr[i]];
      rsd[i] = E.lnrs[tr[i]];
    }
    nvm += 2 * RI;
    // phase 1, per row fragment: the row sums of this wave's 96 columns -> LDS, and the fragment's dgamma / dbeta
    // partial row (the sum over its 16 rows = the 16 lanes of a DPP row) -> part[slot]
#pragma unroll
    for (int i = 0; i < RI; ++i) {
      const float* xr = E.lnx + tr[i] * E.lnldx;
      float xh[24];
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float4 q = *(const float4*)(xr + c8[p] + 16 * h);
          xh[p * 8 + h * 4 + 0] = q.x; xh[p * 8 + h * 4 + 1] = q.y;
          xh[p * 8 + h * 4 + 2] = q.z; xh[p * 8 + h * 4 + 3] = q.w;
        }
      nvm += 2 * NP;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < 24; ++j) {
        const int p = j >> 3, h = (j >> 2) & 1, c4 = j & 3, cc = c8[p] + 16 * h + c4;
        const float v = acc[i][2 * p + h][c4] * E.acc_scale;
        xh[j] = cc < C ? (xh[j] - mu[i]) * rsd[i] : 0.f;
        const float gy = v * sBias[cc - n0];
        s1 += gy;
        s2 += gy * xh[j];
      }
      s1 += __shfl_xor(s1, 16);
      s1 += __shfl_xor(s1, 32);
      s2 += __shfl_xor(s2, 16);
      s2 += __shfl_xor(s2, 32);
      if (fq == 0) {
        xch[((rw * 2 + wn) * 32 + i * 16 + fr) * 2] = s1;
        xch[((rw * 2 + wn) * 32 + i * 16 + fr) * 2 + 1] = s2;
      }
      float* const pg = E.lnpart + (slot0 + i) * 2 * C;
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float dg[4], db[4];
#pragma unroll
          for (int c4 = 0; c4 < 4; ++c4) {
            const float v = acc[i][2 * p + h][c4] * E.acc_scale;
            dg[c4] = row16_sum(v * xh[p * 8 + h * 4 + c4]);
            db[c4] = row16_sum(v);
          }
          const int c = c8[p] + 16 * h;
          if (fr == 0 && c < C) {
            *(float4*)(pg + c) = make_float4(dg[0], dg[1], dg[2], dg[3]);
            *(float4*)(pg + C + c) = make_float4(db[0], db[1], db[2], db[3]);
          }
          nvm += n0 + wn * WC + 32 * p + 16 * h < C ? 2 : 0;   // (lane fq = 0's column: at least that lane stores)
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's row sums are in LDS
    if (lane == 0) flg[wave] = ct + 1;
    while (flg[wave ^ 1] != ct + 1) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
    // phase 2, per row fragment and 4-column chunk: the partner's sums, D += dx, the operand copy
#pragma unroll
    for (int i = 0; i < RI; ++i) {
      const volatile float* a0 = xch + ((rw * 2 + 0) * 32 + i * 16 + fr) * 2;
      const volatile float* a1 = xch + ((rw * 2 + 1) * 32 + i * 16 + fr) * 2;
      const float S1 = (a0[0] + a1[0]) / (float)C, S2 = (a0[1] + a1[1]) / (float)C;   // column half 0 + half 1
      float sc = E.cps;
      if (E.cprs) {
        sc *= E.cprs[fdiv((int)tr[i], E.d_cprps)];
        nvm += 1;
      }
      const long cr = E.cpo ? token_to_win(tr[i], E.cpwin) : 0;
      const float* xr = E.lnx + tr[i] * E.lnldx;
      float* const dr = (float*)E.out + tr[i] * E.ldo;
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int c = c8[p] + 16 * h;
          const float4 xq = *(const float4*)(xr + c), dq = *(const float4*)(dr + c);
          const float xa[4] = {xq.x, xq.y, xq.z, xq.w}, da[4] = {dq.x, dq.y, dq.z, dq.w};
          float o[4];
#pragma unroll
          for (int c4 = 0; c4 < 4; ++c4) {
            const int cc = c + c4;
            const float v = acc[i][2 * p + h][c4] * E.acc_scale;
            const float xhat = (xa[c4] - mu[i]) * rsd[i];
            o[c4] = da[c4] + (cc < C ? rsd[i] * (v * sBias[cc - n0] - S1 - xhat * S2) : 0.f);
          }
          if (okm[i]) {
            *(float4*)(dr + c) = make_float4(o[0], o[1], o[2], o[3]);
            if (E.cpo) {
              f16x4 hi, lo;
#pragma unroll
              for (int c4 = 0; c4 < 4; ++c4) {
                const float w = opaque(o[c4] * sc);   // (common.h opaque: no fused conversion)
                hi[c4] = (f16)w;
                lo[c4] = (f16)(w - (float)hi[c4]);
              }
              *(f16x4*)((f16*)E.cpo + cr * E.cpld + c) = hi;
              *(f16x4*)((f16*)E.cplo + cr * E.cpld + c) = lo;
            }
          }
        }
      nvm += 4 * NP + (__ballot(okm[i]) != 0 ? 2 * NP * (E.cpo ? 3 : 1) : 0);
    }
#pragma unroll
    for (int i = 0; i < RI; ++i)
#pragma unroll
      for (int jn = 0; jn < RN; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};
    return nvm;
  };
  // multiply the fragments in registers into acc; the tile's last chunk also runs its epilogue, its operands
  // loaded after the MFMAs (the partner group's phase covers their latency) and used in the same straight-line
  // branch (no control-flow merge between a load and its use: hipcc never holds a pending load across the loop
  // back-edge).
  // Returns the vector-memory instructions issued (epilogue loads + the stores that MUST issue: rows with at least
  // one valid lane in the wave -- a compiler that also issues fully masked ones only makes later waits stricter).
  auto compute = [&](bool tile_end, int ct) __attribute__((always_inline)) -> int {
    if (!tile_end || KAIR_DBG(E.dbg & 1)) {
      mfma_chunk();
      return 0;
    }
    int nvm = 0;
    int rowv[RI];
    long roff[RI];   // the shuffled forms' row part of the store offset
    bool okm[RI];
    const int m0 = m_base + (mt0 + ct * mstride) * BM + grp * (BM / 2) + wm * (BM / 4) + fr;
#pragma unroll
    for (int i = 0; i < RI; ++i) {
      const int m = m0 + i * 16;
      okm[i] = m < (int)E.M;
      const int mm = okm[i] ? m : 0;
      roff[i] = 0;
      if constexpr (EM == XE_QKV) {
        const int win = fdiv(mm, E.d_tok);
        rowv[i] = win * E.nh * E.tok + (mm - win * E.tok);
      } else if constexpr (EM == XE_PSHUF) {   // pixel (b, y, x) of [psH, psW] -> (b, y r, x r) of the r-times image
        const int hw = E.psH * E.psW, b = mm / hw, pp = mm - b * hw, y = pp / E.psW, x = pp - y * E.psW;
        rowv[i] = mm;
        roff[i] = (((long)b * E.psH * E.r + (long)y * E.r) * ((long)E.psW * E.r) + (long)x * E.r) * E.ldo;
      } else if constexpr (EM == XE_PUNSHUF) {   // pixel (b, Y, X) of the r-times image -> row (b, Y/r, X/r), block (Y%r, X%r)
        const int Wr = E.psW * E.r, HWr = E.psH * E.r * Wr, b = mm / HWr, pp = mm - b * HWr, Y = pp / Wr, X = pp - Y * Wr;
        const int y = Y / E.r, x = X / E.r;
        rowv[i] = mm;
        roff[i] = (((long)b * E.psH + y) * E.psW + x) * E.ldo + (long)((Y - y * E.r) * E.r + (X - x * E.r)) * E.N;
      } else {
        rowv[i] = win_to_token32(mm, E.win);
      }
    }
    mfma_chunk();   // (the fragments die here: the epilogue operands load after it, under the partner's work)
    if constexpr (EX == EX_LNB) return ln_epilogue(ct, rowv, okm, nvm);
    float4 ex[RI][NP][2];
    float rs[RI];
#pragma unroll
    for (int i = 0; i < RI; ++i) rs[i] = 1.f;
    if constexpr (EX != EX_NONE) {
#pragma unroll
      for (int i = 0; i < RI; ++i)
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          const float* src = EX == EX_RESID ? E.resid + (long)rowv[i] * E.ldr : (const float*)E.gate + (long)rowv[i] * E.ldg;
          ex[i][p][0] = *(const float4*)(src + c8[p]);
          ex[i][p][1] = *(const float4*)(src + c8[p] + CB);
        }
      nvm += 2 * RI * NP;
    }
    if constexpr (EX == EX_RESID) {
      const bool hs = E.rowscale != nullptr;
#pragma unroll
      for (int i = 0; i < RI; ++i) {
        const float r = *(hs ? E.rowscale + fdiv(rowv[i], E.d_rps) : (const float*)g_kair_zero_line);
        rs[i] = hs ? r : 1.f;
      }
      nvm += RI;
    }
    const int nst = EM == XE_ROWS_F32 ? (E.pre ? 4 : 2) : (E.out_lo ? 2 : 1) + (EM == XE_ROWS_PAIR && E.pre ? 2 : 0);
#pragma unroll
    for (int i = 0; i < RI; ++i) nvm += __ballot(okm[i]) != 0 ? NP * nst : 0;
#pragma unroll
    for (int i = 0; i < RI; ++i)
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        float v[8];
        const float4 b0 = *(const float4*)(sBias + c8[p] - n0), b1 = *(const float4*)(sBias + c8[p] + CB - n0);
        const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if constexpr (SW) {
            const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * p][c]),
                                                            __float_as_uint(acc[i][2 * p + 1][c]), false, false);
            v[c] = __uint_as_float(r[0]) * E.acc_scale + bv[c];
            v[4 + c] = __uint_as_float(r[1]) * E.acc_scale + bv[4 + c];
          } else {
            v[c] = acc[i][2 * p][c] * E.acc_scale + bv[c];
            v[4 + c] = acc[i][2 * p + 1][c] * E.acc_scale + bv[4 + c];
          }
        }
        const int n = c8[p];
        if constexpr (EM == XE_QKV) {
          if (okm[i]) store8_f16pair(E.out, E.out_lo, colo[p] + (long)rowv[i] * E.hdp, v, E.oscale);
        } else {
          float pre[8];
#pragma unroll
          for (int c = 0; c < 8; ++c) pre[c] = v[c];
          if constexpr (ACT == XA_GELU) {   // GELU and GELU' of element pairs (packed fp32 polynomials)
#pragma unroll
            for (int c = 0; c < 8; c += 2) {
              f32x2 y2, d2;
              gelu_erf_pair2((f32x2){v[c], v[c + 1]}, y2, d2);
              v[c] = y2.x;
              v[c + 1] = y2.y;
              pre[c] = d2.x;
              pre[c + 1] = d2.y;
            }
          } else if constexpr (ACT == XA_GELU_X) {
#pragma unroll
            for (int c = 0; c < 8; c += 2) {
              const f32x2 x2 = {v[c], v[c + 1]};
              const f32x2 y2 = x2 * (0.5f * (1.0f + erf_f32x2(x2 * 0.70710678118654752f)));
              v[c] = y2.x;
              v[c + 1] = y2.y;
            }
          } else if constexpr (ACT == XA_LEAKY) {
#pragma unroll
            for (int c = 0; c < 8; ++c) v[c] = v[c] > 0.f ? v[c] : v[c] * E.slope;
          }
          if constexpr (EX != EX_NONE) {
            const float x8[8] = {ex[i][p][0].x, ex[i][p][0].y, ex[i][p][0].z, ex[i][p][0].w,
                                 ex[i][p][1].x, ex[i][p][1].y, ex[i][p][1].z, ex[i][p][1].w};
#pragma unroll
            for (int c = 0; c < 8; ++c) {
              if constexpr (EX == EX_RESID) v[c] = x8[c] + rs[i] * v[c];
              else if constexpr (GK == XG_MUL) v[c] *= x8[c];
              else v[c] *= (x8[c] > 0.f ? 1.f : E.slope);
            }
          }
#pragma unroll
          for (int c = 0; c < 8; ++c) v[c] = c == oc[p] ? 1.f : v[c];   // the ones column (lane-varying select)
          const long rr = rowv[i];
          // (ablation bit 128: every value computed, no store issued -- the store path's share of the epilogue)
          const bool st = !KAIR_DBG(E.dbg & 128) || v[0] == 1.2345e-30f;
          if (okm[i] && st) {
            if constexpr (EM == XE_ROWS_PAIR) {
              store8_f16pair(E.out, E.out_lo, rr * E.ldo + n, v, E.oscale);
            } else {
              float* d = (float*)E.out + (EM == XE_PSHUF || EM == XE_PUNSHUF ? roff[i] + colo[p] : rr * E.ldo + n);
              *(float4*)d = make_float4(v[0], v[1], v[2], v[3]);
              *(float4*)(d + CB) = make_float4(v[4], v[5], v[6], v[7]);
            }
            if (E.pre) {
              float* d = (float*)E.pre + rr * E.ldp + n;
              *(float4*)d = make_float4(pre[0], pre[1], pre[2], pre[3]);
              *(float4*)(d + CB) = make_float4(pre[4], pre[5], pre[6], pre[7]);
            }
          }
        }
      }
#pragma unroll
    for (int i = 0; i < RI; ++i)
#pragma unroll
      for (int jn = 0; jn < RN; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};
    return nvm;
  };

  const bool stamping = KAIR_DBG(E.dbg & 8) && blockIdx.x < XS_CTAS;
  unsigned long long* stp = g_x3_stamps + ((long)blockIdx.x * 8 + wave) * XS_IT * XS_N;
  auto stamp = [&](int t, int k) __attribute__((always_inline)) {
    if (stamping && t < XS_IT) {
      const unsigned long long tt = x3_now();
      if (lane == 0) stp[t * XS_N + k] = tt;
    }
  };
  // The interval loop, specialised per group (a run-time group test would keep every register of both roles
  // live across the loop).  Consumer state: the chunk this wave multiplies next (k-chunk kc of tile ct) and the
  // stages of the chunk whose fragments it reads next.  Both loops pass the same barriers (one per interval).
  auto run = [&](auto G) __attribute__((always_inline)) {
    constexpr int g = decltype(G)::value;
    int kc = 0, ct = 0, ra = 0, rb = 0;
    int e1 = 0, e2 = 0;   // non-DMA vector-memory instructions this wave issued in intervals t-1, t-2
    for (int t = 0; t <= total; ++t) {
      stamp(t, 0);
      if (t < total) {   // chunk t (its B part: issued in interval t-2)
        const int n = e2 + nA(t - 1) + nB(t - 1) + e1;
        if (n == RI + BI) {   // the steady state (no epilogue stores pending): one immediate wait, not the branch tree
          if constexpr (RI + BI == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
          else if constexpr (RI + BI == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
          else if constexpr (RI + BI == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        } else {
          vm_wait(n);
        }
      }
      stamp(t, 1);
      ring_barrier();   // chunk t is in LDS for every wave; chunk t-1's stages are free
      if (nA(t)) issue_a();
      if (nB(t)) issue_b();
      stamp(t, 2);
      int e0 = 0;
      if constexpr (g == 0) {   // read chunk t, multiply it
        if (t < total) {
          load_frags(ra, rb);
          stamp(t, 3);
          e0 = compute(kc == nk - 1, ct);
          if (++kc == nk) { kc = 0; ++ct; }
        }
      } else {                  // multiply chunk t-1, read chunk t
        if (t >= 1) {
          e0 = compute(kc == nk - 1, ct);
          if (++kc == nk) { kc = 0; ++ct; }
        }
        stamp(t, 3);
        if (t < total) load_frags(ra, rb);
      }
      if (t < total) {
        if (++ra == NA) ra = 0;
        if (++rb == XR_NB) rb = 0;
      }
      stamp(t, 4);
      e2 = e1;
      e1 = e0;
    }
  };
  if (grp == 0) {
    run(std::integral_constant<int, 0>{});
  } else {
    // the second-dispatched half loses VALU arbitration to its SIMD partner by age; a static raise evens it
    // (MI355X_MICROARCH "Two waves per SIMD", item 4)
    __builtin_amdgcn_s_setprio(1);
    run(std::integral_constant<int, 1>{});
  }
}

// ------------------------------------------------------------------------------------------
// TN ring (x3): the weight gradients of the Swin linears and the 192-channel 3x3 convs from fp32 operands.
//   P[s][n][k] = sum_{m in split s} A[m][n] B[m][k],  one 192 x 192 (n, k) tile per CTA, one CTA per CU.
// A and B row chunks (32 rows x 192 fp32 columns, 24 KiB each) stream through an XR_TNS-deep LDS ring by
// LDS-DMA; 16-byte unit u of chunk row r sits at slot u ^ (((r >> 3) & 3) << 2), so a fragment's column
// read (8 rows per 16-lane group, the four groups 8 rows apart) touches 64 distinct banks.  Fragments are
// eight ds_read_b32 down a column, split into the fp16 pair at the read (each operand's 2^e); D = B^T A,
// so each lane stores 4 consecutive k (16 B).  8 waves as 2 (n) x 4 (k), wave tile 96 x 48.
// BT_TAP: B is the 3x3 / pad-1 im2col of a 192-channel map and K-tile tk IS tap tk (row m reads pixel
// m + dy W + dx; a zero line outside the image): the conv weight gradient reads each operand ~once.
// Rows past the split read a zero line.  B's bias "ones" column must already be in the data.
// ------------------------------------------------------------------------------------------
constexpr int XT_RB = 32, XT_NS = 3;
constexpr int XT_PART = XT_RB * 192 * 4, XT_STAGE = 2 * XT_PART;   // 24 + 24 KiB
constexpr int XT_DMA = 6;   // DMA wave-instructions per wave per chunk (3 A + 3 B)
static_assert(XT_DMA * (XT_NS - 2) == 6, "the steady-state wait immediate in gemm_tn_x3_ring");
enum { BT_ROWS = 0, BT_TAP = 1 };

// PR (BT_ROWS only): A and B are fp16 pairs (hi plane ptr, lo plane lo_ptr, values x 2^e): a chunk row holds the
// 192 hi columns in logical units 0..23 and the 192 lo columns in units 24..47 (8 halves per unit), unit u at slot
// u ^ xt_swz_pair(r); fragments are two ds_read_b64_tr_b16 per plane (the 4 x 16 transposed read: a lane's 8
// halves are column lane & 15 over rows 8 (lane >> 4) .. + 7), so no split at the read.  The swizzle spreads the
// four rows of one transposed read over four 8-bank groups and the two 16-lane halves of a 32-lane group over
// the two bank halves: conflict-free.
KAIR_DEV int xt_swz_pair(int r) { return ((r & 3) << 1) | (((r >> 3) & 1) << 3); }

// one CTA's (tile, split) of the TN ring: the launch forms below (one product, or a group of them) pick its operands
template <int BT, bool PR>
KAIR_DEV void tn_x3_body(const Op& A, const Op& B, float* ws, int M, int N, int K, int tilesK, int tile, int split, int rps,
                         float acc_scale, char* smem) {
  static_assert(!PR || BT == BT_ROWS, "fp16-pair operands: row operands only");
  constexpr int ES = PR ? 2 : 4;   // operand element bytes
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave >> 2, wk = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const int n0 = (tile / tilesK) * 192, k0 = (tile % tilesK) * 192;
  const int mbeg = split * rps;
  const int mend = mbeg + rps < M ? mbeg + rps : M;
  const int nch = mbeg < mend ? (mend - mbeg + XT_RB - 1) / XT_RB : 0;
  const char* zero = (const char*)g_kair_zero_line;

  // DMA geometry of this lane (the same for every chunk): wave-instruction g covers slots [64 g, 64 g + 64)
  // tap form: the lane's 4 columns k .. k + 3 of the K = 9 C contraction are channels c .. c + 3 of tap k / C (C % 4
  // == 0), so each lane reads ONE shifted image (its own dy, dx) for the whole launch
  // pair form: the lane's 8 columns of one plane (pl = 0 hi, 1 lo)
  int dr[3], dcA[3], dcB[3], dy[3], dx[3];
  const char* baseA[3];
  const char* baseB[3];
#pragma unroll
  for (int ii = 0; ii < 3; ++ii) {
    const int s = (wave * 3 + ii) * 64 + lane;
    const int r = s / 48, q = s - r * 48;
    dr[ii] = r;
    dy[ii] = dx[ii] = 0;
    if constexpr (PR) {
      const int u = q ^ xt_swz_pair(r);
      const int pl = u >= 24 ? 1 : 0, col = (u - 24 * pl) * 8;
      dcA[ii] = n0 + col < N ? n0 + col : -1;
      dcB[ii] = k0 + col < K ? k0 + col : -1;
      baseA[ii] = (const char*)(pl ? A.lo_ptr : A.ptr);
      baseB[ii] = (const char*)(pl ? B.lo_ptr : B.ptr);
    } else {
      const int u = q ^ (((r >> 3) & 3) << 2);
      dcA[ii] = n0 + u * 4 < N ? n0 + u * 4 : -1;
      const int k = k0 + u * 4;
      baseA[ii] = (const char*)A.ptr;
      baseB[ii] = (const char*)B.ptr;
      if constexpr (BT == BT_TAP) {
        const int tap = k < K ? k / B.imC : 0;
        dcB[ii] = k < K ? k - tap * B.imC : -1;
        dy[ii] = tap / 3 - 1;
        dx[ii] = tap - (tap / 3) * 3 - 1;
      } else {
        dcB[ii] = k < K ? k : -1;
      }
    }
  }
  int lc = 0, ls = 0;   // next chunk to issue, its stage
  // Identity row maps (the engine's operands: both in token order or both in window order): each lane's three
  // source rows advance by XT_RB rows per chunk, so the addresses are kept as running pointers (and, for the
  // tap form, the row's pixel column / row for the halo test) instead of being rebuilt per chunk
  const bool lin = A.win.ws == 0 && (BT == BT_TAP || B.win.ws == 0);
  const char* pa[3];
  const char* pb[3];
  int px[3], py[3];
#pragma unroll
  for (int ii = 0; ii < 3; ++ii) {
    const long m = mbeg + dr[ii];
    pa[ii] = baseA[ii] + (m * A.ld + (dcA[ii] >= 0 ? dcA[ii] : 0)) * ES;
    if constexpr (BT == BT_ROWS) {
      pb[ii] = baseB[ii] + (m * B.ld + (dcB[ii] >= 0 ? dcB[ii] : 0)) * ES;
      px[ii] = py[ii] = 0;
    } else {
      const int mm = m < M ? (int)m : 0;
      const int p = mm - fdiv(mm, B.d_hw) * B.d_hw.d;
      py[ii] = fdiv(p, B.d_imW);
      px[ii] = p - py[ii] * B.imW;
      pb[ii] = baseB[ii] + ((m + (long)dy[ii] * B.imW + dx[ii]) * B.ld + (dcB[ii] >= 0 ? dcB[ii] : 0)) * ES;
    }
  }
  auto issue_next = [&]() {
    char* st = smem + ls * XT_STAGE;
    const int m0 = mbeg + lc * XT_RB;
#pragma unroll
    for (int ii = 0; ii < 3; ++ii) {
      const int m = m0 + dr[ii];
      const bool ok = m < mend;
      const void* sa = zero;
      const void* sb = zero;
      if (lin) {
        if (ok && dcA[ii] >= 0) sa = pa[ii];
        if constexpr (BT == BT_ROWS) {
          if (ok && dcB[ii] >= 0) sb = pb[ii];
        } else {
          const int yy = py[ii] + dy[ii], xx = px[ii] + dx[ii];
          if (ok && dcB[ii] >= 0 && yy >= 0 && yy < B.imH && xx >= 0 && xx < B.imW) sb = pb[ii];
          px[ii] += XT_RB;
          while (px[ii] >= B.imW) {   // (once per chunk for image widths >= 32)
            px[ii] -= B.imW;
            if (++py[ii] == B.imH) py[ii] = 0;
          }
        }
        pa[ii] += (long)XT_RB * A.ld * ES;
        pb[ii] += (long)XT_RB * B.ld * ES;
      } else {
        const int mm = ok ? m : 0;
        if (ok && dcA[ii] >= 0) sa = baseA[ii] + ((long)win_to_token32(mm, A.win) * A.ld + dcA[ii]) * ES;
        if constexpr (BT == BT_ROWS) {
          if (ok && dcB[ii] >= 0) sb = baseB[ii] + ((long)win_to_token32(mm, B.win) * B.ld + dcB[ii]) * ES;
        } else {
          const int hw = B.d_hw.d;
          const int b = fdiv(mm, B.d_hw), p = mm - b * hw;
          const int y = fdiv(p, B.d_imW), x = p - y * B.imW;
          const int yy = y + dy[ii], xx = x + dx[ii];
          if (ok && dcB[ii] >= 0 && yy >= 0 && yy < B.imH && xx >= 0 && xx < B.imW)
            sb = baseB[ii] + (((long)b * hw + (long)yy * B.imW + xx) * B.ld + dcB[ii]) * ES;
        }
      }
      glds16(sa, st + (wave * 3 + ii) * 1024);
      glds16(sb, st + XT_PART + (wave * 3 + ii) * 1024);
    }
    ++lc;
    if (++ls == XT_NS) ls = 0;
  };

#pragma unroll
  for (int j = 0; j < XT_NS - 1; ++j)
    if (lc < nch) issue_next();

  f32x4 acc[3][6];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const float sa = A.x3s, sb = B.x3s;
  // B's injected ones column (the bias gradient of a conv weight gradient: k = ones_col reads 1.0 for every row,
  // whatever the data / halo there), as its K-tile column (-1: none in this tile)
  const int bones = !PR && B.ones_col >= 0 && !B.ones_in_data && B.ones_col >= k0 && B.ones_col < k0 + 192 ? B.ones_col - k0 : -1;
  // a lane's column c of a chunk part: byte (fq * 8 + j) * 768 + slot(c) * 16 + (c & 3) * 4 for rows j = 0..7
  auto frag = [&](const char* part, int c, float s, f16x8& hi, f16x8& lo) {
    const char* p = part + fq * 8 * 768 + ((((c >> 2) ^ (fq << 2))) << 4) + (c & 3) * 4;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float w = *(const float*)(p + j * 768) * s;
      hi[j] = (f16)w;
      lo[j] = (f16)(w - (float)hi[j]);
    }
  };
  // pair form: the 16-column fragment at column cb (% 16 == 0) of plane pl: rows 8 fq + q4 and + 4 (q4 = (lane & 15) >> 2),
  // columns cb + 4 (lane & 3) .. + 3 in each 4 x 16 transposed read
  const int q4 = (lane & 15) >> 2, p4 = (lane & 3) * 4;
  auto frag_tr = [&](const char* part, int pl, int cb) -> f16x8 {
    const int c = cb + p4, u = pl * 24 + (c >> 3), ob = (c & 7) * 2;
    const int r0 = fq * 8 + q4, r1 = r0 + 4;
    const char* a0 = part + r0 * 768 + ((u ^ xt_swz_pair(r0)) << 4) + ob;
    const char* a1 = part + r1 * 768 + ((u ^ xt_swz_pair(r1)) << 4) + ob;
    const short4v x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)a0);
    const short4v y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)a1);
    short __attribute__((ext_vector_type(8))) s8 = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
    return __builtin_bit_cast(f16x8, s8);
  };
  int cs = 0;
  for (int j = 0; j < nch; ++j) {
    const int ahead = (nch - 1 - j) < (XT_NS - 2) ? (nch - 1 - j) : (XT_NS - 2);
    if (ahead == XT_NS - 2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // XT_DMA * (XT_NS - 2): steady state
    else vm_wait(XT_DMA * ahead);
    ring_barrier();   // chunk j in LDS for every wave; stage (j - 1) % NS free
    if (lc < nch) issue_next();
    const char* st = smem + cs * XT_STAGE;
    f16x8 ah[6], al[6], bh[3], bl[3];
    if constexpr (PR) {
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        ah[i] = frag_tr(st, 0, wn * 96 + i * 16);
        al[i] = frag_tr(st, 1, wn * 96 + i * 16);
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        bh[i] = frag_tr(st + XT_PART, 0, wk * 48 + i * 16);
        bl[i] = frag_tr(st + XT_PART, 1, wk * 48 + i * 16);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 6; ++i) frag(st, wn * 96 + i * 16 + fr, sa, ah[i], al[i]);
#pragma unroll
      for (int i = 0; i < 3; ++i) frag(st + XT_PART, wk * 48 + i * 16 + fr, sb, bh[i], bl[i]);
      if (bones >= 0) {   // (uniform: only the K tile holding the ones column) its lanes' fragment reads 1.0 in every row
        const f16 oh = (f16)sb, ol = (f16)(sb - (float)oh);
#pragma unroll
        for (int i = 0; i < 3; ++i)
          if (wk * 48 + i * 16 + fr == bones) {
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
              bh[i][jj] = oh;
              bl[i][jj] = ol;
            }
          }
      }
    }
#pragma unroll
    for (int ik = 0; ik < 3; ++ik)
#pragma unroll
      for (int in = 0; in < 6; ++in) {
        acc[ik][in] = mfma16(bh[ik], ah[in], acc[ik][in]);
        acc[ik][in] = mfma16(bl[ik], ah[in], acc[ik][in]);
        acc[ik][in] = mfma16(bh[ik], al[in], acc[ik][in]);
      }
    if (++cs == XT_NS) cs = 0;
  }
  float* P = ws + (long)split * N * K;
#pragma unroll
  for (int ik = 0; ik < 3; ++ik)
#pragma unroll
    for (int in = 0; in < 6; ++in) {
      const int k = k0 + wk * 48 + ik * 16 + fq * 4, n = n0 + wn * 96 + in * 16 + fr;
      if (n < N && k < K)
        *(float4*)(P + (long)n * K + k) = make_float4(acc[ik][in][0] * acc_scale, acc[ik][in][1] * acc_scale,
                                                      acc[ik][in][2] * acc_scale, acc[ik][in][3] * acc_scale);
    }
}

template <int BT, bool PR>
__global__ __launch_bounds__(512, 1) void gemm_tn_x3_ring(Op A, Op B, float* ws, int M, int N, int K, int tilesK, int ntiles,
                                                         int rps, float acc_scale) {
  __shared__ __attribute__((aligned(16))) char smem[XT_NS * XT_STAGE];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  tn_x3_body<BT, PR>(A, B, ws, M, N, K, tilesK, bid % ntiles, bid / ntiles, rps, acc_scale, smem);
}

// Grouped form (kair_wgrad_grouped with fp16-pair operands): the weight gradients of several Swin linears -- an
// RSTB's, queued for the side stream -- in ONE launch.  Every job is a pair-row product P = A^T B over the same M rows
// in `splits` row ranges; CTA -> (split, global tile), the job found by a scalar scan of the tile offsets.  One launch
// instead of one per linear: the partial planes are (CTAs x one tile) for the whole group rather than per linear (an
// RSTB's 24 linears at B = 32: 28 MB instead of 24 x 28 MB written and read back by the finalize), and small batches
// get long enough workgroups.  The job table is the kernel argument (captured by value).
struct TnX3Job {
  const void* ah; const void* al; const void* bh; const void* bl;   // hi / lo planes of A (gradient) and B (activation)
  float* ws;                                                        // this job's [splits][N][K] partial planes
  long lda, ldb;
  int N, K, tilesK, tile0;
  float acc_scale;
};
struct TnX3Group {
  TnX3Job j[KAIR_WG_MAX];
  int njobs, ntiles, M, rps;
};

__global__ __launch_bounds__(512, 1) void gemm_tn_x3_ring_grouped(const TnX3Group g) {
  __shared__ __attribute__((aligned(16))) char smem[XT_NS * XT_STAGE];
  const int cta = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = cta % g.ntiles, split = cta / g.ntiles;
  int ji = 0;
  for (int i = 1; i < g.njobs; ++i)
    if (g.j[i].tile0 <= tile) ji = i;
  ji = __builtin_amdgcn_readfirstlane(ji);
  const TnX3Job& jb = g.j[ji];
  Op a{}, b{};   // the fields the pair-row body reads: planes, strides, no window map / ones column
  a.ptr = jb.ah; a.lo_ptr = jb.al; a.ld = jb.lda; a.ones_col = -1; a.x3s = 1.f;
  b.ptr = jb.bh; b.lo_ptr = jb.bl; b.ld = jb.ldb; b.ones_col = -1; b.x3s = 1.f;
  tn_x3_body<BT_ROWS, true>(a, b, jb.ws, g.M, jb.N, jb.K, jb.tilesK, tile - jb.tile0, split, g.rps, jb.acc_scale, smem);
}


int g_x3_cus = 0;
int x3_cus() {
  if (g_x3_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      g_x3_cus = n;
    if (g_x3_cus <= 0) g_x3_cus = 256;
  }
  return g_x3_cus;
}

template <typename TA, int AM, int BM, int BN>
int launch_nt_x3(const Op& A, const Op& B, const Epi& E, long M, int N, int K, hipStream_t s) {
  const long tilesM = (M + BM - 1) / BM;
  const int tilesN = (N + BN - 1) / BN;
  const long nwg = tilesM * tilesN;
  if (nwg > 0x7fffffff) return kair_set_error(KAIR_ERR_ARG, "gemm_nt x3: grid too large");
  KAIR_LAUNCH((gemm_nt_x3_kernel<TA, AM, BM, BN>), dim3((unsigned)nwg), dim3(NT), 0, s, A, B, E, K, tilesN, (int)nwg);
  KAIR_CHECK_LAUNCH();
  return 0;
}

// tile: 32 / 64 / 128 columns by N; 128 rows, 64 when that leaves fewer than two workgroups per CU
template <typename TA, int AM>
int nt_x3_tiles(const Op& A, const Op& B, const Epi& E, long M, int N, int K, hipStream_t s) {
  const long min_wg = 2L * x3_cus();
  if (N <= 32) return launch_nt_x3<TA, AM, 128, 32>(A, B, E, M, N, K, s);
  if (N <= 64) {
    if ((M + 127) / 128 >= min_wg) return launch_nt_x3<TA, AM, 128, 64>(A, B, E, M, N, K, s);
    return launch_nt_x3<TA, AM, 64, 64>(A, B, E, M, N, K, s);
  }
  if ((M + 127) / 128 * ((N + 127) / 128) >= min_wg) return launch_nt_x3<TA, AM, 128, 128>(A, B, E, M, N, K, s);
  return launch_nt_x3<TA, AM, 64, 128>(A, B, E, M, N, K, s);
}

template <typename TA, typename TB, int AMB>
int launch_tn_x3(const Op& a, const Op& b, float* ws, int splits, long M, int N, int K, long rps, float acc_scale,
                 hipStream_t s) {
  if (N <= 64 && K <= 64) {
    KAIR_LAUNCH((gemm_tn_x3_kernel<TA, TB, AMB, 64, 64>), dim3(1, splits), dim3(NT), 0, s, a, b, ws, M, N, K, rps, 1,
                       acc_scale);
  } else {
    const int tilesN = (N + 127) / 128, tilesK = (K + 127) / 128;
    KAIR_LAUNCH((gemm_tn_x3_kernel<TA, TB, AMB, 128, 128>), dim3(tilesN * tilesK, splits), dim3(NT), 0, s, a, b, ws,
                       M, N, K, rps, tilesK, acc_scale);
  }
  KAIR_CHECK_LAUNCH();
  return 0;
}

template <typename TA>
int tn_x3_b(const Op& a, const Op& b, int bmode, int bdt, float* ws, int splits, long M, int N, int K, long rps,
            float acc_scale, hipStream_t s) {
  if (bmode == KAIR_LD_ROWS)
    return bdt == KAIR_F16 ? launch_tn_x3<TA, f16, AM_ROWS>(a, b, ws, splits, M, N, K, rps, acc_scale, s)
                           : launch_tn_x3<TA, float, AM_ROWS>(a, b, ws, splits, M, N, K, rps, acc_scale, s);
  return bdt == KAIR_F16 ? launch_tn_x3<TA, f16, AM_IM2COL>(a, b, ws, splits, M, N, K, rps, acc_scale, s)
                         : launch_tn_x3<TA, float, AM_IM2COL>(a, b, ws, splits, M, N, K, rps, acc_scale, s);
}

// the ring's N-tile for N columns (0: none): 192 for multiples of 192, else one tile of 64 or tiles of 128
int nt_x3_ring_bn(int N) {
  if (N % 192 == 0) return 192;
  if (N == 64) return 64;
  return N % 128 == 0 ? 128 : 0;
}

// the ring takes N-tiles of 192 columns, 32-deep k-chunks (im2col: one tap per chunk) and 16-byte aligned rows
bool nt_x3_ring_ok(const kair_operand* A, const kair_operand* B, const kair_epilogue* E, int N, int K) {
  static const int off = [] { const char* e = getenv("KAIR_X3_RING"); return e && e[0] == '0'; }();
  if (off || nt_x3_ring_bn(N) == 0 || K % 32 != 0 || (uintptr_t)B->ptr % 16 != 0 || (uintptr_t)A->ptr % 16 != 0) return false;
  // epilogues: fp32 rows (bias, activation [+ pre], residual [x row scale] or fp32 gate, ones column) or fp16
  // pair rows / head-blocked q, k, v (bias); 16-byte aligned rows throughout
  const bool pair = E->out_dtype == KAIR_F16;
  if (E->out_mode == KAIR_OUT_PSHUF_SPM || E->out_mode == KAIR_OUT_PUNSHUF_SPM) {   // fp32, bias only
    const int r = E->ps_r;
    if (pair || E->act || E->out_pre || E->resid || E->gate || E->rowscale || E->resid2 || E->a_copy || E->out_lo ||
        E->out_ones_col_p1 > 0 || E->win_ws || r < 1 || E->ldo % 4 || (uintptr_t)E->out % 16 || N % 8 ||
        nt_x3_ring_bn(N) != 128)   // 128-column tiles only: the x4 upsampling convs' forward (N = 256; 64-column
                                   // tiles lose to the generic kernel at K = 2,304: 799 vs 546 us in-step)
      return false;
    if (E->out_mode == KAIR_OUT_PSHUF_SPM && (N % (r * r) || (N / (r * r)) % 8)) return false;
  } else if (E->out_mode == KAIR_OUT_QKVBLK) {
    if (nt_x3_ring_bn(N) != 192 || !pair || E->qkv_hdp % 8 || (uintptr_t)E->out % 16 || E->act || E->out_pre || E->resid || E->gate || E->rowscale) return false;
  } else {
    if (E->out_mode != KAIR_OUT_ROWS || E->ldo % 4 || (uintptr_t)E->out % 16) return false;
    if (E->resid2 || E->a_copy || (E->resid && E->gate)) return false;
    // fp16-pair rows: plain (bias), GELU with its fp32 GELU' (the fc1 forward: h as the fc2 operand pair), or the
    // fp32 multiply gate (the fc2 input gradient: dU as the fc1 dgrad / wgrad operand pair)
    if (pair && (E->resid || E->ldo % 8 || (E->act && (E->act != KAIR_ACT_GELU || !E->pre_kind || !E->out_pre)) ||
                 (E->out_pre && !E->act) || (E->gate && E->gate_kind != XG_MUL)))
      return false;
    if (E->out_pre && (E->pre_dtype != KAIR_F32 || E->ldp % 4 || (uintptr_t)E->out_pre % 16)) return false;
    if (E->resid && (E->ldr % 4 || (uintptr_t)E->resid % 16)) return false;
    if (E->gate && (E->gate_dtype != KAIR_F32 || E->ldg % 4 || (uintptr_t)E->gate % 16)) return false;
    if (E->rowscale && !E->resid) return false;
    // the instantiated forms: activation (GELU / LeakyReLU) only without residual / gate; gates 4 (multiply) and 2
    if (E->act && (E->resid || E->gate || (E->act != KAIR_ACT_GELU && E->act != KAIR_ACT_LEAKY))) return false;
    if (E->gate && E->gate_kind != XG_MUL && E->gate_kind != XG_LEAKY) return false;
    if (nt_x3_ring_bn(N) != 192 &&   // the 64 / 128 / 256-column tiles carry the tail's forms only
        (pair || E->resid || E->out_pre || (E->gate && E->gate_kind != XG_LEAKY) || (E->act && E->act != KAIR_ACT_LEAKY)))
      return false;
  }
  if (A->mode == KAIR_LD_ROWS) return A->dtype == KAIR_F16 ? A->ld % 8 == 0 : A->ld % 4 == 0;
  return A->mode == KAIR_LD_IM2COL3 && A->dtype == KAIR_F32 && A->im_C % 32 == 0 && K == 9 * A->im_C &&
         (A->ld == 0 ? A->im_C : A->ld) % 4 == 0;
}

// rows [m_base, M) of the product
template <typename TA, int AM, int BN, int BM>
int launch_nt_x3_ring(const Op& a, const Op& b, const Epi& e, long M, int N, int K, hipStream_t s, long m_base = 0) {
  const int tilesN = N / BN;
  const int tilesM = (int)((M - m_base + BM - 1) / BM);
  int per = x3_cus() / tilesN;
  if (per < 1) per = 1;
  const int rounds = (tilesM + per - 1) / per;
  per = (tilesM + rounds - 1) / rounds;   // the same makespan on as few CUs as it needs
  const dim3 g(per * tilesN), bl(512);
#define XR_LAUNCH(EM, EX, ACT, GK) \
  KAIR_LAUNCH((gemm_nt_x3_ring<TA, AM, EM, EX, ACT, GK, BN, BM>), g, bl, 0, s, a, b, e, K, tilesN, tilesM, (int)m_base)
  if constexpr (BN == 192) {   // the Swin linears and the 192-channel convs: every epilogue form
    if constexpr (sizeof(TA) == 2 && AM == AM_ROWS && BM == 64) {   // fp16-pair rows: the LayerNorm-backward epilogue
      if (e.lnx) {
        XR_LAUNCH(XE_ROWS_F32, EX_LNB, XA_NONE, 0);
        KAIR_CHECK_LAUNCH();
        return 0;
      }
    }
    if (e.omode == KAIR_OUT_QKVBLK) XR_LAUNCH(XE_QKV, EX_NONE, XA_NONE, 0);
    else if (e.odt == KAIR_F16 && e.gate) XR_LAUNCH(XE_ROWS_PAIR, EX_GATE_F32, XA_NONE, XG_MUL);
    else if (e.odt == KAIR_F16 && e.act == KAIR_ACT_GELU) XR_LAUNCH(XE_ROWS_PAIR, EX_NONE, XA_GELU, 0);
    else if (e.odt == KAIR_F16) XR_LAUNCH(XE_ROWS_PAIR, EX_NONE, XA_NONE, 0);
    else if (e.resid) XR_LAUNCH(XE_ROWS_F32, EX_RESID, XA_NONE, 0);
    else if (e.gate && e.gkind == XG_MUL) XR_LAUNCH(XE_ROWS_F32, EX_GATE_F32, XA_NONE, XG_MUL);
    else if (e.gate) XR_LAUNCH(XE_ROWS_F32, EX_GATE_F32, XA_NONE, XG_LEAKY);
    else if (e.act == KAIR_ACT_GELU && e.prek) XR_LAUNCH(XE_ROWS_F32, EX_NONE, XA_GELU, 0);
    else if (e.act == KAIR_ACT_GELU) XR_LAUNCH(XE_ROWS_F32, EX_NONE, XA_GELU_X, 0);
    else if (e.act == KAIR_ACT_LEAKY) XR_LAUNCH(XE_ROWS_F32, EX_NONE, XA_LEAKY, 0);
    else XR_LAUNCH(XE_ROWS_F32, EX_NONE, XA_NONE, 0);
  } else {   // the reconstruction tail's narrow / wide convs: fp32 rows, LeakyReLU or its gate, shuffles (nt_x3_ring_ok)
    if (e.omode == KAIR_OUT_PSHUF_SPM) XR_LAUNCH(XE_PSHUF, EX_NONE, XA_NONE, 0);
    else if (e.omode == KAIR_OUT_PUNSHUF_SPM) XR_LAUNCH(XE_PUNSHUF, EX_NONE, XA_NONE, 0);
    else if (e.gate) XR_LAUNCH(XE_ROWS_F32, EX_GATE_F32, XA_NONE, XG_LEAKY);
    else if (e.act == KAIR_ACT_LEAKY) XR_LAUNCH(XE_ROWS_F32, EX_NONE, XA_LEAKY, 0);
    else XR_LAUNCH(XE_ROWS_F32, EX_NONE, XA_NONE, 0);
  }
#undef XR_LAUNCH
  KAIR_CHECK_LAUNCH();
  return 0;
}

// the row tile of the 192-column NT ring: 64-row tiles when they finish sooner -- rounds of tiles per CU
// (x3_cus / N-tiles CTAs per N-tile) at a 64-row tile's cost of 0.66 of a 128-row one (profiles/r06_bm64_ab.txt:
// the same rows take 1.31x as long in 64-row tiles).  B = 4 (M = 9,216): N = 192 -> 64 rows (1 round of 144 tiles
// instead of 72 on 72 CUs), N = 384 / 576 -> 128 rows (one round; 64-row tiles need two); B = 32: 128 rows everywhere
int nt_x3_bm192(long M, int N) {
  const long per = x3_cus() / (N / 192) > 0 ? x3_cus() / (N / 192) : 1;
  const long r128 = ((M + XR_BM - 1) / XR_BM + per - 1) / per, r64 = ((M + 63) / 64 + per - 1) / per;
  return 66 * r64 < 100 * r128 ? 64 : XR_BM;
}

template <typename TA, int AM>
int nt_x3_ring_dispatch(const Op& a, const Op& b, const Epi& e, long M, int N, int K, hipStream_t s) {
  switch (nt_x3_ring_bn(N)) {
    case 64: return launch_nt_x3_ring<TA, AM, 64, XR_BM>(a, b, e, M, N, K, s);
    case 128: return launch_nt_x3_ring<TA, AM, 128, XR_BM>(a, b, e, M, N, K, s);
    default:
      if (nt_x3_bm192(M, N) == 64) return launch_nt_x3_ring<TA, AM, 192, 64>(a, b, e, M, N, K, s);
      // (a last round of 128-row tiles at most half full -- B = 32, N = 192: 576 tiles = 2 rounds of 256 + 64 -- run
      // as 64-row tiles in a second launch from m_base measured slower: B = 32 650 -> 638, B = 16 548 -> 522 patches/s;
      // the side stream's weight gradients already fill the idle CUs; profiles/r06_nt_split_ab.txt)
      return launch_nt_x3_ring<TA, AM, 192, XR_BM>(a, b, e, M, N, K, s);
  }
}

// the TN ring: fp32 rows (16-byte aligned, N and K % 4), B rows or the per-lane-tap im2col of a C-channel (C % 4)
// map (K = 9 C, no flip / upsample); B's bias ones column as data (ones_in_data) or injected, A's only as data
bool tn_x3_ring_ok(const kair_operand* A, const kair_operand* B, int N, int K) {
  static const int off = [] { const char* e = getenv("KAIR_X3_RING"); return e && e[0] == '0'; }();
  if (off) return false;
  if (A->dtype == KAIR_F16 && B->dtype == KAIR_F16) {   // fp16 pairs: row operands, 16-byte aligned 8-column units
    return A->mode == KAIR_LD_ROWS && B->mode == KAIR_LD_ROWS && N % 8 == 0 && K % 8 == 0 && A->ld % 8 == 0 &&
           B->ld % 8 == 0 && (uintptr_t)A->ptr % 16 == 0 && (uintptr_t)A->lo_ptr % 16 == 0 && (uintptr_t)B->ptr % 16 == 0 &&
           (uintptr_t)B->lo_ptr % 16 == 0 && !A->rowscale && !B->rowscale && (A->ones_col < 0 || A->ones_in_data) &&
           (B->ones_col < 0 || B->ones_in_data);
  }
  if (A->dtype != KAIR_F32 || B->dtype != KAIR_F32 || A->mode != KAIR_LD_ROWS || N % 4 || K % 4) return false;
  if (A->ld % 4 || (uintptr_t)A->ptr % 16 || (uintptr_t)B->ptr % 16 || A->rowscale || B->rowscale) return false;
  if (A->ones_col >= 0 && !A->ones_in_data) return false;
  if (B->mode == KAIR_LD_ROWS) return B->ld % 4 == 0;
  const long ld = B->ld == 0 ? B->im_C : B->ld;
  // (192-column N tiles: the RSTB / conv_after_body convs; the tail's N = 64 / 256 convs measured faster on the
  // generic kernel, 190 vs 398 and 428 vs 452 us)
  return B->mode == KAIR_LD_IM2COL3 && B->im_C % 4 == 0 && K == 9 * B->im_C && !B->im_flip && B->im_up != 2 && ld % 4 == 0 &&
         B->win_ws == 0 && N % 192 == 0;
}

// an x3 operand: fp32, or an fp16 hi plane with its 16-byte aligned lo plane
int x3_operand_ok(const kair_operand* o, const char* what) {
  KAIR_CHECK_ARG(o->dtype == KAIR_F32 || (o->dtype == KAIR_F16 && o->lo_ptr && ((uintptr_t)o->lo_ptr % 16) == 0),
                 "%s: x3 operands are fp32 or fp16 hi planes with their lo plane (lo_ptr)", what);
  KAIR_CHECK_ARG(o->x3_exp > -100 && o->x3_exp < 100, "%s: x3 exponent out of range", what);
  // no per-row scale rides on a stored pair (an injected ones column reads 2^x3_exp)
  KAIR_CHECK_ARG(!o->rowscale || o->dtype == KAIR_F32, "%s: x3 row scale needs an fp32 operand", what);
  return 0;
}

}  // namespace

// every job fp16 pairs in rows, 16-byte aligned 8-column units, no window map (tn_x3_ring_ok's pair branch)
int kair_wgrad_grouped_x3(const kair_wgrad_job* jobs, int njobs, long M, float* ws, int splits, void* stream) {
  TnX3Group g;
  FinGroup f;
  memset(&g, 0, sizeof(g));
  memset(&f, 0, sizeof(f));
  long rps = (M + splits - 1) / splits;
  rps = (rps + XT_RB - 1) / XT_RB * XT_RB;
  long tile0 = 0, off = 0, blk0 = 0;
  for (int i = 0; i < njobs; ++i) {
    const kair_wgrad_job& J = jobs[i];
    KAIR_CHECK_ARG(J.A.dtype == KAIR_F16 && J.B.dtype == KAIR_F16 && tn_x3_ring_ok(&J.A, &J.B, J.N, J.K) &&
                       J.A.win_ws == 0 && J.B.win_ws == 0,
                   "wgrad_grouped x3: job %d: fp16-pair row operands (16-byte aligned, N, K %% 8, no window map)", i);
    KAIR_CHECK_ARG(J.grad && J.map.kind == 0 && (long)J.map.nG * J.map.nGp == J.N && (long)J.map.kG * J.map.kGp == J.K,
                   "wgrad_grouped x3: job %d needs a linear map whose packed dims are (N, K)", i);
    KAIR_CHECK_ARG(!J.bias_grad || (J.ones_col >= 0 && J.ones_col < J.K), "wgrad_grouped x3: job %d bias needs ones_col", i);
    const int tilesK = (J.K + 191) / 192;
    TnX3Job& t = g.j[i];
    t.ah = J.A.ptr; t.al = J.A.lo_ptr; t.bh = J.B.ptr; t.bl = J.B.lo_ptr;
    t.ws = ws + off;
    t.lda = J.A.ld; t.ldb = J.B.ld;
    t.N = J.N; t.K = J.K; t.tilesK = tilesK; t.tile0 = (int)tile0;
    t.acc_scale = ldexpf(1.f, -(J.A.x3_exp + J.B.x3_exp));
    tile0 += (long)((J.N + 191) / 192) * tilesK;
    FinJob& q = f.j[i];
    q.part = ws + off; q.grad = J.grad; q.bias = J.bias_grad; q.mp = J.map; q.ones_col = J.bias_grad ? J.ones_col : -1;
    q.Kt = J.K; q.plane = (long)J.N * J.K; q.blk0 = blk0;
    blk0 += ((long)J.N * J.K / 4 + 63) / 64;
    off += (long)splits * J.N * J.K;
  }
  g.njobs = njobs; g.ntiles = (int)tile0; g.M = (int)M; g.rps = (int)rps;
  f.njobs = njobs; f.splits = splits; f.nblocks = blk0;
  hipStream_t s = (hipStream_t)stream;
  KAIR_LAUNCH(gemm_tn_x3_ring_grouped, dim3((unsigned)(tile0 * splits)), dim3(512), 0, s, g);
  KAIR_CHECK_LAUNCH();
  return kair_launch_finalize_grouped(f, s);
}

// copy the NT ring's phase stamps to the host and clear them (perf investigation only; zeros in release builds)
extern "C" int kair_debug_x3_stamps(unsigned long long* host, int n) {
  KAIR_CHECK_ARG(host && n > 0 && n <= XS_CTAS * 8 * XS_IT * XS_N, "debug_x3_stamps: bad args");
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_x3_stamps), sizeof(unsigned long long) * n, 0, hipMemcpyDeviceToHost) !=
      hipSuccess)
    return kair_set_error(KAIR_ERR_HIP, "debug_x3_stamps: copy failed");
  void* dev = nullptr;
  if (hipGetSymbolAddress(&dev, HIP_SYMBOL(g_x3_stamps)) != hipSuccess ||
      hipMemset(dev, 0, sizeof(unsigned long long) * XS_CTAS * 8 * XS_IT * XS_N) != hipSuccess)
    return kair_set_error(KAIR_ERR_HIP, "debug_x3_stamps: clear failed");
  return 0;
}

int kair_gemm_nt_x3(const kair_operand* A, const kair_operand* B, const kair_epilogue* E, long M, int N, int K,
                    void* stream) {
  int rc;
  if ((rc = x3_operand_ok(A, "gemm_nt x3 A"))) return rc;
  KAIR_CHECK_ARG(M > 0 && N > 0 && K > 0 && K % 8 == 0, "gemm_nt x3: bad M/N/K (%ld,%d,%d)", M, N, K);
  KAIR_CHECK_ARG(A->mode == KAIR_LD_ROWS || A->mode == KAIR_LD_IM2COL3, "gemm_nt x3: A rows or im2col");
  KAIR_CHECK_ARG(A->ones_col < 0 && !A->rowscale, "gemm_nt x3: no ones column / row scale on A");
  KAIR_CHECK_ARG(B->mode == KAIR_LD_ROWS && B->dtype == KAIR_F16 && B->win_ws == 0 && B->ld >= 2L * ((K + 63) / 64) * 64 &&
                     B->ld % 8 == 0,
                 "gemm_nt x3: B must be split-packed fp16 weight rows of >= 2*ceil(K/64)*64 columns");
  KAIR_CHECK_ARG(E->out_dtype != KAIR_F16 || E->out_mode == KAIR_OUT_ROWS || E->out_mode == KAIR_OUT_QKVBLK,
                 "gemm_nt x3: an fp16 pair output is ROWS or QKVBLK");
  KAIR_CHECK_ARG(E->out_dtype != KAIR_BF16 && !E->a_copy, "gemm_nt x3: fp32 or fp16-pair outputs, no a_copy");
  KAIR_CHECK_ARG(!E->out_lo || E->out_dtype == KAIR_F16, "gemm_nt x3: out_lo is the lo plane of an fp16 output");
  KAIR_CHECK_ARG(E->out_mode != KAIR_OUT_QKVBLK || (E->qkv_hdp % 8 == 0 && E->qkv_tok > 0), "gemm_nt x3: qkv epilogue");
  KAIR_CHECK_ARG((E->out_mode != KAIR_OUT_PSHUF && E->out_mode != KAIR_OUT_PUNSHUF && E->out_mode != KAIR_OUT_PSHUF_NCHW &&
                  E->out_mode != KAIR_OUT_PSHUF_SPM && E->out_mode != KAIR_OUT_PUNSHUF_SPM) || E->ps_r > 0,
                 "gemm_nt x3: pixel shuffle r");
  KAIR_CHECK_ARG(M < KAIR_MAX_MAPPED_ROWS && N < KAIR_MAX_MAPPED_ROWS && K < KAIR_MAX_MAPPED_ROWS,
                 "gemm_nt x3: dimensions must be < 2^24");
  const Op a = make_op(*A, M), b = make_op(*B, N);
  Epi e = make_epi(*E, M, N);
  e.acc_scale = ldexpf(1.f, -(A->x3_exp + B->x3_exp));
  hipStream_t s = (hipStream_t)stream;
  if (nt_x3_ring_ok(A, B, E, N, K)) {
    if (A->mode == KAIR_LD_IM2COL3) return nt_x3_ring_dispatch<float, AM_IM2COL>(a, b, e, M, N, K, s);
    return A->dtype == KAIR_F16 ? nt_x3_ring_dispatch<f16, AM_ROWS>(a, b, e, M, N, K, s)
                                : nt_x3_ring_dispatch<float, AM_ROWS>(a, b, e, M, N, K, s);
  }
  if (A->dtype == KAIR_F16)
    return A->mode == KAIR_LD_ROWS ? nt_x3_tiles<f16, AM_ROWS>(a, b, e, M, N, K, s) : nt_x3_tiles<f16, AM_IM2COL>(a, b, e, M, N, K, s);
  return A->mode == KAIR_LD_ROWS ? nt_x3_tiles<float, AM_ROWS>(a, b, e, M, N, K, s) : nt_x3_tiles<float, AM_IM2COL>(a, b, e, M, N, K, s);
}

extern "C" long kair_gemm_nt_x3_lnbwd_parts(long M, int N) {
  if (M <= 0 || N != 192) return 0;
  return (M + 63) / 64 * 4;   // (64-row tile, row wave): 16 rows each
}

extern "C" int kair_gemm_nt_x3_lnbwd(const kair_operand* A, const kair_operand* B, long M, int N, int K, int win_H,
                                     int win_W, int win_ws, int win_shift, const float* x, long ldx, const float* gamma,
                                     const float* mean, const float* rstd, int C, float* D, long ldd, float* part,
                                     const kair_copy_desc* copy, void* stream) {
  int rc;
  if ((rc = x3_operand_ok(A, "gemm_nt_x3_lnbwd A"))) return rc;
  KAIR_CHECK_ARG(x && gamma && mean && rstd && D && part, "gemm_nt_x3_lnbwd: null pointer");
  KAIR_CHECK_ARG(N == 192 && C > 0 && C <= N && C % 4 == 0 && M > 0 && M < KAIR_MAX_MAPPED_ROWS,
                 "gemm_nt_x3_lnbwd: one 192-column tile holding the C <= 192 channels (C %% 4 == 0)");
  KAIR_CHECK_ARG(A->dtype == KAIR_F16 && A->mode == KAIR_LD_ROWS, "gemm_nt_x3_lnbwd: A must be fp16-pair rows");
  KAIR_CHECK_ARG(ldx % 4 == 0 && ldd % 4 == 0 && ldx >= N && ldd >= N && ((uintptr_t)x % 16) == 0 && ((uintptr_t)D % 16) == 0,
                 "gemm_nt_x3_lnbwd: x / D rows of >= 192 columns, 16-byte aligned");
  kair_epilogue E;
  memset(&E, 0, sizeof(E));
  E.out = D; E.out_dtype = KAIR_F32; E.out_mode = KAIR_OUT_ROWS; E.ldo = ldd;
  E.win_H = win_H; E.win_W = win_W; E.win_ws = win_ws; E.win_shift = win_shift;
  E.bias = gamma;
  KAIR_CHECK_ARG(nt_x3_ring_ok(A, B, &E, N, K), "gemm_nt_x3_lnbwd: shape / operands outside the NT ring");
  KAIR_CHECK_ARG(win_ws == 0 || (win_H % win_ws == 0 && win_W % win_ws == 0), "gemm_nt_x3_lnbwd: window geometry");
  const Op a = make_op(*A, M), b = make_op(*B, N);
  Epi e = make_epi(E, M, N);
  e.acc_scale = ldexpf(1.f, -(A->x3_exp + B->x3_exp));
  e.lnx = x; e.lnldx = ldx; e.lnmu = mean; e.lnrs = rstd; e.lnpart = part; e.lnC = C;
  if (copy && copy->out) {
    KAIR_CHECK_ARG(copy->dtype == KAIR_F16 && copy->out_lo && copy->ld % 4 == 0 && copy->ld >= N &&
                       ((uintptr_t)copy->out % 8) == 0 && ((uintptr_t)copy->out_lo % 8) == 0,
                   "gemm_nt_x3_lnbwd: the copy is an fp16 pair (out + out_lo, 8-byte aligned, ld %% 4 == 0)");
    KAIR_CHECK_ARG(copy->win_ws == 0 || (copy->win_H % copy->win_ws == 0 && copy->win_W % copy->win_ws == 0),
                   "gemm_nt_x3_lnbwd: copy window geometry");
    e.cpo = copy->out; e.cplo = copy->out_lo; e.cpld = copy->ld;
    e.cprs = copy->rowscale;
    e.d_cprps = make_fdiv(copy->rows_per_scale > 0 ? copy->rows_per_scale : 1);
    e.cpwin = make_winmap(copy->win_H, copy->win_W, copy->win_ws, copy->win_shift);
    e.cps = ldexpf(1.f, copy->x3_exp);
  }
  // 64-row tiles at every M: with this epilogue the 128-row form exceeds the 256 VGPRs of two waves per SIMD (spills)
  return launch_nt_x3_ring<f16, AM_ROWS, 192, 64>(a, b, e, M, N, K, (hipStream_t)stream);
}

int kair_gemm_tn_x3(const kair_operand* A, const kair_operand* B, float* ws, int splits, long M, int N, int K,
                    void* stream) {
  int rc;
  if ((rc = x3_operand_ok(A, "gemm_tn x3 A"))) return rc;
  if ((rc = x3_operand_ok(B, "gemm_tn x3 B"))) return rc;
  KAIR_CHECK_ARG(A->mode == KAIR_LD_ROWS && (B->mode == KAIR_LD_ROWS || B->mode == KAIR_LD_IM2COL3),
                 "gemm_tn x3: A rows, B rows or im2col");
  KAIR_CHECK_ARG(M < KAIR_MAX_MAPPED_ROWS && N < KAIR_MAX_MAPPED_ROWS && K < KAIR_MAX_MAPPED_ROWS,
                 "gemm_tn x3: dimensions must be < 2^24");
  const Op a = make_op(*A, M), b = make_op(*B, M);
  long rps = (M + splits - 1) / splits;
  rps = (rps + 31) / 32 * 32;
  const float sc = ldexpf(1.f, -(A->x3_exp + B->x3_exp));
  hipStream_t s = (hipStream_t)stream;
  if (tn_x3_ring_ok(A, B, N, K)) {
    const int tilesN = (N + 191) / 192, tilesK = (K + 191) / 192, nt = tilesN * tilesK;
    const dim3 g(nt * splits), bl(512);
      if (A->dtype == KAIR_F16)
      KAIR_LAUNCH((gemm_tn_x3_ring<BT_ROWS, true>), g, bl, 0, s, a, b, ws, (int)M, N, K, tilesK, nt, (int)rps, sc);
    else if (B->mode == KAIR_LD_IM2COL3)
      KAIR_LAUNCH((gemm_tn_x3_ring<BT_TAP, false>), g, bl, 0, s, a, b, ws, (int)M, N, K, tilesK, nt, (int)rps, sc);
    else
      KAIR_LAUNCH((gemm_tn_x3_ring<BT_ROWS, false>), g, bl, 0, s, a, b, ws, (int)M, N, K, tilesK, nt, (int)rps, sc);
    KAIR_CHECK_LAUNCH();
    return 0;
  }
  return A->dtype == KAIR_F16 ? tn_x3_b<f16>(a, b, B->mode, B->dtype, ws, splits, M, N, K, rps, sc, s)
                              : tn_x3_b<float>(a, b, B->mode, B->dtype, ws, splits, M, N, K, rps, sc, s);
}
