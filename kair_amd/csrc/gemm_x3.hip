// The fp32 engine's contractions on the 16-bit matrix cores ("x3" arithmetic, KAIR_COMPUTE_X3): every
// operand x enters as an fp16 pair of x * 2^e (hi = f16(x 2^e), lo = f16(x 2^e - hi)) and every product as
// hi.hi + hi.lo + lo.hi (v_mfma_f32_16x16x32_f16, fp32 accumulation), the accumulator rescaled by 2^-(eA+eB).
// The pair carries 22 of fp32's 24 mantissa bits, so a product is exact to ~2^-21 -- the precision class of
// the fp32 reference (SwinIR classical x4 trains in fp32: models/model_plain.py:31-36 with no amp_enabled in
// options/swinir/train_swinir_sr_classical.json); the power-of-2 exponent keeps the operand inside fp16's
// range (weights 2^KAIR_X3_WEXP, activations 2^0, gradients 2^(log2 of the loss normalisation)).
//
//   kair_gemm_nt_x3 : C[m,n] = sum_k A[m,k] B[n,k]            (nn.Linear / 3x3 nn.Conv2d forward + dgrad)
//   kair_gemm_tn_x3 : P[s][n,k] = sum_{m in s} A[m,n] B[m,k]   (their weight gradients, split over m)
//
// Operands: fp32 (split at the LDS commit, read from HBM once) or fp16 hi planes with their lo planes
// (kair_operand.lo_ptr).  LDS holds hi and lo planes of both operands; 32-deep k-steps (NT) / 32-row
// reduction steps (TN), double-buffered by register staging as the bf16 kernels (gemm.hip).
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
  hipLaunchKernelGGL((gemm_nt_x3_kernel<TA, AM, BM, BN>), dim3((unsigned)nwg), dim3(NT), 0, s, A, B, E, K, tilesN, (int)nwg);
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
    hipLaunchKernelGGL((gemm_tn_x3_kernel<TA, TB, AMB, 64, 64>), dim3(1, splits), dim3(NT), 0, s, a, b, ws, M, N, K, rps, 1,
                       acc_scale);
  } else {
    const int tilesN = (N + 127) / 128, tilesK = (K + 127) / 128;
    hipLaunchKernelGGL((gemm_tn_x3_kernel<TA, TB, AMB, 128, 128>), dim3(tilesN * tilesK, splits), dim3(NT), 0, s, a, b, ws,
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
  if (A->dtype == KAIR_F16)
    return A->mode == KAIR_LD_ROWS ? nt_x3_tiles<f16, AM_ROWS>(a, b, e, M, N, K, s) : nt_x3_tiles<f16, AM_IM2COL>(a, b, e, M, N, K, s);
  return A->mode == KAIR_LD_ROWS ? nt_x3_tiles<float, AM_ROWS>(a, b, e, M, N, K, s) : nt_x3_tiles<float, AM_IM2COL>(a, b, e, M, N, K, s);
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
  return A->dtype == KAIR_F16 ? tn_x3_b<f16>(a, b, B->mode, B->dtype, ws, splits, M, N, K, rps, sc, s)
                              : tn_x3_b<float>(a, b, B->mode, B->dtype, ws, splits, M, N, K, rps, sc, s);
}
