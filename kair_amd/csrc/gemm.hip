// Implicit-GEMM kernels for gfx950 (CDNA4): the contractions of nn.Linear and 3x3 nn.Conv2d on the
// KAIR hot path (forward, input gradient and weight gradient), with fused prologue address maps
// (Swin window partition + cyclic shift, im2col, head-blocked q/k/v) and fused epilogues
// (bias, GELU / LeakyReLU, residual add, DropPath scale, PixelShuffle store, NCHW image store,
// act' gating).
//
//   kair_gemm_nt : C[m,n] = sum_k A[m,k] B[n,k]            (forward, input gradient)
//   kair_gemm_tn : P[s][n,k] = sum_{m in s} A[m,n] B[m,k]   (weight gradient, split over m)
//
// Structure (both): 256 threads = 4 waves (2x2), 128x128 (or smaller) output tile, K-step 64
// (bf16) / 32 (fp32), double-buffered LDS filled by register staging: the next K-step's global
// loads are issued before the current step's MFMAs and written to the other LDS buffer after them,
// one barrier per K-step.  Operand modes are template parameters and every per-row address is
// computed once before the K loop.  bf16 compute uses v_mfma_f32_16x16x32_bf16 fed by
// ds_read_b128 (NT) or ds_read_b64_tr_b16 (TN, m-major tiles); fp32 (parity) compute uses the exact
// v_mfma_f32_16x16x4_f32.  The NT epilogue stages the accumulator tile through LDS so every thread
// finishes 8 consecutive columns of one row with 16-byte loads/stores.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gemm_common.h"

namespace {

// ------------------------------------------------------------------------------------------
// NT kernel
// ------------------------------------------------------------------------------------------
template <typename CT, typename TA, int AM, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(NT, 2) void gemm_nt_kernel(Op A, Op B, Epi E, int K, int tilesN, int nwg) {
  constexpr int BK = KStep<CT>::BK;
  constexpr int LD = BK + (sizeof(CT) == 2 ? 8 : 2);
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int RM = TM / 16, RN = TN / 16;
  constexpr int CPR = BK / 8;                      // chunks per tile row
  constexpr int CA = BM * CPR, CB = BN * CPR;
  constexpr int PA = (CA + NT - 1) / NT, PB = (CB + NT - 1) / NT;
  constexpr int STAGE = (BM + BN) * LD;            // elements per LDS stage
  constexpr int EPI_LD = BN + 4;                   // fp32 epilogue tile row stride
  constexpr int LDS_BYTES_MAIN = 2 * STAGE * (int)sizeof(CT);
  constexpr int LDS_BYTES_EPI = BM * EPI_LD * 4;
  constexpr int LDS_BYTES = LDS_BYTES_MAIN > LDS_BYTES_EPI ? LDS_BYTES_MAIN : LDS_BYTES_EPI;
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  CT* lds = (CT*)smem;

  const int tile = xcd_remap(blockIdx.x, nwg);
  const int tm = tile / tilesN, tn = tile - tm * tilesN;
  const long m0 = (long)tm * BM;
  const int n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  RowState ra[PA], rb[PB];
#pragma unroll
  for (int p = 0; p < PA; ++p) {
    const int c = tid + p * NT;
    ra[p] = row_state<AM, TA>(A, c < CA ? m0 + c / CPR : A.M);
  }
#pragma unroll
  for (int p = 0; p < PB; ++p) {
    const int c = tid + p * NT;
    rb[p] = row_state<AM_ROWS, CT>(B, c < CB ? (long)(n0 + c / CPR) : B.M);
  }
  Raw<TA> va[PA];
  Raw<CT> vb[PB];
  Pend pa[PA], pb[PB];
  // hi/lo split weights (bf16): K-step kt reads A columns of step kt >> 1 and B columns kt * BK of
  // the interleaved [hi | lo] rows, so the A chunk is fetched twice from L1/L2 but once from HBM.
  // hi/lo split activations (A.asplit) add a third product per K step, a_lo . w_hi: the lo half
  // formed from the fp32 source at commit, or read from the lo plane of a bf16 source.
  const int wsp = (sizeof(CT) == 2 && B.wsplit) ? 1 : 0;
  const int asp = (sizeof(CT) == 2 && A.asplit == 1) ? 1 : 0;   // a_split 2: the lo half is in the image
  const int NP = 1 + wsp + asp;   // products per K step: (a_hi, w_hi) [, (a_hi, w_lo)] [, (a_lo, w_hi)]
  const int nks = (K + BK - 1) / BK;
  const int nk = nks * NP;
  const int KB = wsp ? 2 * nks * BK : K;
  bool pend_lo = false;   // the chunk in flight is the lo half of an fp32 A
  auto gload = [&](int kt) {
    const int st = kt / NP, pp = kt - st * NP;
    const bool alo = asp && pp == NP - 1;
    const int ka = st * BK, kb = (wsp ? 2 * st + (pp == 1 && !alo) : st) * BK;
    const void* abase = (alo && sizeof(TA) == 2) ? A.lo_ptr : A.ptr;
    pend_lo = alo && sizeof(TA) == 4;
#pragma unroll
    for (int p = 0; p < PA; ++p) issue_chunk<AM, TA>(A, ra[p], ka + ((tid + p * NT) % CPR) * 8, K, va[p], pa[p], abase);
#pragma unroll
    for (int p = 0; p < PB; ++p) issue_chunk<AM_ROWS, CT>(B, rb[p], kb + ((tid + p * NT) % CPR) * 8, KB, vb[p], pb[p]);
  };
  auto sstore = [&](int st) {
    CT* sA = lds + st * STAGE;
    CT* sB = sA + BM * LD;
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int c = tid + p * NT;
      if (c < CA) commit_chunk<CT, TA>(sA + (c / CPR) * LD + (c % CPR) * 8, va[p], pa[p], pend_lo);
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int c = tid + p * NT;
      if (c < CB) commit_chunk<CT, CT>(sB + (c / CPR) * LD + (c % CPR) * 8, vb[p], pb[p]);
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const CT* sA = lds + st * STAGE;
    const CT* sB = sA + BM * LD;
    if constexpr (sizeof(CT) == 2) {
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        bf16x8 af[RM], bfr[RN];
#pragma unroll
        for (int i = 0; i < RM; ++i) af[i] = *(const bf16x8*)(sA + (wm * TM + i * 16 + fr) * LD + ks * 32 + fq * 8);
#pragma unroll
        for (int j = 0; j < RN; ++j) bfr[j] = *(const bf16x8*)(sB + (wn * TN + j * 16 + fr) * LD + ks * 32 + fq * 8);
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
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
    if (kt + 1 < nk) sstore(st ^ 1);
    __syncthreads();
  }
  // epilogue: accumulator tile -> LDS (fp32) -> 8-column row chunks
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
    epi_chunk(E, m0 + row, n0 + col, v);
  }
}

// ------------------------------------------------------------------------------------------
// 4-column register epilogue (ring kernel): lane holds columns [n, n+4) of one output row.
// ------------------------------------------------------------------------------------------
enum { EM_ROWS = 0, EM_QKV = 1 };

KAIR_DEV void ld4_any(const void* p, int dt, long off, float (&g)[4]) {
  if (dt == KAIR_BF16) {
    const bf16x4 q = *(const bf16x4*)((const bf16*)p + off);
    g[0] = (float)q[0]; g[1] = (float)q[1]; g[2] = (float)q[2]; g[3] = (float)q[3];
  } else {
    const float4 a = *(const float4*)((const float*)p + off);
    g[0] = a.x; g[1] = a.y; g[2] = a.z; g[3] = a.w;
  }
}
KAIR_DEV void st4_any(void* p, int dt, long off, const float (&v)[4]) {
  if (dt == KAIR_BF16) {
    bf16x4 q = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    *(bf16x4*)((bf16*)p + off) = q;
  } else {
    *(float4*)((float*)p + off) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// 16-byte store with a cache policy: 0 plain, 1 nt, 2 sc1 (write-through)
typedef unsigned __attribute__((ext_vector_type(4))) u32x4;
KAIR_DEV void st16_pol(void* p, u32x4 v, int pol) {
  if (pol == 1) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
  else if (pol == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  else *(u32x4*)p = v;
}

// 8 consecutive columns: one 16-byte store for bf16, two for fp32
KAIR_DEV void st8_any(void* p, int dt, long off, const float (&v)[8], int pol = 0) {
  if (dt == KAIR_BF16) {
    const bf16x8 q = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3], (bf16)v[4], (bf16)v[5], (bf16)v[6], (bf16)v[7]};
    st16_pol((bf16*)p + off, __builtin_bit_cast(u32x4, q), pol);
  } else {
    const u32x4 a = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
    const u32x4 b = {__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]), __float_as_uint(v[7])};
    st16_pol((float*)p + off, a, pol);
    st16_pol((float*)p + off + 4, b, pol);
  }
}

template <int EM>
KAIR_DEV void epi4(const Epi& e, long m, long row, float rs, int n, float (&v)[4]) {
  if (e.bias) {
    const float4 b = *(const float4*)(e.bias + n);
    v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
  }
  if constexpr (EM == EM_QKV) {
    const int pw = e.nh * e.hdp;
    const int part = fdiv(n, e.d_pw), rr = n - part * pw;
    const int h = fdiv(rr, e.d_hdp), d = rr - h * e.hdp;
    const long win = fdiv((int)m, e.d_tok);
    const int t = (int)(m - win * e.tok);
    st4_any(e.out, e.odt, (long)part * e.M * pw + ((win * e.nh + h) * e.tok + t) * e.hdp + d, v);
  } else {
    float pre[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pre[j] = v[j];
      if (e.act == KAIR_ACT_GELU) {
        float y, dy;
        gelu_pair_fast(v[j], y, dy);
        v[j] = y;
        if (e.prek) pre[j] = dy;
      } else if (e.act == KAIR_ACT_LEAKY) v[j] = v[j] > 0.f ? v[j] : v[j] * e.slope;
      else if (e.act == KAIR_ACT_RELU) v[j] = fmaxf(v[j], 0.f);
    }
    if (e.gate) {
      float g[4];
      ld4_any(e.gate, e.gdt, row * e.ldg + n, g);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (e.gkind == 1) v[j] *= gelu_grad_fast(g[j]);
        else if (e.gkind == 2) v[j] *= (g[j] > 0.f ? 1.f : e.slope);
        else if (e.gkind == 4) v[j] *= g[j];
        else v[j] *= (g[j] > 0.f ? 1.f : 0.f);
      }
    }
    if (e.resid) {
      const float4 r = *(const float4*)(e.resid + row * e.ldr + n);
      v[0] = r.x + rs * v[0]; v[1] = r.y + rs * v[1]; v[2] = r.z + rs * v[2]; v[3] = r.w + rs * v[3];
    }
    if (e.ones_col >= n && e.ones_col < n + 4) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (n + j == e.ones_col) v[j] = 1.f;
    }
    st4_any(e.out, e.odt, row * e.ldo + n, v);
    if (e.pre) st4_any(e.pre, e.pdt, row * e.ldp + n, pre);
  }
}

// ------------------------------------------------------------------------------------------
// NT ring kernel (bf16 A rows / head-blocked q,k,v; K % 64 == 0, K <= 576): one 512-thread CTA
// per CU, persistent over the M-tiles of ONE N-tile.
//  * the CTA's BN x K slice of the packed weights is loaded into LDS once and stays resident;
//  * A streams through an NS-deep ring of 128x64 bf16 chunks filled by LDS-DMA
//    (global_load_lds_dwordx4, 2 wave-instructions per wave per chunk, source-address XOR swizzle
//    so the lane-linear image reads conflict-light), waited with a counted vmcnt and a raw
//    s_barrier, so NS-2 chunks stay in flight across barriers and across tile boundaries;
//  * MFMA operands are swapped (D = B . A^T) so each lane owns 4 consecutive output columns of one
//    row: the fused epilogue runs from the accumulators with 8/16-byte vector accesses;
//  * vmcnt counts the epilogue's stores too (in issue order with the LDS-DMA loads), so the chunk
//    wait adds the stores this wave issued after the awaited chunk: a tile's stores drain under the
//    next tile's MFMAs instead of being waited for at its first chunk.  The count used is the number
//    of store instructions that MUST have issued (fragments with at least one valid lane); a
//    compiler that also issues fully masked ones only makes the wait stricter.
// ------------------------------------------------------------------------------------------
constexpr int RING_BM = 128, RING_BK = 64;
constexpr int RING_B_ELEMS = 38400;   // max BN * (Kr + 8) over the (BN, K) pairs dispatched below (Kr: K up to 64)
constexpr int RING_RS_MAX = 1024;     // per-sample residual scales kept in LDS by the ring kernel


template <int BN, int NS, int AM, int EM, int EX>
__global__ __launch_bounds__(512, 1) void gemm_nt_ring(Op A, Op B, Epi E, int K, int tilesN, int tilesM) {
  constexpr int BM = RING_BM, BK = RING_BK;
  // 8 waves as WM (rows) x WN (columns); each wave's columns split into 16-wide fragment pairs
  constexpr int WN = BN == 96 ? 1 : 2, WM = 8 / WN, WROWS = BM / WM;
  // K % 64 != 0 (head-padded projections, e.g. 6 heads x 16 = 96): the last chunk is partial -- its pieces past K
  // load the zero line and the B slice is zero there, so the chunk contracts exact zeros
  constexpr int TN = BN / WN, RM = WROWS / 16, RN = TN / 16;
  constexpr int STAGE_BYTES = BM * BK * 2;   // 16 KiB
  constexpr int NP = RN / 2;                  // fragment pairs per wave row (8-column epilogue groups)
  static_assert(RN % 2 == 0, "fragment pairs");
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE_BYTES + RING_B_ELEMS * 2 + RING_RS_MAX * 4];
  bf16* sB = (bf16*)(smem + NS * STAGE_BYTES);
  float* sRS = (float*)(smem + NS * STAGE_BYTES + RING_B_ELEMS * 2);
  const int Kr = (K + BK - 1) / BK * BK;
  const int LDB = Kr + 8;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int fr = lane & 15, fq = lane >> 4;
  const int cta = xcd_remap(blockIdx.x, gridDim.x);
  const int nt = cta % tilesN;
  const int mstride = gridDim.x / tilesN;
  const int mt0 = cta / tilesN;
  if (mt0 >= tilesM) return;
  const int ntile_m = (tilesM - mt0 + mstride - 1) / mstride;
  const int nk = Kr / BK;
  const int total = ntile_m * nk;
  const int n0 = nt * BN;

  // resident B slice [BN][K] (rows >= N are zero)
  {
    const bf16* bp = (const bf16*)B.ptr;
    // all loads first (<= 10 16-byte pieces per thread: BN * K <= RING_B_ELEMS), then the LDS
    // stores, so the slice costs one L2 round trip rather than one per piece
    constexpr int PER = (RING_B_ELEMS / 8 + 511) / 512;
    const int cpr = Kr / 8;
    uint4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * 512;
      const int r = c / cpr, k8 = (c - r * cpr) * 8;
      // unconditional (clamped) loads, zeroed after: a conditional load becomes a branch with its
      // own wait, i.e. one L2 round trip per piece
      const bool ok = c < BN * cpr && n0 + r < B.M && k8 < K;
      const long row = ok ? n0 + r : 0;
      v[i] = *(const uint4*)(bp + row * B.ld + (ok ? k8 : 0));
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * 512;
      const int r = c / cpr, k8 = (c - r * cpr) * 8;
      if (!(c < BN * cpr && n0 + r < B.M && k8 < K)) v[i] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * 512;
      const int r = c / cpr, k8 = (c - r * cpr) * 8;
      if (c < BN * cpr) *(uint4*)(sB + r * LDB + k8) = v[i];
    }
  }
  // per-sample residual scales (DropPath) in LDS: the epilogue reads them without a global load
  if constexpr (EX == EX_RESID) {
    if (E.rowscale) {
      const int nrs = (int)((E.M + E.rps - 1) / E.rps);
      for (int i = tid; i < nrs; i += 512) sRS[i] = E.rowscale[i];
    }
  }

  // Epilogue columns (fixed per CTA).  After a v_permlane16_swap of fragment pair (2p, 2p+1) a
  // lane owns 8 consecutive columns of fragment 2p + (fq & 1): c8 = that fragment's base +
  // (fq >> 1) * 8, so bf16 outputs leave as one 16-byte store per lane instead of two 8-byte ones.
  int c8v[NP];
  long colo[NP];   // ROWS: output column; QKV: column part of the head-blocked offset
  float4 bias8[NP][2];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int n = n0 + wn * TN + (2 * p + (fq & 1)) * 16 + (fq >> 1) * 8;
    c8v[p] = n;
    const int nn = n < E.N ? n : 0;
    if constexpr (EM == EM_QKV) {
      const int pw = E.nh * E.hdp;
      const int part = fdiv(nn, E.d_pw), rr = nn - part * pw;
      const int h = fdiv(rr, E.d_hdp), d = rr - h * E.hdp;
      colo[p] = (long)part * E.M * pw + (long)h * E.tok * E.hdp + d;
    } else {
      colo[p] = nn;
    }
    // unconditional loads (a zero line stands in for a missing bias / column)
    bias8[p][0] = *(const float4*)(E.bias && n < E.N ? E.bias + n : (const float*)g_kair_zero_line);
    bias8[p][1] = *(const float4*)(E.bias && n + 4 < E.N ? E.bias + n + 4 : (const float*)g_kair_zero_line);
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) { land(bias8[p][0]); land(bias8[p][1]); }
  const int st_per_frag = (EM == EM_ROWS && E.pre) ? 2 : 1;

  // loader state: this lane's two rows of the chunk being LOADED
  const int q8 = lane & 7;
  long rbase[2];
  int rsw[2];   // row & 7 (swizzle key)
  auto load_rows = [&](int i) {
    const int mt = mt0 + i * mstride;
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      const int r = (wave * 2 + ii) * 8 + (lane >> 3);
      int m = mt * BM + r;
      if (m >= (int)A.M) m = 0;   // rows past M load row 0; the epilogue skips them
      rsw[ii] = r & 7;
      if constexpr (AM == AM_ROWS) {
        rbase[ii] = (long)win_to_token32(m, A.win) * A.ld;
      } else {
        const int win = fdiv(m, A.d_tok), t = m - win * A.tok;
        rbase[ii] = ((long)win * A.nh * A.tok + t) * A.hdp;
      }
    }
  };
  // loader cursor: the next chunk to issue is lj = lt * nk + lkc, into stage ls (all wave-uniform
  // counters advanced incrementally -- no per-chunk divisions)
  int lj = 0, lt = 0, lkc = 0, ls = 0;
  auto issue_next = [&]() {
    if (lkc == 0) load_rows(lt);
    if (!KAIR_DBG(E.dbg & 4)) {
      char* st = smem + ls * STAGE_BYTES;
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int k = lkc * BK + ((q8 ^ rsw[ii]) << 3);
        const int kk = k < K ? k : 0;
        long off;
        if constexpr (AM == AM_ROWS) {
          off = rbase[ii] + kk;
        } else {
          const int pw = A.d_pw.d;
          const int part = fdiv(kk, A.d_pw), rr = kk - part * pw;
          const int h = fdiv(rr, A.d_hdp), d = rr - h * A.hdp;
          off = (long)part * A.M * pw + rbase[ii] + (long)h * A.tok * A.hdp + d;
        }
        glds16(k < K ? (const void*)((const bf16*)A.ptr + off) : (const void*)g_kair_zero_line, st + (wave * 2 + ii) * 1024);
      }
    }
    ++lj;
    if (++lkc == nk) { lkc = 0; ++lt; }
    if (++ls == NS) ls = 0;
  };

  // prologue: B slice visible to every wave, then NS-1 chunks in flight
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (lj < total) issue_next();

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int jn = 0; jn < RN; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};

  static_assert(NS == 5, "the store bookkeeping below assumes chunk j is issued at iteration j-4");
  int sq1 = 0, sq2 = 0, sq3 = 0, sq4 = 0;   // store instructions this wave issued at iterations j-1 .. j-4
  const bool early = KAIR_DBG(E.dbg & 32);     // tile end: issue the deferred chunk before the stores
  int kc = 0, cs = 0, ct = 0;      // consumer cursor: chunk j = ct * nk + kc, in stage cs
  for (int j = 0; j < total; ++j) {
    // chunk j landed for this wave: younger than it are min(NS-2, total-1-j) chunks (2 DMA
    // instructions each) and the stores of the epilogues run at iterations j-3 .. j-1
    const int ahead = (total - 1 - j) < (NS - 2) ? (total - 1 - j) : (NS - 2);
    vm_wait(2 * ahead + sq1 + sq2 + sq3 + (early ? sq4 : 0));
    ring_barrier();   // every wave's part of chunk j is in LDS; stage (j-1)%NS is free
    const bool tile_end = kc == nk - 1;
    if (!tile_end && lj < total) issue_next();   // lj == j + NS - 1
    const char* st = smem + cs * STAGE_BYTES;
#pragma unroll
    for (int ks = 0; ks < (KAIR_DBG(E.dbg & 2) ? 0 : BK / 32); ++ks) {
      bf16x8 af[RM], bfr[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int r = wm * WROWS + i * 16 + fr;
        af[i] = *(const bf16x8*)(st + r * 128 + (((ks * 4 + fq) ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int jn = 0; jn < RN; ++jn)
        bfr[jn] = *(const bf16x8*)(sB + (wn * TN + jn * 16 + fr) * LDB + kc * BK + ks * 32 + fq * 8);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int jn = 0; jn < RN; ++jn)
          acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[jn], af[i], acc[i][jn], 0, 0, 0);
    }
    int sj = 0;
    const int pol = KAIR_DEBUG_ABLATIONS ? (E.dbg >> 3) & 3 : 0;
    if (tile_end && early && lj < total) issue_next();
    if (tile_end) {
      // Epilogue from registers: fragment pairs are re-laid by v_permlane16_swap so each lane
      // holds 8 consecutive columns of one row; every epilogue load is issued before the first
      // store and landed at once (no path leaves a load pending into the next chunk, where hipcc
      // would drain the ring for it).
      const int mt = mt0 + ct * mstride;
      int mv[RM], rowv[RM];
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int m = mt * BM + wm * WROWS + i * 16 + fr;
        mv[i] = m;
        const int mm = m < (int)E.M ? m : 0;
        if constexpr (EM == EM_ROWS) {
          rowv[i] = win_to_token32(mm, E.win);
        } else {
          const int win = fdiv(mm, E.d_tok);
          rowv[i] = win * E.nh * E.tok + (mm - win * E.tok);
        }
      }
      float4 ex[RM][NP][2];
      if constexpr (EX != EX_NONE) {
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int p = 0; p < NP; ++p) {
            const long rr = rowv[i];
            const long c = colo[p];   // clamped rows / columns read valid memory
            if constexpr (EX == EX_RESID) {
              ex[i][p][0] = *(const float4*)(E.resid + rr * E.ldr + c);
              ex[i][p][1] = *(const float4*)(E.resid + rr * E.ldr + c + 4);
            } else if constexpr (EX == EX_GATE_BF16) {
              const bf16x8 g = *(const bf16x8*)((const bf16*)E.gate + rr * E.ldg + c);
              ex[i][p][0] = make_float4((float)g[0], (float)g[1], (float)g[2], (float)g[3]);
              ex[i][p][1] = make_float4((float)g[4], (float)g[5], (float)g[6], (float)g[7]);
            } else {
              ex[i][p][0] = *(const float4*)((const float*)E.gate + rr * E.ldg + c);
              ex[i][p][1] = *(const float4*)((const float*)E.gate + rr * E.ldg + c + 4);
            }
          }
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int p = 0; p < NP; ++p) { land(ex[i][p][0]); land(ex[i][p][1]); }
      }
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          float v[8];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * p][c]),
                                                            __float_as_uint(acc[i][2 * p + 1][c]), false, false);
            v[c] = __uint_as_float(r[0]);
            v[4 + c] = __uint_as_float(r[1]);
          }
          const int n = c8v[p];
          const bool ok = mv[i] < (int)E.M && n < E.N && !KAIR_DBG(E.dbg & 1);   // N % 8 == 0: whole groups
          const float b8[8] = {bias8[p][0].x, bias8[p][0].y, bias8[p][0].z, bias8[p][0].w,
                               bias8[p][1].x, bias8[p][1].y, bias8[p][1].z, bias8[p][1].w};
#pragma unroll
          for (int c = 0; c < 8; ++c) v[c] += b8[c];
          if constexpr (EM == EM_QKV) {
            const long off = colo[p] + (long)rowv[i] * E.hdp;
            if (ok) st8_any(E.out, E.odt, off, v, pol);
            sj += __ballot(ok) != 0 ? 1 : 0;
          } else {
            float pre[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) {
              pre[c] = v[c];
              if (E.act == KAIR_ACT_GELU) {
                float y, dy;
                gelu_pair_fast(v[c], y, dy);
                v[c] = y;
                if (E.prek) pre[c] = dy;
              } else if (E.act == KAIR_ACT_LEAKY) v[c] = v[c] > 0.f ? v[c] : v[c] * E.slope;
              else if (E.act == KAIR_ACT_RELU) v[c] = fmaxf(v[c], 0.f);
            }
            if constexpr (EX != EX_NONE) {
              const float x8[8] = {ex[i][p][0].x, ex[i][p][0].y, ex[i][p][0].z, ex[i][p][0].w,
                                   ex[i][p][1].x, ex[i][p][1].y, ex[i][p][1].z, ex[i][p][1].w};
              if constexpr (EX == EX_RESID) {
                const float rs = E.rowscale ? sRS[fdiv(rowv[i], E.d_rps)] : 1.f;
#pragma unroll
                for (int c = 0; c < 8; ++c) v[c] = x8[c] + rs * v[c];
              } else {
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                  if (E.gkind == 1) v[c] *= gelu_grad_fast(x8[c]);
                  else if (E.gkind == 2) v[c] *= (x8[c] > 0.f ? 1.f : E.slope);
                  else if (E.gkind == 4) v[c] *= x8[c];
                  else v[c] *= (x8[c] > 0.f ? 1.f : 0.f);
                }
              }
            }
            if (E.ones_col >= n && E.ones_col < n + 8) {
#pragma unroll
              for (int c = 0; c < 8; ++c)
                if (n + c == E.ones_col) v[c] = 1.f;
            }
            const long rr = rowv[i];
            if (ok) {
              st8_any(E.out, E.odt, rr * E.ldo + n, v, pol);
              if (E.pre) st8_any(E.pre, E.pdt, rr * E.ldp + n, pre, pol);
            }
            sj += __ballot(ok) != 0 ? st_per_frag : 0;
          }
        }
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int jn = 0; jn < RN; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (!early && lj < total) issue_next();
    }
    sq4 = sq3; sq3 = sq2; sq2 = sq1; sq1 = sj;
    if (++kc == nk) { kc = 0; ++ct; }
    if (++cs == NS) cs = 0;
  }
}

// ------------------------------------------------------------------------------------------
// TN ring kernel (weight gradients of the Swin block projections, bf16):
//   P[s][n][k] = sum_{m in split s} A[m][n] * B[m][k],   one 192x192 (n,k) tile per CTA.
// 512 threads, one CTA per CU; A and B row chunks (32 rows) stream through a 6-deep LDS ring by
// LDS-DMA (3 wave-instructions per wave per chunk), counted vmcnt + raw barrier; fragments are
// ds_read_b64_tr_b16 transposed reads; D = B^T.A so each lane stores 4 consecutive k (16 B).
// Rows past the split (and columns past N / K) read a zero line.  The bias-gradient "ones" column
// must already be in B (kair_operand.ones_in_data).
// BM_TAP: B is a 3x3 / pad-1 im2col of a bf16 NHWC image with exactly TNR_BK (192) channels, so
// K-tile tk IS tap tk: row m of the tile reads pixel m + dy*W + dx of the image (a zero line where the
// tap leaves the image).  The 9 taps of one row split are consecutive CTAs (one XCD: xcd_remap), so
// the image rows and the A rows come from L2 after the first tap -- the conv weight gradient moves
// ~1x its operands instead of the 9x re-read of a per-K-tile im2col.
// ------------------------------------------------------------------------------------------

#ifndef KAIR_TNR_NSG
#define KAIR_TNR_NSG 6
#endif
constexpr int TNR_BN = 192, TNR_BK = 192, TNR_RB = 32, TNR_NS = 6;
// the grouped launch runs on the side stream beside the data-gradient chain: a shallower ring
// (TNR_NSG stages, 96 KiB) leaves room on each CU for a chain workgroup of <= 64 KiB LDS
constexpr int TNR_NSG = KAIR_TNR_NSG;
constexpr int BM_ROWS = 0, BM_TAP = 1, BM_TAP3 = 2;

// One CTA's share of a TN ring product: rows [mbeg, mend) of the (n0, k0) 192x192 tile -> plane P.
struct TnRingTile {
  const bf16* Ap; const bf16* Bp;
  long Ald, Bld;
  int N, K, M;                                  // M: operand rows (q/k/v part stride)
  int n0, k0, mbeg, mend;
  float* P;                                     // this split's fp32 [N][K] plane
};

// the chunk permutation of LDS row r (see tn_ring_body): rows {0, 2, 8, 10} + 16 k and {1, 3, 9, 11} + 16 k
// -- the rows one 32-lane half reads together -- get distinct chunk offsets 0 / 2 / 4 / 6
KAIR_DEV int tn_sw(int r) { return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }

template <int AMA, int BMB, int NS>
KAIR_DEV void tn_ring_body(const TnRingTile& t, const Op& A, const Op& Bo, char* smem) {
  constexpr int BNt = TNR_BN, BKt = TNR_BK, RB = TNR_RB;
  static_assert(NS >= 3 && NS <= 6, "ring depth: the counted waits below cover 1..4 chunks ahead");
  constexpr int PART = RB * BNt * 2;            // 12 KiB (A part; B part the same since BKt == BNt)
  constexpr int STAGE = 2 * PART;
  constexpr int ROWB = BNt * 2;                  // 384 B per LDS row
  constexpr int RN = 6, RK = 3;                  // wave tile 96 (n) x 48 (k)
  const int n0 = t.n0, k0 = t.k0, mbeg = t.mbeg, mend = t.mend, N = t.N, K = t.K, M = t.M;
  const int nchunks = mbeg < mend ? (mend - mbeg + RB - 1) / RB : 0;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave >> 2, wk = wave & 3;

  // operand bases as scalars: selecting A or B fields per lane below would otherwise read the
  // kernel-argument struct through a VGPR pointer (a global load + vmcnt(0) before every DMA)
  const bf16* const Ap = t.Ap;
  const bf16* const Bp = t.Bp;
  const long Ald = t.Ald, Bld = t.Bld;
  // BM_TAP: this tile's tap (dy, dx) and its row offset in the image
  const int tap = BMB == BM_TAP ? k0 / BKt : 0;
  const int tdy = tap / 3 - 1, tdx = tap - 3 * (tap / 3) - 1;
  const int tshift = BMB == BM_TAP ? tdy * Bo.imW + tdx : 0;
  // LDS rows of 384 B put rows r and r + 2 (and r + 8) on the same banks: the transposed fragment reads
  // (rows g8 + q and + 4 of a 32-lane half) were 4-way conflicted (PMC: 75 % of the LDS cycles).  The
  // 16-byte chunks of row r sit XOR-permuted by tn_sw(r) (even, < 8: a chunk pair stays adjacent, a row
  // stays within its 24 chunks); the DMA fetches, for each LDS slot, the logical chunk that lands there.
  auto issue = [&](int j) {
    const int m0 = mbeg + j * RB;
    char* st = smem + (j % NS) * STAGE;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int g = wave * 3 + i;                // 0..23: 12 KiB of A then 12 KiB of B
      const bool isB = g >= 12;
      const int off = (isB ? g - 12 : g) * 1024 + lane * 16;
      const int r = off / ROWB, c = (((off - (off / ROWB) * ROWB) >> 4) ^ tn_sw(r)) << 3;
      const int m = m0 + r;
      const void* src = g_kair_zero_line;
      if (m < mend) {
        if (isB) {
          if constexpr (BMB == BM_TAP) {
            const int p = m - fdiv(m, Bo.d_hw) * Bo.d_hw.d;   // pixel within the image
            const int y = fdiv(p, Bo.d_imW), x = p - y * Bo.imW;
            if ((unsigned)(y + tdy) < (unsigned)Bo.imH && (unsigned)(x + tdx) < (unsigned)Bo.imW)
              src = Bp + (long)(m + tshift) * Bld + c;
          } else if constexpr (BMB == BM_TAP3) {   // 64-channel image: K tile tk = taps 3 tk .. 3 tk + 2
            const int tp = 3 * (k0 / BKt) + (c >> 6);
            const int dy = tp / 3 - 1, dx = tp - 3 * (tp / 3) - 1;
            const int p = m - fdiv(m, Bo.d_hw) * Bo.d_hw.d;
            const int y = fdiv(p, Bo.d_imW), x = p - y * Bo.imW;
            if ((unsigned)(y + dy) < (unsigned)Bo.imH && (unsigned)(x + dx) < (unsigned)Bo.imW)
              src = Bp + (long)(m + dy * Bo.imW + dx) * Bld + (c & 63);
          } else if (k0 + c < K) {
            src = Bp + (long)m * Bld + k0 + c;
          }
        } else if (n0 + c < N) {
          if constexpr (AMA == AM_ROWS) {
            src = Ap + (long)m * Ald + n0 + c;
          } else {
            const int n = n0 + c, pw = A.d_pw.d;
            const int part = fdiv(n, A.d_pw), rr = n - part * pw;
            const int h = fdiv(rr, A.d_hdp), d = rr - h * A.hdp;
            const int win = fdiv(m, A.d_tok), tk = m - win * A.tok;
            src = Ap + (long)part * M * pw + (((long)win * A.nh + h) * A.tok + tk) * A.hdp + d;
          }
        }
      }
      glds16(src, st + (isB ? PART : 0) + (g % 12) * 1024);
    }
  };

#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (j < nchunks) issue(j);

  f32x4 acc[RK][RN];
#pragma unroll
  for (int j = 0; j < RK; ++j)
#pragma unroll
    for (int i = 0; i < RN; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int q = (lane & 15) >> 2, p4 = (lane & 3) * 4, g8 = (lane >> 4) * 8;
  const int R0 = g8 + q, sw0 = tn_sw(R0), sw4 = tn_sw(R0 + 4);   // this lane's two fragment rows
  for (int j = 0; j < nchunks; ++j) {
    const int ahead = (nchunks - 1 - j) < (NS - 2) ? (nchunks - 1 - j) : (NS - 2);
    if (ahead >= 4) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (ahead == 3) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
    else if (ahead == 2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ring_barrier();
    if (j + NS - 1 < nchunks) issue(j + NS - 1);
    const bf16* sA = (const bf16*)(smem + (j % NS) * STAGE);
    const bf16* sB = sA + RB * BNt;
    bf16x8 af[RN], bfr[RK];
#pragma unroll
    for (int i = 0; i < RN; ++i) {
      const int ch = wn * 12 + 2 * i + (p4 >> 3);   // logical 16-byte chunk of the 8-byte read
      const bf16* base = sA + R0 * BNt + ((ch ^ sw0) << 3) + (p4 & 7);
      const bf16* base4 = sA + (R0 + 4) * BNt + ((ch ^ sw4) << 3) + (p4 & 7);
      const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)base);
      const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)base4);
      short __attribute__((ext_vector_type(8))) s8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      af[i] = __builtin_bit_cast(bf16x8, s8);
    }
#pragma unroll
    for (int jk = 0; jk < RK; ++jk) {
      const int ch = wk * 6 + 2 * jk + (p4 >> 3);
      const bf16* base = sB + R0 * BKt + ((ch ^ sw0) << 3) + (p4 & 7);
      const bf16* base4 = sB + (R0 + 4) * BKt + ((ch ^ sw4) << 3) + (p4 & 7);
      const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)base);
      const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)base4);
      short __attribute__((ext_vector_type(8))) s8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      bfr[jk] = __builtin_bit_cast(bf16x8, s8);
    }
#pragma unroll
    for (int jk = 0; jk < RK; ++jk)
#pragma unroll
      for (int i = 0; i < RN; ++i)
        acc[jk][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[jk], af[i], acc[jk][i], 0, 0, 0);
  }
  // lane holds k = kb + 4*(lane>>4) + r (r < 4) of column n = nb + (lane & 15)
  float* P = t.P;
#pragma unroll
  for (int jk = 0; jk < RK; ++jk)
#pragma unroll
    for (int i = 0; i < RN; ++i) {
      const int n = n0 + wn * 96 + i * 16 + (lane & 15);
      const int k = k0 + wk * 48 + jk * 16 + 4 * (lane >> 4);
      if (n < N && k < K) *(float4*)(P + (long)n * K + k) = make_float4(acc[jk][i][0], acc[jk][i][1], acc[jk][i][2], acc[jk][i][3]);
    }
}

// BM_TAP (the conv weight gradients, side stream) runs the grouped launch's shallower ring
template <int AMA, int BMB>
__global__ __launch_bounds__(512, 1) void gemm_tn_ring(Op A, Op B, float* ws, int M, int N, int K, int tilesK, int ntiles,
                                                       int rows_per_split) {
  constexpr int NS = BMB == BM_TAP ? TNR_NSG : TNR_NS;
  __shared__ __attribute__((aligned(16))) char smem[NS * 2 * TNR_RB * TNR_BN * 2];
  const int cta = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = cta % ntiles, split = cta / ntiles;
  const int tn = tile / tilesK, tk = tile - (tile / tilesK) * tilesK;
  TnRingTile t;
  t.Ap = (const bf16*)A.ptr; t.Bp = (const bf16*)B.ptr;
  t.Ald = A.ld; t.Bld = B.ld;
  t.N = N; t.K = K; t.M = M;
  t.n0 = tn * TNR_BN; t.k0 = tk * TNR_BK;
  t.mbeg = split * rows_per_split;
  t.mend = t.mbeg + rows_per_split < M ? t.mbeg + rows_per_split : M;
  t.P = ws + (long)split * N * K;
  tn_ring_body<AMA, BMB, NS>(t, A, B, smem);
}

// ------------------------------------------------------------------------------------------
// Grouped TN ring (kair_wgrad_grouped): the weight gradients of several layers in ONE launch.
// Every job is a bf16 [M][N]^T x [M][K] product split into `splits` row ranges; CTA ->
// (split, global tile) with the job found by a scalar scan of the tile offsets.  The job table is
// the kernel argument (no device table: graph capture keeps the pointers by value).
// ------------------------------------------------------------------------------------------
constexpr int WG_MAX = 24;
struct TnJob {
  const bf16* a; const bf16* b; float* ws;      // ws: this job's [splits][N][K] planes
  int lda, ldb, N, K, tilesK, tile0, qkv, pad;
};
struct TnGroup {
  TnJob j[WG_MAX];
  int njobs, ntiles, M, rps;
  Op qa;                                        // q/k/v geometry shared by the QKVBLK jobs
};

__global__ __launch_bounds__(512, 1) void gemm_tn_ring_grouped(const TnGroup g) {
  __shared__ __attribute__((aligned(16))) char smem[TNR_NSG * 2 * TNR_RB * TNR_BN * 2];
  const int cta = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = cta % g.ntiles, split = cta / g.ntiles;
  int ji = 0;
  for (int i = 1; i < g.njobs; ++i)
    if (g.j[i].tile0 <= tile) ji = i;
  ji = __builtin_amdgcn_readfirstlane(ji);
  const TnJob& jb = g.j[ji];
  const int lt = tile - jb.tile0;
  const int tn = lt / jb.tilesK, tk = lt - (lt / jb.tilesK) * jb.tilesK;
  TnRingTile t;
  t.Ap = jb.a; t.Bp = jb.b;
  t.Ald = jb.lda; t.Bld = jb.ldb;
  t.N = jb.N; t.K = jb.K; t.M = g.M;
  t.n0 = tn * TNR_BN; t.k0 = tk * TNR_BK;
  t.mbeg = split * g.rps;
  t.mend = t.mbeg + g.rps < g.M ? t.mbeg + g.rps : g.M;
  t.P = jb.ws + (long)split * jb.N * jb.K;
  if (jb.qkv) tn_ring_body<AM_QKV, BM_ROWS, TNR_NSG>(t, g.qa, g.qa, smem);
  else tn_ring_body<AM_ROWS, BM_ROWS, TNR_NSG>(t, g.qa, g.qa, smem);
}

// ------------------------------------------------------------------------------------------
// TN kernel (weight gradient): P[s][n][k] = sum_{m in split s} A[m][n] * B[m][k]
// LDS holds both operands m-major ([BMr m][BN], [BMr m][BKo]) as loaded; bf16 fragments (8
// consecutive m of one column) come from two ds_read_b64_tr_b16 transposed reads.
// ------------------------------------------------------------------------------------------
template <typename CT, typename TA, typename TB, int AMA, int AMB, int BN, int BKo>
__global__ __launch_bounds__(NT, 2) void gemm_tn_kernel(Op A, Op B, float* ws, long M, int N, int K, long rows_per_split,
                                                        int tilesK) {
  constexpr int BMr = sizeof(CT) == 2 ? 64 : 32;   // reduction rows per step
  constexpr int LDA = BN + 8, LDB = BKo + 8;
  constexpr int WN = 2, WK = 2;
  constexpr int TN_ = BN / WN, TK_ = BKo / WK;
  constexpr int RN = TN_ / 16, RK = TK_ / 16;
  constexpr int CPA = BN / 8, CPB = BKo / 8;
  constexpr int CA = BMr * CPA, CB = BMr * CPB;
  constexpr int PA = (CA + NT - 1) / NT, PB = (CB + NT - 1) / NT;
  constexpr int STAGE = BMr * (LDA + LDB);
  __shared__ __attribute__((aligned(16))) CT lds[2 * STAGE];

  const int tn = blockIdx.x / tilesK, tk = blockIdx.x - (blockIdx.x / tilesK) * tilesK;
  const int n0 = tn * BN, k0 = tk * BKo;
  const long mbeg = (long)blockIdx.y * rows_per_split;
  long mend = mbeg + rows_per_split;
  if (mend > M) mend = M;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave / WK, wk = wave % WK;

  Raw<TA> va[PA];
  Raw<TB> vb[PB];
  Pend pa[PA], pb[PB];
  auto gload = [&](long mb) {
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int c = tid + p * NT;
      if (c < CA) {
        const long m = mb + c / CPA;
        const RowState r = row_state<AMA, TA>(A, m < mend ? m : A.M);
        issue_chunk<AMA, TA>(A, r, n0 + (c % CPA) * 8, N, va[p], pa[p]);
      }
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int c = tid + p * NT;
      if (c < CB) {
        const long m = mb + c / CPB;
        const RowState r = row_state<AMB, TB>(B, m < mend ? m : B.M);
        issue_chunk<AMB, TB>(B, r, k0 + (c % CPB) * 8, K, vb[p], pb[p]);
      }
    }
  };
  auto sstore = [&](int st) {
    CT* sA = lds + st * STAGE;
    CT* sB = sA + BMr * LDA;
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int c = tid + p * NT;
      if (c < CA) commit_chunk<CT, TA>(sA + (c / CPA) * LDA + (c % CPA) * 8, va[p], pa[p]);
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int c = tid + p * NT;
      if (c < CB) commit_chunk<CT, TB>(sB + (c / CPB) * LDB + (c % CPB) * 8, vb[p], pb[p]);
    }
  };

  f32x4 acc[RN][RK];
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int j = 0; j < RK; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  const int nsteps = mbeg < mend ? (int)((mend - mbeg + BMr - 1) / BMr) : 0;
  if (nsteps > 0) {
    gload(mbeg);
    sstore(0);
    __syncthreads();
  }
  for (int it = 0; it < nsteps; ++it) {
    const int st = it & 1;
    if (it + 1 < nsteps) gload(mbeg + (long)(it + 1) * BMr);
    const CT* sA = lds + st * STAGE;
    const CT* sB = sA + BMr * LDA;
    if constexpr (sizeof(CT) == 2) {
      const int q = (lane & 15) >> 2, p4 = (lane & 3) * 4, g8 = (lane >> 4) * 8;
#pragma unroll
      for (int ks = 0; ks < BMr / 32; ++ks) {
        bf16x8 af[RN], bfr[RK];
#pragma unroll
        for (int i = 0; i < RN; ++i) {
          const CT* base = sA + (ks * 32 + g8 + q) * LDA + wn * TN_ + i * 16 + p4;
          const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)base);
          const short4v hi =
              __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)(base + 4 * LDA));
          short __attribute__((ext_vector_type(8))) s8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          af[i] = __builtin_bit_cast(bf16x8, s8);
        }
#pragma unroll
        for (int j = 0; j < RK; ++j) {
          const CT* base = sB + (ks * 32 + g8 + q) * LDB + wk * TK_ + j * 16 + p4;
          const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)base);
          const short4v hi =
              __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)(base + 4 * LDB));
          short __attribute__((ext_vector_type(8))) s8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          bfr[j] = __builtin_bit_cast(bf16x8, s8);
        }
#pragma unroll
        for (int i = 0; i < RN; ++i)
#pragma unroll
          for (int j = 0; j < RK; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < BMr / 4; ++s) {
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
    if (it + 1 < nsteps) sstore(st ^ 1);
    __syncthreads();
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

// ------------------------------------------------------------------------------------------
// dispatch
// ------------------------------------------------------------------------------------------
template <typename CT, typename TA, int AM, int BM, int BN, int WM, int WN>
int launch_nt(const Op& A, const Op& B, const Epi& E, long M, int N, int K, hipStream_t s) {
  const long tilesM = (M + BM - 1) / BM;
  const int tilesN = (N + BN - 1) / BN;
  const long nwg = tilesM * tilesN;
  if (nwg > 0x7fffffff) return kair_set_error(KAIR_ERR_ARG, "gemm_nt: grid too large");
  KAIR_LAUNCH((gemm_nt_kernel<CT, TA, AM, BM, BN, WM, WN>), dim3((unsigned)nwg), dim3(NT), 0, s, A, B, E, K, tilesN,
                     (int)nwg);
  KAIR_CHECK_LAUNCH();
  return 0;
}

static int g_num_cus = 0;
static const int g_ring_mode = 1;   // the LDS-DMA ring kernels (measured A/B switch in round 1)
static const int g_halo_mode = 1;
static long g_ring_min_tiles = -1;

static void init_num_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    n = 256;
  g_num_cus = n > 0 ? n : 256;
  g_ring_min_tiles = g_num_cus;   // the persistent ring kernel only with >= one tile per CU
}

// Tile choice of the register-staged kernel: the largest tile that still gives >= 2 CTAs per CU
// (small per-GPU batches, e.g. 4 patches/GPU at 8 GPUs, would otherwise leave most CUs idle).
template <typename CT, typename TA, int AM>
int nt_tiles(const Op& A, const Op& B, const Epi& E, long M, int N, int K, hipStream_t s) {
  if (N <= 16) return launch_nt<CT, TA, AM, 256, 16, 4, 1>(A, B, E, M, N, K, s);
  if (g_num_cus == 0) init_num_cus();
  // 32x32 tiles for N <= 32 (RRDB dense-block convs, growth 32; ResUNet level-2 convs): no half-empty
  // 64-wide N tile, twice the CTAs on these small-M, long-K convs (RRDBNet B=16: 421 -> 436
  // patches/s; 64x32 tiles 429).  (measured against 64x32 and 64x64)
  constexpr int n32 = 2;
  if (N <= 32 && n32 == 1) return launch_nt<CT, TA, AM, 64, 32, 2, 2>(A, B, E, M, N, K, s);
  if (N <= 32 && n32 == 2) return launch_nt<CT, TA, AM, 32, 32, 2, 2>(A, B, E, M, N, K, s);
  const long tm = (M + 127) / 128;
  // (thresholds at >= 1 or 0.5 CTAs per CU measured slower at B = 4: 476 -> 460 / 390 patches/s)
  const long min_ctas = 2L * g_num_cus;
  if (N > 64 && tm * ((N + 127) / 128) >= min_ctas) return launch_nt<CT, TA, AM, 128, 128, 2, 2>(A, B, E, M, N, K, s);
  if (tm * ((N + 63) / 64) >= min_ctas || M <= 64) return launch_nt<CT, TA, AM, 128, 64, 2, 2>(A, B, E, M, N, K, s);
  return launch_nt<CT, TA, AM, 64, 64, 2, 2>(A, B, E, M, N, K, s);
}

// 4-column register epilogue: ROWS / QKV outputs whose vectors are 4-aligned
static bool epi4_ok(const Epi& e, int N) {
  if (N % 4 != 0 || N < 64 || e.resid2) return false;
  if (e.omode == KAIR_OUT_QKVBLK) return e.hdp % 4 == 0;
  if (e.omode != KAIR_OUT_ROWS) return false;
  return e.ldo % 4 == 0 && (!e.pre || e.ldp % 4 == 0) && (!e.resid || e.ldr % 4 == 0) && (!e.gate || e.ldg % 4 == 0);
}

template <int BN, int NS, int AM>
int launch_ring(const Op& A, const Op& B, const Epi& E, long M, int N, int K, hipStream_t s) {
  const int tilesN = (N + BN - 1) / BN;
  const int tilesM = (int)((M + RING_BM - 1) / RING_BM);
  int grid = (g_num_cus / tilesN) * tilesN;
  if (grid < tilesN) grid = tilesN;
  const int need = tilesM * tilesN;
  if (grid > need) grid = need;
  const dim3 g(grid), b(512);
  if (E.omode == KAIR_OUT_QKVBLK)
    KAIR_LAUNCH((gemm_nt_ring<BN, NS, AM, EM_QKV, EX_NONE>), g, b, 0, s, A, B, E, K, tilesN, tilesM);
  else if (E.resid)
    KAIR_LAUNCH((gemm_nt_ring<BN, NS, AM, EM_ROWS, EX_RESID>), g, b, 0, s, A, B, E, K, tilesN, tilesM);
  else if (E.gate && E.gdt == KAIR_BF16)
    KAIR_LAUNCH((gemm_nt_ring<BN, NS, AM, EM_ROWS, EX_GATE_BF16>), g, b, 0, s, A, B, E, K, tilesN, tilesM);
  else if (E.gate)
    KAIR_LAUNCH((gemm_nt_ring<BN, NS, AM, EM_ROWS, EX_GATE_F32>), g, b, 0, s, A, B, E, K, tilesN, tilesM);
  else
    KAIR_LAUNCH((gemm_nt_ring<BN, NS, AM, EM_ROWS, EX_NONE>), g, b, 0, s, A, B, E, K, tilesN, tilesM);
  KAIR_CHECK_LAUNCH();
  return 0;
}

// The ring's N tile.  Narrow outputs take ONE N tile, so A streams through the ring once: N <= 64 (the
// SwinIR-lightweight block's Cp = 64 projections: fc2 / proj forward, fc1 input gradient) a 64-wide tile,
// N <= 96 a 96-wide one, N <= 128 at K <= 256 (its fc1 forward and gated fc2 input gradient, Hdp = 128) a 128-wide
// one (against a 192-wide tile, whose second wave column had 32 of 96 columns to store: C2 2,171 -> 2,240 patches/s) rather than two
// 96-wide tiles that read A twice.  Wider outputs (the classical Cp = 192 geometry): a gated
// epilogue (the fc2 input gradient, N = 384) four 96-wide N tiles rather than two 192-wide ones -- each CTA's
// epilogue reads half the gate columns per tile (B = 32: 1015 -> 1019 patches/s); one 192-wide N tile leaves the
// persistent CTAs unevenly loaded (B = 32: 576 M-tiles on 256 CUs -> 3 vs 2.25 on average), two 96-wide tiles
// balance better (815 -> 823 patches/s) except for the q/k/v output.
static const int g_ring_bn128 = [] {   // KAIR_RING_BN128=0: N <= 128 on the 192-wide tile (A/B)
  const char* e = getenv("KAIR_RING_BN128");
  return e && atoi(e) == 0 ? 0 : 1;
}();
static int ring_bn_of(const Epi& E, int N, int K) {
  K = (K + RING_BK - 1) / RING_BK * RING_BK;   // the chunked K
  if (N <= 64) return 64;
  if (N <= 96 && K <= 384) return 96;
  if (N <= 128 && K <= 256 && g_ring_bn128) return 128;
  if (N <= 128 && K <= 192) return 192;
  if (E.gate && K <= 192) return 96;
  if (K <= 192 && !(N <= 192 && E.omode != KAIR_OUT_QKVBLK)) return 192;
  if (K <= 384) return 96;
  return 64;
}

// ring kernel: bf16 A (rows, optionally window-mapped, or head-blocked q/k/v) with no row scale
static bool ring_ok(int amode, const Op& A, const Op& B, const Epi& e, long M, int N, int K) {
  if (K % 8 != 0 || K > 576 || M >= (1L << 30)) return false;
  if (amode != KAIR_LD_ROWS && amode != KAIR_LD_QKVBLK) return false;
  if (A.rowscale || A.ones_col >= 0 || A.asplit || e.out_lo) return false;
  if (amode == KAIR_LD_ROWS && A.ld % 8 != 0) return false;
  if (amode == KAIR_LD_QKVBLK && (A.hdp % 8 != 0)) return false;
  if (B.ld % 8 != 0 || B.ones_col >= 0 || B.wsplit) return false;
  if (e.resid && e.gate) return false;   // one epilogue operand per ring kernel
  // 8-column epilogue groups: whole groups, 16-byte aligned rows / pointers
  if (N % 8 != 0) return false;
  auto al16 = [](const void* q) { return ((unsigned long)q & 15) == 0; };
  if (!al16(e.out) || (e.pre && !al16(e.pre)) || (e.gate && !al16(e.gate)) || (e.resid && !al16(e.resid)))
    return false;
  if ((e.odt == KAIR_BF16 && e.ldo % 8) || (e.pre && e.pdt == KAIR_BF16 && e.ldp % 8) ||
      (e.gate && e.gdt == KAIR_BF16 && e.ldg % 8))
    return false;
  if (e.omode == KAIR_OUT_QKVBLK && e.hdp % 8) return false;
  if (e.rowscale && (!e.resid || (M + e.rps - 1) / e.rps > RING_RS_MAX)) return false;
  if (e.omode == KAIR_OUT_QKVBLK) {         // the staged store groups whole heads per wave
    const int bn = ring_bn_of(e, N, K);
    const int TN = bn == 96 ? 96 : bn / 2;
    if (e.hdp <= 0 || TN % e.hdp != 0) return false;
  }
  return epi4_ok(e, N);
}

template <int AM>
int ring_bn(const Op& A, const Op& B, const Epi& E, long M, int N, int K, hipStream_t s) {
  const int bn = ring_bn_of(E, N, K);
  if (bn == 192) return launch_ring<192, 5, AM>(A, B, E, M, N, K, s);
  if (bn == 128) return launch_ring<128, 5, AM>(A, B, E, M, N, K, s);
  if (bn == 96) return launch_ring<96, 5, AM>(A, B, E, M, N, K, s);
  return launch_ring<64, 5, AM>(A, B, E, M, N, K, s);
}

// ------------------------------------------------------------------------------------------
// 3x3 conv (stride 1, pad 1; forward, or input gradient with flipped taps) as implicit GEMM with
// the input tile's halo resident in LDS.  Tile = 96 output pixels (96/W whole image rows of width
// W <= 96, or 96 pixels of a wider row) x all N <= 192 output channels; one 512-thread CTA per CU,
// persistent over tiles.  Each input pixel is fetched once per tile instead of once per tap (the
// register-staged im2col GEMM re-reads it 9 times and is L2-bandwidth bound); the weights
// [N][9 Cin] stream through a double-buffered LDS stage, two k-steps ahead in registers.
// MFMA operands swapped (D = W . X^T) so each lane finishes 4 consecutive channels of a pixel.
// ------------------------------------------------------------------------------------------
constexpr int HC_BM = 96, HC_BN = 192, HC_BK = 64;
constexpr int HC_HALO_ELEMS = 40960;   // bf16 elements: (RPT + 2) x (XW + 2) x (Cin + 8)
constexpr int HC_PER = HC_HALO_ELEMS / 8 / 512;
constexpr int HC_EM_ROWS = 0, HC_EM_PSHUF = 1, HC_EM_PUNSHUF = 2;   // epilogue: token rows / PixelShuffle
                                                                  // sub-pixel-major (PSHUF_SPM) / its inverse

// BN: output channels per tile (192, or 128 for N in (192, 256]: N tiles of one M tile run on
// consecutive workgroups, each with its own weight rows; the persistent grid is a multiple of the
// N-tile count so a workgroup's N tile -- its bias and weight rows -- never changes).
// bf16 A with a_split == 2: the image's channels are [hi | lo] halves of one activation and the
// weights (hi/lo split, tied over the halves) give 4 chunk products per tap; the lo.lo one is skipped.
// BM: output pixels per tile, 96 or (128-wide N tiles of images with <= 128 channels) 192 -- twice the
// pixels per streamed weight chunk, so half the weight traffic from L2 (the upsampling convs' bound).
template <int BM> struct HaloSize { static constexpr int ELEMS = BM == 192 ? 57344 : HC_HALO_ELEMS; };
// CGM > 1: an image of C = 64 CGM channels (C > 192: the upsampling convs' input gradients, C = 256) in
// CGM passes over the tile, pass p holding channels [64 p, 64 p + 64) in the halo and running the nine
// weight chunks of that channel group, accumulating.
template <typename TA, int EX, int NPASS, int BN, int EM, int BM, int CGM>
__global__ __launch_bounds__(512, 1) void conv3x3_halo_kernel(Op A, Op B, Epi E, int K, int tilesM) {
  constexpr int WM = 2, WN = 4, TM = BM / WM, TN = BN / WN, RM = TM / 16, RN = TN / 16;
  constexpr int NI = BN / 64;   // LDS-DMA wave-instructions per weight chunk (8 rows x 128 B each)
  constexpr int HALO = HaloSize<BM>::ELEMS, HPER = HALO / 8 / 512;
  __shared__ __attribute__((aligned(16))) bf16 sHalo[HALO];
  __shared__ __attribute__((aligned(16))) bf16 sBw[3][BN * HC_BK];   // LDS-DMA ring of weight chunks
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int fr = lane & 15, fq = lane >> 4;
  const int H = A.imH, W = A.imW, C = A.imC;
  constexpr bool CG = CGM > 1;
  const int XW = W < BM ? W : BM, RPT = BM / XW, HWD = XW + 2, HR = RPT + 2, PS = (CG ? HC_BK : C) + 8;
  const int sh = B.wsplit;   // hi/lo split weights: weight chunk j pairs with halo chunk j >> 1
  // NPASS 2 -- hi/lo split activations (fp32 A, kair_operand.a_split): a second pass over the tile with
  // the halo refilled by the lo halves bf16(x - bf16(x)) and only the hi weight chunks (the a_lo . w_hi
  // product), accumulating into the same tile
  constexpr int npass = CG ? CGM : NPASS;
  const int cpt = C / HC_BK, nks = (9 * cpt) << sh, c8n = (CG ? HC_BK : C) / 8;
  const bool pair = sizeof(TA) == 2 && A.asplit == 2 && sh && cpt == 2;   // skip lo . lo (chunk 4t + 3)
  const int halo_pieces = HR * HWD * c8n;
  const TA* Ap = (const TA*)A.ptr;
  const int N = E.N;
  const int tilesN = (N + BN - 1) / BN, tn = blockIdx.x % tilesN, n0 = tn * BN;
  const bf16* Bp = (const bf16*)B.ptr + (long)n0 * B.ld;   // this workgroup's weight rows
  const int Nt = N - n0 < BN ? N - n0 : BN;                 // real rows of the tile

  // per-lane constants: halo element offset of each fragment row's centre pixel, weight rows
  int hb[RM];
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    const int row = wm * TM + i * 16 + fr;
    const int ry = row / XW, rx = row - (row / XW) * XW;
    hb[i] = ((ry + 1) * HWD + rx + 1) * PS;
  }
  int nrow[RN];
#pragma unroll
  for (int jn = 0; jn < RN; ++jn) nrow[jn] = wn * TN + jn * 16 + fr;
  float4 bias4[RN];
#pragma unroll
  for (int jn = 0; jn < RN; ++jn) {
    const int n = n0 + wn * TN + jn * 16 + fq * 4;
    bias4[jn] = *(const float4*)(E.bias && n < N ? E.bias + n : (const float*)g_kair_zero_line);
  }
#pragma unroll
  for (int jn = 0; jn < RN; ++jn) land(bias4[jn]);

  // weight chunk j (BN rows x 64 k) -> ring stage js % 3 by LDS-DMA: NI wave-instructions per wave,
  // each 8 rows x 128 B; source pieces XOR-swizzled by row so the fragment reads are conflict-light.
  // Rows >= Nt re-read row Nt-1: they only feed output columns >= N, never stored.
  auto bissue = [&](int js, int j) {
    char* st = (char*)sBw[js % 3];
#pragma unroll
    for (int ii = 0; ii < NI; ++ii) {
      const int r = (wave * NI + ii) * 8 + (lane >> 3), q = lane & 7;
      const int rr = r < Nt ? r : Nt - 1;
      glds16(Bp + (long)rr * B.ld + j * HC_BK + ((q ^ (r & 7)) << 3), st + (wave * NI + ii) * 1024);
    }
  };
  f32x4 acc[RM][RN];
  auto compute = [&](int buf, int jw) {
    const int j = jw >> sh;
    const int tap = j / cpt, cc = j - tap * cpt;
    int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
    if (A.flip) { dy = -dy; dx = -dx; }
    const int hoff = (dy * HWD + dx) * PS + (CG ? 0 : cc * HC_BK);   // CG: the halo holds one channel group
#pragma unroll
    for (int ks = 0; ks < HC_BK / 32; ++ks) {
      bf16x8 af[RM], bfr[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) af[i] = *(const bf16x8*)(sHalo + hb[i] + hoff + ks * 32 + fq * 8);
#pragma unroll
      for (int jn = 0; jn < RN; ++jn)
        bfr[jn] = *(const bf16x8*)(&sBw[buf][nrow[jn] * HC_BK + (((ks * 4 + fq) ^ (nrow[jn] & 7)) << 3)]);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int jn = 0; jn < RN; ++jn)
          acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[jn], af[i], acc[i][jn], 0, 0, 0);
    }
  };

  for (int t = blockIdx.x / tilesN; t < tilesM; t += gridDim.x / tilesN) {
    const long p0 = (long)t * BM;
    const int b = (int)(p0 / ((long)H * W));
    const int rem = (int)(p0 - (long)b * H * W);
    const int y0 = rem / W, x0 = rem - (rem / W) * W;
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int jn = 0; jn < RN; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};
    float4 ex[RM][RN];
    // epilogue operand (fp32 residual): loaded two k-chunks before the end of the last pass, after that
    // chunk's ring wait, so its latency hides under the last chunks' MFMAs instead of following them
    // (the younger DMA count is then 0: no chunk is issued after the last one)
    auto load_resid = [&]() {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int jn = 0; jn < RN; ++jn) {
          const long m = p0 + wm * TM + i * 16 + fr;
          const int n = n0 + wn * TN + jn * 16 + fq * 4;
          ex[i][jn] = *(const float4*)(E.resid + m * E.ldr + (n < N ? n : 0));
        }
    };
#pragma unroll
    for (int pass = 0; pass < npass; ++pass) {
    const bool last = pass == npass - 1;
    __syncthreads();   // every wave is done reading the previous tile's (or pass's) halo and ring
    // halo of this tile:
    // all loads first, then the converts and LDS writes
    {
      // (1) every load issued unconditionally (clamped address), (2) landed in order, (3) masked,
      // converted and written: a load whose value a path ignores becomes a branch + wait each
      constexpr int HP = 5;   // pieces per batch (register budget for fp32 pieces)
#pragma unroll
      for (int h0 = 0; h0 < HPER; h0 += HP) {
        uint4 lo[HP], hi[HP];
        bool okv[HP];
#pragma unroll
        for (int i = 0; i < HP; ++i) {
          const int idx = tid + 512 * (h0 + i);
          const int pix = idx / c8n, c8 = idx - (idx / c8n) * c8n;
          const int hr = pix / HWD, hc = pix - (pix / HWD) * HWD;
          const int y = y0 - 1 + hr, x = x0 - 1 + hc;
          okv[i] = idx < halo_pieces && y >= 0 && y < H && x >= 0 && x < W;
          const long src = okv[i] ? ((long)(b * H + y) * W + x) * A.ld + (CG ? HC_BK * pass : 0) + c8 * 8 : 0;
          lo[i] = *(const uint4*)(Ap + src);
          if constexpr (sizeof(TA) == 4) hi[i] = *(const uint4*)(Ap + src + 4);
        }
#pragma unroll
        for (int i = 0; i < HP; ++i) {
          asm volatile("" : "+v"(lo[i].x), "+v"(lo[i].y), "+v"(lo[i].z), "+v"(lo[i].w));
          if constexpr (sizeof(TA) == 4) asm volatile("" : "+v"(hi[i].x), "+v"(hi[i].y), "+v"(hi[i].z), "+v"(hi[i].w));
        }
#pragma unroll
        for (int i = 0; i < HP; ++i) {
          const int idx = tid + 512 * (h0 + i);
          uint4 q;
          if constexpr (sizeof(TA) == 4) {
            const float4 u = __builtin_bit_cast(float4, lo[i]), v = __builtin_bit_cast(float4, hi[i]);
            const float f[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
            bf16x8 qq;
#pragma unroll
            for (int e8 = 0; e8 < 8; ++e8) qq[e8] = (NPASS == 2 && pass) ? (bf16)(f[e8] - (float)(bf16)f[e8]) : (bf16)f[e8];
            q = __builtin_bit_cast(uint4, qq);
          } else {
            q = lo[i];
          }
          if (!okv[i]) q = make_uint4(0, 0, 0, 0);
          if (idx < halo_pieces) {
            const int pix = idx / c8n, c8 = idx - (idx / c8n) * c8n;
            *(uint4*)(sHalo + pix * PS + c8 * 8) = q;
            if (E.acopy && pass == 0 && tn == 0) {   // the tile's own pixels (halo interior): bf16 copy for the weight gradient
              const int hr = pix / HWD, hc = pix - (pix / HWD) * HWD;
              if (hr >= 1 && hr <= RPT && hc >= 1 && hc <= XW) {
                uint4 qc = q;
                const int oc = E.acones - c8 * 8;
                if ((unsigned)oc < 8u) {
                  bf16x8 v8 = __builtin_bit_cast(bf16x8, qc);
                  v8[oc] = (bf16)1.f;
                  qc = __builtin_bit_cast(uint4, v8);
                }
                const long px = ((long)(b * H + y0 + hr - 1) * W + x0 + hc - 1);
                *(uint4*)(E.acopy + px * E.ldac + c8 * 8) = qc;
              }
            }
          }
        }
      }
    }
    __syncthreads();   // halo visible
    // pass 1 (lo halo): the hi weight chunks only, chunk j of the pass = weight chunk j << sh;
    // a [hi | lo] pair image: per tap the weight chunks 4t, 4t+1, 4t+2 (hi.w_hi, hi.w_lo, lo.w_hi)
    // CG pass p: the nine taps of channel group p, weight chunk tap * cpt + p
    const int nkp = CG ? 9 : (pass ? nks >> sh : (pair ? nks / 4 * 3 : nks)), wsh = (!CG && pass) ? sh : 0;
    auto wchunk = [&](int j) { return CG ? j * cpt + pass : (pass ? j << wsh : (pair ? (j / 3) * 4 + j % 3 : j)); };
    bissue(0, wchunk(0));   // (a channel-group pass starts at weight chunk `pass`)
    if (1 < nkp) bissue(1, wchunk(1));
    for (int j = 0; j < nkp; ++j) {
      // chunk j landed for this wave (younger: chunk j+1's NI DMA instructions), then all waves
      if (j + 1 < nkp) {
        if constexpr (NI == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        else if constexpr (NI == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      ring_barrier();   // chunk j visible; stage (j+2) % 3 = (j-1) % 3 is free
      if (j + 2 < nkp) bissue(j + 2, wchunk(j + 2));
      if constexpr (EX == EX_RESID) {
        if (last && j == nkp - 2) load_resid();
      }
      compute(j % 3, wchunk(j));
    }
    }   // pass
    // epilogue: bias (+ act) (+ fp32 residual), 4 consecutive channels per lane
    if constexpr (EX == EX_RESID) {
      if (!CG && (nks >> (npass - 1 ? sh : 0)) < 2) load_resid();
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int jn = 0; jn < RN; ++jn) land(ex[i][jn]);
    }
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int jn = 0; jn < RN; ++jn) {
        const long m = p0 + wm * TM + i * 16 + fr;
        const int n = n0 + wn * TN + jn * 16 + fq * 4;
        const float4 bb = bias4[jn];
        float v[4] = {acc[i][jn][0] + bb.x, acc[i][jn][1] + bb.y, acc[i][jn][2] + bb.z, acc[i][jn][3] + bb.w};
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          if (E.act == KAIR_ACT_GELU) v[q4] = gelu_fast(v[q4]);
          else if (E.act == KAIR_ACT_LEAKY) v[q4] = v[q4] > 0.f ? v[q4] : v[q4] * E.slope;
          else if (E.act == KAIR_ACT_RELU) v[q4] = fmaxf(v[q4], 0.f);
        }
        if constexpr (EX == EX_RESID) {
          v[0] += ex[i][jn].x; v[1] += ex[i][jn].y; v[2] += ex[i][jn].z; v[3] += ex[i][jn].w;
        }
        if (E.ones_col >= n && E.ones_col < n + 4) {
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4)
            if (n + q4 == E.ones_col) v[q4] = 1.f;
        }
        if (E.gate && n < N) {   // act'(gate) of the same row (ROWS): the input gradient's activation gate
          float gv[4];
          ld4_any(E.gate, E.gdt, m * E.ldg + n, gv);
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) {
            if (E.gkind == 2) v[q4] *= (gv[q4] > 0.f ? 1.f : E.slope);
            else if (E.gkind == 4) v[q4] *= gv[q4];
            else v[q4] *= (gv[q4] > 0.f ? 1.f : 0.f);
          }
        }
        if (n < N) {
          long o = m * E.ldo + n;
          if constexpr (EM == HC_EM_PSHUF) {   // sub-pixel-major columns: n = (i r + j) nf + c -> pixel (y r + i, x r + j)
            const int r = E.r, nf = N / (r * r);
            const int bi = (int)(m / ((long)H * W)), pp = (int)(m - (long)bi * H * W), yy = pp / W, xx = pp - yy * W;
            const int sp = n / nf, cc = n - sp * nf, ii = sp / r, jj = sp - ii * r;
            o = (((long)bi * H * r + (long)yy * r + ii) * ((long)W * r) + (long)xx * r + jj) * E.ldo + cc;
          } else if constexpr (EM == HC_EM_PUNSHUF) {   // pixel (y, x) of the r-times grid -> pre-shuffle row
            const int r = E.r;                          // (y / r, x / r), column (i r + j) N + n
            const int bi = (int)(m / ((long)H * W)), pp = (int)(m - (long)bi * H * W), yy = pp / W, xx = pp - yy * W;
            const int yl = yy / r, xl = xx / r;
            o = (((long)bi * (H / r) + yl) * (W / r) + xl) * E.ldo + ((yy - yl * r) * r + (xx - xl * r)) * N + n;
          }
          st4_any(E.out, E.odt, o, v);
          if (E.out_lo) {
            const bf16x4 ql = {(bf16)(v[0] - (float)(bf16)v[0]), (bf16)(v[1] - (float)(bf16)v[1]),
                               (bf16)(v[2] - (float)(bf16)v[2]), (bf16)(v[3] - (float)(bf16)v[3])};
            *(bf16x4*)(E.out_lo + o) = ql;
          }
        }
      }
  }
}

// halo conv applicability (host): geometry, epilogue features and alignment the kernel assumes
// The halo tile's pixel count: 96 (whole rows of a width dividing 96, or 96-pixel pieces of a row 96 divides), else
// 128 for a plain ROWS conv with <= 64 outputs (SwinIR-lightweight's 64-pixel rows, Cp = 64: two whole rows per tile;
// neither 96 | 64 nor 64 | 96, so its RSTB convs ran on the register-staged im2col kernel at 201 us), else 0 (none).
static int halo_bm_of(int H, int W, int C, int N, const Epi& e) {
  auto fits = [&](int bm) { return W <= bm ? (bm % W == 0 && H % (bm / W) == 0) : W % bm == 0; };
  if (fits(HC_BM)) return HC_BM;
  if (fits(128) && N <= 64 && C <= 192 && e.omode == KAIR_OUT_ROWS && !e.acopy && !e.gate) return 128;
  return 0;
}

template <typename TA>
static bool conv_halo_ok(const Op& A, const Op& B, const Epi& e, long M, int N, int K) {
  const int H = A.imH, W = A.imW, C = A.imC;
  if (A.up_sh != 0 || C % HC_BK != 0 || C > 256 || K != 9 * C || N > 256 || N % 4 != 0) return false;
  // C in (192, 256]: channel-group passes, plain bf16 operands, 64 outputs
  if (C > 192 && (C != 256 || sizeof(TA) != 2 || A.asplit || B.wsplit || N > 64 || e.resid || e.acopy)) return false;
  // the two-pass split forms lo from an fp32 image; a bf16 image carries it as its [hi | lo] halves (a_split 2)
  if (A.asplit && !(sizeof(TA) == 4 ? A.asplit == 1 : (A.asplit == 2 && C == 128 && B.wsplit))) return false;
  if (W <= 0 || H <= 0) return false;
  const int bm = halo_bm_of(H, W, C, N, e);
  if (bm == 0) return false;
  const int XW = W < bm ? W : bm, RPT = bm / XW;
  if ((long)(RPT + 2) * (XW + 2) * ((C > 192 ? HC_BK : C) + 8) > HC_HALO_ELEMS) return false;   // the halo of one pass
  if (M % bm != 0 || M % ((long)H * W) != 0) return false;
  if (A.ld % 8 != 0 || ((unsigned long)A.ptr & 15) || B.ld % 8 != 0 || ((unsigned long)B.ptr & 15)) return false;
  if (e.omode != KAIR_OUT_ROWS && !(e.omode == KAIR_OUT_PSHUF_SPM && e.psH == H && e.psW == W && e.r > 0 &&
                                    N % (e.r * e.r) == 0 && (N / (e.r * e.r)) % 4 == 0 && !e.resid && !e.acopy) &&
      !(e.omode == KAIR_OUT_PUNSHUF_SPM && C > 192 && e.r > 0 && e.psH * e.r == H && e.psW * e.r == W && N % 4 == 0 &&
        e.ldo >= (long)N * e.r * e.r && !e.resid && !e.acopy))
    return false;
  // a gate only on ROWS outputs with 4-aligned rows (bf16 8-byte / fp32 16-byte loads), no residual
  if (e.gate && (e.omode != KAIR_OUT_ROWS || e.resid || e.ldg % 4 != 0 || e.gkind == 1 || ((unsigned long)e.gate & 15)))
    return false;
  if (e.win.ws != 0 || e.pre || e.resid2 || e.rowscale) return false;
  if (e.ldo % 4 != 0 || ((unsigned long)e.out & 15) || (e.resid && (e.ldr % 4 != 0 || ((unsigned long)e.resid & 15))))
    return false;
  if (e.acopy && (e.ldac % 8 != 0 || e.ldac < C || ((unsigned long)e.acopy & 15))) return false;
  return true;
}

// the geometry half of conv_halo_ok, for hosts that pick a_copy (16-byte aligned rows, ld = C, plain
// ROWS epilogue assumed)
extern "C" int kair_conv3x3_halo_geometry(int H, int W, int C, long M, int N) {
  if (C % HC_BK != 0 || C > 192 || N > HC_BN || N % 4 != 0 || W <= 0 || H <= 0 || M <= 0) return 0;
  if (W <= HC_BM) {
    if (HC_BM % W != 0 || H % (HC_BM / W) != 0) return 0;
  } else if (W % HC_BM != 0) {
    return 0;
  }
  const int XW = W < HC_BM ? W : HC_BM, RPT = HC_BM / XW;
  if ((long)(RPT + 2) * (XW + 2) * (C + 8) > HC_HALO_ELEMS) return 0;
  return M % HC_BM == 0 && M % ((long)H * W) == 0 && C % 8 == 0;
}

// the 192-pixel tile (128-wide N tiles only): whole rows of width W <= 192 or 192-pixel row pieces
static bool halo_bm192_ok(const Op& A, long M) {
  const int H = A.imH, W = A.imW, C = A.imC;
  if (W <= 192) {
    if (192 % W != 0 || H % (192 / W) != 0) return false;
  } else if (W % 192 != 0) {
    return false;
  }
  const int XW = W < 192 ? W : 192, RPT = 192 / XW;
  return (long)(RPT + 2) * (XW + 2) * (C + 8) <= HaloSize<192>::ELEMS && M % 192 == 0 && M % ((long)H * W) == 0;
}

template <typename TA>
static int launch_conv_halo(const Op& A, const Op& B, const Epi& E, long M, int K, hipStream_t s) {
  if (g_num_cus == 0) init_num_cus();
  const bool wide = E.N > HC_BN;   // N in (192, 256]: two 128-wide N tiles
  const bool big = wide && !E.resid && A.asplit != 1 && halo_bm192_ok(A, M);   // (the two-pass form would spill)
  const bool t128 = halo_bm_of(A.imH, A.imW, A.imC, E.N, E) == 128;           // (N <= 64, ROWS: one 64-wide N tile)
  const int tilesM = (int)(M / (big ? 192 : (t128 ? 128 : HC_BM)));
  // few M tiles (small batches: 96 tiles at 4 patches per GPU): 64-wide N tiles put 3x the workgroups
  // on the chip, each a third of the weight chunks
  const bool slim = !wide && E.omode == KAIR_OUT_ROWS && E.N > 64 && 2L * tilesM <= g_num_cus;
  const int tilesN = wide ? (E.N + 127) / 128 : (slim ? (E.N + 63) / 64 : 1);
  long tiles = (long)tilesM * tilesN;
  int grid = (int)(tiles < g_num_cus ? tiles : (g_num_cus / tilesN) * tilesN);   // a multiple of tilesN
#define KAIR_HALO(NP, EXV, BNV, EMV, BMV) \
  KAIR_LAUNCH((conv3x3_halo_kernel<TA, EXV, NP, BNV, EMV, BMV, 1>), dim3(grid), dim3(512), 0, s, A, B, E, K, tilesM)
  if constexpr (sizeof(TA) == 2) {
    if (A.imC > 192) {   // conv_halo_ok: 64 outputs, plain operands, C = 256 in four channel-group passes
      if (A.imC != 256) return kair_set_error(KAIR_ERR_ARG, "halo conv: C in (192, 256) has no channel-group form");
      if (E.omode == KAIR_OUT_PUNSHUF_SPM)
        KAIR_LAUNCH((conv3x3_halo_kernel<TA, EX_NONE, 1, 64, HC_EM_PUNSHUF, 96, 4>), dim3(grid), dim3(512), 0, s, A, B,
                           E, K, tilesM);
      else
        KAIR_LAUNCH((conv3x3_halo_kernel<TA, EX_NONE, 1, 64, HC_EM_ROWS, 96, 4>), dim3(grid), dim3(512), 0, s, A, B, E,
                           K, tilesM);
      KAIR_CHECK_LAUNCH();
      return 0;
    }
  }
#define KAIR_HALO_NP(NP)                                                                           \
  if (t128 && E.resid) KAIR_HALO(NP, EX_RESID, 64, HC_EM_ROWS, 128);                               \
  else if (t128) KAIR_HALO(NP, EX_NONE, 64, HC_EM_ROWS, 128);                                      \
  else if (E.resid && slim) KAIR_HALO(NP, EX_RESID, 64, HC_EM_ROWS, 96);                           \
  else if (E.resid) KAIR_HALO(NP, EX_RESID, 192, HC_EM_ROWS, 96);                                  \
  else if (E.omode == KAIR_OUT_PSHUF_SPM && big) KAIR_HALO(NP, EX_NONE, 128, HC_EM_PSHUF, 192);     \
  else if (E.omode == KAIR_OUT_PSHUF_SPM && wide) KAIR_HALO(NP, EX_NONE, 128, HC_EM_PSHUF, 96);     \
  else if (E.omode == KAIR_OUT_PSHUF_SPM) KAIR_HALO(NP, EX_NONE, 192, HC_EM_PSHUF, 96);             \
  else if (big) KAIR_HALO(NP, EX_NONE, 128, HC_EM_ROWS, 192);                                       \
  else if (wide) KAIR_HALO(NP, EX_NONE, 128, HC_EM_ROWS, 96);                                       \
  else if (E.N <= 64 || slim) KAIR_HALO(NP, EX_NONE, 64, HC_EM_ROWS, 96);                           \
  else KAIR_HALO(NP, EX_NONE, 192, HC_EM_ROWS, 96);
  if constexpr (sizeof(TA) == 4) {
    if (A.asplit) {   // conv_halo_ok: the two-pass split takes an fp32 A only
      KAIR_HALO_NP(2)
      KAIR_CHECK_LAUNCH();
      return 0;
    }
  }
  KAIR_HALO_NP(1)
#undef KAIR_HALO_NP
#undef KAIR_HALO
  KAIR_CHECK_LAUNCH();
  return 0;
}

template <typename CT, typename TA>
int nt_modes(int mode, const Op& A, const Op& B, const Epi& E, long M, int N, int K, hipStream_t s) {
  if constexpr (sizeof(CT) == 2) {
    if (mode == KAIR_LD_IM2COL3 && g_halo_mode != 0 && conv_halo_ok<TA>(A, B, E, M, N, K))
      return launch_conv_halo<TA>(A, B, E, M, K, s);
    if (E.acopy) return kair_set_error(KAIR_ERR_ARG, "gemm_nt: a_copy needs the 3x3 halo-conv path (geometry / epilogue)");
  }
  if constexpr (sizeof(CT) == 2 && sizeof(TA) == 2) {
    if (g_ring_mode && ring_ok(mode, A, B, E, M, N, K)) {
      if (g_num_cus == 0) init_num_cus();
      const int bn = ring_bn_of(E, N, K);
      const long tiles = ((M + RING_BM - 1) / RING_BM) * ((N + bn - 1) / bn);
      if (tiles >= g_ring_min_tiles) {
        if (mode == KAIR_LD_ROWS) return ring_bn<AM_ROWS>(A, B, E, M, N, K, s);
        return ring_bn<AM_QKV>(A, B, E, M, N, K, s);
      }
    }
  }
  if (mode == KAIR_LD_ROWS) return nt_tiles<CT, TA, AM_ROWS>(A, B, E, M, N, K, s);
  if (mode == KAIR_LD_IM2COL3) return nt_tiles<CT, TA, AM_IM2COL>(A, B, E, M, N, K, s);
  if (mode == KAIR_LD_S2D) return nt_tiles<CT, TA, AM_S2D>(A, B, E, M, N, K, s);
  if constexpr (sizeof(TA) == sizeof(CT)) return nt_tiles<CT, TA, AM_QKV>(A, B, E, M, N, K, s);
  return kair_set_error(KAIR_ERR_ARG, "gemm_nt: q/k/v operand must have the compute dtype");
}

// Cp = 192 conv weight gradients (N = 192, K = 9 * 192): one 192-wide N tile instead of a full
// and a half-empty 128-wide one (B = 32: 946 -> 953 patches/s; B = 4 unchanged)
static bool tn192_shape(int N, int K) { return N > 128 && N <= 192 && K > 128; }
// narrow weight gradients (N <= 32 output channels, e.g. RRDB's growth-32 dense-block convs): a
// 128 x 128 tile would be 3/4 empty along N; a 32 x 256 one does the same work in half the tiles
static bool tn_narrow_shape(int N, int K) { return N <= 32 && K > 64; }
static bool tn_narrow64_shape(int N, int K) { return N > 32 && N <= 64 && K > 64; }

template <typename CT, typename TA, typename TB, int AMA, int AMB>
int launch_tn(const Op& a, const Op& b, float* ws, int splits, long M, int N, int K, long rps, hipStream_t s) {
  if (tn192_shape(N, K)) {   // one 192-wide N tile (Cp = 192 conv weight gradients): no half-empty tile
    const int tilesK = (K + 127) / 128;
    KAIR_LAUNCH((gemm_tn_kernel<CT, TA, TB, AMA, AMB, 192, 128>), dim3(tilesK, splits), dim3(NT), 0, s, a, b,
                       ws, M, N, K, rps, tilesK);
  } else if (tn_narrow_shape(N, K) && K <= 160) {   // e.g. 16 -> 16-channel 3x3 convs (K = 144): one 32 x 160 tile
    KAIR_LAUNCH((gemm_tn_kernel<CT, TA, TB, AMA, AMB, 32, 160>), dim3(1, splits), dim3(NT), 0, s, a, b,
                       ws, M, N, K, rps, 1);
  } else if (tn_narrow_shape(N, K)) {   // N <= 32 (dense-block growth convs): one 32 x 256 tile, no 3/4-empty N
    const int tilesK = (K + 255) / 256;
    KAIR_LAUNCH((gemm_tn_kernel<CT, TA, TB, AMA, AMB, 32, 256>), dim3(tilesK, splits), dim3(NT), 0, s, a, b,
                       ws, M, N, K, rps, tilesK);
  } else if (tn_narrow64_shape(N, K)) {   // 32 < N <= 64: one 64 x 128 tile, no half-empty 128-wide N
    const int tilesK = (K + 127) / 128;
    KAIR_LAUNCH((gemm_tn_kernel<CT, TA, TB, AMA, AMB, 64, 128>), dim3(tilesK, splits), dim3(NT), 0, s, a, b,
                       ws, M, N, K, rps, tilesK);
  } else if (N <= 64 && K <= 64) {
    const int tilesN = (N + 63) / 64, tilesK = (K + 63) / 64;
    KAIR_LAUNCH((gemm_tn_kernel<CT, TA, TB, AMA, AMB, 64, 64>), dim3(tilesN * tilesK, splits), dim3(NT), 0, s, a, b,
                       ws, M, N, K, rps, tilesK);
  } else {
    const int tilesN = (N + 127) / 128, tilesK = (K + 127) / 128;
    KAIR_LAUNCH((gemm_tn_kernel<CT, TA, TB, AMA, AMB, 128, 128>), dim3(tilesN * tilesK, splits), dim3(NT), 0, s, a,
                       b, ws, M, N, K, rps, tilesK);
  }
  KAIR_CHECK_LAUNCH();
  return 0;
}

template <typename CT, typename TA, int AMA>
int tn_b(int bmode, int bdt, const Op& a, const Op& b, float* ws, int splits, long M, int N, int K, long rps, hipStream_t s) {
  if (bmode == KAIR_LD_ROWS)
    return bdt == KAIR_BF16 ? launch_tn<CT, TA, bf16, AMA, AM_ROWS>(a, b, ws, splits, M, N, K, rps, s)
                            : launch_tn<CT, TA, float, AMA, AM_ROWS>(a, b, ws, splits, M, N, K, rps, s);
  if (bmode == KAIR_LD_S2D)
    return bdt == KAIR_BF16 ? launch_tn<CT, TA, bf16, AMA, AM_S2D>(a, b, ws, splits, M, N, K, rps, s)
                            : launch_tn<CT, TA, float, AMA, AM_S2D>(a, b, ws, splits, M, N, K, rps, s);
  return bdt == KAIR_BF16 ? launch_tn<CT, TA, bf16, AMA, AM_IM2COL>(a, b, ws, splits, M, N, K, rps, s)
                          : launch_tn<CT, TA, float, AMA, AM_IM2COL>(a, b, ws, splits, M, N, K, rps, s);
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

int kair_dbg_env(const char* name) {
#if KAIR_DEBUG_ABLATIONS
  const char* v = getenv(name);
  return v ? atoi(v) : 0;
#else
  (void)name;
  return 0;
#endif
}

extern "C" int kair_device_arch(char* buf, int len) {
  hipDeviceProp_t p;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess)
    return kair_set_error(KAIR_ERR_HIP, "no HIP device");
  snprintf(buf, len, "%s", p.gcnArchName);
  return 0;
}

int kair_check_operand(const kair_operand* o, const char* what) {
  KAIR_CHECK_ARG(o && o->ptr, "%s: null operand", what);
  KAIR_CHECK_ARG(o->dtype == KAIR_F32 || o->dtype == KAIR_BF16 || o->dtype == KAIR_F16, "%s: bad dtype", what);
  KAIR_CHECK_ARG(o->mode >= 0 && o->mode <= 3, "%s: bad mode", what);
  const int esz = o->dtype == KAIR_F32 ? 4 : 2;
  KAIR_CHECK_ARG(((uintptr_t)o->ptr % 16) == 0, "%s: pointer not 16-byte aligned", what);
  if (o->mode == KAIR_LD_ROWS) KAIR_CHECK_ARG((o->ld * esz) % 16 == 0, "%s: row stride not 16-byte aligned", what);
  if (o->mode == KAIR_LD_IM2COL3) {
    KAIR_CHECK_ARG(o->im_C % 8 == 0 && o->im_H > 0 && o->im_W > 0, "%s: im2col geometry", what);
    KAIR_CHECK_ARG(o->ld == 0 || (o->ld >= o->im_C && (o->ld * esz) % 16 == 0), "%s: im2col pixel stride", what);
    KAIR_CHECK_ARG(o->im_up == 0 || o->im_up == 1 || (o->im_up == 2 && o->im_H % 2 == 0 && o->im_W % 2 == 0),
                   "%s: im2col upsample factor", what);
  }
  if (o->mode == KAIR_LD_S2D) {
    KAIR_CHECK_ARG(o->im_C % 8 == 0 && o->im_H > 0 && o->im_W > 0, "%s: space-to-depth geometry", what);
    KAIR_CHECK_ARG(o->ld == 0 || (o->ld >= o->im_C && (o->ld * esz) % 16 == 0), "%s: space-to-depth pixel stride", what);
  }
  if (o->mode == KAIR_LD_QKVBLK) KAIR_CHECK_ARG(o->qkv_hdp % 8 == 0 && o->qkv_tok > 0 && o->qkv_nh > 0, "%s: qkv geometry", what);
  if (o->win_ws > 0)
    KAIR_CHECK_ARG(o->win_H % o->win_ws == 0 && o->win_W % o->win_ws == 0, "%s: window map geometry", what);
  return 0;
}

extern "C" int kair_gemm_nt(const kair_operand* A, const kair_operand* B, const kair_epilogue* E, long M, int N, int K,
                            int compute, void* stream) {
  int rc;
  if ((rc = kair_check_operand(A, "gemm_nt A"))) return rc;
  if ((rc = kair_check_operand(B, "gemm_nt B"))) return rc;
  KAIR_CHECK_ARG(E && E->out, "gemm_nt: null epilogue/out");
  if (compute == KAIR_COMPUTE_X3) return kair_gemm_nt_x3(A, B, E, M, N, K, stream);   // gemm_x3.hip
  KAIR_CHECK_ARG(M > 0 && N > 0 && K > 0 && K % 8 == 0, "gemm_nt: bad M/N/K (%ld,%d,%d), K%%8 must be 0", M, N, K);
  KAIR_CHECK_ARG(B->mode == KAIR_LD_ROWS && B->dtype == compute && B->win_ws == 0,
                 "gemm_nt: B must be packed rows of the compute dtype");
  KAIR_CHECK_ARG(compute == KAIR_BF16 || A->dtype == KAIR_F32, "gemm_nt: fp32 compute needs fp32 A");
  KAIR_CHECK_ARG(!B->w_split || (compute == KAIR_BF16 && B->ld >= 2L * ((K + 63) / 64) * 64),
                 "gemm_nt: hi/lo split weights need bf16 compute and rows of 2*ceil(K/64)*64 columns");
  KAIR_CHECK_ARG(!A->w_split, "gemm_nt: w_split is a B-operand flag");
  KAIR_CHECK_ARG(!B->a_split, "gemm_nt: a_split is an A-operand flag");
  KAIR_CHECK_ARG(A->a_split != 1 || (compute == KAIR_BF16 && (A->mode == KAIR_LD_ROWS || A->mode == KAIR_LD_IM2COL3) &&
                                      !A->rowscale && A->ones_col < 0 &&
                                      (A->dtype == KAIR_F32 || (A->lo_ptr && ((uintptr_t)A->lo_ptr % 16) == 0))),
                 "gemm_nt: a_split needs bf16 compute, a ROWS / IM2COL3 A without rowscale or ones column, and for a "
                 "bf16 A its 16-byte aligned lo plane");
  KAIR_CHECK_ARG(A->a_split >= 0 && A->a_split <= 2, "gemm_nt: a_split must be 0, 1 or 2");
  KAIR_CHECK_ARG(A->a_split != 2 || (compute == KAIR_BF16 && A->dtype == KAIR_BF16 && A->mode == KAIR_LD_IM2COL3 &&
                                      B->w_split && A->im_C % 2 == 0),
                 "gemm_nt: a_split 2 marks a bf16 [hi | lo] pair image read through tied hi/lo split weights");
  KAIR_CHECK_ARG(!E->out_lo || (E->out_dtype == KAIR_BF16 &&
                                (E->out_mode == KAIR_OUT_ROWS || E->out_mode == KAIR_OUT_PSHUF_SPM ||
                                 E->out_mode == KAIR_OUT_QKVBLK) &&
                                ((uintptr_t)E->out_lo % 16) == 0),
                 "gemm_nt: out_lo needs a bf16 ROWS / PSHUF_SPM / QKVBLK output and a 16-byte aligned lo plane");
  KAIR_CHECK_ARG(!E->a_copy || (compute == KAIR_BF16 && A->mode == KAIR_LD_IM2COL3 && A->im_up <= 1),
                 "gemm_nt: a_copy is a side output of the bf16 3x3 conv (no upsample)");
  KAIR_CHECK_ARG((E->out_mode != KAIR_OUT_PSHUF && E->out_mode != KAIR_OUT_PUNSHUF && E->out_mode != KAIR_OUT_PSHUF_NCHW &&
                  E->out_mode != KAIR_OUT_PSHUF_SPM && E->out_mode != KAIR_OUT_PUNSHUF_SPM) ||
                     E->ps_r > 0, "gemm_nt: pixel shuffle r");
  KAIR_CHECK_ARG(E->out_mode != KAIR_OUT_PSHUF_SPM || N % (E->ps_r * E->ps_r) == 0, "gemm_nt: PSHUF_SPM needs N %% r^2 == 0");
  KAIR_CHECK_ARG(E->out_mode != KAIR_OUT_PUNSHUF_SPM || E->ldo >= (long)N * E->ps_r * E->ps_r,
                 "gemm_nt: PUNSHUF_SPM needs ldo >= N * r^2");
  KAIR_CHECK_ARG(E->out_mode != KAIR_OUT_QKVBLK || (E->qkv_hdp % 8 == 0 && E->qkv_tok > 0), "gemm_nt: qkv epilogue");
  KAIR_CHECK_ARG(M < KAIR_MAX_MAPPED_ROWS && N < KAIR_MAX_MAPPED_ROWS && K < KAIR_MAX_MAPPED_ROWS,
                 "gemm_nt: dimensions must be < 2^24");
  const Op a = make_op(*A, M), b = make_op(*B, N);
  const Epi e = make_epi(*E, M, N);
  hipStream_t s = (hipStream_t)stream;
  if (compute == KAIR_BF16) {
    if (A->dtype == KAIR_BF16) return nt_modes<bf16, bf16>(A->mode, a, b, e, M, N, K, s);
    return nt_modes<bf16, float>(A->mode, a, b, e, M, N, K, s);
  }
  if (compute == KAIR_F32) return nt_modes<float, float>(A->mode, a, b, e, M, N, K, s);
  return kair_set_error(KAIR_ERR_ARG, "gemm_nt: bad compute type");
}

static bool tn_ring_shape(long M, int N, int K) {
  return N <= 576 && K <= 576 && N % 8 == 0 && K % 8 == 0 && N > 64 && K > 64 && M < (1L << 30);
}
// the grouped launch takes narrow linears too (SwinIR-lightweight: Cp = 64 with Hdp = 128 and 6 x 16 heads): one
// 192 x 192 tile holds a whole 64 x 128 weight -- its pieces past N / K load the zero line -- and the group's
// splits fill the chip (the single-linear path keeps N, K > 64: its split count is shared with the generic kernel)
static bool tn_ring_shape_grouped(long M, int N, int K) {
  return N <= 576 && K <= 576 && N % 8 == 0 && K % 8 == 0 && N >= 16 && K >= 16 && M < (1L << 30);
}
// 3x3 conv weight gradient over a 192-channel image: the ring with one tap per K tile (BM_TAP)
static bool tn_tap_shape(long M, int N, int K) {
  return N <= 576 && N % 8 == 0 && N > 64 && K == 9 * TNR_BK && M < (1L << 30);
}

extern "C" int kair_wgrad_splits(long M, int N, int K) {
  if (tn_ring_shape(M, N, K) || tn_tap_shape(M, N, K)) {   // ring kernel: one 192x192 tile per CTA, one CTA per CU
    if (g_num_cus == 0) init_num_cus();
    const int tiles = ((N + TNR_BN - 1) / TNR_BN) * ((K + TNR_BK - 1) / TNR_BK);
    long s = g_num_cus / tiles;
    // >= 128 rows per split (binds only at small M: at B = 4, 256 -> 128 rows
    // measured 311 -> 316-320 patches/s, 64 / 32 no better, 512 / 1024 slower)
    constexpr long min_rows = 128;
    const long maxs = (M + min_rows - 1) / min_rows;
    if (s > maxs) s = maxs;
    return (int)(s < 1 ? 1 : s);
  }
  const long tiles = tn_narrow_shape(N, K) ? (K + 255) / 256
                     : (N <= 64 && K <= 64) ? 1 : (long)((N + 127) / 128) * ((K + 127) / 128);
  // enough (tile, split) CTAs for ~2 per CU, but >= 1024 rows per split so the fp32 partial
  // planes stay small next to the operand traffic (wgrad_finalize reads them all back)
  long s = 512 / (tiles > 0 ? tiles : 1);
  if (tn192_shape(N, K)) {   // 192-wide tiles: one CTA per CU (LDS)
    if (g_num_cus == 0) init_num_cus();
    s = g_num_cus / ((K + 127) / 128);
  }
  // (narrow tiles: >= 512 rows -- their partial planes are 1/4 the size, and the half-as-many tiles
  // need the splits to fill the CUs)
  const long maxs = tn_narrow_shape(N, K) || tn_narrow64_shape(N, K) ? (M + 511) / 512 : (M + 1023) / 1024;
  if (s > maxs) s = maxs;
  if (s < 1) s = 1;
  return (int)s;
}

extern "C" int kair_gemm_tn(const kair_operand* A, const kair_operand* B, float* ws, int splits, long M, int N, int K,
                            int compute, void* stream) {
  int rc;
  if ((rc = kair_check_operand(A, "gemm_tn A"))) return rc;
  if ((rc = kair_check_operand(B, "gemm_tn B"))) return rc;
  KAIR_CHECK_ARG(ws, "gemm_tn: null workspace");
  KAIR_CHECK_ARG(M > 0 && N > 0 && K > 0 && N % 8 == 0 && K % 8 == 0 && splits > 0, "gemm_tn: bad sizes");
  KAIR_CHECK_ARG(A->mode != KAIR_LD_IM2COL3 && A->mode != KAIR_LD_S2D, "gemm_tn: A cannot be im2col / space-to-depth");
  KAIR_CHECK_ARG(B->mode != KAIR_LD_QKVBLK, "gemm_tn: B cannot be q/k/v blocked");
  if (compute == KAIR_COMPUTE_X3) return kair_gemm_tn_x3(A, B, ws, splits, M, N, K, stream);   // gemm_x3.hip
  KAIR_CHECK_ARG(compute == KAIR_BF16 || (A->dtype == KAIR_F32 && B->dtype == KAIR_F32),
                 "gemm_tn: fp32 compute needs fp32 operands");
  KAIR_CHECK_ARG(A->mode != KAIR_LD_QKVBLK || A->dtype == compute, "gemm_tn: q/k/v operand dtype");
  KAIR_CHECK_ARG(M < KAIR_MAX_MAPPED_ROWS && N < KAIR_MAX_MAPPED_ROWS && K < KAIR_MAX_MAPPED_ROWS,
                 "gemm_tn: dimensions must be < 2^24");
  const Op a = make_op(*A, M), b = make_op(*B, M);
  hipStream_t s0 = (hipStream_t)stream;
  if (g_ring_mode && compute == KAIR_BF16 && tn_ring_shape(M, N, K) && A->dtype == KAIR_BF16 && B->dtype == KAIR_BF16 &&
      (A->mode == KAIR_LD_ROWS || A->mode == KAIR_LD_QKVBLK) && B->mode == KAIR_LD_ROWS && !A->rowscale && !B->rowscale &&
      A->win_ws == 0 && B->win_ws == 0 && A->ones_col < 0 && (B->ones_col < 0 || B->ones_in_data) &&
      (A->mode != KAIR_LD_ROWS || A->ld % 8 == 0) && B->ld % 8 == 0 && (A->mode != KAIR_LD_QKVBLK || A->qkv_hdp % 8 == 0)) {
    const int tilesN = (N + TNR_BN - 1) / TNR_BN, tilesK = (K + TNR_BK - 1) / TNR_BK;
    const int ntiles = tilesN * tilesK;
    long rps = (M + splits - 1) / splits;
    rps = (rps + TNR_RB - 1) / TNR_RB * TNR_RB;
    const long grid = (long)ntiles * splits;
    if (A->mode == KAIR_LD_ROWS)
      KAIR_LAUNCH((gemm_tn_ring<AM_ROWS, BM_ROWS>), dim3((unsigned)grid), dim3(512), 0, s0, a, b, ws, (int)M, N, K, tilesK,
                         ntiles, (int)rps);
    else
      KAIR_LAUNCH((gemm_tn_ring<AM_QKV, BM_ROWS>), dim3((unsigned)grid), dim3(512), 0, s0, a, b, ws, (int)M, N, K, tilesK,
                         ntiles, (int)rps);
    KAIR_CHECK_LAUNCH();
    return 0;
  }
  // conv weight gradient, bf16 rows x bf16 192-channel image (ones column, if any, stored in the data)
  if (g_ring_mode && compute == KAIR_BF16 && tn_tap_shape(M, N, K) && A->dtype == KAIR_BF16 && B->dtype == KAIR_BF16 &&
      A->mode == KAIR_LD_ROWS && B->mode == KAIR_LD_IM2COL3 && B->im_C == TNR_BK && !B->im_flip && B->im_up <= 1 &&
      !A->rowscale && !B->rowscale && A->win_ws == 0 && A->ones_col < 0 && (B->ones_col < 0 || B->ones_in_data) &&
      A->ld % 8 == 0 && b.ld % 8 == 0 && (long)B->im_H * B->im_W > 0 && M % ((long)B->im_H * B->im_W) == 0) {
    const int tilesN = (N + TNR_BN - 1) / TNR_BN, tilesK = 9;
    const int ntiles = tilesN * tilesK;
    long rps = (M + splits - 1) / splits;
    rps = (rps + TNR_RB - 1) / TNR_RB * TNR_RB;
    const long grid = (long)ntiles * splits;
    KAIR_LAUNCH((gemm_tn_ring<AM_ROWS, BM_TAP>), dim3((unsigned)grid), dim3(512), 0, s0, a, b, ws, (int)M, N, K, tilesK,
                       ntiles, (int)rps);
    KAIR_CHECK_LAUNCH();
    return 0;
  }
  // conv weight gradient over a 64-channel bf16 image (the reconstruction tail's upsampling convs): the
  // ring with three taps per 192-wide K tile, each image row fetched once per tile instead of once
  // per im2col column block
  if (g_ring_mode && compute == KAIR_BF16 && tn_ring_shape(M, N, K) && K == 9 * 64 && A->dtype == KAIR_BF16 &&
      B->dtype == KAIR_BF16 && A->mode == KAIR_LD_ROWS && B->mode == KAIR_LD_IM2COL3 && B->im_C == 64 && !B->im_flip &&
      B->im_up <= 1 && !A->rowscale && !B->rowscale && A->win_ws == 0 && A->ones_col < 0 && B->ones_col < 0 &&
      A->ld % 8 == 0 && b.ld % 8 == 0 && (long)B->im_H * B->im_W > 0 && M % ((long)B->im_H * B->im_W) == 0) {
    const int tilesN = (N + TNR_BN - 1) / TNR_BN, tilesK = 3;
    const int ntiles = tilesN * tilesK;
    long rps = (M + splits - 1) / splits;
    rps = (rps + TNR_RB - 1) / TNR_RB * TNR_RB;
    const long grid = (long)ntiles * splits;
    KAIR_LAUNCH((gemm_tn_ring<AM_ROWS, BM_TAP3>), dim3((unsigned)grid), dim3(512), 0, s0, a, b, ws, (int)M, N, K, tilesK,
                       ntiles, (int)rps);
    KAIR_CHECK_LAUNCH();
    return 0;
  }
  const int BMr = compute == KAIR_BF16 ? 64 : 32;
  long rps = (M + splits - 1) / splits;
  rps = (rps + BMr - 1) / BMr * BMr;
  hipStream_t s = (hipStream_t)stream;
  if (compute == KAIR_BF16) {
    if (A->mode == KAIR_LD_QKVBLK) return tn_b<bf16, bf16, AM_QKV>(B->mode, B->dtype, a, b, ws, splits, M, N, K, rps, s);
    if (A->dtype == KAIR_BF16) return tn_b<bf16, bf16, AM_ROWS>(B->mode, B->dtype, a, b, ws, splits, M, N, K, rps, s);
    return tn_b<bf16, float, AM_ROWS>(B->mode, B->dtype, a, b, ws, splits, M, N, K, rps, s);
  }
  if (A->mode == KAIR_LD_QKVBLK) {
    if (B->mode == KAIR_LD_ROWS) return launch_tn<float, float, float, AM_QKV, AM_ROWS>(a, b, ws, splits, M, N, K, rps, s);
    return launch_tn<float, float, float, AM_QKV, AM_IM2COL>(a, b, ws, splits, M, N, K, rps, s);
  }
  if (B->mode == KAIR_LD_ROWS) return launch_tn<float, float, float, AM_ROWS, AM_ROWS>(a, b, ws, splits, M, N, K, rps, s);
  if (B->mode == KAIR_LD_S2D) return launch_tn<float, float, float, AM_ROWS, AM_S2D>(a, b, ws, splits, M, N, K, rps, s);
  return launch_tn<float, float, float, AM_ROWS, AM_IM2COL>(a, b, ws, splits, M, N, K, rps, s);
}

static int grouped_splits(long M, long tiles) {
  if (g_num_cus == 0) init_num_cus();
  long s = g_num_cus / (tiles > 0 ? tiles : 1);
  const long maxs = (M + 255) / 256;   // >= 256 rows per split
  if (s > maxs) s = maxs;
  return (int)(s < 1 ? 1 : s);
}

static long grouped_tiles(const kair_wgrad_job* jobs, int njobs) {
  long t = 0;
  for (int i = 0; i < njobs; ++i) t += (long)((jobs[i].N + TNR_BN - 1) / TNR_BN) * ((jobs[i].K + TNR_BK - 1) / TNR_BK);
  return t;
}

// max_ctas > 0: at most that many (tile, split) workgroups -- fewer splits, so the launch holds only part
// of the chip (the deferred gradient work beside the data-gradient chain, which needs the rest)
// max_ctas < 0: -max_ctas times the default splits (shorter workgroups, which hand the CUs back to a
// concurrent chain sooner; the workspace grows by the same factor), at >= 32 rows per split
static int grouped_splits_capped(long M, long ntiles, int max_ctas) {
  int s = grouped_splits(M, ntiles);
  if (max_ctas > 0) {
    const long cap = max_ctas / (ntiles > 0 ? ntiles : 1);
    if (s > cap) s = (int)(cap < 1 ? 1 : cap);
  } else if (max_ctas < 0) {
    long t = (long)s * -max_ctas;
    const long maxs = (M + TNR_RB - 1) / TNR_RB;
    s = (int)(t < maxs ? t : maxs);
  }
  return s;
}

// fp32x3 pair jobs (gemm_x3.hip): 192 x 192 tiles
static long grouped_tiles_x3(const kair_wgrad_job* jobs, int njobs) {
  long t = 0;
  for (int i = 0; i < njobs; ++i) t += (long)((jobs[i].N + 191) / 192) * ((jobs[i].K + 191) / 192);
  return t;
}
int kair_wgrad_grouped_x3(const kair_wgrad_job* jobs, int njobs, long M, float* ws, int splits, void* stream);

extern "C" long kair_wgrad_grouped_ws(const kair_wgrad_job* jobs, int njobs, long M) {
  if (!jobs || njobs <= 0 || M <= 0) return 0;
  const bool x3 = jobs[0].A.dtype == KAIR_F16;
  const int splits = grouped_splits(M, x3 ? grouped_tiles_x3(jobs, njobs) : grouped_tiles(jobs, njobs));
  long nk = 0;
  for (int i = 0; i < njobs; ++i) nk += (long)jobs[i].N * jobs[i].K;
  return (long)splits * nk;
}

extern "C" int kair_wgrad_grouped_ex(const kair_wgrad_job* jobs, int njobs, long M, float* ws, int max_ctas,
                                     void* stream);
extern "C" int kair_wgrad_grouped(const kair_wgrad_job* jobs, int njobs, long M, float* ws, void* stream) {
  return kair_wgrad_grouped_ex(jobs, njobs, M, ws, 0, stream);
}

extern "C" int kair_wgrad_grouped_ex(const kair_wgrad_job* jobs, int njobs, long M, float* ws, int max_ctas,
                                     void* stream) {
  KAIR_CHECK_ARG(jobs && ws && njobs > 0 && njobs <= KAIR_WG_MAX && M > 0 && M < (1L << 30),
                 "wgrad_grouped: 1..%d jobs, M > 0 and a workspace", KAIR_WG_MAX);
  KAIR_CHECK_ARG(((uintptr_t)ws % 16) == 0, "wgrad_grouped: workspace not 16-byte aligned");
  int rc;
  if (jobs[0].A.dtype == KAIR_F16) {   // fp32x3: fp16-pair operands on the x3 TN ring
    for (int i = 0; i < njobs; ++i) {
      if ((rc = kair_check_operand(&jobs[i].A, "wgrad_grouped A"))) return rc;
      if ((rc = kair_check_operand(&jobs[i].B, "wgrad_grouped B"))) return rc;
    }
    return kair_wgrad_grouped_x3(jobs, njobs, M, ws, grouped_splits_capped(M, grouped_tiles_x3(jobs, njobs), max_ctas),
                                 stream);
  }
  TnGroup g;
  FinGroup f;
  memset(&g, 0, sizeof(g));
  memset(&f, 0, sizeof(f));
  const long ntiles = grouped_tiles(jobs, njobs);
  const int splits = grouped_splits_capped(M, ntiles, max_ctas);
  long rps = (M + splits - 1) / splits;
  rps = (rps + TNR_RB - 1) / TNR_RB * TNR_RB;
  int qkv_seen = 0;
  long tile0 = 0, off = 0, blk0 = 0;
  for (int i = 0; i < njobs; ++i) {
    const kair_wgrad_job& J = jobs[i];
    if ((rc = kair_check_operand(&J.A, "wgrad_grouped A"))) return rc;
    if ((rc = kair_check_operand(&J.B, "wgrad_grouped B"))) return rc;
    KAIR_CHECK_ARG(J.A.dtype == KAIR_BF16 && J.B.dtype == KAIR_BF16, "wgrad_grouped: job %d operands must be bf16", i);
    KAIR_CHECK_ARG((J.A.mode == KAIR_LD_ROWS || J.A.mode == KAIR_LD_QKVBLK) && J.B.mode == KAIR_LD_ROWS,
                   "wgrad_grouped: job %d: A rows or q/k/v blocked, B rows", i);
    KAIR_CHECK_ARG(!J.A.rowscale && !J.B.rowscale && J.A.win_ws == 0 && J.B.win_ws == 0 && J.A.ones_col < 0 &&
                       (J.B.ones_col < 0 || J.B.ones_in_data),
                   "wgrad_grouped: job %d: no row scale / window map / injected ones column", i);
    KAIR_CHECK_ARG(tn_ring_shape_grouped(M, J.N, J.K) && (J.A.mode != KAIR_LD_ROWS || J.A.ld % 8 == 0) && J.B.ld % 8 == 0,
                   "wgrad_grouped: job %d shape (N %d, K %d) / strides", i, J.N, J.K);
    KAIR_CHECK_ARG(J.grad && J.map.kind == 0 && (long)J.map.nG * J.map.nGp == J.N && (long)J.map.kG * J.map.kGp == J.K,
                   "wgrad_grouped: job %d needs a linear map whose packed dims are (N, K)", i);
    KAIR_CHECK_ARG(!J.bias_grad || (J.ones_col >= 0 && J.ones_col < J.K), "wgrad_grouped: job %d bias needs ones_col", i);
    if (J.A.mode == KAIR_LD_QKVBLK) {
      if (!qkv_seen) g.qa = make_op(J.A, M);
      KAIR_CHECK_ARG(!qkv_seen || (J.A.qkv_nh == g.qa.nh && J.A.qkv_hdp == g.qa.hdp && J.A.qkv_tok == g.qa.tok),
                     "wgrad_grouped: q/k/v jobs must share one geometry");
      qkv_seen = 1;
    }
    const int tilesK = (J.K + TNR_BK - 1) / TNR_BK;
    TnJob& t = g.j[i];
    t.a = (const bf16*)J.A.ptr; t.b = (const bf16*)J.B.ptr; t.ws = ws + off;
    t.lda = (int)J.A.ld; t.ldb = (int)J.B.ld; t.N = J.N; t.K = J.K; t.tilesK = tilesK; t.tile0 = (int)tile0;
    t.qkv = J.A.mode == KAIR_LD_QKVBLK;
    tile0 += (long)((J.N + TNR_BN - 1) / TNR_BN) * tilesK;
    FinJob& q = f.j[i];
    q.part = ws + off; q.grad = J.grad; q.bias = J.bias_grad; q.mp = J.map; q.ones_col = J.bias_grad ? J.ones_col : -1;
    q.Kt = J.K; q.plane = (long)J.N * J.K; q.blk0 = blk0;
    blk0 += ((long)J.N * J.K / 4 + 63) / 64;
    off += (long)splits * J.N * J.K;
  }
  g.njobs = njobs; g.ntiles = (int)ntiles; g.M = (int)M; g.rps = (int)rps;
  f.njobs = njobs; f.splits = splits; f.nblocks = blk0;
  hipStream_t s = (hipStream_t)stream;
  KAIR_LAUNCH(gemm_tn_ring_grouped, dim3((unsigned)(ntiles * splits)), dim3(512), 0, s, g);
  KAIR_CHECK_LAUNCH();
  return kair_launch_finalize_grouped(f, s);
}
