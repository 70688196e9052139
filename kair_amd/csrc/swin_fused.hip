// Fused Swin Transformer block halves for gfx950 (bf16 MFMA, fp32 accumulation): the attention half
//
//   mid = x + s * proj( W-MSA( LN1(x) ) )          network_swinir.py:239-272 (SwinTransformerBlock
//                                                   .forward up to the first residual) with
//                                                   WindowAttention.forward :114-145
//
// as ONE launch: one workgroup per 8x8 window, one wave per head (nh = 6, Cp = 32 * nh = 192).
//   A  LN1 of the window's 64 token rows (read through the cyclic-shift + window-partition row map)
//      into an LDS tile (bf16), also stored for backward (window order, ones column at C) with the
//      per-token mean / rstd;
//   B  per head: Q^T = Wq_h . LN^T, K^T = Wk_h . LN^T, V = LN . Wv_h^T with v_mfma_f32_32x32x16_bf16;
//      the accumulators ARE the attention operands -- register r of lane half hh holds d =
//      acc_row(r, hh), so packing registers 8s..8s+7 gives an MFMA fragment whose contraction
//      index runs over a permutation of d that is the same for q and k (and of the keys for P and
//      v): q, k, v never pass through LDS.  Stored head-blocked for backward;
//   C  S^T = K Q^T * scale + rel-pos bias (+ shift-region mask), wave64 softmax, O^T = V^T P^T;
//      O stored for backward (ones column) and into the LDS tile (LN no longer needed);
//   D  proj: wave w makes output channels [32w, 32w+32) of the 64 rows, + bias, * DropPath scale,
//      + the fp32 residual x, scattered back to token order (window_reverse + reverse roll).
// The saved tensors are exactly those of the unfused path (ln1, m1, r1, qkv, O, lse), so the
// backward program is unchanged.  Per window the kernel moves x (49 KB fp32) in and mid (49 KB)
// + ln1 / O (2 x 24.6 KB) + q/k/v (73.7 KB) out: 221 KB, against ~4x that across the separate
// LayerNorm / QKV / attention / proj kernels it replaces.
#include <stdlib.h>

#include <type_traits>

#include "common.h"

namespace {

constexpr int TOK = 64, WSZ = 8;
#ifndef KAIR_ATTN12
#define KAIR_ATTN12 1
#endif

KAIR_DEV int acc_row32(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }
KAIR_DEV int shift_region(int coord, int n, int shift) { return coord < n - WSZ ? 0 : (coord < n - shift ? 1 : 2); }

// perf-investigation phase stamps of the fused attention half (debug builds, KAIR_ATTN_DBG bit 8): per
// wave, s_memtime at the phase boundaries of its workgroup's last window (kair_debug_fused_stamps)
constexpr int FST_WAVES = 4096, FST_N = 8;
__device__ unsigned long long g_fused_stamps[FST_WAVES * FST_N];
KAIR_DEV unsigned long long fst_now() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

struct AttnFwdArgs {
  const float* x; long ldx;                  // residual stream fp32 [M][ldx], token order
  const float* gamma; const float* beta;     // LN1
  float eps; int C;
  bf16* ln; long ldln;                       // saved LN1 output, window order, ones column at C
  float* mean; float* rstd;                  // [M], token order
  const bf16* wqkv; const float* bqkv;       // fragment order (pack kind 10) of [3*nh*32][Cp], bias
  bf16* qkv;                                 // head-blocked [3][nWin][nh][64][32]
  const float* table; float scale;           // [225][nh]
  bf16* O; long ldo; int o_ones_col;         // [M][ldo], window order
  float* lse;                                // [nWin][nh][64]
  const bf16* wproj; const float* bproj;     // fragment order (pack kind 10) of [Cp][nh*32], bias
  const float* rowscale; int win_per_scale;  // DropPath per-sample scale (NULL = 1)
  float* out; long ldout;                    // mid fp32 [M][ldout], token order
  long nWin; int H, W, shift;
  WinMap wm;
  int dbg;   // ablation bits (KAIR_ATTN_DBG, perf investigation only): 1 no q/k/v stores, 2 no end-of-window stores
};

KAIR_DEV bf16x8 pack8r(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)a[8 * s + j];
  return r;
}

// Persistent: one workgroup per CU loops over windows.  Memory-operation order: vmcnt counts
// loads AND stores in issue order, so a wait for a load issued after a store also waits for that
// store.  The NEXT window's x rows and first weight fragments are issued before the O-tile barrier
// and waited for (behind the proj GEMM) before this window's stores are issued, so no later wait
// drains those stores.  One window is ~37 k cycles of barrier-separated phases, issue-bound on the
// two SIMDs that carry two of the six waves (tools/attn_fwd_stamps.py).  The fp32 x
// rows also stay in LDS for the residual, so nothing is re-read.

// NS = 2: hi/lo split weights (pack kind 12), each k-step multiplies the same LN / O fragment by
// the hi and the lo half, so the products see the fp32 master weights to ~16 mantissa bits.
template <int NH, int NS>
__global__ __launch_bounds__(64 * NH) void swin_attn_fwd_kernel(const AttnFwdArgs a) {
  constexpr int CP = 32 * NH, LDT = CP + 8, LDX = CP + 4, KB = CP / 16;
  constexpr int RPW = (TOK + NH - 1) / NH, PF = NS == 1 ? 3 : 2, WS = 512 * NS;   // WS: k-step stride
  static_assert(KB % PF == 0, "k-steps must be a multiple of the prefetch depth");
  __shared__ __attribute__((aligned(16))) bf16 sT[TOK * LDT];   // LN1 tile
  __shared__ __attribute__((aligned(16))) bf16 sO[TOK * LDT];   // O tile
  __shared__ __attribute__((aligned(16))) float sX[TOK * LDX];  // x rows (fp32) for the residual
  __shared__ float sTabR[NH][232];          // relative-position bias, REVERSED: sTabR[h][224 - idx]
  __shared__ float sBias[3 * NH * 32];       // qkv bias (packed, head-padded)
  __shared__ float sGB[2][CP];               // LN1 gamma, beta (0 past C)
  __shared__ int sReg[TOK];
  __shared__ int sRow[TOK];
  __shared__ float sMean[TOK], sRstd[TOK];
  constexpr int LDV = 40;                    // v transpose scratch row stride (80 B, 16 B aligned)
  __shared__ __attribute__((aligned(16))) bf16 sV[NH][TOK * LDV];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l31 = lane & 31, hh = lane >> 5;
  const long M = a.nWin * TOK;
  bf16* sVw = sV[w];
  const int h = w;
  const int c = 32 * w + l31;   // phase D output channel of this lane
  long win = blockIdx.x;

  // ---- prologue: first window's x rows, first q/k/v weight fragments, per-head tables ------------
  // x rows: 16 lanes per row (lane group g, lane jl in it), channels 4 jl + 64 k (k < 3: 768 B
  // of a row per 16 lanes, coalesced); pass p covers row index i = 4 p + g of the wave's rows
  // w + NH i.
  static_assert(CP == 192, "the fused attention kernel is laid out for Cp = 192");
  constexpr int NPASS = (RPW + 3) / 4;
  const int g = lane >> 4, jl = lane & 15;
  // Branch-free (lanes past the window's rows re-read its row 0, past the last window the last window),
  // so the compiler's vmcnt bookkeeping stays exact across it: the waits for older loads then count
  // the newer loads and stores instead of draining every store in flight.
  float4 xv[NPASS][3];
  auto load_x = [&](long wn) {
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      const int i = 4 * p + g, r = w + NH * i;
      const long wc = wn < a.nWin ? wn : a.nWin - 1;
      const int rr = i < RPW && r < TOK ? r : 0;
      const long base = win_to_token(wc * TOK + rr, a.wm) * a.ldx;
#pragma unroll
      for (int k = 0; k < 3; ++k) xv[p][k] = *(const float4*)(a.x + base + 4 * jl + 64 * k);
    }
  };
  load_x(win);
  const bf16* wq = a.wqkv + (long)((0 * NH + h) * KB) * WS + lane * 8;
  const bf16* wk = a.wqkv + (long)((1 * NH + h) * KB) * WS + lane * 8;
  const bf16* wv = a.wqkv + (long)((2 * NH + h) * KB) * WS + lane * 8;
  const bf16* wp = a.wproj + (long)(w * KB) * WS + lane * 8;
  bf16x8 pq[PF][NS], pk[PF][NS], pv[PF][NS];
  auto load_w = [&]() {
#pragma unroll
    for (int i = 0; i < PF; ++i)
#pragma unroll
      for (int e = 0; e < NS; ++e) {
        pq[i][e] = *(const bf16x8*)(wq + i * WS + e * 512);
        pk[i][e] = *(const bf16x8*)(wk + i * WS + e * 512);
        pv[i][e] = *(const bf16x8*)(wv + i * WS + e * 512);
      }
  };
  load_w();
  for (int i = lane; i < (2 * WSZ - 1) * (2 * WSZ - 1); i += 64) sTabR[w][224 - i] = a.table[i * NH + w];
  for (int i = tid; i < 3 * NH * 32; i += 64 * NH) sBias[i] = a.bqkv[i];
  for (int i = tid; i < CP; i += 64 * NH) {
    sGB[0][i] = i < a.C ? a.gamma[i] : 0.f;
    sGB[1][i] = i < a.C ? a.beta[i] : 0.f;
  }
  const float bvl = a.bqkv[(2 * NH + h) * 32 + l31];
  const float bc = a.bproj[c];
  __syncthreads();   // sTabR, sBias, sGB visible
  const float inv_c = 1.0f / (float)a.C;
  const int nWw = a.W / WSZ, nW = (a.H / WSZ) * nWw;

  unsigned long long fts[FST_N];
  const bool fstamp = KAIR_DBG(a.dbg & 8) && (long)blockIdx.x * NH + w < FST_WAVES;
  for (; win < a.nWin; win += gridDim.x) {
    const bool fst_on = fstamp;   // every window; the workgroup's last one is what stays
    if (fst_on) fts[0] = fst_now();
    // row map and shift regions of this window (readers are behind the LN barrier; the previous
    // iteration's last readers are behind its closing barrier)
    const int wi = (int)(win % nW), wy = wi / nWw, wx = wi - wy * nWw;
    if (tid < TOK) {
      sRow[tid] = (int)win_to_token(win * TOK + tid, a.wm);
      sReg[tid] = a.shift > 0 ? shift_region(wy * WSZ + (tid >> 3), a.H, a.shift) * 3 +
                                    shift_region(wx * WSZ + (tid & 7), a.W, a.shift)
                              : 0;
    }
    const bool mixed = a.shift > 0 && (wy == a.H / WSZ - 1 || wx == nWw - 1);

    // ---- A: LayerNorm, 16 lanes per row (DPP sums, no LDS permutes); x rows -> sX (fp32), LN rows
    // -> sT (bf16, 1.0 in column C)
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      const int i = 4 * p + g, r = w + NH * i;
      const bool ok = i < RPW && r < TOK;
      float sm = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int cb = 4 * jl + 64 * k;
        sm += (cb + 0 < a.C ? xv[p][k].x : 0.f) + (cb + 1 < a.C ? xv[p][k].y : 0.f) +
              (cb + 2 < a.C ? xv[p][k].z : 0.f) + (cb + 3 < a.C ? xv[p][k].w : 0.f);
      }
      const float mu = dpp_sum16(sm) * inv_c;
      float q = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int cb = 4 * jl + 64 * k;
        const float vv[4] = {xv[p][k].x, xv[p][k].y, xv[p][k].z, xv[p][k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = cb + j < a.C ? vv[j] - mu : 0.f;
          q += d * d;
        }
      }
      const float rs = rsqrtf(dpp_sum16(q) * inv_c + a.eps);
      if (ok) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int cb = 4 * jl + 64 * k;
          const float vv[4] = {xv[p][k].x, xv[p][k].y, xv[p][k].z, xv[p][k].w};
          bf16x4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int cc = cb + j;
            o[j] = (bf16)(cc < a.C ? (vv[j] - mu) * rs * sGB[0][cc] + sGB[1][cc] : (cc == a.C ? 1.f : 0.f));
          }
          *(bf16x4*)(sT + r * LDT + cb) = o;
          *(float4*)(sX + r * LDX + cb) = xv[p][k];
        }
        if (jl == 0) {
          sMean[r] = mu;
          sRstd[r] = rs;
        }
      }
    }
    __syncthreads();           // LN tile, sX, sRow, sReg visible
    if (fst_on) fts[1] = fst_now();

    // ---- B: q^T, k^T, v of head h = w (weight fragments PF k-steps ahead) -----------------------
    f32x16 QT[2], KT[2], V[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) QT[t][r] = KT[t][r] = V[t][r] = 0.f;
    // k-steps in groups of PF; the last group refills nothing, so the loads stay unconditional and the
    // compiler's vmcnt bookkeeping exact across the loop (a conditional load makes it wait for all)
    auto qkv_steps = [&](int kb0, auto refill) {
#pragma unroll
      for (int sl = 0; sl < PF; ++sl) {
        const int kb = kb0 + sl;
        bf16x8 fl[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) fl[t] = *(const bf16x8*)(sT + (t * 32 + l31) * LDT + kb * 16 + 8 * hh);
#pragma unroll
        for (int e = 0; e < NS; ++e)
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            QT[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pq[sl][e], fl[t], QT[t], 0, 0, 0);
            KT[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pk[sl][e], fl[t], KT[t], 0, 0, 0);
            V[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fl[t], pv[sl][e], V[t], 0, 0, 0);
          }
        // refill the slot after its MFMAs: the load lands in the same registers (no loop-carried
        // copies, whose reads would make every iteration wait for the loads just issued)
        if constexpr (decltype(refill)::value) {
#pragma unroll
          for (int e = 0; e < NS; ++e) {
            pq[sl][e] = *(const bf16x8*)(wq + (kb + PF) * WS + e * 512);
            pk[sl][e] = *(const bf16x8*)(wk + (kb + PF) * WS + e * 512);
            pv[sl][e] = *(const bf16x8*)(wv + (kb + PF) * WS + e * 512);
          }
        }
      }
    };
#pragma unroll 1
    for (int kb0 = 0; kb0 < KB - PF; kb0 += PF) qkv_steps(kb0, std::true_type{});
    qkv_steps(KB - PF, std::false_type{});
    if (fst_on) fts[2] = fst_now();
    // proj weight fragments for the first PF k-steps of phase D, in flight during the attention
    bf16x8 pw[PF][NS];
#pragma unroll
    for (int i = 0; i < PF; ++i)
#pragma unroll
      for (int e = 0; e < NS; ++e) pw[i][e] = *(const bf16x8*)(wp + i * WS + e * 512);
    // + bias, round to bf16 (the values attention and the saved q/k/v both use)
    const float* bq = sBias + (0 * NH + h) * 32;
    const float* bk = sBias + (1 * NH + h) * 32;
    bf16x8 Fq[2][2], Fk[2][2], Fv[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int d = acc_row32(8 * s + j, hh);
          Fq[t][s][j] = (bf16)(QT[t][8 * s + j] + bq[d]);
          Fk[t][s][j] = (bf16)(KT[t][8 * s + j] + bk[d]);
          Fv[t][s][j] = (bf16)(V[t][8 * s + j] + bvl);
        }

    // the saved q / k / v go out now (their registers are needed until the attention's last MFMA
    // anyway); the loads after them (proj weights) were issued before
    if (!KAIR_DBG(a.dbg & 1)) {   // q / k / v, head-blocked [part][win][h][tok][32]
      const long part = M * NH * 32;
      bf16* qb = a.qkv + (win * NH + h) * TOK * 32;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int tok = t * 32 + l31;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d0 = 8 * g + 4 * hh, s = g >> 1, j0 = 4 * (g & 1);
          const bf16x4 q4 = {Fq[t][s][j0], Fq[t][s][j0 + 1], Fq[t][s][j0 + 2], Fq[t][s][j0 + 3]};
          const bf16x4 k4 = {Fk[t][s][j0], Fk[t][s][j0 + 1], Fk[t][s][j0 + 2], Fk[t][s][j0 + 3]};
          *(bf16x4*)(qb + tok * 32 + d0) = q4;
          *(bf16x4*)(qb + part + tok * 32 + d0) = k4;
        }
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j) sVw[(t * 32 + acc_row32(8 * s + j, hh)) * LDV + l31] = Fv[t][s][j];
      }
      // v: lane = d in registers -> token rows through the wave's LDS scratch, 16-byte stores
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int id = lane + 64 * i, tok = id >> 2, q8 = (id & 3) * 8;
        *(uint4*)(qb + 2 * part + tok * 32 + q8) = *(const uint4*)(sVw + tok * LDV + q8);
      }
    }

    if (fst_on) fts[3] = fst_now();
    // ---- C: attention of head h ------------------------------------------------------------------
    f32x16 S[2][2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int r = 0; r < 16; ++r) S[kt][qt][r] = 0.f;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
          S[kt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Fk[kt][s], Fq[qt][s], S[kt][qt], 0, 0, 0);
    float lse_v[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int qi = qt * 32 + l31;
      // rel index = (qy - ky + 7) * 15 + (qx - kx + 7); in the reversed table the key part is a
      // compile-time offset per register: 15 ky + kx = 15 (4 kt + r / 4) + r % 4 + 4 hh
      const float* tb = &sTabR[h][112 - 15 * (qi >> 3) - (qi & 7) + 4 * hh];
      float mx = -3.0e38f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float sc = fmaf(S[kt][qt][r], a.scale, tb[15 * (4 * kt + (r >> 2)) + (r & 3)]);
          S[kt][qt][r] = sc;
          mx = fmaxf(mx, sc);
        }
      if (mixed) {   // shifted block, window on the image's last window row / column: region mask
        const int rq = sReg[qi];
        mx = -3.0e38f;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            if (sReg[kt * 32 + acc_row32(r, hh)] != rq) S[kt][qt][r] += -100.f;
            mx = fmaxf(mx, S[kt][qt][r]);
          }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      float sum = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = __expf(S[kt][qt][r] - mx);
          S[kt][qt][r] = e;
          sum += e;
        }
      sum += __shfl_xor(sum, 32, 64);
      const float inv = 1.f / sum;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) S[kt][qt][r] *= inv;
      lse_v[qt] = mx + __logf(sum);
    }
    if (fst_on) fts[4] = fst_now();
    // O^T = V^T P^T: lane = query, registers = d -> the O tile (LDS)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      f32x16 o;
#pragma unroll
      for (int r = 0; r < 16; ++r) o[r] = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int s = 0; s < 2; ++s) o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Fv[kt][s], pack8r(S[kt][qt], s), o, 0, 0, 0);
      const int qi = qt * 32 + l31;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = 8 * g + 4 * hh;
        float r4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) r4[j] = (h * 32 + d0 + j == a.o_ones_col) ? 1.f : o[4 * g + j];
        *(bf16x4*)(sO + qi * LDT + h * 32 + d0) = bf16x4{(bf16)r4[0], (bf16)r4[1], (bf16)r4[2], (bf16)r4[3]};
      }
    }
    load_x(win + gridDim.x);   // the next window's rows and first q/k/v weight fragments, in flight
    load_w();                  // through phase D
    const float rs = a.rowscale ? a.rowscale[win / a.win_per_scale] : 1.f;
    __syncthreads();           // the O tile is complete
    if (fst_on) fts[5] = fst_now();

    // ---- D: proj + bias, DropPath scale, fp32 residual from sX ------------------------------------
    f32x16 P[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) P[t][r] = 0.f;
    auto proj_steps = [&](int kb0, auto refill) {
#pragma unroll
      for (int sl = 0; sl < PF; ++sl) {
        const int kb = kb0 + sl;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const bf16x8 fo = *(const bf16x8*)(sO + (t * 32 + l31) * LDT + kb * 16 + 8 * hh);
#pragma unroll
          for (int e = 0; e < NS; ++e) P[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fo, pw[sl][e], P[t], 0, 0, 0);
        }
        if constexpr (decltype(refill)::value) {
#pragma unroll
          for (int e = 0; e < NS; ++e) pw[sl][e] = *(const bf16x8*)(wp + (kb + PF) * WS + e * 512);
        }
      }
    };
#pragma unroll 1
    for (int kb0 = 0; kb0 < KB - PF; kb0 += PF) proj_steps(kb0, std::true_type{});
    proj_steps(KB - PF, std::false_type{});
    if (fst_on) fts[6] = fst_now();
    // the next window's x rows (and with them the weight fragments) have landed by now, behind the
    // proj GEMM: waiting for them HERE, before this window's stores are issued, keeps the next LN
    // from waiting for those stores to drain (vmcnt retires loads and stores in issue order)
#pragma unroll
    for (int p = 0; p < NPASS; ++p)
#pragma unroll
      for (int k = 0; k < 3; ++k) asm volatile("" ::"v"(xv[p][k].x), "v"(xv[p][k].y), "v"(xv[p][k].z), "v"(xv[p][k].w));

    // ---- stores: mid (token order), then everything saved for backward ---------------------------
    // mid = x + s * (proj + bias), formed in place in sX, then stored row-contiguous
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float* px = sX + (t * 32 + acc_row32(r, hh)) * LDX + c;
        *px = *px + rs * (P[t][r] + bc);
      }
    __syncthreads();
    constexpr int C4 = CP / 4;
    for (int i = tid; i < (KAIR_DBG(a.dbg & 2) ? 0 : TOK * C4); i += 64 * NH) {
      const int r = i / C4, q = (i - (i / C4) * C4) * 4;
      *(float4*)(a.out + (long)sRow[r] * a.ldout + q) = *(const float4*)(sX + r * LDX + q);
    }
    if (hh == 0 && !KAIR_DBG(a.dbg & 2)) {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) a.lse[(win * NH + h) * TOK + qt * 32 + l31] = lse_v[qt];
    }
    // LN1 rows and O rows from LDS, 16 bytes per lane (window order)
    constexpr int CH = CP / 8;   // 16-byte chunks per row
    for (int i = tid; i < (KAIR_DBG(a.dbg & 2) ? 0 : TOK * CH); i += 64 * NH) {
      const int r = i / CH, q = (i - (i / CH) * CH) * 8;
      *(uint4*)(a.ln + (win * TOK + r) * a.ldln + q) = *(const uint4*)(sT + r * LDT + q);
      *(uint4*)(a.O + (win * TOK + r) * a.ldo + q) = *(const uint4*)(sO + r * LDT + q);
    }
    if (tid < TOK && !KAIR_DBG(a.dbg & 2)) {
      const long t = sRow[tid];
      a.mean[t] = sMean[tid];
      a.rstd[t] = sRstd[tid];
    }
    __syncthreads();   // every LDS tile / row map of this window consumed
    if (fst_on) {
      fts[7] = fst_now();
      if (lane < FST_N) {
        // the stamp of phase 0 carries the wave's SIMD (HW_ID bits 5:4) in its top byte
        const unsigned hwid = __builtin_amdgcn_s_getreg(4 | (31 << 11));
        unsigned long long v = (fts[0] & 0x00FFFFFFFFFFFFFFull) | ((unsigned long long)((hwid >> 4) & 3) << 56);
#pragma unroll
        for (int i = 1; i < FST_N; ++i)
          if (lane == i) v = fts[i];
        g_fused_stamps[((long)blockIdx.x * NH + w) * FST_N + lane] = v;
      }
    }
  }
}


// ---- attention half, 12 waves: two per head ------------------------------------------------------
// The same program as swin_attn_fwd_kernel, balanced over the four SIMDs: wave w = 2 h + q owns head h
// and query / token tile q (tokens 32 q .. 32 q + 31) of the window, so every SIMD carries three waves
// and 1.5 heads' work (the 6-wave kernel's SIMDs 0 / 1 carry two heads each and set the pace of every
// head phase).  Per window:
//   A  LayerNorm, rows w + 12 i (16 rows per SIMD);
//   B  q^T, k^T and v of head h for the wave's 32 tokens (36 MFMAs 32x32x16 instead of 72): its k half
//      goes to the partner wave through LDS in MFMA-fragment form, its v half through the v-transpose
//      scratch that also feeds the saved v rows;
//   C  S^T of the wave's 32 queries x 64 keys, softmax, O^T = V^T P^T into the O tile;
//   D  proj: wave w makes output channels 32 (w >> 1) .. +31 of token tile w & 1;
// then the stores, spread over all twelve waves.  Saves exactly what the 6-wave kernel saves.
template <int NH>
__global__ __launch_bounds__(128 * NH) void swin_attn_fwd12_kernel(const AttnFwdArgs a) {
  constexpr int CP = 32 * NH, LDT = CP + 8, LDX = CP + 4, KB = CP / 16;
  constexpr int NW = 2 * NH, PF = 3, WS = 512;
  constexpr int RPW = (TOK + NW - 1) / NW;   // LN rows per wave (6)
  static_assert(KB % PF == 0, "k-steps must be a multiple of the prefetch depth");
  static_assert(CP == 192, "laid out for Cp = 192");
  __shared__ __attribute__((aligned(16))) bf16 sT[TOK * LDT];   // LN1 tile
  // O tile; before phase C it carries the k fragments exchanged between the two waves of a head
  __shared__ __attribute__((aligned(16))) bf16 sO[TOK * LDT];
  __shared__ __attribute__((aligned(16))) float sX[TOK * LDX];  // x rows (fp32) for the residual
  __shared__ float sTabR[NH][232];
  __shared__ float sBias[3 * NH * 32];
  __shared__ float sGB[2][CP];
  __shared__ int sReg[TOK];
  __shared__ int sRow[TOK];
  __shared__ float sMean[TOK], sRstd[TOK];
  constexpr int LDV = 40;
  __shared__ __attribute__((aligned(16))) bf16 sV[NH][TOK * LDV];   // v rows [tok][d] of each head
  static_assert(NH * 2 * 2 * 64 * 8 <= TOK * LDT, "the k exchange must fit the O tile");
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l31 = lane & 31, hh = lane >> 5;
  const int h = w >> 1, q = w & 1;   // head, token / query tile
  const long M = a.nWin * TOK;
  bf16* sVh = sV[h];
  bf16* sK = sO;   // [NH][2 tiles][2 s][64 lanes][8]
  const int c = 32 * h + l31;   // phase D output channel of this lane (channel block h, token tile q)
  long win = blockIdx.x;

  constexpr int NPASS = (RPW + 3) / 4;
  const int g = lane >> 4, jl = lane & 15;
  float4 xv[NPASS][3];
  auto load_x = [&](long wn) {
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      const int i = 4 * p + g, r = w + NW * i;
      const long wc = wn < a.nWin ? wn : a.nWin - 1;
      const int rr = i < RPW && r < TOK ? r : 0;
      const long base = win_to_token(wc * TOK + rr, a.wm) * a.ldx;
#pragma unroll
      for (int k = 0; k < 3; ++k) xv[p][k] = *(const float4*)(a.x + base + 4 * jl + 64 * k);
    }
  };
  load_x(win);
  const bf16* wq = a.wqkv + (long)((0 * NH + h) * KB) * WS + lane * 8;
  const bf16* wk = a.wqkv + (long)((1 * NH + h) * KB) * WS + lane * 8;
  const bf16* wv = a.wqkv + (long)((2 * NH + h) * KB) * WS + lane * 8;
  const bf16* wp = a.wproj + (long)(h * KB) * WS + lane * 8;
  bf16x8 pq[PF], pk[PF], pv[PF];
  auto load_w = [&]() {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      pq[i] = *(const bf16x8*)(wq + i * WS);
      pk[i] = *(const bf16x8*)(wk + i * WS);
      pv[i] = *(const bf16x8*)(wv + i * WS);
    }
  };
  load_w();
  if (q == 0)
    for (int i = lane; i < (2 * WSZ - 1) * (2 * WSZ - 1); i += 64) sTabR[h][224 - i] = a.table[i * NH + h];
  for (int i = tid; i < 3 * NH * 32; i += 64 * NW) sBias[i] = a.bqkv[i];
  for (int i = tid; i < CP; i += 64 * NW) {
    sGB[0][i] = i < a.C ? a.gamma[i] : 0.f;
    sGB[1][i] = i < a.C ? a.beta[i] : 0.f;
  }
  const float bvl = a.bqkv[(2 * NH + h) * 32 + l31];
  const float bc = a.bproj[c];
  __syncthreads();
  const float inv_c = 1.0f / (float)a.C;
  const int nWw = a.W / WSZ, nW = (a.H / WSZ) * nWw;

  for (; win < a.nWin; win += gridDim.x) {
    // lane-derived values from an opaque copy of the lane id, per window: hoisted out of the loop they
    // would hold ~30 VGPRs of addresses and masks for its whole length (12 waves: 168 VGPRs each)
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int l31 = lane & 31, hh = lane >> 5, g = lane >> 4, jl = lane & 15;
    const int c = 32 * h + l31;
    const int wi = (int)(win % nW), wy = wi / nWw, wx = wi - wy * nWw;
    if (tid < TOK) {
      sRow[tid] = (int)win_to_token(win * TOK + tid, a.wm);
      sReg[tid] = a.shift > 0 ? shift_region(wy * WSZ + (tid >> 3), a.H, a.shift) * 3 +
                                    shift_region(wx * WSZ + (tid & 7), a.W, a.shift)
                              : 0;
    }
    const bool mixed = a.shift > 0 && (wy == a.H / WSZ - 1 || wx == nWw - 1);

    // ---- A: LayerNorm (16 lanes per row), rows w + 12 i -------------------------------------------
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      const int i = 4 * p + g, r = w + NW * i;
      const bool ok = i < RPW && r < TOK;
      float sm = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int cb = 4 * jl + 64 * k;
        sm += (cb + 0 < a.C ? xv[p][k].x : 0.f) + (cb + 1 < a.C ? xv[p][k].y : 0.f) +
              (cb + 2 < a.C ? xv[p][k].z : 0.f) + (cb + 3 < a.C ? xv[p][k].w : 0.f);
      }
      const float mu = dpp_sum16(sm) * inv_c;
      float qq = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int cb = 4 * jl + 64 * k;
        const float vv[4] = {xv[p][k].x, xv[p][k].y, xv[p][k].z, xv[p][k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = cb + j < a.C ? vv[j] - mu : 0.f;
          qq += d * d;
        }
      }
      const float rs = rsqrtf(dpp_sum16(qq) * inv_c + a.eps);
      if (ok) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int cb = 4 * jl + 64 * k;
          const float vv[4] = {xv[p][k].x, xv[p][k].y, xv[p][k].z, xv[p][k].w};
          bf16x4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int cc = cb + j;
            o[j] = (bf16)(cc < a.C ? (vv[j] - mu) * rs * sGB[0][cc] + sGB[1][cc] : (cc == a.C ? 1.f : 0.f));
          }
          *(bf16x4*)(sT + r * LDT + cb) = o;
          *(float4*)(sX + r * LDX + cb) = xv[p][k];
        }
        if (jl == 0) {
          sMean[r] = mu;
          sRstd[r] = rs;
        }
      }
    }
    __syncthreads();           // LN tile, sX, sRow, sReg visible

    // ---- B: q^T, k^T, v of head h for token tile q ----------------------------------------------
    f32x16 QT, KT, V;
#pragma unroll
    for (int r = 0; r < 16; ++r) QT[r] = KT[r] = V[r] = 0.f;
    auto qkv_steps = [&](int kb0, auto refill) {
#pragma unroll
      for (int sl = 0; sl < PF; ++sl) {
        const int kb = kb0 + sl;
        const bf16x8 fl = *(const bf16x8*)(sT + (q * 32 + l31) * LDT + kb * 16 + 8 * hh);
        QT = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pq[sl], fl, QT, 0, 0, 0);
        KT = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pk[sl], fl, KT, 0, 0, 0);
        V = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fl, pv[sl], V, 0, 0, 0);
        if constexpr (decltype(refill)::value) {
          pq[sl] = *(const bf16x8*)(wq + (kb + PF) * WS);
          pk[sl] = *(const bf16x8*)(wk + (kb + PF) * WS);
          pv[sl] = *(const bf16x8*)(wv + (kb + PF) * WS);
        }
      }
    };
#pragma unroll 1
    for (int kb0 = 0; kb0 < KB - PF; kb0 += PF) qkv_steps(kb0, std::true_type{});
    qkv_steps(KB - PF, std::false_type{});
    bf16x8 pw[PF];
#pragma unroll
    for (int i = 0; i < PF; ++i) pw[i] = *(const bf16x8*)(wp + i * WS);
    const float* bq = sBias + (0 * NH + h) * 32;
    const float* bk = sBias + (1 * NH + h) * 32;
    // fragments [s]: this wave's token tile (Fk / Fv), the partner's (Fk2 / Fv2) -- named, never indexed
    // by the run-time tile q (a register array indexed at run time goes to scratch)
    bf16x8 Fq[2], Fk[2], Fv[2], Fk2[2], Fv2[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int d = acc_row32(8 * s2 + j, hh);
        Fq[s2][j] = (bf16)(QT[8 * s2 + j] + bq[d]);
        Fk[s2][j] = (bf16)(KT[8 * s2 + j] + bk[d]);
        Fv[s2][j] = (bf16)(V[8 * s2 + j] + bvl);
      }
    // k fragments to the partner (O tile, unused until phase C writes it), v rows to the scratch
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) *(bf16x8*)(sK + (((h * 2 + q) * 2 + s2) * 64 + lane) * 8) = Fk[s2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 8; ++j) sVh[(q * 32 + acc_row32(8 * s2 + j, hh)) * LDV + l31] = Fv[s2][j];
    if (!KAIR_DBG(a.dbg & 1)) {   // saved q / k of this tile, head-blocked [part][win][h][tok][32]
      const long part = M * NH * 32;
      bf16* qb = a.qkv + (win * NH + h) * TOK * 32;
      const int tok = q * 32 + l31;
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int d0 = 8 * gg + 4 * hh, s2 = gg >> 1, j0 = 4 * (gg & 1);
        const bf16x4 q4 = {Fq[s2][j0], Fq[s2][j0 + 1], Fq[s2][j0 + 2], Fq[s2][j0 + 3]};
        const bf16x4 k4 = {Fk[s2][j0], Fk[s2][j0 + 1], Fk[s2][j0 + 2], Fk[s2][j0 + 3]};
        *(bf16x4*)(qb + tok * 32 + d0) = q4;
        *(bf16x4*)(qb + part + tok * 32 + d0) = k4;
      }
    }
    __syncthreads();   // k fragments and v rows of both tiles visible
    if (!KAIR_DBG(a.dbg & 1)) {   // saved v rows of this tile, 16-byte stores
      bf16* vb = a.qkv + 2 * M * NH * 32 + (win * NH + h) * TOK * 32;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int id = lane + 64 * i, tok = q * 32 + (id >> 2), q8 = (id & 3) * 8;
        *(uint4*)(vb + tok * 32 + q8) = *(const uint4*)(sVh + tok * LDV + q8);
      }
    }
    // the partner's k (fragment form) and v (from the scratch rows: register j of lane (d = l31, hh) is
    // token row acc_row32(8 s + j, hh) of the other tile)
    const int o = 1 - q;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      Fk2[s2] = *(const bf16x8*)(sK + (((h * 2 + o) * 2 + s2) * 64 + lane) * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) Fv2[s2][j] = sVh[(o * 32 + acc_row32(8 * s2 + j, hh)) * LDV + l31];
    }

    // ---- C: attention of head h, queries of tile q ----------------------------------------------
    // S[0]: keys of this wave's tile q, S[1]: keys of the partner's tile o (key tile kt[i] below)
    f32x16 S[2];
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int r = 0; r < 16; ++r) S[i2][r] = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      S[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Fk[s2], Fq[s2], S[0], 0, 0, 0);
      S[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Fk2[s2], Fq[s2], S[1], 0, 0, 0);
    }
    const int ktile[2] = {q, o};
    __syncthreads();   // every wave has its partner's k: the O tile is free
    float lse_v;
    {
      const int qi = q * 32 + l31;
      const float* tb = &sTabR[h][112 - 15 * (qi >> 3) - (qi & 7) + 4 * hh];
      float mx = -3.0e38f;
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2) {
        const float* tbk = tb + 60 * ktile[i2];   // 15 * 4 * kt
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float sc = fmaf(S[i2][r], a.scale, tbk[15 * (r >> 2) + (r & 3)]);
          S[i2][r] = sc;
          mx = fmaxf(mx, sc);
        }
      }
      if (mixed) {
        const int rq = sReg[qi];
        mx = -3.0e38f;
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            if (sReg[ktile[i2] * 32 + acc_row32(r, hh)] != rq) S[i2][r] += -100.f;
            mx = fmaxf(mx, S[i2][r]);
          }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      float sum = 0.f;
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = __expf(S[i2][r] - mx);
          S[i2][r] = e;
          sum += e;
        }
      sum += __shfl_xor(sum, 32, 64);
      const float inv = 1.f / sum;
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int r = 0; r < 16; ++r) S[i2][r] *= inv;
      lse_v = mx + __logf(sum);
      f32x16 ov;
#pragma unroll
      for (int r = 0; r < 16; ++r) ov[r] = 0.f;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        ov = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Fv[s2], pack8r(S[0], s2), ov, 0, 0, 0);
        ov = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Fv2[s2], pack8r(S[1], s2), ov, 0, 0, 0);
      }
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int d0 = 8 * gg + 4 * hh;
        float r4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) r4[j] = (h * 32 + d0 + j == a.o_ones_col) ? 1.f : ov[4 * gg + j];
        *(bf16x4*)(sO + qi * LDT + h * 32 + d0) = bf16x4{(bf16)r4[0], (bf16)r4[1], (bf16)r4[2], (bf16)r4[3]};
      }
    }
    load_x(win + gridDim.x);   // the next window's rows and first q/k/v weight fragments, in flight
    load_w();                  // through phase D
    const float rs = a.rowscale ? a.rowscale[win / a.win_per_scale] : 1.f;
    __syncthreads();           // the O tile is complete

    // ---- D: proj of token tile q, output channels 32 h .. 32 h + 31 ------------------------------
    f32x16 P;
#pragma unroll
    for (int r = 0; r < 16; ++r) P[r] = 0.f;
    auto proj_steps = [&](int kb0, auto refill) {
#pragma unroll
      for (int sl = 0; sl < PF; ++sl) {
        const int kb = kb0 + sl;
        const bf16x8 fo = *(const bf16x8*)(sO + (q * 32 + l31) * LDT + kb * 16 + 8 * hh);
        P = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fo, pw[sl], P, 0, 0, 0);
        if constexpr (decltype(refill)::value) pw[sl] = *(const bf16x8*)(wp + (kb + PF) * WS);
      }
    };
#pragma unroll 1
    for (int kb0 = 0; kb0 < KB - PF; kb0 += PF) proj_steps(kb0, std::true_type{});
    proj_steps(KB - PF, std::false_type{});
#pragma unroll
    for (int p = 0; p < NPASS; ++p)
#pragma unroll
      for (int k = 0; k < 3; ++k) asm volatile("" ::"v"(xv[p][k].x), "v"(xv[p][k].y), "v"(xv[p][k].z), "v"(xv[p][k].w));
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float* px = sX + (q * 32 + acc_row32(r, hh)) * LDX + c;
      *px = *px + rs * (P[r] + bc);
    }
    __syncthreads();
    constexpr int C4 = CP / 4;
    for (int i = tid; i < (KAIR_DBG(a.dbg & 2) ? 0 : TOK * C4); i += 64 * NW) {
      const int r = i / C4, qq = (i - (i / C4) * C4) * 4;
      *(float4*)(a.out + (long)sRow[r] * a.ldout + qq) = *(const float4*)(sX + r * LDX + qq);
    }
    if (hh == 0 && !KAIR_DBG(a.dbg & 2)) a.lse[(win * NH + h) * TOK + q * 32 + l31] = lse_v;
    constexpr int CH = CP / 8;
    for (int i = tid; i < (KAIR_DBG(a.dbg & 2) ? 0 : TOK * CH); i += 64 * NW) {
      const int r = i / CH, qq = (i - (i / CH) * CH) * 8;
      *(uint4*)(a.ln + (win * TOK + r) * a.ldln + qq) = *(const uint4*)(sT + r * LDT + qq);
      *(uint4*)(a.O + (win * TOK + r) * a.ldo + qq) = *(const uint4*)(sO + r * LDT + qq);
    }
    if (tid < TOK && !KAIR_DBG(a.dbg & 2)) {
      const long t = sRow[tid];
      a.mean[t] = sMean[tid];
      a.rstd[t] = sRstd[tid];
    }
    __syncthreads();   // every LDS tile / row map of this window consumed
  }
}


// ---- MLP half ------------------------------------------------------------------------------------
//   out = mid + s * fc2( GELU( fc1( LN2(mid) ) ) )      network_swinir.py:274-276 + Mlp.forward :24-30
// Persistent, one 1024-thread workgroup per CU looping over 64-row tiles of token rows, WARP-
// SPECIALISED: 12 compute waves never issue a global store, 4 store waves never issue a load.
// On gfx950 vmcnt counts loads and stores in issue order, so in a wave that stores a tile's outputs
// every later load (the streamed weight fragments of the next k-steps, the next tile's rows) waits
// for those stores to drain; here the compute waves' loads wait only for loads, and the store
// waves drain the outputs from LDS while the compute waves run the next phase.
// The hidden layer runs in two 192-column halves so the whole working set fits one CU's LDS:
//   compute: LN2 (x rows prefetched a tile ahead in registers) -> sT, x -> sX (fp32)
//            per half: fc1 (one 32x32 tile per wave) -> u -> sU | GELU pair: h -> sU, g -> sG |
//            fc2 partial (one 32x32 output tile per wave, accumulated over both halves)
//            out = x + s * (fc2 + b2) in place in sX
//   store:   ln2 / mean / rstd from sT | per half g, h from sG, sU | out rows from sX
// Saved for backward as the unfused path stores them (pre_kind 1): LN2 output (1.0 at column C),
// mean / rstd, g = GELU'(u) of the fc1 pre-activation, h = GELU(u) (1.0 at column hd).  Per 64
// rows it moves mid in (49 KB fp32, once) and ln2 (24.6 KB) + g + h (2 x 49 KB) + out (49 KB) out.
struct MlpFwdArgs {
  const float* x; long ldx;                  // mid fp32 [M][ldx]
  const float* gamma; const float* beta;     // LN2
  float eps; int C;
  bf16* ln; long ldln;                       // saved LN2 output, 1.0 at column C
  float* mean; float* rstd;                  // [M]
  const bf16* w1; const float* b1;           // fragment order [HP/32][CP/16][S][64][8], bias [HP]
  bf16* u; bf16* hact; long ldh; int hd;     // GELU'(pre-activation) / GELU output [M][ldh], 1.0 at h column hd
  const bf16* w2; const float* b2;           // fragment order [CP/32][HP/16][S][64][8], bias [CP]
  const float* rowscale; int tiles_per_scale;
  float* out; long ldout;
  long nTiles;
  int dbg;   // ablation bits (KAIR_MLP_DBG, perf investigation only): 1 no fc1 MFMA, 2 no fc2 MFMA, 4 no store-wave stores
};

template <int S>
__global__ __launch_bounds__(1024) void swin_mlp_fwd_kernel(const MlpFwdArgs a) {
  constexpr int NC = 12, NST = 256, CP = 192, HP = 384, HH = HP / 2;
  constexpr int LDT = CP + 8, LDU = HH + 8, LDX = CP + 4;
  constexpr int KB1 = CP / 16, KB2 = HP / 16, KBH = HH / 16, WS = 512 * S, PF = S == 1 ? 4 : 3;
  constexpr int RPW = (TOK + NC - 1) / NC, NPASS = (RPW + 3) / 4;   // LN rows per compute wave
  static_assert(KB1 % PF == 0 && KBH % PF == 0, "k-steps must be a multiple of the prefetch depth");
  __shared__ __attribute__((aligned(16))) bf16 sT[TOK * LDT];    // LN2 tile
  __shared__ __attribute__((aligned(16))) bf16 sU[TOK * LDU];    // h of one hidden half
  __shared__ __attribute__((aligned(16))) bf16 sG[TOK * LDU];    // GELU'(u) of one hidden half
  __shared__ __attribute__((aligned(16))) float sX[TOK * LDX];   // x rows (fp32), then the output rows
  __shared__ __attribute__((aligned(16))) float sB1[HP];
  __shared__ __attribute__((aligned(16))) float sB2[CP];
  __shared__ float sGB[2][CP];
  __shared__ float sMean[TOK], sRstd[TOK];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bool compute = w < NC;
  const int sid = tid - 64 * NC;   // store-wave thread index (0..255)
  const int l31 = lane & 31, hh = lane >> 5;
  const int g = lane >> 4, jl = lane & 15;

  for (int i = tid; i < HP; i += 1024) sB1[i] = a.b1[i];
  for (int i = tid; i < CP; i += 1024) {
    sB2[i] = a.b2[i];
    sGB[0][i] = i < a.C ? a.gamma[i] : 0.f;
    sGB[1][i] = i < a.C ? a.beta[i] : 0.f;
  }
  // compute wave w owns one 32x32 tile of each GEMM: columns 32 (w % 6) (of the hidden half for
  // fc1, of the output for fc2), token rows 32 (w / 6).  MFMA D = W . X^T: lane = token row,
  // registers = columns.
  const int ct = w % 6, rt = w / 6;
  float4 xv[NPASS][3];
  auto load_x = [&](long tl) {
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      const int i = 4 * p + g, r = w + NC * i;
      const bool ok = tl < a.nTiles && i < RPW && r < TOK;
      const long base = ok ? (tl * TOK + r) * a.ldx : 0;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        xv[p][k] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ok) xv[p][k] = *(const float4*)(a.x + base + 4 * jl + 64 * k);
      }
    }
  };
  long tile = blockIdx.x;
  if (compute) load_x(tile);
  __syncthreads();   // sB1, sB2, sGB visible
  const float inv_c = 1.0f / (float)a.C;

  for (; tile < a.nTiles; tile += gridDim.x) {
    const long row0 = tile * TOK;
    // ---- [compute] LayerNorm 2 (16 lanes per row, DPP sums) -> sT (bf16, 1.0 in column C); x -> sX
    if (compute) {
#pragma unroll
      for (int p = 0; p < NPASS; ++p) {
        const int i = 4 * p + g, r = w + NC * i;
        const bool ok = i < RPW && r < TOK;
        float sm = 0.f;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int cb = 4 * jl + 64 * k;
          sm += (cb + 0 < a.C ? xv[p][k].x : 0.f) + (cb + 1 < a.C ? xv[p][k].y : 0.f) +
                (cb + 2 < a.C ? xv[p][k].z : 0.f) + (cb + 3 < a.C ? xv[p][k].w : 0.f);
        }
        const float mu = dpp_sum16(sm) * inv_c;
        float q = 0.f;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int cb = 4 * jl + 64 * k;
          const float vv[4] = {xv[p][k].x, xv[p][k].y, xv[p][k].z, xv[p][k].w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float d = cb + j < a.C ? vv[j] - mu : 0.f;
            q += d * d;
          }
        }
        const float rs = rsqrtf(dpp_sum16(q) * inv_c + a.eps);
        if (ok) {
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const int cb = 4 * jl + 64 * k;
            const float vv[4] = {xv[p][k].x, xv[p][k].y, xv[p][k].z, xv[p][k].w};
            bf16x4 o;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int cc = cb + j;
              o[j] = (bf16)(cc < a.C ? (vv[j] - mu) * rs * sGB[0][cc] + sGB[1][cc] : (cc == a.C ? 1.f : 0.f));
            }
            *(bf16x4*)(sT + r * LDT + cb) = o;
            *(float4*)(sX + r * LDX + cb) = xv[p][k];
          }
          if (jl == 0) {
            sMean[r] = mu;
            sRstd[r] = rs;
          }
        }
      }
    }
    __syncthreads();   // (1) LN tile and x rows visible; the previous tile's output rows are stored
    if (!compute && !KAIR_DBG(a.dbg & 4)) {   // ---- [store] LN2 rows and statistics
      constexpr int CH = CP / 8;
      for (int i = sid; i < TOK * CH; i += NST) {
        const int r = i / CH, q = (i - (i / CH) * CH) * 8;
        *(uint4*)(a.ln + (row0 + r) * a.ldln + q) = *(const uint4*)(sT + r * LDT + q);
      }
      if (sid < TOK) {
        a.mean[row0 + sid] = sMean[sid];
        a.rstd[row0 + sid] = sRstd[sid];
      }
    }
    f32x16 O2;
#pragma unroll
    for (int r = 0; r < 16; ++r) O2[r] = 0.f;
#pragma unroll 1
    for (int half = 0; half < 2; ++half) {
      if (compute) {
        // ---- [compute] fc1, hidden columns 192 half + 32 ct.., rows 32 rt..
        const bf16* w1p = a.w1 + (long)(6 * half + ct) * KB1 * WS + lane * 8;
        bf16x8 pw[PF][S];
#pragma unroll
        for (int i = 0; i < PF; ++i)
#pragma unroll
          for (int e = 0; e < S; ++e) pw[i][e] = *(const bf16x8*)(w1p + i * WS + e * 512);
        f32x16 U;
#pragma unroll
        for (int r = 0; r < 16; ++r) U[r] = 0.f;
#pragma unroll 1
        for (int kb0 = 0; kb0 < (KAIR_DBG(a.dbg & 1) ? 0 : KB1); kb0 += PF) {
#pragma unroll
          for (int sl = 0; sl < PF; ++sl) {
            const int kb = kb0 + sl;
            bf16x8 fw[S];
#pragma unroll
            for (int e = 0; e < S; ++e) {
              fw[e] = pw[sl][e];
              if (kb + PF < KB1) pw[sl][e] = *(const bf16x8*)(w1p + (kb + PF) * WS + e * 512);
            }
            const bf16x8 fl = *(const bf16x8*)(sT + (rt * 32 + l31) * LDT + kb * 16 + 8 * hh);
#pragma unroll
            for (int e = 0; e < S; ++e) U = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[e], fl, U, 0, 0, 0);
          }
        }
        // pre-activation x = acc + b1 (fp32) -> h = GELU(x) -> sU, g = GELU'(x) -> sG (bf16): lane row
        // 32 rt + l31, half-local columns 32 ct + 8 gg + 4 hh + e; h is 1.0 at column hd, 0 past it
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          const int col = 32 * ct + 8 * gg + 4 * hh;
          const float4 bb = *(const float4*)(sB1 + HH * half + col);
          const float xs[4] = {U[4 * gg] + bb.x, U[4 * gg + 1] + bb.y, U[4 * gg + 2] + bb.z, U[4 * gg + 3] + bb.w};
          bf16x4 hv, gv;
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            f32x2 y, dy;
            gelu_pair_fast2((f32x2){xs[e], xs[e + 1]}, y, dy);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              const int cc = HH * half + col + e + q;
              hv[e + q] = cc < a.hd ? (bf16)y[q] : (bf16)(cc == a.hd ? 1.f : 0.f);
              gv[e + q] = (bf16)dy[q];
            }
          }
          *(bf16x4*)(sU + (rt * 32 + l31) * LDU + col) = hv;
          *(bf16x4*)(sG + (rt * 32 + l31) * LDU + col) = gv;
        }
      }
      __syncthreads();   // (3) h and g halves complete
      if (!compute) {
        if (!KAIR_DBG(a.dbg & 4)) {   // ---- [store] g and h of this half
          constexpr int CH = HH / 8;
          for (int i = sid; i < TOK * CH; i += NST) {
            const int r = i / CH, q = (i - (i / CH) * CH) * 8;
            *(uint4*)(a.u + (row0 + r) * a.ldh + HH * half + q) = *(const uint4*)(sG + r * LDU + q);
            *(uint4*)(a.hact + (row0 + r) * a.ldh + HH * half + q) = *(const uint4*)(sU + r * LDU + q);
          }
        }
      } else {
        if (half == 1) load_x(tile + gridDim.x);   // the next tile's rows (nothing to wait behind)
        // ---- [compute] fc2 partial over this half's 192 hidden rows
        const bf16* w2p = a.w2 + ((long)ct * KB2 + KBH * half) * WS + lane * 8;
        bf16x8 pw[PF][S];
#pragma unroll
        for (int i = 0; i < PF; ++i)
#pragma unroll
          for (int e = 0; e < S; ++e) pw[i][e] = *(const bf16x8*)(w2p + i * WS + e * 512);
#pragma unroll 1
        for (int kb0 = 0; kb0 < (KAIR_DBG(a.dbg & 2) ? 0 : KBH); kb0 += PF) {
#pragma unroll
          for (int sl = 0; sl < PF; ++sl) {
            const int kb = kb0 + sl;
            bf16x8 fw[S];
#pragma unroll
            for (int e = 0; e < S; ++e) {
              fw[e] = pw[sl][e];
              if (kb + PF < KBH) pw[sl][e] = *(const bf16x8*)(w2p + (kb + PF) * WS + e * 512);
            }
            const bf16x8 fh = *(const bf16x8*)(sU + (rt * 32 + l31) * LDU + kb * 16 + 8 * hh);
#pragma unroll
            for (int e = 0; e < S; ++e) O2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[e], fh, O2, 0, 0, 0);
          }
        }
      }
      __syncthreads();   // (4) the h / g halves are no longer read (fc2, the stores)
    }
    if (compute) {   // ---- [compute] out = x + s * (fc2 + b2), in place in sX
      const float rs = a.rowscale ? a.rowscale[tile / a.tiles_per_scale] : 1.f;
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int col = 32 * ct + 8 * gg + 4 * hh;
        const float4 bb = *(const float4*)(sB2 + col);
        float* px = sX + (rt * 32 + l31) * LDX + col;
        const float4 xr = *(const float4*)px;
        *(float4*)px = make_float4(xr.x + rs * (O2[4 * gg] + bb.x), xr.y + rs * (O2[4 * gg + 1] + bb.y),
                                   xr.z + rs * (O2[4 * gg + 2] + bb.z), xr.w + rs * (O2[4 * gg + 3] + bb.w));
      }
    }
    __syncthreads();   // (5) output rows complete
    if (!compute && !KAIR_DBG(a.dbg & 4)) {   // ---- [store] output rows (the next LN waits at barrier 1... via (6))
      constexpr int C4 = CP / 4;
      for (int i = sid; i < TOK * C4; i += NST) {
        const int r = i / C4, q = (i - (i / C4) * C4) * 4;
        *(float4*)(a.out + (row0 + r) * a.ldout + q) = *(const float4*)(sX + r * LDX + q);
      }
    }
    __syncthreads();   // (6) sX / sT free for the next tile
  }
}


// ---- MLP half, weights resident in registers (the default, S = 1) --------------------------------
// Same maths and saved tensors as swin_mlp_fwd_kernel, re-laid out for short dependent chains:
// one 12-wave workgroup per CU loads BOTH weight matrices once into registers (wave w: W1 rows
// [32w, 32w+32) -- kind 10, 12 fragments -- and W2 rows [16w, 16w+16) -- kind 14, 12 fragments;
// 96 VGPRs) and then loops over 32-row tiles.  A tile's chain is LN2 -> fc1 (12 MFMAs per wave,
// LN rows from LDS) -> GELU pair -> fc2 (24 v_mfma_f32_16x16x32 per wave, h from LDS) -> residual,
// with no weight traffic at all: the streamed-fragment waits that bounded the 64-row kernel (three
// L2 / HBM round trips per GEMM phase, a whole tile per CU in flight) are gone, and 32-row tiles
// give the B = 4 step (M = 9216) 288 tiles for the 256 CUs instead of 144.  The next tile's x rows
// are issued before this tile's stores (vmcnt retires in issue order); every store reads LDS and
// writes whole 16-byte row chunks; the output rows of tile t are stored during tile t + G's fc1
// (sX double-buffered).
__global__ __launch_bounds__(768, 1) void swin_mlp_fwd_wr_kernel(const MlpFwdArgs a) {
  constexpr int NW = 12, NT = 64 * NW, RT = 32, CP = 192, HP = 384;
  constexpr int LDT = CP + 8, LDH = HP + 8, LDX = CP + 4;
  constexpr int KB1 = CP / 16, KB2 = HP / 32;   // 12 k-steps each
  typedef __attribute__((address_space(3))) float lds_f;
  __shared__ __attribute__((aligned(16))) bf16 sT[RT * LDT];        // LN2 rows (bf16, 1.0 at column C)
  __shared__ __attribute__((aligned(16))) bf16 sH[RT * LDH];        // h = GELU(u)
  __shared__ __attribute__((aligned(16))) bf16 sG[RT * LDH];        // g = GELU'(u)
  __shared__ __attribute__((aligned(16))) float sX[2][RT * LDX];    // x rows, then the output rows
  __shared__ __attribute__((aligned(16))) float sC[HP + 3 * CP];    // b1 | b2 | gamma | beta (0 past C)
  __shared__ float sMean[RT], sRstd[RT];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l31 = lane & 31, hh = lane >> 5, l15 = lane & 15, q4 = lane >> 4;
  const long G = gridDim.x;
  long tile = blockIdx.x;
  if (tile >= a.nTiles) return;

  // resident weights: W1 fragments (nb = w, kb) of kind 10 and W2 fragments (nb = w, kb) of kind 14
  bf16x8 w1r[KB1], w2r[KB2];
#pragma unroll
  for (int kb = 0; kb < KB1; ++kb) w1r[kb] = *(const bf16x8*)(a.w1 + ((long)(w * KB1 + kb) * 64 + lane) * 8);
#pragma unroll
  for (int kb = 0; kb < KB2; ++kb) w2r[kb] = *(const bf16x8*)(a.w2 + ((long)(w * KB2 + kb) * 64 + lane) * 8);
  for (int i = tid; i < HP; i += NT) sC[i] = a.b1[i];
  for (int i = tid; i < CP; i += NT) {
    sC[HP + i] = a.b2[i];
    sC[HP + CP + i] = i < a.C ? a.gamma[i] : 0.f;
    sC[HP + 2 * CP + i] = i < a.C ? a.beta[i] : 0.f;
  }
  const long M = a.nTiles * RT;
  const BufRsrc rx = buf_rsrc(a.x, M * a.ldx * 4), rln = buf_rsrc(a.ln, M * a.ldln * 2);
  const BufRsrc rmu = buf_rsrc(a.mean, M * 4), rrs = buf_rsrc(a.rstd, M * 4);
  const BufRsrc ru = buf_rsrc(a.u, M * a.ldh * 2), rh = buf_rsrc(a.hact, M * a.ldh * 2);
  const BufRsrc ro = buf_rsrc(a.out, M * a.ldout * 4);
  // LN layout: threads 0..511, row lr = tid / 16, lane jl: columns 4 jl + 64 k (k < 3)
  auto load_x = [&](long t, float4 (&xv)[3], int ti) {
    const int lr = (ti >> 4) & (RT - 1), jl = ti & 15;
    const unsigned xoff = ((unsigned)lr * (unsigned)a.ldx + 4u * jl) * 4u;
    if (ti < 16 * RT && t < a.nTiles) {
      const unsigned so = (unsigned)(t * RT * a.ldx * 4);
#pragma unroll
      for (int k = 0; k < 3; ++k) xv[k] = buf_ld4(rx, xoff + 256u * k, so);
    }
  };
  const float inv_c = 1.0f / (float)a.C;
  // output rows of tile t from sX[b] (fp32, 16-byte chunks, 2 per thread)
  auto store_out = [&](long t, int b, int ti) {
    constexpr int C4 = CP / 4;
    const unsigned so = (unsigned)(t * RT * a.ldout * 4);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = ti + NT * j, r = i / C4, c = (i - r * C4) * 4;
      buf_st4(ro, ((unsigned)r * (unsigned)a.ldout + c) * 4u, so, *(const float4*)(&sX[b][r * LDX + c]));
    }
  };

  auto run_tile = [&](long t, int b, float4 (&xv)[3], float4 (&xn)[3], long prev) {
    const long row0 = t * RT;
    // Registers belong to the resident weights: the LDS constants, the lane-derived addresses and the
    // column masks are recomputed per tile instead of being hoisted out of the tile loop (opaque copies
    // of their inputs; the recomputation is a few VALU ops per tile)
    const lds_f* cst = (const lds_f*)sC;
    int ti = tid, C = a.C, hd = a.hd;
    asm volatile("" : "+v"(cst), "+v"(ti), "+s"(C), "+s"(hd));
    const int lane = ti & 63, l31 = lane & 31, hh = lane >> 5, l15 = lane & 15, q4 = lane >> 4;
    const int lr = (ti >> 4) & (RT - 1), jl = ti & 15;
    load_x(t + G, xn, ti);   // the next tile's rows, ahead of every store of this one
    // ---- LN2 of this tile's rows -> sT (bf16), sX[b] (fp32 x), statistics
    if (ti < 16 * RT) {   // LN layout: threads 0..511, row lr, lane jl: columns 4 jl + 64 k (k < 3)
      float sm = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int cb = 4 * jl + 64 * k;
        sm += (cb + 0 < C ? xv[k].x : 0.f) + (cb + 1 < C ? xv[k].y : 0.f) + (cb + 2 < C ? xv[k].z : 0.f) +
              (cb + 3 < C ? xv[k].w : 0.f);
      }
      const float mu = dpp_sum16(sm) * inv_c;
      float qv = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int cb = 4 * jl + 64 * k;
        const float vv[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = cb + j < C ? vv[j] - mu : 0.f;
          qv += d * d;
        }
      }
      const float rs = rsqrtf(dpp_sum16(qv) * inv_c + a.eps);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int cb = 4 * jl + 64 * k;
        const float vv[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int cc = cb + j;
          o[j] = (bf16)(cc < C ? (vv[j] - mu) * rs * cst[HP + CP + cc] + cst[HP + 2 * CP + cc] : (cc == C ? 1.f : 0.f));
        }
        *(bf16x4*)(sT + lr * LDT + cb) = o;
        *(float4*)(&sX[b][lr * LDX + cb]) = xv[k];
      }
      if (jl == 0) {
        sMean[lr] = mu;
        sRstd[lr] = rs;
      }
    }
    __syncthreads();   // (1) LN tile, x rows, statistics visible
    // ---- stores: LN2 rows + statistics of this tile (one 16-byte chunk per thread), output rows of the
    // previous tile
    {
      constexpr int CH = CP / 8;
      const int r = ti / CH, c = (ti - r * CH) * 8;
      buf_st16(rln, ((unsigned)r * (unsigned)a.ldln + c) * 2u, (unsigned)(row0 * a.ldln * 2),
               *(const uint4*)(sT + r * LDT + c));
      if (ti < RT) {
        buf_st1(rmu, 4u * ti, (unsigned)(row0 * 4), sMean[ti]);
        buf_st1(rrs, 4u * ti, (unsigned)(row0 * 4), sRstd[ti]);
      }
      if (prev >= 0) store_out(prev, b ^ 1, ti);
    }
    // ---- fc1: hidden columns [32w, 32w+32), rows 0..31: D = W1 . LN^T (lane = row, registers = columns)
    {
      f32x16 U;
#pragma unroll
      for (int r = 0; r < 16; ++r) U[r] = 0.f;
      // LDS operand reads in groups of 4 k-steps (a scheduling barrier between groups keeps them from all
      // being hoisted: the resident weights leave ~70 VGPRs for everything else)
#pragma unroll
      for (int k0 = 0; k0 < KB1; k0 += 4) {
        bf16x8 fl[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) fl[i] = *(const bf16x8*)(sT + l31 * LDT + (k0 + i) * 16 + 8 * hh);
#pragma unroll
        for (int i = 0; i < 4; ++i) U = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1r[k0 + i], fl[i], U, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      // pre-activation u = acc + b1 (fp32) -> h = GELU(u) -> sH, g = GELU'(u) -> sG; h is 1.0 at
      // column hd and 0 past it
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int col = 32 * w + 8 * gg + 4 * hh;
        const float xs[4] = {U[4 * gg] + cst[col], U[4 * gg + 1] + cst[col + 1], U[4 * gg + 2] + cst[col + 2],
                             U[4 * gg + 3] + cst[col + 3]};
        bf16x4 hv, gv;
#if KAIR_MLP_VAR == 1
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int cc = col + e;
          hv[e] = cc < hd ? (bf16)gelu_fast(xs[e]) : (bf16)(cc == hd ? 1.f : 0.f);
          gv[e] = (bf16)gelu_grad_fast(xs[e]);
        }
#else
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          f32x2 y, dy;
          gelu_pair_fast2((f32x2){xs[e], xs[e + 1]}, y, dy);
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int cc = col + e + q;
            hv[e + q] = cc < hd ? (bf16)y[q] : (bf16)(cc == hd ? 1.f : 0.f);
            gv[e + q] = (bf16)dy[q];
          }
        }
#endif
        *(bf16x4*)(sH + l31 * LDH + col) = hv;
        *(bf16x4*)(sG + l31 * LDH + col) = gv;
#if KAIR_MLP_VAR == 2
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
      }
    }
    __syncthreads();   // (2) h, g complete; sT free
    // ---- stores: g and h rows of this tile (2 x 2 chunks per thread)
    {
      constexpr int CH = HP / 8;
      const unsigned so = (unsigned)(row0 * a.ldh * 2);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int i = ti + NT * j, r = i / CH, c = (i - r * CH) * 8;
        const unsigned vo = ((unsigned)r * (unsigned)a.ldh + c) * 2u;
        buf_st16(ru, vo, so, *(const uint4*)(sG + r * LDH + c));
        buf_st16(rh, vo, so, *(const uint4*)(sH + r * LDH + c));
      }
    }
    // ---- fc2: output columns [16w, 16w+16) for rows 16 rb + (lane & 15); D = W2 . h^T with
    // v_mfma_f32_16x16x32 (lane: row 16 rb + lane % 16, registers: columns 16w + 4 (lane / 16) + r)
    {
      f32x4 Y[2];
      Y[0] = Y[1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k0 = 0; k0 < KB2; k0 += 2) {
        bf16x8 fh[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) fh[i][rb] = *(const bf16x8*)(sH + (16 * rb + l15) * LDH + (k0 + i) * 32 + 8 * q4);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) Y[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2r[k0 + i], fh[i][rb], Y[rb], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      const float rsc = a.rowscale ? a.rowscale[t / a.tiles_per_scale] : 1.f;
      const int col = 16 * w + 4 * q4;
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        float* px = &sX[b][(16 * rb + l15) * LDX + col];
        const float4 xr = *(const float4*)px;
        *(float4*)px = make_float4(xr.x + rsc * (Y[rb][0] + cst[HP + col]), xr.y + rsc * (Y[rb][1] + cst[HP + col + 1]),
                                   xr.z + rsc * (Y[rb][2] + cst[HP + col + 2]), xr.w + rsc * (Y[rb][3] + cst[HP + col + 3]));
      }
    }
    __syncthreads();   // (3) output rows in sX[b] complete; sH / sG free
  };

  float4 x0[3], x1[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) x0[k] = x1[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  load_x(tile, x0, tid);
  __syncthreads();   // sC visible
  long prev = -1;
  int b = 0;
  for (;;) {   // unrolled by two so the double-buffered x rows stay in fixed registers
    run_tile(tile, b, x0, x1, prev);
    prev = tile; b ^= 1; tile += G;
    if (tile >= a.nTiles) break;
    run_tile(tile, b, x1, x0, prev);
    prev = tile; b ^= 1; tile += G;
    if (tile >= a.nTiles) break;
  }
  store_out(prev, b ^ 1, tid);
}

// ---- MLP half, backward ---------------------------------------------------------------------------
// Given D = dL/dout (fp32) and Dc = s_mlp * D (bf16), one persistent warp-specialised launch makes
//   dU   = (Dc . W2) * GELU'(u)                       (fc2 input gradient through the stored gate)
//   dxn  = dU . W1                                    (fc1 input gradient)
//   D   += LN2-backward(dxn)   -> dL/dmid             (network_swinir.py:274-276 backward)
//   Dco  = s_attn * dL/dmid   (bf16, window order: the proj input-gradient operand)
//   dgamma / dbeta partials of LN2 per workgroup
// replacing the fc2 / fc1 input-gradient GEMMs and the LayerNorm backward: dxn never touches HBM,
// dU is written once (the fc1 weight gradient reads it), D is read and written once.
// 12 compute waves run only the GEMMs (they issue no global store, so their streamed weight
// fragments never wait behind one); 4 memory waves store dU and run the LayerNorm backward of the
// PREVIOUS tile (dxn from LDS, x / D / statistics from HBM, results stored straight from
// registers) while the compute waves run this tile's first GEMM.  Hidden dimension in two
// 192-wide halves; weights in transposed fragment order (pack kind 13).
struct MlpBwdArgs {
  const bf16* dc; long lddc;                 // s_mlp * dL/dout, token rows
  const bf16* gd; long ldg;                  // GELU'(fc1 pre-activation), token rows
  const bf16* w2t; const bf16* w1t;          // kind 13 of fc2 ([HP/32][CP/16]) and fc1 ([CP/32][HP/16])
  bf16* du; long lddu;                       // out: dL/d(fc1 pre-activation)
  const float* x; long ldx;                  // LN2 input (mid), token rows
  const float* gamma; const float* mean; const float* rstd; int C;
  float* D; long ldD;                        // dL/dout in, dL/dmid out (token rows)
  bf16* dco; long lddo;                      // out: s_attn * dL/dmid, window-order rows
  const float* rowscale; int tiles_per_scale;
  WinMap wm;
  float* part;                               // [gridDim][2][CP]
  long nTiles;
  int dbg;   // ablation bits (KAIR_MLPB_DBG, perf only): 1 no dH GEMM, 2 no dxn GEMM, 4 no memory-wave work
};

__global__ __launch_bounds__(512) void swin_mlp_bwd_kernel(const MlpBwdArgs a) {
  constexpr int NC = 6, NT = 512, NST = NT - 64 * NC, NG = NST / 16, CP = 192, HH = 192, LDA = CP + 8, LDY = CP + 4;
  constexpr int KBC = CP / 16, KBH = HH / 16, PF = 4;
  static_assert(KBC % PF == 0 && KBH % PF == 0, "k-steps must be a multiple of the prefetch depth");
  __shared__ __attribute__((aligned(16))) bf16 sA[TOK * LDA];    // Dc tile
  __shared__ __attribute__((aligned(16))) bf16 sU[TOK * LDA];    // dU half
  __shared__ __attribute__((aligned(16))) bf16 sG[TOK * LDA];    // GELU' half
  __shared__ __attribute__((aligned(16))) float sY[TOK * LDY];   // dxn (fp32) of the last tile
  __shared__ float sGam[CP];
  __shared__ float sPart[NG][2][CP];   // LN2 parameter-gradient partials, one row per memory-wave row group
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bool compute = w < NC;
  const int sid = tid - 64 * NC;
  const int l31 = lane & 31, hh = lane >> 5;
  const int ct = w;   // compute wave w: hidden / output column tile w, both 32-row tiles
  // memory waves: 16 lanes per LN row, NG rows per pass (row group sg = sid / 16, lane sj)
  const int sg = sid >> 4, sj = sid & 15;
  for (int i = tid; i < CP; i += NT) sGam[i] = i < a.C ? a.gamma[i] : 0.f;
  for (int i = tid; i < NG * 2 * CP; i += NT) (&sPart[0][0][0])[i] = 0.f;
  __syncthreads();
  const float inv_c = 1.0f / (float)a.C;

  // LayerNorm-2 backward of tile tl (dxn in sY) by the memory waves: D += rstd (g dy - mean(g dy) -
  // xh mean(g dy xh)); the finished rows also as s_attn * row (bf16, window order)
  auto ln_bwd = [&](long tl) {
    const long row0 = tl * TOK;
    const float sc = a.rowscale ? a.rowscale[tl / a.tiles_per_scale] : 1.f;
#pragma unroll 1
    for (int p = 0; p < TOK / NG; ++p) {
      const int r = NG * p + sg;
      const long t = row0 + r;
      const float mu = a.mean[t], rs = a.rstd[t];
      float4 xq[3], dcur[3], dv[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        dcur[k] = *(const float4*)(a.D + t * a.ldD + 4 * sj + 64 * k);
        xq[k] = *(const float4*)(a.x + t * a.ldx + 4 * sj + 64 * k);
        dv[k] = *(const float4*)(sY + r * LDY + 4 * sj + 64 * k);
      }
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int cb = 4 * sj + 64 * k;
        const float xa[4] = {xq[k].x, xq[k].y, xq[k].z, xq[k].w};
        const float da[4] = {dv[k].x, dv[k].y, dv[k].z, dv[k].w};
        float4 pgv = *(const float4*)&sPart[sg][0][cb], pbv = *(const float4*)&sPart[sg][1][cb];
        float pgs[4] = {pgv.x, pgv.y, pgv.z, pgv.w}, pbs[4] = {pbv.x, pbv.y, pbv.z, pbv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool in = cb + e < a.C;
          const float xh = in ? (xa[e] - mu) * rs : 0.f;
          const float d = in ? da[e] : 0.f;
          const float gy = d * sGam[cb + e];
          pgs[e] += d * xh;
          pbs[e] += d;
          s1 += gy;
          s2 += gy * xh;
        }
        *(float4*)&sPart[sg][0][cb] = make_float4(pgs[0], pgs[1], pgs[2], pgs[3]);
        *(float4*)&sPart[sg][1][cb] = make_float4(pbs[0], pbs[1], pbs[2], pbs[3]);
      }
      s1 = dpp_sum16(s1) * inv_c;
      s2 = dpp_sum16(s2) * inv_c;
      const long wr = token_to_win(t, a.wm);
#pragma unroll
      for (int k = 0; k < 3; ++k) {   // second pass: x-hat and gamma * dy recomputed, not kept live
        const int cb = 4 * sj + 64 * k;
        const float xa[4] = {xq[k].x, xq[k].y, xq[k].z, xq[k].w};
        const float da[4] = {dv[k].x, dv[k].y, dv[k].z, dv[k].w};
        const float cu[4] = {dcur[k].x, dcur[k].y, dcur[k].z, dcur[k].w};
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool in = cb + e < a.C;
          const float xh = (xa[e] - mu) * rs, gy = da[e] * sGam[cb + e];
          o[e] = cu[e] + (in ? rs * (gy - s1 - xh * s2) : 0.f);
        }
        *(float4*)(a.D + t * a.ldD + cb) = make_float4(o[0], o[1], o[2], o[3]);
        *(bf16x4*)(a.dco + wr * a.lddo + cb) = bf16x4{(bf16)(sc * o[0]), (bf16)(sc * o[1]), (bf16)(sc * o[2]), (bf16)(sc * o[3])};
      }
    }
  };

  long prev = -1;
  for (long tile = blockIdx.x; tile < a.nTiles; tile += gridDim.x) {
    const long row0 = tile * TOK;
    if (compute) {
      // Dc tile and the first GELU' half into LDS
      constexpr int CH = CP / 8;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = tid + 64 * NC * k, r = i / CH, q = (i - (i / CH) * CH) * 8;
        *(uint4*)(sA + r * LDA + q) = *(const uint4*)(a.dc + (row0 + r) * a.lddc + q);
        *(uint4*)(sG + r * LDA + q) = *(const uint4*)(a.gd + (row0 + r) * a.ldg + q);
      }
    }
    __syncthreads();   // (1) Dc tile and GELU' half 0 visible
    // the previous tile's LayerNorm backward (memory waves), under this tile's first GEMM
    if (!compute && prev >= 0 && !KAIR_DBG(a.dbg & 4)) ln_bwd(prev);
    uint4 g1[4];
    if (compute) {   // the second GELU' half, into registers until half 0 has consumed the first
      constexpr int CH = CP / 8;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = tid + 64 * NC * k, r = i / CH, q = (i - (i / CH) * CH) * 8;
        g1[k] = *(const uint4*)(a.gd + (row0 + r) * a.ldg + HH + q);
      }
    }
    f32x16 DX[2];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) DX[rt][r] = 0.f;
#pragma unroll 1
    for (int half = 0; half < 2; ++half) {
      if (compute) {
        // dH tile (hidden columns 192 half + 32 ct.., rows 32 rt..) = W2^T . Dc^T, times GELU'
        const bf16* wp = a.w2t + ((long)(6 * half + ct) * KBC * 64 + lane) * 8;
        bf16x8 pw[PF];
#pragma unroll
        for (int i = 0; i < PF; ++i) pw[i] = *(const bf16x8*)(wp + i * 512);
        f32x16 U[2];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
          for (int r = 0; r < 16; ++r) U[rt][r] = 0.f;
#pragma unroll 1
        for (int kb0 = 0; kb0 < (KAIR_DBG(a.dbg & 1) ? 0 : KBC); kb0 += PF) {
#pragma unroll
          for (int sl = 0; sl < PF; ++sl) {
            const int kb = kb0 + sl;
            const bf16x8 fw = pw[sl];
            if (kb + PF < KBC) pw[sl] = *(const bf16x8*)(wp + (kb + PF) * 512);
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) {
              const bf16x8 fa = *(const bf16x8*)(sA + (rt * 32 + l31) * LDA + kb * 16 + 8 * hh);
              U[rt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw, fa, U[rt], 0, 0, 0);
            }
          }
        }
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
          for (int gg = 0; gg < 4; ++gg) {
            const int col = 32 * ct + 8 * gg + 4 * hh;
            const bf16x4 gv = *(const bf16x4*)(sG + (rt * 32 + l31) * LDA + col);
            *(bf16x4*)(sU + (rt * 32 + l31) * LDA + col) =
                bf16x4{(bf16)(U[rt][4 * gg] * (float)gv[0]), (bf16)(U[rt][4 * gg + 1] * (float)gv[1]),
                       (bf16)(U[rt][4 * gg + 2] * (float)gv[2]), (bf16)(U[rt][4 * gg + 3] * (float)gv[3])};
          }
      }
      __syncthreads();   // (2) dU half complete; GELU' half and the previous dxn no longer read
      if (!compute) {   // ---- [memory] dU half
        constexpr int CH = HH / 8;
        for (int i = sid; i < (KAIR_DBG(a.dbg & 4) ? 0 : TOK * CH); i += NST) {
          const int r = i / CH, q = (i - (i / CH) * CH) * 8;
          *(uint4*)(a.du + (row0 + r) * a.lddu + HH * half + q) = *(const uint4*)(sU + r * LDA + q);
        }
      } else {
        if (half == 0) {   // the second GELU' half into LDS
          constexpr int CH = HH / 8;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int i = tid + 64 * NC * k, r = i / CH, q = (i - (i / CH) * CH) * 8;
            *(uint4*)(sG + r * LDA + q) = g1[k];
          }
        }
        // dxn tile (columns 32 ct.., rows 32 rt..) += W1^T(half) . dU_half^T
        const bf16* wp = a.w1t + ((long)ct * (2 * KBH) + KBH * half) * 512 + lane * 8;
        bf16x8 pw[PF];
#pragma unroll
        for (int i = 0; i < PF; ++i) pw[i] = *(const bf16x8*)(wp + i * 512);
#pragma unroll 1
        for (int kb0 = 0; kb0 < (KAIR_DBG(a.dbg & 2) ? 0 : KBH); kb0 += PF) {
#pragma unroll
          for (int sl = 0; sl < PF; ++sl) {
            const int kb = kb0 + sl;
            const bf16x8 fw = pw[sl];
            if (kb + PF < KBH) pw[sl] = *(const bf16x8*)(wp + (kb + PF) * 512);
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) {
              const bf16x8 fu = *(const bf16x8*)(sU + (rt * 32 + l31) * LDA + kb * 16 + 8 * hh);
              DX[rt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw, fu, DX[rt], 0, 0, 0);
            }
          }
        }
      }
      __syncthreads();   // (3) dU half consumed (fc1 input gradient, stores); GELU' half 1 visible
    }
    if (compute) {
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg)
          *(float4*)(sY + (rt * 32 + l31) * LDY + 32 * ct + 8 * gg + 4 * hh) =
              make_float4(DX[rt][4 * gg], DX[rt][4 * gg + 1], DX[rt][4 * gg + 2], DX[rt][4 * gg + 3]);
    }
    __syncthreads();   // (4) dxn tile complete
    prev = tile;
  }
  if (!compute && prev >= 0 && !KAIR_DBG(a.dbg & 4)) ln_bwd(prev);
  // LN2 parameter-gradient partials: the 16 memory-wave row groups, summed in a fixed order
  __syncthreads();
  for (int i = tid; i < 2 * CP; i += NT) {
    const int which = i / CP, c = i - which * CP;
    float sum = 0.f;
#pragma unroll
    for (int q = 0; q < NG; ++q) sum += sPart[q][which][c];
    a.part[(long)blockIdx.x * 2 * CP + i] = sum;
  }
}

// dgamma / dbeta (+)= sum over workgroups of the partials, fixed order
__global__ __launch_bounds__(256) void mlp_bwd_param_reduce(const float* __restrict__ part, int nb, int C, int CPd,
                                                            float* dgamma, float* dbeta, int acc) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= 2 * C) return;
  const int which = i / C, c = i - which * C;
  float s = 0.f;
  for (int b = 0; b < nb; ++b) s += part[(long)b * 2 * CPd + which * CPd + c];
  float* o = which == 0 ? dgamma + c : dbeta + c;
  *o = acc ? *o + s : s;
}

}  // namespace

extern "C" int kair_swin_attn_fwd(const float* x, long ldx, const float* gamma, const float* beta, float eps, int C,
                                  void* ln, long ldln, float* mean, float* rstd, const void* wqkv, const float* bqkv,
                                  void* qkv, const float* table, float scale, void* O, long ldo, int o_ones_col,
                                  float* lse, const void* wproj, const float* bproj, const float* rowscale,
                                  int rows_per_scale, float* out, long ldout, long nWin, int nh, int H, int W, int shift,
                                  int w_split, void* stream) {
  KAIR_CHECK_ARG(x && gamma && beta && ln && mean && rstd && wqkv && bqkv && qkv && table && O && lse && wproj && bproj && out,
                 "swin_attn_fwd: null pointer");
  KAIR_CHECK_ARG(nh == 6 && C > 0 && C < 32 * nh && C % nh == 0 && C / nh <= 32,
                 "swin_attn_fwd: nh must be 6 with C < 32*nh (C %d, nh %d)", C, nh);
  KAIR_CHECK_ARG(H % WSZ == 0 && W % WSZ == 0 && (shift == 0 || (shift > 0 && shift < WSZ)), "swin_attn_fwd: geometry");
  KAIR_CHECK_ARG(nWin > 0 && nWin * TOK < KAIR_MAX_MAPPED_ROWS && (nWin * TOK) % ((long)H * W) == 0,
                 "swin_attn_fwd: nWin * 64 must be a whole number of H x W images, < 2^24");
  KAIR_CHECK_ARG(ldx >= 32 * nh && ldx % 4 == 0 && ldout >= 32 * nh && ldln >= 32 * nh && ldln % 4 == 0 && ldo >= 32 * nh &&
                     ldo % 4 == 0 && ((uintptr_t)x & 15) == 0,
                 "swin_attn_fwd: strides");
  KAIR_CHECK_ARG(!rowscale || (rows_per_scale > 0 && rows_per_scale % TOK == 0), "swin_attn_fwd: rows_per_scale");
  AttnFwdArgs a;
  a.x = x; a.ldx = ldx; a.gamma = gamma; a.beta = beta; a.eps = eps; a.C = C;
  a.ln = (bf16*)ln; a.ldln = ldln; a.mean = mean; a.rstd = rstd;
  a.wqkv = (const bf16*)wqkv; a.bqkv = bqkv; a.qkv = (bf16*)qkv;
  a.table = table; a.scale = scale;
  a.O = (bf16*)O; a.ldo = ldo; a.o_ones_col = o_ones_col; a.lse = lse;
  a.wproj = (const bf16*)wproj; a.bproj = bproj;
  a.rowscale = rowscale; a.win_per_scale = rowscale ? rows_per_scale / TOK : 1;
  a.out = out; a.ldout = ldout;
  a.nWin = nWin; a.H = H; a.W = W; a.shift = shift;
  a.wm = make_winmap(H, W, WSZ, shift);
  static const int dbg = kair_dbg_env("KAIR_ATTN_DBG");
  a.dbg = dbg;
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      ncu <= 0)
    ncu = 256;
  const long grid = nWin < ncu ? nWin : ncu;   // persistent: one workgroup per CU
  if (w_split)
    KAIR_LAUNCH((swin_attn_fwd_kernel<6, 2>), dim3((unsigned)grid), dim3(64 * 6), 0, (hipStream_t)stream, a);
  else if (KAIR_ATTN12)   // two waves per head (A/B: -DKAIR_ATTN12=0 builds the 6-wave kernel)
    KAIR_LAUNCH((swin_attn_fwd12_kernel<6>), dim3((unsigned)grid), dim3(128 * 6), 0, (hipStream_t)stream, a);
  else
    KAIR_LAUNCH((swin_attn_fwd_kernel<6, 1>), dim3((unsigned)grid), dim3(64 * 6), 0, (hipStream_t)stream, a);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_swin_mlp_fwd(const float* x, long ldx, const float* gamma, const float* beta, float eps, int C,
                                 void* ln, long ldln, float* mean, float* rstd, const void* w1, const float* b1, void* u,
                                 void* h, long ldh, int hd, const void* w2, const float* b2, const float* rowscale,
                                 int rows_per_scale, float* out, long ldout, long M, int Cp, int Hp, int w_split,
                                 void* stream) {
  KAIR_CHECK_ARG(x && gamma && beta && ln && mean && rstd && w1 && b1 && u && h && w2 && b2 && out,
                 "swin_mlp_fwd: null pointer");
  KAIR_CHECK_ARG(Cp == 192 && Hp == 384 && C > 0 && C < Cp && hd > 0 && hd < Hp,
                 "swin_mlp_fwd: laid out for Cp 192 / hidden 384 (C %d, Cp %d, hd %d, Hp %d)", C, Cp, hd, Hp);
  KAIR_CHECK_ARG(M > 0 && M % (w_split ? TOK : 32) == 0, "swin_mlp_fwd: M must be a multiple of %d", w_split ? TOK : 32);
  KAIR_CHECK_ARG(ldx >= Cp && ldx % 4 == 0 && ldout >= Cp && ldout % 4 == 0 && ldln >= Cp && ldln % 8 == 0 && ldh >= Hp &&
                     ldh % 8 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 15) == 0 && ((uintptr_t)b2 & 15) == 0,
                 "swin_mlp_fwd: strides / alignment");
  KAIR_CHECK_ARG(!rowscale || (rows_per_scale > 0 && rows_per_scale % (w_split ? TOK : 32) == 0), "swin_mlp_fwd: rows_per_scale");
  MlpFwdArgs a;
  a.x = x; a.ldx = ldx; a.gamma = gamma; a.beta = beta; a.eps = eps; a.C = C;
  a.ln = (bf16*)ln; a.ldln = ldln; a.mean = mean; a.rstd = rstd;
  a.w1 = (const bf16*)w1; a.b1 = b1; a.u = (bf16*)u; a.hact = (bf16*)h; a.ldh = ldh; a.hd = hd;
  a.w2 = (const bf16*)w2; a.b2 = b2;
  const int rt = w_split ? TOK : 32;   // rows per tile
  a.tiles_per_scale = rowscale ? rows_per_scale / rt : 1;
  a.ldout = ldout;
  static const int dbg = kair_dbg_env("KAIR_MLP_DBG");
  a.dbg = dbg;
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      ncu <= 0)
    ncu = 256;
  // The weight-resident kernel addresses x / out / ln / u / h through buffer resources with 32-bit byte offsets
  // (num_records 0x7fffffff): launch it over row ranges whose every stream stays below 2^31 bytes, each range
  // a whole number of tiles and of DropPath scale groups (the rowscale pointer advances with it).
  long row_bytes = ldx * 4;
  if (ldout * 4 > row_bytes) row_bytes = ldout * 4;
  if (ldln * 2 > row_bytes) row_bytes = ldln * 2;
  if (ldh * 2 > row_bytes) row_bytes = ldh * 2;
  const long unit = rowscale ? (long)rows_per_scale : (long)rt;
  const long chunk = ((0x7fffffffL / row_bytes) / unit) * unit;
  KAIR_CHECK_ARG(chunk > 0, "swin_mlp_fwd: a DropPath scale group exceeds the 2 GiB range of one launch");
  for (long r0 = 0; r0 < M; r0 += chunk) {
    const long rows = M - r0 < chunk ? M - r0 : chunk;
    a.x = x + r0 * ldx; a.out = out + r0 * ldout;
    a.ln = (bf16*)ln + r0 * ldln; a.mean = mean + r0; a.rstd = rstd + r0;
    a.u = (bf16*)u + r0 * ldh; a.hact = (bf16*)h + r0 * ldh;
    a.rowscale = rowscale ? rowscale + r0 / rows_per_scale : nullptr;
    a.nTiles = rows / rt;
    const long grid = a.nTiles < ncu ? a.nTiles : ncu;   // persistent: one workgroup per CU
    if (w_split)
      KAIR_LAUNCH(swin_mlp_fwd_kernel<2>, dim3((unsigned)grid), dim3(1024), 0, (hipStream_t)stream, a);
    else
      KAIR_LAUNCH(swin_mlp_fwd_wr_kernel, dim3((unsigned)grid), dim3(768), 0, (hipStream_t)stream, a);
    KAIR_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" long kair_swin_mlp_bwd_ws(void) {
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      ncu <= 0)
    ncu = 256;
  return (long)ncu * 2 * 192;
}

extern "C" int kair_swin_mlp_bwd(const void* dc, long lddc, const void* gd, long ldg, const void* w2t, const void* w1t,
                                 void* du, long lddu, const float* x, long ldx, const float* gamma, const float* mean,
                                 const float* rstd, int C, float* D, long ldD, void* dco, long lddo, const float* rowscale,
                                 int rows_per_scale, int H, int W, int shift, float* dgamma, float* dbeta, int dparam_acc,
                                 float* ws, long M, int Cp, int Hp, void* stream) {
  KAIR_CHECK_ARG(dc && gd && w2t && w1t && du && x && gamma && mean && rstd && D && dco && dgamma && dbeta && ws,
                 "swin_mlp_bwd: null pointer");
  KAIR_CHECK_ARG(Cp == 192 && Hp == 384 && C > 0 && C < Cp, "swin_mlp_bwd: laid out for Cp 192 / hidden 384");
  KAIR_CHECK_ARG(M > 0 && M % TOK == 0 && M < KAIR_MAX_MAPPED_ROWS, "swin_mlp_bwd: M must be a multiple of 64");
  KAIR_CHECK_ARG(H % WSZ == 0 && W % WSZ == 0 && shift >= 0 && shift < WSZ && M % ((long)H * W) == 0, "swin_mlp_bwd: geometry");
  KAIR_CHECK_ARG(lddc >= Cp && lddc % 8 == 0 && ldg >= Hp && ldg % 8 == 0 && lddu >= Hp && lddu % 8 == 0 && ldx >= Cp &&
                     ldx % 4 == 0 && ldD >= Cp && ldD % 4 == 0 && lddo >= Cp && lddo % 8 == 0,
                 "swin_mlp_bwd: strides");
  KAIR_CHECK_ARG(dco != dc, "swin_mlp_bwd: dco must not alias dc (rows are read and written by different tiles)");
  KAIR_CHECK_ARG(!rowscale || (rows_per_scale > 0 && rows_per_scale % TOK == 0), "swin_mlp_bwd: rows_per_scale");
  MlpBwdArgs a;
  a.dc = (const bf16*)dc; a.lddc = lddc; a.gd = (const bf16*)gd; a.ldg = ldg;
  a.w2t = (const bf16*)w2t; a.w1t = (const bf16*)w1t; a.du = (bf16*)du; a.lddu = lddu;
  a.x = x; a.ldx = ldx; a.gamma = gamma; a.mean = mean; a.rstd = rstd; a.C = C;
  a.D = D; a.ldD = ldD; a.dco = (bf16*)dco; a.lddo = lddo;
  a.rowscale = rowscale; a.tiles_per_scale = rowscale ? rows_per_scale / TOK : 1;
  a.wm = make_winmap(H, W, WSZ, shift);
  a.part = ws;
  a.nTiles = M / TOK;
  static const int dbg = kair_dbg_env("KAIR_MLPB_DBG");
  a.dbg = dbg;
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      ncu <= 0)
    ncu = 256;
  const long grid = a.nTiles < ncu ? a.nTiles : ncu;
  KAIR_LAUNCH(swin_mlp_bwd_kernel, dim3((unsigned)grid), dim3(512), 0, (hipStream_t)stream, a);
  KAIR_CHECK_LAUNCH();
  KAIR_LAUNCH(mlp_bwd_param_reduce, dim3((unsigned)((2 * C + 255) / 256)), dim3(256), 0, (hipStream_t)stream, ws,
                     (int)grid, C, 192, dgamma, dbeta, dparam_acc);
  KAIR_CHECK_LAUNCH();
  return 0;
}

// copy the fused-attention phase stamps to the host (perf investigation only; zeros in release builds)
extern "C" int kair_debug_fused_stamps(unsigned long long* host, int n) {
  KAIR_CHECK_ARG(host && n > 0 && n <= FST_WAVES * FST_N, "debug_fused_stamps: bad args");
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fused_stamps), sizeof(unsigned long long) * n, 0, hipMemcpyDeviceToHost) !=
      hipSuccess)
    return kair_set_error(KAIR_ERR_HIP, "debug_fused_stamps: copy failed");
  void* dev = nullptr;   // cleared after the read, so the next read holds only the next launch's windows
  if (hipGetSymbolAddress(&dev, HIP_SYMBOL(g_fused_stamps)) != hipSuccess ||
      hipMemset(dev, 0, sizeof(unsigned long long) * FST_WAVES * FST_N) != hipSuccess)
    return kair_set_error(KAIR_ERR_HIP, "debug_fused_stamps: clear failed");
  return 0;
}
