// Fused Swin window attention for gfx950 (network_swinir.py:114-145, WindowAttention.forward):
//   S = (q*scale) k^T + table[relative_position_index] (+ shifted-window region mask, -100)
//   P = softmax(S) ; O = P v          per (window, head), window 8x8 = 64 tokens, head_dim <= 32
// and its backward (dq, dk, dv, d table), flash-style: P is recomputed from q, k and the saved
// row log-sum-exp, nothing of size 64x64 per (window, head) touches HBM.
//
// One wave64 owns one (window, head) tile at a time; q/k/v (4 KB each in bf16) are staged
// global -> LDS with 16-byte coalesced loads.  bf16 mode uses v_mfma_f32_32x32x16_bf16, the
// accumulator of the first product feeds the second directly as an MFMA operand (k order permuted
// in-register, the other operand fetched with ds_read_b64_tr_b16 in the matching order).  fp32
// (parity) mode uses v_mfma_f32_32x32x2_f32 with the same dataflow.  The relative position bias
// and the shift mask are computed from indices (no 64x64 tables are read).
#include <stdlib.h>

#include <string.h>

#include "attn_common.h"

namespace {

template <bool BF> constexpr int NWAVES = BF ? 4 : 2;  // fp32 tiles need twice the LDS

template <bool BF> struct AT {
  using T = typename std::conditional<BF, bf16, float>::type;
  static constexpr int LD = BF ? 40 : 33;  // LDS row stride (elements) of a [64][32] tile
};

// stage a [64][32] tile (element type T in global, contiguous rows of `ld` elements starting at
// column c0) into LDS with row stride LD
template <bool BF>
KAIR_DEV void stage_tile(typename AT<BF>::T* lds, const typename AT<BF>::T* g, long ld, int lane) {
  using T = typename AT<BF>::T;
  constexpr int LD = AT<BF>::LD;
  constexpr int EPC = 16 / sizeof(T);              // elements per 16-byte chunk
  constexpr int CPR = HDP / EPC;                   // chunks per row
#pragma unroll
  for (int i = 0; i < TOK * CPR / 64; ++i) {
    const int c = lane + 64 * i;
    const int row = c / CPR, col = (c % CPR) * EPC;
    if constexpr (BF) {
      *(bf16x8*)(lds + row * LD + col) = *(const bf16x8*)(g + row * ld + col);
    } else {
      const float4 v = *(const float4*)(g + row * ld + col);
      float* d = (float*)lds + row * LD + col;
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
  }
}


// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
template <bool BF>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const typename AT<BF>::T* __restrict__ qkv,
                                                       const float* __restrict__ table, typename AT<BF>::T* __restrict__ O,
                                                       long ldo, float* __restrict__ lse, long nWin, int nh, float scale,
                                                       int H, int W, int shift, int ones_col,
                                                       const float* __restrict__ amask, int mask_nw) {
  using T = typename AT<BF>::T;
  constexpr int LD = AT<BF>::LD;
  constexpr int WAVES = NWAVES<BF>;
  __shared__ __attribute__((aligned(16))) T sQ[WAVES][TOK * LD];
  __shared__ __attribute__((aligned(16))) T sK[WAVES][TOK * LD];
  __shared__ __attribute__((aligned(16))) T sV[WAVES][TOK * LD];
  __shared__ float sTab[WAVES][232];
  __shared__ int sReg[WAVES][TOK];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long task = (long)blockIdx.x * WAVES + w;
  if (task >= nWin * nh) return;
  const long win = task / nh;
  const int h = (int)(task - win * nh);
  const long M = nWin * TOK;
  const long blk = (win * nh + h) * TOK * HDP;
  const long part = M * nh * HDP;
  T* q = sQ[w]; T* k = sK[w]; T* v = sV[w];
  stage_tile<BF>(q, qkv + blk, HDP, lane);
  stage_tile<BF>(k, qkv + part + blk, HDP, lane);
  stage_tile<BF>(v, qkv + 2 * part + blk, HDP, lane);
  for (int i = lane; i < (2 * WS - 1) * (2 * WS - 1); i += 64) sTab[w][i] = table[i * nh + h];
  const int nW = (H / WS) * (W / WS);
  const int wi = (int)(win % nW);
  sReg[w][lane] = shift > 0 ? token_region(wi, lane, H, W, shift) : 0;
  wave_sync();

  // S^T = K Q^T : tiles [kt][qt], lane column = query, registers = keys
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const int l31 = lane & 31, hh = lane >> 5;
  if constexpr (BF) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 fk[2], fq[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        fk[t] = frag_cols(k, LD, t * 32 + l31, s, lane);
        fq[t] = frag_cols(q, LD, t * 32 + l31, s, lane);
      }
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
          acc[kt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fk[kt], fq[qt], acc[kt][qt], 0, 0, 0);
    }
  } else {
#pragma unroll 4
    for (int s = 0; s < HDP / 2; ++s) {
      float fk[2], fq[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        fk[t] = k[(t * 32 + l31) * LD + 2 * s + hh];
        fq[t] = q[(t * 32 + l31) * LD + 2 * s + hh];
      }
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
          acc[kt][qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(fk[kt], fq[qt], acc[kt][qt], 0, 0, 0);
    }
  }
  // scores: scale, bias, mask ; softmax over keys (registers + lane^32)
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qi = qt * 32 + l31;
    const int rq = sReg[w][qi];
    float mx = -3.0e38f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ki = kt * 32 + acc_row(r, hh);
        float sc = acc[kt][qt][r] * scale + sTab[w][relidx(qi, ki)];
        if (shift > 0 && sReg[w][ki] != rq) sc += -100.f;
        if (amask) sc += amask[((win % mask_nw) * TOK + qi) * TOK + ki];
        acc[kt][qt][r] = sc;
        mx = fmaxf(mx, sc);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __expf(acc[kt][qt][r] - mx);
        acc[kt][qt][r] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 32, 64);
    const float inv = 1.f / sum;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[kt][qt][r] *= inv;
    if (hh == 0) lse[task * TOK + qi] = mx + __logf(sum);
  }
  // O = P V : out tile [qt] rows = query, columns = d (lane)
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    f32x16 o;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] = 0.f;
    if constexpr (BF) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pack8(acc[kt][qt], s), frag_rows_perm(v, kt * 32, s, lane), o, 0, 0, 0);
    } else {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int s = 0; s < 16; ++s)
          o = __builtin_amdgcn_mfma_f32_32x32x2f32(acc[kt][qt][s], v[(kt * 32 + acc_row(s, hh)) * LD + l31], o, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qi = qt * 32 + acc_row(r, hh);
      O[(win * TOK + qi) * ldo + h * HDP + l31] = (T)(h * HDP + l31 == ones_col ? 1.f : o[r]);
    }
  }
}

// ------------------------------------------------------------------------------------------
// bf16 forward: q / k fragments straight from global into registers (the frag_cols layout the
// S^T = K Q^T product consumes), only v staged in LDS (for the transposed P.V fragments), so a
// wave needs 6 KiB of LDS and 8 waves fit a CU; O is produced transposed (O^T = V^T P^T: lane =
// query, 4 consecutive d per register group) and stored 8 bytes at a time.
// Each wave runs `tpw` consecutive (window, head) tasks and loads the next task's q / k / v fragments and
// bias-table column while the current one computes (2 waves per SIMD: one task per wave left every load's
// latency exposed -- 1.75 TB/s at SwinIR-lightweight's shapes).
// HP: the head pad of the q / k / v / O layout -- 32, or 16 for head dims below 16 (SwinIR-lightweight's 10,
// network_swinir.py:85 with embed_dim 60 / 6 heads): one K = 16 step for S, half the HBM bytes per head; the
// P.V product keeps its 32-row MFMA tile (rows d >= 16 read zeroed LDS columns and are not stored).
// ------------------------------------------------------------------------------------------
template <int HP>
__global__ __launch_bounds__(256, 2) void attn_fwd_bf16_kernel(const bf16* __restrict__ qkv, const float* __restrict__ table,
                                                            bf16* __restrict__ O, long ldo, float* __restrict__ lse,
                                                            long nWin, int nh, float scale, int H, int W, int shift,
                                                            int ones_col, const float* __restrict__ amask, int mask_nw,
                                                            int tpw) {
  constexpr int LD = AT<true>::LD, NW = 4, NS = HP / 16, NT = ((2 * WS - 1) * (2 * WS - 1) + 63) / 64;
  static_assert(HP == 16 || HP == 32, "head pad");
  __shared__ __attribute__((aligned(16))) bf16 sV[NW][TOK * LD];
  __shared__ float sTab[NW][NT * 64];
  __shared__ int sReg[NW][TOK];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long ntask = nWin * nh;
  const long task0 = ((long)blockIdx.x * NW + w) * tpw;
  if (task0 >= ntask) return;
  const long task1 = task0 + tpw < ntask ? task0 + tpw : ntask;
  const long M = nWin * TOK;
  const long part = M * nh * HP;
  const int l31 = lane & 31, hh = lane >> 5;
  const int nW = (H / WS) * (W / WS);
  bf16x8 Fq[2][NS], Fk[2][NS], Fv[2][NS];
  float Ft[NT];
  auto load_task = [&](long task) {
    const long win = task / nh;
    const int h = (int)(task - win * nh);
    const long blk = (win * nh + h) * TOK * HP;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const long o = (long)(t * 32 + l31) * HP + 16 * s + 8 * hh;
        Fq[t][s] = *(const bf16x8*)(qkv + blk + o);
        Fk[t][s] = *(const bf16x8*)(qkv + part + blk + o);
        Fv[t][s] = *(const bf16x8*)(qkv + 2 * part + blk + o);
      }
#pragma unroll
    for (int i = 0; i < NT; ++i) {   // clamped index: unconditional loads (no branch, no extra wait)
      const int ti = lane + 64 * i < (2 * WS - 1) * (2 * WS - 1) ? lane + 64 * i : 0;
      Ft[i] = table[ti * nh + h];
    }
  };
  load_task(task0);
  bf16* v = sV[w];
  for (long task = task0; task < task1; ++task) {
    const long win = task / nh;
    const int h = (int)(task - win * nh);
    wave_sync();   // the previous task's LDS reads are complete
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 z = {};
        *(bf16x8*)(v + (t * 32 + l31) * LD + 16 * s + 8 * hh) = s < NS ? Fv[t][s < NS ? s : 0] : z;
      }
#pragma unroll
    for (int i = 0; i < NT; ++i) sTab[w][lane + 64 * i] = Ft[i];
    sReg[w][lane] = shift > 0 ? token_region((int)(win % nW), lane, H, W, shift) : 0;

    // S^T = K Q^T : tiles [kt][qt], lane column = query, registers = keys
    f32x16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
          acc[kt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Fk[kt][s], Fq[qt][s], acc[kt][qt], 0, 0, 0);
    // the next task's fragments load under this task's softmax, P.V and stores (the last task reloads itself,
    // so every path reaches the loop back-edge with the same loads pending)
    load_task(task + 1 < task1 ? task + 1 : task);
    wave_sync();
    // scores: scale, bias, mask ; softmax over keys (registers + lane^32)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int qi = qt * 32 + l31;
      const int rq = sReg[w][qi];
      float mx = -3.0e38f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ki = kt * 32 + acc_row(r, hh);
          float sc = acc[kt][qt][r] * scale + sTab[w][relidx(qi, ki)];
          if (shift > 0 && sReg[w][ki] != rq) sc += -100.f;
          if (amask) sc += amask[((win % mask_nw) * TOK + qi) * TOK + ki];
          acc[kt][qt][r] = sc;
          mx = fmaxf(mx, sc);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      float sum = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = __expf(acc[kt][qt][r] - mx);
          acc[kt][qt][r] = e;
          sum += e;
        }
      sum += __shfl_xor(sum, 32, 64);
      const float inv = 1.f / sum;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[kt][qt][r] *= inv;
      if (hh == 0) lse[task * TOK + qi] = mx + __logf(sum);
    }
    // O^T = V^T P^T : tile [qt] rows = d, lane = query
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      f32x16 o;
#pragma unroll
      for (int r = 0; r < 16; ++r) o[r] = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_rows_perm(v, kt * 32, s, lane), pack8(acc[kt][qt], s), o, 0, 0, 0);
      const int qi = qt * 32 + l31;
      bf16* orow = O + (win * TOK + qi) * ldo + h * HP;
#pragma unroll
      for (int g = 0; g < HP / 8; ++g) {
        const int d0 = 8 * g + 4 * hh;
        float r4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) r4[j] = (h * HP + d0 + j == ones_col) ? 1.f : o[4 * g + j];
        const bf16x4 q4 = {(bf16)r4[0], (bf16)r4[1], (bf16)r4[2], (bf16)r4[3]};
        *(bf16x4*)(orow + d0) = q4;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// backward: one wave per (head, group of windows); dS summed over the group in registers for the
// relative-position-bias gradient
// ------------------------------------------------------------------------------------------
template <bool BF>
__global__ __launch_bounds__(256) void attn_bwd_kernel(const typename AT<BF>::T* __restrict__ qkv,
                                                       const typename AT<BF>::T* __restrict__ O, long ldo,
                                                       const typename AT<BF>::T* __restrict__ dO, long lddo,
                                                       const float* __restrict__ table, const float* __restrict__ lse,
                                                       typename AT<BF>::T* __restrict__ dqkv, float* __restrict__ dB_part,
                                                       long nWin, int nh, int wpg, float scale, int H, int W, int shift,
                                                       const float* __restrict__ amask, int mask_nw) {
  using T = typename AT<BF>::T;
  constexpr int LD = AT<BF>::LD;
  constexpr int WAVES = NWAVES<BF>;
  constexpr int LDS_ = 72;  // dS tile row stride (bf16: 144 B; fp32 reads use 65)
  __shared__ __attribute__((aligned(16))) T sQ[WAVES][TOK * LD];
  __shared__ __attribute__((aligned(16))) T sK[WAVES][TOK * LD];
  __shared__ __attribute__((aligned(16))) T sV[WAVES][TOK * LD];
  __shared__ __attribute__((aligned(16))) T sdO[WAVES][TOK * LD];
  __shared__ __attribute__((aligned(16))) T sdS[WAVES][TOK * (BF ? LDS_ : 65)];
  __shared__ float sTab[WAVES][232];
  __shared__ float sRow[WAVES][2][TOK];  // lse, delta
  __shared__ int sReg[WAVES][TOK];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long gtask = (long)blockIdx.x * WAVES + w;
  const long ngroups = (nWin + wpg - 1) / wpg;
  if (gtask >= ngroups * nh) return;
  const int h = (int)(gtask % nh);
  const long grp = gtask / nh;
  const long M = nWin * TOK;
  const long part = M * nh * HDP;
  const int l31 = lane & 31, hh = lane >> 5;
  T* q = sQ[w]; T* k = sK[w]; T* v = sV[w]; T* go = sdO[w]; T* ds = sdS[w];
  for (int i = lane; i < (2 * WS - 1) * (2 * WS - 1); i += 64) sTab[w][i] = table[i * nh + h];
  const int nW = (H / WS) * (W / WS);

  // dS accumulator for the bias gradient: S-layout tiles [qt][kt], lane = key, regs = query
  f32x16 dB[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) dB[a][b][r] = 0.f;

  const long w0 = grp * wpg;
  long w1 = w0 + wpg;
  if (w1 > nWin) w1 = nWin;
  for (long win = w0; win < w1; ++win) {
    const long blk = (win * nh + h) * TOK * HDP;
    wave_sync();
    stage_tile<BF>(q, qkv + blk, HDP, lane);
    stage_tile<BF>(k, qkv + part + blk, HDP, lane);
    stage_tile<BF>(v, qkv + 2 * part + blk, HDP, lane);
    stage_tile<BF>(go, dO + win * TOK * lddo + h * HDP, lddo, lane);
    {
      // delta[q] = sum_d dO[q][d] * O[q][d]  (lane = query)
      const T* orow = O + (win * TOK + lane) * ldo + h * HDP;
      const T* grow = dO + (win * TOK + lane) * lddo + h * HDP;
      float d = 0.f;
#pragma unroll
      for (int c = 0; c < HDP; ++c) d += (float)orow[c] * (float)grow[c];
      sRow[w][1][lane] = d;
      sRow[w][0][lane] = lse[((long)win * nh + h) * TOK + lane];
      sReg[w][lane] = shift > 0 ? token_region((int)(win % nW), lane, H, W, shift) : 0;
    }
    wave_sync();

    // S = Q K^T and dP = dO V^T : tiles [qt][kt], lane = key, regs = query
    f32x16 S[2][2], dP[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) { S[a][b][r] = 0.f; dP[a][b][r] = 0.f; }
    if constexpr (BF) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 fq[2], fk[2], fg[2], fv[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          fq[t] = frag_cols(q, LD, t * 32 + l31, s, lane);
          fk[t] = frag_cols(k, LD, t * 32 + l31, s, lane);
          fg[t] = frag_cols(go, LD, t * 32 + l31, s, lane);
          fv[t] = frag_cols(v, LD, t * 32 + l31, s, lane);
        }
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            S[qt][kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fq[qt], fk[kt], S[qt][kt], 0, 0, 0);
            dP[qt][kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fg[qt], fv[kt], dP[qt][kt], 0, 0, 0);
          }
      }
    } else {
#pragma unroll 4
      for (int s = 0; s < HDP / 2; ++s) {
        float fq[2], fk[2], fg[2], fv[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          fq[t] = q[(t * 32 + l31) * LD + 2 * s + hh];
          fk[t] = k[(t * 32 + l31) * LD + 2 * s + hh];
          fg[t] = go[(t * 32 + l31) * LD + 2 * s + hh];
          fv[t] = v[(t * 32 + l31) * LD + 2 * s + hh];
        }
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            S[qt][kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(fq[qt], fk[kt], S[qt][kt], 0, 0, 0);
            dP[qt][kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(fg[qt], fv[kt], dP[qt][kt], 0, 0, 0);
          }
      }
    }
    // P = exp(S*scale + bias + mask - lse) ; dS = P (dP - delta).  Lane = key ki, register r of
    // tile qt = query qi = 32 qt + 8 (r/4) + r%4 + 4 hh, so every per-element LDS operand sits at a
    // compile-time offset from a per-lane base: relidx(qi, ki) = 15 (4 qt + r/4) + r%4 + [15 (7 - ky)
    // + 7 - kx + 4 hh]; lse / delta / region of qi at [32 qt + 8 (r/4) + r%4] + 4 hh.  The reads
    // issue back to back instead of one dependent address computation each.
    const int wi_img = (int)(win % nW), nWw = W / WS;
    const bool mixed = shift > 0 && ((wi_img / nWw) == H / WS - 1 || (wi_img % nWw) == nWw - 1);
    const float* rl = &sRow[w][0][4 * hh];
    const float* rd = &sRow[w][1][4 * hh];
    const int* rg = &sReg[w][4 * hh];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int ki = kt * 32 + l31;
      const int rk = sReg[w][ki];
      const float* tb = &sTab[w][15 * (WS - 1 - (ki >> 3)) + (WS - 1 - (ki & 7)) + 4 * hh];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int o = 32 * qt + 8 * (r >> 2) + (r & 3);
          float sc = S[qt][kt][r] * scale + tb[15 * (4 * qt + (r >> 2)) + (r & 3)];
          if (mixed && rg[o] != rk) sc += -100.f;
          if (amask) sc += amask[((win % mask_nw) * TOK + qt * 32 + acc_row(r, hh)) * TOK + ki];
          const float p = __expf(sc - rl[o]);
          S[qt][kt][r] = p;
          const float d = p * (dP[qt][kt][r] - rd[o]);
          dP[qt][kt][r] = d;
          dB[qt][kt][r] += d;
        }
    }
    // dV = P^T dO and dK = scale * dS^T Q : tiles [kt], rows = key, lane = d
    T* dq_out = dqkv + blk;
    T* dk_out = dqkv + part + blk;
    T* dv_out = dqkv + 2 * part + blk;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      f32x16 av, ak;
#pragma unroll
      for (int r = 0; r < 16; ++r) { av[r] = 0.f; ak[r] = 0.f; }
      if constexpr (BF) {
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            av = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pack8(S[qt][kt], s), frag_rows_perm(go, qt * 32, s, lane), av, 0, 0, 0);
            ak = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pack8(dP[qt][kt], s), frag_rows_perm(q, qt * 32, s, lane), ak, 0, 0, 0);
          }
      } else {
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int s = 0; s < 16; ++s) {
            const int qr = (qt * 32 + acc_row(s, hh)) * LD + l31;
            av = __builtin_amdgcn_mfma_f32_32x32x2f32(S[qt][kt][s], go[qr], av, 0, 0, 0);
            ak = __builtin_amdgcn_mfma_f32_32x32x2f32(dP[qt][kt][s], q[qr], ak, 0, 0, 0);
          }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ki = kt * 32 + acc_row(r, hh);
        dv_out[ki * HDP + l31] = (T)av[r];
        dk_out[ki * HDP + l31] = (T)(ak[r] * scale);
      }
    }
    // dQ = scale * dS K : dS through LDS ([q][key] row-major)
    constexpr int LDD = BF ? LDS_ : 65;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) ds[(qt * 32 + acc_row(r, hh)) * LDD + kt * 32 + l31] = (T)dP[qt][kt][r];
    wave_sync();
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      f32x16 aq;
#pragma unroll
      for (int r = 0; r < 16; ++r) aq[r] = 0.f;
      if constexpr (BF) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
          aq = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_cols(ds, LDD, qt * 32 + l31, s, lane),
                                                      frag_rows_nat(k, 0, s, lane), aq, 0, 0, 0);
      } else {
#pragma unroll 8
        for (int s = 0; s < 32; ++s)
          aq = __builtin_amdgcn_mfma_f32_32x32x2f32(ds[(qt * 32 + l31) * LDD + 2 * s + hh], k[(2 * s + hh) * LD + l31], aq,
                                                   0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) dq_out[(qt * 32 + acc_row(r, hh)) * HDP + l31] = (T)(aq[r] * scale);
    }
  }
  // partial bias gradient of this (group, head): [q][key] through the wave's (free) dS tile, binned
  wave_sync();
  float* dbt = (float*)sdS[w];   // fp32: [64][65]; bf16: [64][72] bf16 = [64][36] floats -- too small
  static_assert(!BF, "the binned bias gradient needs the fp32 dS tile (the bf16 mode uses attn_bwd_bf16_kernel)");
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) dbt[(qt * 32 + acc_row(r, hh)) * 65 + kt * 32 + l31] = dB[qt][kt][r];
  wave_sync();
  bin_dbias<false>(dbt, 65, (float*)sQ[w], dB_part + (grp * nh + h) * NBIN, lane);
}

// perf-investigation phase stamps (KAIR_ATTN_STAMP=1, read with kair_debug_attn_stamps): per wave,
// s_memtime at the phase boundaries of its third window
constexpr int STAMP_WAVES = 8192, STAMP_N = 8;
__device__ unsigned long long g_attn_stamps[STAMP_WAVES * STAMP_N];
KAIR_DEV unsigned long long stamp_now() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// ------------------------------------------------------------------------------------------
// bf16 backward, software-pipelined.  Per wave: one head, a group of windows.  The q/k/v/dO/O
// fragments of the NEXT window are loaded into registers (16-byte loads, the frag_cols layout the
// S / dP products consume directly) while the current window is computed; q, k and dO are also
// written to LDS for the transposed fragment reads of dV, dK and dQ.  delta = rowsum(dO o O)
// comes from the register fragments (lane half + partner lane).  dV, dK and dQ are produced
// transposed (D[d][token]: lane = token, 4 consecutive d per register group), so each lane
// stores 8 bytes at a time instead of 2.
// ------------------------------------------------------------------------------------------
template <int NW, int HP>
__global__ __launch_bounds__(64 * NW) void attn_bwd_bf16_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ O,
                                                            long ldo, const bf16* __restrict__ dO, long lddo,
                                                            const float* __restrict__ table, const float* __restrict__ lse,
                                                            bf16* __restrict__ dqkv, float* __restrict__ dB_part,
                                                            long nWin, int nh, int wpg, float scale, int H, int W,
                                                            int shift, const float* __restrict__ amask, int mask_nw,
                                                            int stamp, int rows) {
  constexpr int LD = AT<true>::LD, LDD = 72, LDB = 72, NS = HP / 16;
  static_assert(HP == 16 || HP == 32, "head pad");
  static_assert(TOK * LDD <= 2 * TOK * LD, "the dS tile reuses the q / dO tiles");
  // per wave: q and dO tiles (after dV / dK they hold the dS tile), k tile, and the running bias
  // gradient [q][key] in fp32 (row stride 72: the two lane halves' rows 4 apart fall in opposite
  // bank halves) -- in LDS rather than 64 accumulator registers the kernel does not have
  __shared__ __attribute__((aligned(16))) bf16 sQG[NW][2 * TOK * LD];
  __shared__ __attribute__((aligned(16))) bf16 sK[NW][TOK * LD];
  __shared__ __attribute__((aligned(16))) float sDB[NW][TOK * LDB];
  __shared__ float sTab[NW][232];
  __shared__ float sRow[NW][2][TOK];  // lse, delta
  __shared__ int sReg[NW][TOK];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long gtask = (long)blockIdx.x * NW + w;
  const long ngroups = (nWin + wpg - 1) / wpg;
  if (gtask >= ngroups * nh) return;
  const int h = (int)(gtask % nh);
  const long grp = gtask / nh;
  const long M = nWin * TOK;
  const long part = M * nh * HP;
  const int l31 = lane & 31, hh = lane >> 5;
  bf16* q = sQG[w]; bf16* go = sQG[w] + TOK * LD; bf16* k = sK[w]; bf16* ds = sQG[w];
  float* db = sDB[w];
  for (int i = lane; i < (2 * WS - 1) * (2 * WS - 1); i += 64) sTab[w][i] = table[i * nh + h];
  for (int i = lane; i < TOK * LDB / 4; i += 64) ((float4*)db)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  const int nW = (H / WS) * (W / WS);

  // register fragments of one window: rows t*32 + l31, columns 16 s + 8 hh.  HP = 16: the q / k / dO LDS tiles'
  // columns 16..31 feed only the transposed products' rows d >= 16, which are not stored; zeroed once so those
  // rows start from defined values (later windows leave the finite dS tile there)
  if constexpr (HP == 16) {
    const bf16x8 z = {};
    for (int i = lane; i < 3 * TOK * 2; i += 64) {
      const int r = i >> 1;
      bf16* t = r < 2 * TOK ? sQG[w] + r * LD : sK[w] + (r - 2 * TOK) * LD;
      *(bf16x8*)(t + 16 + 8 * (i & 1)) = z;
    }
  }
  bf16x8 Fq[2][NS], Fk[2][NS], Fv[2][NS], Fg[2][NS], Fo[2][NS];
  float Fl[2];
  auto ldfrag = [&](const bf16* g, long ld, bf16x8 (&f)[2][NS]) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < NS; ++s) f[t][s] = *(const bf16x8*)(g + (long)(t * 32 + l31) * ld + 16 * s + 8 * hh);
  };
  auto load_win = [&](long win) {
    const long blk = (win * nh + h) * TOK * HP;
    ldfrag(qkv + blk, HP, Fq);
    ldfrag(qkv + part + blk, HP, Fk);
    ldfrag(qkv + 2 * part + blk, HP, Fv);
    ldfrag(dO + win * TOK * lddo + h * HP, lddo, Fg);
    ldfrag(O + win * TOK * ldo + h * HP, ldo, Fo);
#pragma unroll
    for (int t = 0; t < 2; ++t) Fl[t] = lse[(win * nh + h) * TOK + t * 32 + l31];
  };

  const long w0 = grp * wpg;
  long w1 = w0 + wpg;
  if (w1 > nWin) w1 = nWin;
  load_win(w0);
  unsigned long long ts[STAMP_N];
  const bool stamping = KAIR_DBG(stamp) && gtask < STAMP_WAVES;
  for (long win = w0; win < w1; ++win) {
    const bool st_on = stamping && win == w0 + 2;
    if (st_on) ts[0] = stamp_now();
    const long blk = (win * nh + h) * TOK * HP;
    wave_sync();   // the previous window's LDS tiles are no longer read
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const int o = (t * 32 + l31) * LD + 16 * s + 8 * hh;
        *(bf16x8*)(q + o) = Fq[t][s];
        *(bf16x8*)(k + o) = Fk[t][s];
        *(bf16x8*)(go + o) = Fg[t][s];
      }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float d = 0.f;
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) d += (float)Fg[t][s][j] * (float)Fo[t][s][j];
      d += __shfl_xor(d, 32, 64);
      if (hh == 0) {
        sRow[w][0][t * 32 + l31] = Fl[t];
        sRow[w][1][t * 32 + l31] = d;
      }
    }
    sReg[w][lane] = shift > 0 ? token_region((int)(win % nW), lane, H, W, shift) : 0;
    if (st_on) ts[1] = stamp_now();

    // S = Q K^T and dP = dO V^T : tiles [qt][kt], lane = key, regs = query
    f32x16 S[2][2], dP[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) { S[a][b][r] = 0.f; dP[a][b][r] = 0.f; }
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          S[qt][kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Fq[qt][s], Fk[kt][s], S[qt][kt], 0, 0, 0);
          dP[qt][kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Fg[qt][s], Fv[kt][s], dP[qt][kt], 0, 0, 0);
        }
    // the next window's fragments load under the rest of this window's work (unconditionally --
    // the last window reloads itself -- so every path reaches the loop back-edge with the same
    // loads pending and hipcc can wait for exactly them instead of draining the window's stores)
    load_win(win + 1 < w1 ? win + 1 : win);
    wave_sync();
    if (st_on) ts[2] = stamp_now();

    // P = exp(S*scale + bias + mask - lse) ; dS = P (dP - delta).  Lane = key ki, register r of
    // tile qt = query qi = 32 qt + 8 (r/4) + r%4 + 4 hh, so every per-element LDS operand sits at a
    // compile-time offset from a per-lane base: relidx(qi, ki) = 15 (4 qt + r/4) + r%4 + [15 (7 - ky)
    // + 7 - kx + 4 hh]; lse / delta / region of qi at [32 qt + 8 (r/4) + r%4] + 4 hh.  The reads
    // issue back to back instead of one dependent address computation each.
    const int wi_img = (int)(win % nW), nWw = W / WS;
    const bool mixed = shift > 0 && ((wi_img / nWw) == H / WS - 1 || (wi_img % nWw) == nWw - 1);
    const float* rl = &sRow[w][0][4 * hh];
    const float* rd = &sRow[w][1][4 * hh];
    const int* rg = &sReg[w][4 * hh];
    float* dbl = db + 4 * hh * LDB + l31;
    // Per 16-element block: every LDS read first, then the math, then the dB writes -- no branch
    // and no possibly-aliasing store between the reads, so they issue back to back (one wave per
    // SIMD: an LDS round trip per element would be the whole cost of this phase).
    const bool plain = !mixed && !amask;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int ki = kt * 32 + l31;
      const float* tb = &sTab[w][15 * (WS - 1 - (ki >> 3)) + (WS - 1 - (ki & 7)) + 4 * hh];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        float tv[16], lv[16], dv[16], bv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int o = 32 * qt + 8 * (r >> 2) + (r & 3);
          tv[r] = tb[15 * (4 * qt + (r >> 2)) + (r & 3)];
          lv[r] = rl[o];
          dv[r] = rd[o];
          bv[r] = dbl[o * LDB + 32 * kt];   // each (q, key) entry belongs to one lane / register
        }
        if (!plain) {   // shifted window on the image's last row / column, or an explicit mask
          const int rk = sReg[w][ki];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int o = 32 * qt + 8 * (r >> 2) + (r & 3);
            if (mixed && rg[o] != rk) tv[r] += -100.f;
            if (amask) tv[r] += amask[((win % mask_nw) * TOK + qt * 32 + acc_row(r, hh)) * TOK + ki];
          }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = __expf(fmaf(S[qt][kt][r], scale, tv[r]) - lv[r]);
          S[qt][kt][r] = p;
          const float d = p * (dP[qt][kt][r] - dv[r]);
          dP[qt][kt][r] = d;
          bv[r] += d;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) dbl[(32 * qt + 8 * (r >> 2) + (r & 3)) * LDB + 32 * kt] = bv[r];
      }
    }
    if (st_on) ts[3] = stamp_now();
    // dV^T = dO^T P and dK^T = scale * Q^T dS : tiles [kt], rows = d, lane = key
    // head-blocked [3][nWin][nh][64][32] (token stride 32), or token rows [M][3 nh 32] (rows != 0:
    // columns (part * nh + h) * 32 + d, the q/k/v input-gradient GEMM's plain A operand)
    const long tstr = rows ? 3L * nh * HP : HP;
    bf16* dq_out = rows ? dqkv + win * TOK * tstr + h * HP : dqkv + blk;
    bf16* dk_out = rows ? dq_out + nh * HP : dqkv + part + blk;
    bf16* dv_out = rows ? dq_out + 2 * nh * HP : dqkv + 2 * part + blk;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      f32x16 av, ak;
#pragma unroll
      for (int r = 0; r < 16; ++r) { av[r] = 0.f; ak[r] = 0.f; }
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          av = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_rows_perm(go, qt * 32, s, lane), pack8(S[qt][kt], s), av, 0, 0, 0);
          ak = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_rows_perm(q, qt * 32, s, lane), pack8(dP[qt][kt], s), ak, 0, 0, 0);
        }
      const int key = kt * 32 + l31;
#pragma unroll
      for (int g = 0; g < HP / 8; ++g) {
        const bf16x4 vv = {(bf16)av[4 * g], (bf16)av[4 * g + 1], (bf16)av[4 * g + 2], (bf16)av[4 * g + 3]};
        const bf16x4 kk = {(bf16)(ak[4 * g] * scale), (bf16)(ak[4 * g + 1] * scale), (bf16)(ak[4 * g + 2] * scale),
                           (bf16)(ak[4 * g + 3] * scale)};
        *(bf16x4*)(dv_out + key * tstr + 8 * g + 4 * hh) = vv;
        *(bf16x4*)(dk_out + key * tstr + 8 * g + 4 * hh) = kk;
      }
    }
    if (st_on) ts[4] = stamp_now();
    // dQ^T = scale * K^T dS^T : dS through LDS ([q][key] row-major), written over the q / dO tiles
    wave_sync();   // the dV / dK fragment reads of q and dO are complete
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) ds[(qt * 32 + acc_row(r, hh)) * LDD + kt * 32 + l31] = (bf16)dP[qt][kt][r];
    wave_sync();
    if (st_on) ts[5] = stamp_now();
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      f32x16 aq;
#pragma unroll
      for (int r = 0; r < 16; ++r) aq[r] = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s)
        aq = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_rows_nat(k, 0, s, lane), frag_cols(ds, LDD, qt * 32 + l31, s, lane),
                                                    aq, 0, 0, 0);
      const int qi = qt * 32 + l31;
#pragma unroll
      for (int g = 0; g < HP / 8; ++g) {
        const bf16x4 vq = {(bf16)(aq[4 * g] * scale), (bf16)(aq[4 * g + 1] * scale), (bf16)(aq[4 * g + 2] * scale),
                           (bf16)(aq[4 * g + 3] * scale)};
        *(bf16x4*)(dq_out + qi * tstr + 8 * g + 4 * hh) = vq;
      }
    }
    if (st_on) {
      ts[6] = stamp_now();
      ts[7] = (unsigned long long)(w1 - w0);
      if (lane < STAMP_N) {
        unsigned long long v = ts[0];
#pragma unroll
        for (int i = 1; i < STAMP_N; ++i)
          if (lane == i) v = ts[i];
        g_attn_stamps[gtask * STAMP_N + lane] = v;   // vector store, one lane per stamp
      }
    }
  }
  // partial bias gradient of this (group, head), binned (the q / dO tiles are free scratch now)
  wave_sync();
  static_assert(2 * TOK * LD * sizeof(bf16) >= 1024 * sizeof(float), "bin scratch");
  bin_dbias<true>(db, LDB, (float*)sQG[w], dB_part + (grp * nh + h) * NBIN, lane);
}

// dtable[idx][h] (+)= sum over groups of the binned per-group partials [group][h][idx] (coalesced,
// one thread per (h, idx), the groups split over the 16 waves and summed in fixed order)
__global__ __launch_bounds__(1024) void attn_dtable_sum_kernel(const float* __restrict__ part, long ngroups, int nh,
                                                               float* dtable, int acc) {
  const long n = (long)nh * NBIN;
  const long t = (long)blockIdx.x * 64 + (threadIdx.x & 63);
  const float s = split_sum16(part, ngroups, n, t, t < n);
  if (t < n && threadIdx.x < 64) {
    const int h = (int)(t / NBIN), idx = (int)(t - (long)h * NBIN);
    float* o = dtable + idx * nh + h;
    *o = acc ? *o + s : s;
  }
}

// Grouped bias-table gradient (kair_attn_dtable_grouped): the sum above for every block of a group in
// one launch; a workgroup finds its job by a scalar scan of the first-block offsets.
struct DtabJob { const float* part; float* dtable; long ngroups; int nh, acc, blk0; };
constexpr int DTAB_MAX = 32;
struct DtabGroup { DtabJob j[DTAB_MAX]; int njobs; };

KAIR_DEV int dtab_job(const DtabGroup& g, int b) {
  int ji = 0;
  for (int i = 1; i < g.njobs; ++i)
    if (g.j[i].blk0 <= b) ji = i;
  return __builtin_amdgcn_readfirstlane(ji);
}

__global__ __launch_bounds__(1024) void attn_dtable_grouped(const DtabGroup g) {
  const DtabJob& jb = g.j[dtab_job(g, blockIdx.x)];
  const long n = (long)jb.nh * NBIN;
  const long t = (long)(blockIdx.x - jb.blk0) * 64 + (threadIdx.x & 63);
  const float s = split_sum16(jb.part, jb.ngroups, n, t, t < n);
  if (t < n && threadIdx.x < 64) {
    const int h = (int)(t / NBIN), idx = (int)(t - (long)h * NBIN);
    float* o = jb.dtable + idx * jb.nh + h;
    *o = jb.acc ? *o + s : s;
  }
}

constexpr int WPG = 4;  // windows per backward wave (fp32 parity path)

// bf16 backward: windows per wave so that the (group, head) waves fill every CU's 4 wave slots in
// one round (1 wave per SIMD: the kernel holds ~500 VGPRs) -- e.g. 1152 windows x 6 heads on 256
// CUs -> 7 windows per wave, 990 waves
static int g_attn_ncu = 0;
static int bwd_wpg_bf16(long nWin, int nh) {
  int& ncu = g_attn_ncu;
  if (ncu == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      ncu = n;
    if (ncu <= 0) ncu = 256;
  }
  // windows per group from the groups per head that fit one round: ceil(nWin * nh / slots) could leave
  // ngroups * nh just above the slots (SwinIR-lightweight, 4,096 windows x 6 heads: 24 per wave -> 1,026 waves on
  // 1,024 slots, one workgroup running a second round alone -- the kernel's time doubled)
  long per = 4L * ncu / nh;
  if (per < 1) per = 1;
  const long w = (nWin + per - 1) / per;
  return (int)(w < 1 ? 1 : w);
}
static long bwd_groups(long nWin, int wpg) { return (nWin + wpg - 1) / wpg; }

// bf16 forward: (window, head) tasks per wave so that one round of waves (occ per SIMD: 3 at head pad 16, 2 at
// 32 -- the kernels' register occupancy) covers them all (KAIR_ATTN_FWD_TPW=n forces n: A/B)
static int fwd_tpw_bf16(long tasks, int occ) {
  static const int forced = [] {
    const char* e = getenv("KAIR_ATTN_FWD_TPW");
    return e ? atoi(e) : 0;
  }();
  if (forced > 0) return forced;
  bwd_wpg_bf16(1, 1);   // (initialises the CU count)
  const long slots = 4L * occ * g_attn_ncu;
  const long t = (tasks + slots - 1) / slots;
  return (int)(t < 1 ? 1 : t);
}

}  // namespace

extern "C" int kair_window_attn_fwd_ex(const void* qkv, int dtype, const float* table, void* O, long ldo, float* lse,
                                       long nWin, int nh, int hd, float scale, int H, int W, int shift, int ones_col,
                                       const float* mask, int mask_nw, int head_pad, void* stream) {
  KAIR_CHECK_ARG(!mask || (mask_nw > 0 && shift == 0), "window_attn_fwd: an explicit mask needs mask_nw > 0 and shift 0");
  KAIR_CHECK_ARG(qkv && table && O && lse, "window_attn_fwd: null pointer");
  KAIR_CHECK_ARG(head_pad == HDP || (head_pad == 16 && dtype == KAIR_BF16), "window_attn_fwd: head pad %d (32, or 16 in bf16)",
                 head_pad);
  const int hp = head_pad;
  KAIR_CHECK_ARG(hd > 0 && hd <= hp && nh > 0 && nWin > 0, "window_attn_fwd: head_dim %d must be <= %d", hd, hp);
  KAIR_CHECK_ARG(H % WS == 0 && W % WS == 0 && (shift == 0 || (shift > 0 && shift < WS)),
                 "window_attn_fwd: grid %dx%d / shift %d", H, W, shift);
  KAIR_CHECK_ARG(ldo >= nh * hp && ldo % 8 == 0, "window_attn_fwd: ldo");
  KAIR_CHECK_ARG(ones_col < 0 || (ones_col < nh * hp && ones_col % hp >= hd), "window_attn_fwd: ones column must be a pad column");
  const long tasks = nWin * nh;
  const int nw = dtype == KAIR_BF16 ? NWAVES<true> : NWAVES<false>;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == KAIR_BF16) {
    const int tpw = fwd_tpw_bf16(tasks, hp == 16 ? 3 : 2);
    const long nb = (tasks + (long)nw * tpw - 1) / ((long)nw * tpw);
    if (hp == 16)
      KAIR_LAUNCH(attn_fwd_bf16_kernel<16>, dim3((unsigned)nb), dim3(64 * nw), 0, s, (const bf16*)qkv, table, (bf16*)O, ldo,
                  lse, nWin, nh, scale, H, W, shift, ones_col, mask, mask_nw, tpw);
    else
      KAIR_LAUNCH(attn_fwd_bf16_kernel<32>, dim3((unsigned)nb), dim3(64 * nw), 0, s, (const bf16*)qkv, table, (bf16*)O, ldo,
                  lse, nWin, nh, scale, H, W, shift, ones_col, mask, mask_nw, tpw);
  } else {
    const long nb = (tasks + nw - 1) / nw;
    KAIR_LAUNCH(attn_fwd_kernel<false>, dim3((unsigned)nb), dim3(64 * nw), 0, s, (const float*)qkv, table, (float*)O,
                       ldo, lse, nWin, nh, scale, H, W, shift, ones_col, mask, mask_nw);
  }
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_window_attn_fwd(const void* qkv, int dtype, const float* table, void* O, long ldo, float* lse,
                                    long nWin, int nh, int hd, float scale, int H, int W, int shift, int ones_col,
                                    const float* mask, int mask_nw, void* stream) {
  return kair_window_attn_fwd_ex(qkv, dtype, table, O, ldo, lse, nWin, nh, hd, scale, H, W, shift, ones_col, mask, mask_nw,
                                 HDP, stream);
}

static const int g_stamp = kair_dbg_env("KAIR_ATTN_STAMP");
// waves per workgroup of the bf16 backward: 2 (71 KB of LDS, two workgroups per CU) spreads the
// (group, head) waves over every CU where 4-wave workgroups fill only 216 of 256 at B = 4 (A/B with
// KAIR_ATTN_BWD_NW=4: B = 4 630.7 -> 633.7 patches/s, B = 32 1,430 -> 1,438)
static const int g_bwd_nw = [] {
  const char* e = getenv("KAIR_ATTN_BWD_NW");
  return e && atoi(e) == 4 ? 4 : 2;
}();

// copy the attention-backward phase stamps to the host (perf investigation only)
extern "C" int kair_debug_attn_stamps(unsigned long long* host, int n) {
  KAIR_CHECK_ARG(host && n > 0 && n <= STAMP_WAVES * STAMP_N, "debug_attn_stamps: bad args");
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_attn_stamps), sizeof(unsigned long long) * n, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return kair_set_error(KAIR_ERR_HIP, "debug_attn_stamps: copy failed");
  return 0;
}

extern "C" long kair_window_attn_bwd_ws(long nWin, int nh) {
  const long g32 = bwd_groups(nWin, WPG), g16 = bwd_groups(nWin, bwd_wpg_bf16(nWin, nh));
  const long gx3 = bwd_groups(nWin, (int)kair_attn_x3_wpg(nWin, nh));
  long g = g32 > g16 ? g32 : g16;
  if (gx3 > g) g = gx3;
  return g * nh * NBIN;
}

int kair_attn_dtable_sum(const float* ws, long ngroups, int nh, float* dtable, int accumulate, hipStream_t s) {
  KAIR_LAUNCH(attn_dtable_sum_kernel, dim3((nh * NBIN + 63) / 64), dim3(1024), 0, s, ws, ngroups, nh, dtable,
                     accumulate);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_window_attn_bwd_ex(const void* qkv, const void* O, long ldo, const void* dO, long lddo, int dtype,
                                       const float* table, const float* lse, void* dqkv, int dqkv_rows, float* dtable,
                                       int dtable_accumulate, float* ws, long nWin, int nh, int hd, float scale, int H, int W,
                                       int shift, const float* mask, int mask_nw, int head_pad, void* stream) {
  KAIR_CHECK_ARG(!dqkv_rows || dtype == KAIR_BF16, "window_attn_bwd: token-row dqkv is a bf16 layout");
  KAIR_CHECK_ARG(head_pad == HDP || (head_pad == 16 && dtype == KAIR_BF16), "window_attn_bwd: head pad %d (32, or 16 in bf16)",
                 head_pad);
  KAIR_CHECK_ARG(!mask || (mask_nw > 0 && shift == 0), "window_attn_bwd: an explicit mask needs mask_nw > 0 and shift 0");
  KAIR_CHECK_ARG(qkv && O && dO && table && lse && dqkv && ws, "window_attn_bwd: null pointer");
  KAIR_CHECK_ARG(hd > 0 && hd <= head_pad && nh > 0 && nWin > 0, "window_attn_bwd: head_dim");
  KAIR_CHECK_ARG(H % WS == 0 && W % WS == 0 && (shift == 0 || (shift > 0 && shift < WS)), "window_attn_bwd: geometry");
  KAIR_CHECK_ARG(ldo % 8 == 0 && lddo % 8 == 0, "window_attn_bwd: strides");
  const int wpg = dtype == KAIR_BF16 ? bwd_wpg_bf16(nWin, nh) : WPG;
  const long ngroups = bwd_groups(nWin, wpg);
  const int nw = dtype == KAIR_BF16 ? g_bwd_nw : NWAVES<false>;
  const long nb = (ngroups * nh + nw - 1) / nw;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == KAIR_BF16 && head_pad == 16)
    KAIR_LAUNCH((attn_bwd_bf16_kernel<2, 16>), dim3((unsigned)nb), dim3(64 * nw), 0, s, (const bf16*)qkv, (const bf16*)O,
                       ldo, (const bf16*)dO, lddo, table, lse, (bf16*)dqkv, ws, nWin, nh, wpg, scale, H, W, shift, mask,
                       mask_nw, g_stamp, dqkv_rows);
  else if (dtype == KAIR_BF16 && nw == 2)
    KAIR_LAUNCH((attn_bwd_bf16_kernel<2, 32>), dim3((unsigned)nb), dim3(64 * nw), 0, s, (const bf16*)qkv, (const bf16*)O, ldo,
                       (const bf16*)dO, lddo, table, lse, (bf16*)dqkv, ws, nWin, nh, wpg, scale, H, W, shift, mask, mask_nw,
                       g_stamp, dqkv_rows);
  else if (dtype == KAIR_BF16)
    KAIR_LAUNCH((attn_bwd_bf16_kernel<4, 32>), dim3((unsigned)nb), dim3(64 * nw), 0, s, (const bf16*)qkv, (const bf16*)O, ldo,
                       (const bf16*)dO, lddo, table, lse, (bf16*)dqkv, ws, nWin, nh, wpg, scale, H, W, shift, mask, mask_nw,
                       g_stamp, dqkv_rows);
  else
    KAIR_LAUNCH(attn_bwd_kernel<false>, dim3((unsigned)nb), dim3(64 * nw), 0, s, (const float*)qkv, (const float*)O,
                       ldo, (const float*)dO, lddo, table, lse, (float*)dqkv, ws, nWin, nh, wpg, scale, H, W, shift, mask, mask_nw);
  KAIR_CHECK_LAUNCH();
  if (!dtable) return 0;   // deferred: the per-group partials stay in ws for kair_attn_dtable_grouped
  KAIR_LAUNCH(attn_dtable_sum_kernel, dim3((nh * NBIN + 63) / 64), dim3(1024), 0, s, ws, ngroups, nh, dtable,
                     dtable_accumulate);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_window_attn_bwd(const void* qkv, const void* O, long ldo, const void* dO, long lddo, int dtype,
                                    const float* table, const float* lse, void* dqkv, float* dtable, int dtable_accumulate,
                                    float* ws, long nWin, int nh, int hd, float scale, int H, int W, int shift,
                                    const float* mask, int mask_nw, void* stream) {
  return kair_window_attn_bwd_ex(qkv, O, ldo, dO, lddo, dtype, table, lse, dqkv, 0, dtable, dtable_accumulate, ws, nWin, nh,
                                 hd, scale, H, W, shift, mask, mask_nw, HDP, stream);
}

extern "C" long kair_window_attn_bwd_groups(long nWin, int nh, int dtype) {
  if (nWin <= 0 || nh <= 0) return 0;
  if (dtype == KAIR_COMPUTE_X3) return bwd_groups(nWin, (int)kair_attn_x3_wpg(nWin, nh));
  return bwd_groups(nWin, dtype == KAIR_BF16 ? bwd_wpg_bf16(nWin, nh) : WPG);
}

extern "C" int kair_attn_dtable_grouped(const kair_attn_dtable_job* jobs, int njobs, void* stream) {
  KAIR_CHECK_ARG(jobs && njobs > 0 && njobs <= DTAB_MAX, "attn_dtable_grouped: 1..%d jobs", DTAB_MAX);
  DtabGroup g;
  memset(&g, 0, sizeof(g));
  int b0 = 0;
  for (int i = 0; i < njobs; ++i) {
    const kair_attn_dtable_job& J = jobs[i];
    KAIR_CHECK_ARG(J.ws && J.dtable && J.nh > 0 && J.nWin > 0, "attn_dtable_grouped: job %d", i);
    g.j[i] = DtabJob{J.ws, J.dtable, kair_window_attn_bwd_groups(J.nWin, J.nh, J.dtype), J.nh, J.accumulate ? 1 : 0, b0};
    b0 += (J.nh * NBIN + 63) / 64;
  }
  g.njobs = njobs;
  hipStream_t s = (hipStream_t)stream;
  KAIR_LAUNCH(attn_dtable_grouped, dim3(b0), dim3(1024), 0, s, g);
  KAIR_CHECK_LAUNCH();
  return 0;
}
