// Swin window attention at the fp32 reference's arithmetic on the bf16 matrix cores (network_swinir.py
// :114-145 WindowAttention.forward and its autograd backward; the reference trains classical x4 in fp32,
// models/model_plain.py:31-36 with no amp_enabled in options/swinir/train_swinir_sr_classical.json).
//
// Every operand x is carried as an fp16 pair of x 2^e (hi = f16(x 2^e), lo = f16(x 2^e - hi); e a power-of-2
// exponent that puts the bulk of the tensor at 2^2 .. 2^10, so the lo half stays a normal fp16 number: the
// engine's activation exponent for q/k/v and O, P_EXP for the probabilities, its gradient exponent for dO, dS
// and dq/dk/dv) and every product as three v_mfma_f32_32x32x16_f16:
// hi.hi + hi.lo + lo.hi, fp32 accumulation, rescaled by 2^-(eA + eB).  The pair holds 22 mantissa bits, so a
// product is exact to ~2^-21: the fp32 computation's precision class (a bf16 pair reaches 2^-16, one bf16
// product 2^-8).  The fp32 MFMA (v_mfma_f32_32x32x2_f32) runs at 1/16 of the 16-bit rate; three 16-bit
// products cost 3/16.
//
// Layouts as the bf16 kernels (window_attn.hip): q/k/v head-blocked [3][nWin][nh][64][32], O and dO
// token rows (window order, head h at columns h*32..), lse [nWin][nh][64]; each fp16 tensor has its lo
// plane in a second buffer of the same layout.  The backward writes dq/dk/dv as token rows
// [nWin*64][3*nh*32] (column (part*nh + h)*32 + d), hi and lo planes: the A operand of the q/k/v
// input- and weight-gradient GEMMs.  O and dq/dk/dv may instead be fp32 in natural units (a null lo
// plane): the form the fp32-operand ring GEMMs of gemm_x3.hip stream by LDS-DMA.
#include <string.h>

#include "attn_common.h"

namespace {

constexpr int FWD_NW = 4;
constexpr int P_EXP = 6;   // the probabilities' exponent: P ~ 1/64 -> ~1, its lo half a normal fp16 number

typedef __attribute__((ext_vector_type(8))) short s16x8;
KAIR_DEV f16x8 as_f16(const bf16x8& v) { return __builtin_bit_cast(f16x8, v); }
// MFMA-fragment reads of fp16 LDS tiles through the 16-bit helpers of attn_common.h (bit patterns only)
KAIR_DEV f16x8 hrows_perm(const f16* X, int base, int s, int lane) { return as_f16(frag_rows_perm((const bf16*)X, base, s, lane)); }
KAIR_DEV f16x8 hrows_nat(const f16* X, int base, int s, int lane) { return as_f16(frag_rows_nat((const bf16*)X, base, s, lane)); }
KAIR_DEV f16x8 hcols(const f16* X, int ld, int row, int s, int lane) { return as_f16(frag_cols((const bf16*)X, ld, row, s, lane)); }
KAIR_DEV f32x16 mfma32(const f16x8& a, const f16x8& b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
// the fp16 pair of 8 accumulator elements (the pack8 operand order) scaled by sc
// (products made opaque before the split: common.h opaque)
KAIR_DEV void pack8_pair(const f32x16& a, int s, float sc, f16x8& hi, f16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float v = opaque(a[8 * s + j] * sc);
    hi[j] = (f16)v;
    lo[j] = (f16)(v - (float)hi[j]);
  }
}
KAIR_DEV void pair4(const float (&v)[4], float sc, f16x4& hi, f16x4& lo) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float w = opaque(v[j] * sc);
    hi[j] = (f16)w;
    lo[j] = (f16)(w - (float)hi[j]);
  }
}

// ------------------------------------------------------------------------------------------
// forward: one wave per (window, head).  q / k fragments straight from global into registers (the
// S^T = K Q^T operands), v hi / lo planes staged in LDS for the transposed P.V fragments; O^T = V^T P^T
// (lane = query) stored 8 bytes per plane per register group.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64 * FWD_NW, 3) void attn_fwd_x3_kernel(const f16* __restrict__ qkv, const f16* __restrict__ qkvl,
                                                                  const float* __restrict__ table, f16* __restrict__ O,
                                                                  f16* __restrict__ Ol, long ldo, float* __restrict__ lse,
                                                                  long nWin, int nh, float scale, int H, int W, int shift,
                                                                  int ones_col, int e_in, int e_out) {
  constexpr int LD = ATT_LD, NW = FWD_NW;
  __shared__ __attribute__((aligned(16))) f16 sV[NW][2][TOK * LD];
  __shared__ float sTab[NW][232];
  __shared__ int sReg[NW][TOK];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long task = (long)blockIdx.x * NW + w;
  if (task >= nWin * nh) return;
  const long win = task / nh;
  const int h = (int)(task - win * nh);
  const long M = nWin * TOK;
  const long blk = (win * nh + h) * TOK * HDP;
  const long part = M * nh * HDP;
  const int l31 = lane & 31, hh = lane >> 5;
  f16x8 Qh[2][2], Ql[2][2], Kh[2][2], Kl[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const long o = blk + (long)(t * 32 + l31) * HDP + 16 * s + 8 * hh;
      Qh[t][s] = *(const f16x8*)(qkv + o);
      Ql[t][s] = *(const f16x8*)(qkvl + o);
      Kh[t][s] = *(const f16x8*)(qkv + part + o);
      Kl[t][s] = *(const f16x8*)(qkvl + part + o);
      const int lo = (t * 32 + l31) * LD + 16 * s + 8 * hh;
      *(f16x8*)(sV[w][0] + lo) = *(const f16x8*)(qkv + 2 * part + o);
      *(f16x8*)(sV[w][1] + lo) = *(const f16x8*)(qkvl + 2 * part + o);
    }
  for (int i = lane; i < NBIN; i += 64) sTab[w][i] = table[i * nh + h];
  const int nW = (H / WS) * (W / WS);
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
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        acc[kt][qt] = mfma32(Kh[kt][s], Qh[qt][s], acc[kt][qt]);
        acc[kt][qt] = mfma32(Kh[kt][s], Ql[qt][s], acc[kt][qt]);
        acc[kt][qt] = mfma32(Kl[kt][s], Qh[qt][s], acc[kt][qt]);
      }
  wave_sync();
  const float sqk = scale * ldexpf(1.f, -2 * e_in);   // q.k^T back to natural units, times the attention scale
  // scores: scale, bias, shifted-window mask; softmax over keys (registers + lane^32)
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
        float sc = acc[kt][qt][r] * sqk + sTab[w][relidx(qi, ki)];
        if (shift > 0 && sReg[w][ki] != rq) sc += -100.f;
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
  // O^T = V^T P^T : tile [qt] rows = d, lane = query (P with exponent P_EXP)
  const float so = ldexpf(1.f, e_out - e_in - P_EXP), sone = ldexpf(1.f, e_out), sp = ldexpf(1.f, P_EXP);
  const float so_nat = ldexpf(1.f, -e_in - P_EXP);
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    f32x16 o;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const f16x8 vh = hrows_perm(sV[w][0], kt * 32, s, lane), vl = hrows_perm(sV[w][1], kt * 32, s, lane);
        f16x8 ph, pl;
        pack8_pair(acc[kt][qt], s, sp, ph, pl);
        o = mfma32(vh, ph, o);
        o = mfma32(vh, pl, o);
        o = mfma32(vl, ph, o);
      }
    const int qi = qt * 32 + l31;
    const long orow = (win * TOK + qi) * ldo + h * HDP;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d0 = 8 * g + 4 * hh;
      float v[4];
      if (Ol) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (h * HDP + d0 + j == ones_col) ? sone : o[4 * g + j] * so;
        f16x4 qh, ql;
        pair4(v, 1.f, qh, ql);
        *(f16x4*)(O + orow + d0) = qh;
        *(f16x4*)(Ol + orow + d0) = ql;
      } else {   // fp32 O in natural units
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (h * HDP + d0 + j == ones_col) ? 1.f : o[4 * g + j] * so_nat;
        *(float4*)((float*)O + orow + d0) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// backward: one 2-wave workgroup per (head, group of windows); wave w owns the keys 32 w .. 32 w + 31 of every
// window (S, dP, P, dS, dV, dK of its key half; its partial dQ over those keys, the two halves summed through
// LDS, each wave finishing 32 queries).  50 KB of LDS per workgroup: the window's q / dO hi and lo tiles (each
// wave stages 32 rows), then the two waves' dS tiles; each wave's k tile, then its dQ-partial exchange slot; the
// running bias gradient [q][key] fp32 (each entry belongs to one lane of one wave).  3 workgroups per CU.
// P is recomputed from q, k and the saved log-sum-exp.
// ------------------------------------------------------------------------------------------
constexpr int BWD_NW = 2;
__global__ __launch_bounds__(64 * BWD_NW, 2) void attn_bwd_x3_kernel(const f16* __restrict__ qkv, const f16* __restrict__ qkvl,
                                                            const f16* __restrict__ O, const f16* __restrict__ Ol, long ldo,
                                                            const f16* __restrict__ dO, const f16* __restrict__ dOl, long lddo,
                                                            const float* __restrict__ table, const float* __restrict__ lse,
                                                            f16* __restrict__ dqkv, f16* __restrict__ dqkvl,
                                                            float* __restrict__ dB_part, long nWin, int nh, int wpg,
                                                            float scale, int H, int W, int shift, int e_act, int e_grad) {
  constexpr int LD = ATT_LD, LDB = 72;
  // plane p (0 hi, 1 lo): [q | dO] tiles [64][LD]; after dV / dK wave w's dS tile [q][its 32 keys] at w * TOK * LD
  __shared__ __attribute__((aligned(16))) f16 sQG[2][2 * TOK * LD];
  // [wave][plane]: the wave's k rows [32][LD]; after its dQ MFMAs, its exchange slot (16 floats per lane)
  __shared__ __attribute__((aligned(16))) f16 sK[BWD_NW][2][32 * LD];
  __shared__ __attribute__((aligned(16))) float sDB[TOK * LDB];   // running bias gradient [q][key]
  __shared__ float sTab[232];
  __shared__ float sRow[2][TOK];  // lse, delta
  __shared__ int sReg[TOK];
  static_assert(2 * 32 * LD * sizeof(f16) >= 64 * 16 * sizeof(float), "dQ exchange slot");
  static_assert(2 * 32 * LD * sizeof(f16) >= 1024 * sizeof(float), "bin scratch");
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const long gtask = blockIdx.x;
  const long ngroups = (nWin + wpg - 1) / wpg;
  if (gtask >= ngroups * nh) return;
  const int h = (int)(gtask % nh);
  const long grp = gtask / nh;
  const long M = nWin * TOK;
  const long part = M * nh * HDP;
  const int l31 = lane & 31, hh = lane >> 5;
  for (int i = tid; i < NBIN; i += 64 * BWD_NW) sTab[i] = table[i * nh + h];
  const int nW = (H / WS) * (W / WS);
  const long tstr = 3L * nh * HDP;
  // exponents: q/k/v and O carry e_act, dO / dS / dq,dk,dv carry e_grad; everything below is rescaled
  // to natural units (S, dP, delta, P, dS) before it is combined
  const float s_qk = ldexpf(1.f, -2 * e_act), s_dp = ldexpf(1.f, -(e_grad + e_act));
  const float s_o = ldexpf(1.f, -e_act), s_g = ldexpf(1.f, -e_grad), s_gup = ldexpf(1.f, e_grad);
  const float s_dv = ldexpf(1.f, -P_EXP);    // dO^T P: (e_grad) x (P_EXP) -> e_grad
  const float s_p = ldexpf(1.f, P_EXP);
  const float s_dk = ldexpf(1.f, -e_act);    // Q^T dS, K^T dS^T: (e_act) x (e_grad) -> e_grad
  // (row stride 72: the two lane halves' rows 4 apart fall in opposite bank halves)
  for (int i = tid; i < TOK * LDB / 4; i += 64 * BWD_NW) ((float4*)sDB)[i] = make_float4(0.f, 0.f, 0.f, 0.f);

  // fragment f[s] of token t * 32 + l31 (8 consecutive d at 16 s + 8 hh) and its LDS image (row r0 + l31)
  auto ldfrag = [&](const f16* g, long ld, int t, f16x8 (&f)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 2; ++s) f[s] = *(const f16x8*)(g + (long)(t * 32 + l31) * ld + 16 * s + 8 * hh);
  };
  auto stfrag = [&](f16* tile, int r0, const f16x8 (&f)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 2; ++s) *(f16x8*)(tile + (r0 + l31) * LD + 16 * s + 8 * hh) = f[s];
  };
  // the wave's own token half f[w] of a [2][2] fragment set (a select: a register array indexed by the run-time
  // wave index would live in scratch)
  auto stown = [&](f16* tile, const f16x8 (&f)[2][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 2; ++s) *(f16x8*)(tile + (32 * w + l31) * LD + 16 * s + 8 * hh) = w ? f[1][s] : f[0][s];
  };

  const long w0 = grp * wpg;
  long w1 = w0 + wpg;
  if (w1 > nWin) w1 = nWin;
  const int ki = w * 32 + l31;   // this lane's key
  for (long win = w0; win < w1; ++win) {
    const long blk = (win * nh + h) * TOK * HDP;
    __syncthreads();   // the previous window's tiles and exchange slots are no longer read
    f32x16 S[2], dP[2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) { S[a][r] = 0.f; dP[a][r] = 0.f; }
    {   // S = Q K_w^T : tiles [qt], lane = key, regs = query
      f16x8 Fqh[2][2], Fql[2][2], Fkh[2], Fkl[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        ldfrag(qkv + blk, HDP, t, Fqh[t]);
        ldfrag(qkvl + blk, HDP, t, Fql[t]);
      }
      ldfrag(qkv + part + blk, HDP, w, Fkh);
      ldfrag(qkvl + part + blk, HDP, w, Fkl);
      stown(sQG[0], Fqh);
      stown(sQG[1], Fql);
      stfrag(sK[w][0], 0, Fkh);
      stfrag(sK[w][1], 0, Fkl);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          S[qt] = mfma32(Fqh[qt][s], Fkh[s], S[qt]);
          S[qt] = mfma32(Fqh[qt][s], Fkl[s], S[qt]);
          S[qt] = mfma32(Fql[qt][s], Fkh[s], S[qt]);
        }
    }
    {   // dP = dO V_w^T ; delta = rowsum(dO o O) for the queries 32 w + l31, from the fp32 sums of the planes
      f16x8 Fgh[2][2], Fgl[2][2], Fvh[2], Fvl[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        ldfrag(dO + win * TOK * lddo + h * HDP, lddo, t, Fgh[t]);
        ldfrag(dOl + win * TOK * lddo + h * HDP, lddo, t, Fgl[t]);
      }
      ldfrag(qkv + 2 * part + blk, HDP, w, Fvh);
      ldfrag(qkvl + 2 * part + blk, HDP, w, Fvl);
      stown(sQG[0] + TOK * LD, Fgh);
      stown(sQG[1] + TOK * LD, Fgl);
      float dsum = 0.f;
      if (Ol) {
        f16x8 Foh[2], Fol[2];
        ldfrag(O + win * TOK * ldo + h * HDP, ldo, w, Foh);
        ldfrag(Ol + win * TOK * ldo + h * HDP, ldo, w, Fol);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const f16x8 gh = w ? Fgh[1][s] : Fgh[0][s], gl = w ? Fgl[1][s] : Fgl[0][s];
#pragma unroll
          for (int j = 0; j < 8; ++j) dsum += ((float)gh[j] + (float)gl[j]) * ((float)Foh[s][j] + (float)Fol[s][j]) * s_o;
        }
      } else {   // fp32 O (natural units)
        const float* Of = (const float*)O + win * TOK * ldo + h * HDP;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const float* op = Of + (long)(w * 32 + l31) * ldo + 16 * s + 8 * hh;
          const float4 a = *(const float4*)op, b = *(const float4*)(op + 4);
          const float ov[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
          const f16x8 gh = w ? Fgh[1][s] : Fgh[0][s], gl = w ? Fgl[1][s] : Fgl[0][s];
#pragma unroll
          for (int j = 0; j < 8; ++j) dsum += ((float)gh[j] + (float)gl[j]) * ov[j];
        }
      }
      dsum += __shfl_xor(dsum, 32, 64);
      if (hh == 0) {
        sRow[0][w * 32 + l31] = lse[(win * nh + h) * TOK + w * 32 + l31];
        sRow[1][w * 32 + l31] = dsum * s_g;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          dP[qt] = mfma32(Fgh[qt][s], Fvh[s], dP[qt]);
          dP[qt] = mfma32(Fgh[qt][s], Fvl[s], dP[qt]);
          dP[qt] = mfma32(Fgl[qt][s], Fvh[s], dP[qt]);
        }
    }
    if (w == 0) sReg[lane] = shift > 0 ? token_region((int)(win % nW), lane, H, W, shift) : 0;
    __syncthreads();   // the q / dO tiles, lse / delta and the token regions of both halves

    // P = exp(S*scale + bias + mask - lse) ; dS = P (dP - delta), natural units.  Lane = key ki, register r
    // of tile qt = query 32 qt + 8 (r/4) + r%4 + 4 hh: every LDS operand at a compile-time offset from a
    // per-lane base (the bf16 kernel's indexing).
    const int wi_img = (int)(win % nW), nWw = W / WS;
    const bool mixed = shift > 0 && ((wi_img / nWw) == H / WS - 1 || (wi_img % nWw) == nWw - 1);
    const float* rl = &sRow[0][4 * hh];
    const float* rd = &sRow[1][4 * hh];
    const int* rg = &sReg[4 * hh];
    const float sqk = scale * s_qk;
    {
      const int rk = sReg[ki];
      const float* tb = &sTab[15 * (WS - 1 - (ki >> 3)) + (WS - 1 - (ki & 7)) + 4 * hh];
      float* dbl = sDB + 4 * hh * LDB + ki;
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int r0 = 0; r0 < 16; r0 += 8) {   // 8 elements' LDS operands read back to back, then the math
          float tv[8], lv[8], dv[8], bv[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int r = r0 + u, o = 32 * qt + 8 * (r >> 2) + (r & 3);
            tv[u] = tb[15 * (4 * qt + (r >> 2)) + (r & 3)];
            lv[u] = rl[o];
            dv[u] = rd[o];
            bv[u] = dbl[o * LDB];
          }
          if (mixed) {
#pragma unroll
            for (int u = 0; u < 8; ++u)
              if (rg[32 * qt + 8 * ((r0 + u) >> 2) + ((r0 + u) & 3)] != rk) tv[u] += -100.f;
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int r = r0 + u;
            const float p = __expf(fmaf(S[qt][r], sqk, tv[u]) - lv[u]);
            S[qt][r] = p;
            const float d = p * (dP[qt][r] * s_dp - dv[u]);
            dP[qt][r] = d;
            bv[u] += d;
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) dbl[(32 * qt + 8 * ((r0 + u) >> 2) + ((r0 + u) & 3)) * LDB] = bv[u];
        }
    }
    // dV^T = dO^T P and dK^T = scale * Q^T dS of the wave's keys: rows = d, lane = key; token-row outputs
    // carrying e_grad (dS enters as the pair of dS 2^e_grad)
    f16* dq_out = dqkv + win * TOK * tstr + h * HDP;
    f16* dql_out = dqkvl ? dqkvl + win * TOK * tstr + h * HDP : nullptr;
    float* dqf = (float*)dqkv + win * TOK * tstr + h * HDP;
    const long koff = (long)nh * HDP, voff = 2L * nh * HDP;
    {
      f32x16 av, ak;
#pragma unroll
      for (int r = 0; r < 16; ++r) { av[r] = 0.f; ak[r] = 0.f; }
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const f16x8 gh = hrows_perm(sQG[0] + TOK * LD, qt * 32, s, lane);
          const f16x8 gl = hrows_perm(sQG[1] + TOK * LD, qt * 32, s, lane);
          const f16x8 qh = hrows_perm(sQG[0], qt * 32, s, lane), ql = hrows_perm(sQG[1], qt * 32, s, lane);
          f16x8 ph, pl, dh, dl;
          pack8_pair(S[qt], s, s_p, ph, pl);
          pack8_pair(dP[qt], s, s_gup, dh, dl);
          av = mfma32(gh, ph, av);
          av = mfma32(gh, pl, av);
          av = mfma32(gl, ph, av);
          ak = mfma32(qh, dh, ak);
          ak = mfma32(qh, dl, ak);
          ak = mfma32(ql, dh, ak);
        }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float va[4], ka[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          va[j] = av[4 * g + j] * s_dv;
          ka[j] = ak[4 * g + j] * (scale * s_dk);
        }
        const long o = (long)ki * tstr + 8 * g + 4 * hh;
        if (dqkvl) {
          f16x4 vh, vl, kh, kl;
          pair4(va, 1.f, vh, vl);
          pair4(ka, 1.f, kh, kl);
          *(f16x4*)(dq_out + voff + o) = vh;
          *(f16x4*)(dql_out + voff + o) = vl;
          *(f16x4*)(dq_out + koff + o) = kh;
          *(f16x4*)(dql_out + koff + o) = kl;
        } else {   // fp32 dq/dk/dv in natural units
          *(float4*)(dqf + voff + o) = make_float4(va[0] * s_g, va[1] * s_g, va[2] * s_g, va[3] * s_g);
          *(float4*)(dqf + koff + o) = make_float4(ka[0] * s_g, ka[1] * s_g, ka[2] * s_g, ka[3] * s_g);
        }
      }
    }
    // dQ^T = scale * K^T dS^T, each wave over its keys: its dS pair [q][32 keys] through its half of sQG
    __syncthreads();   // both waves' dV / dK fragment reads of the q / dO tiles are complete
    f16* dsh = sQG[0] + w * TOK * LD;
    f16* dsl = sQG[1] + w * TOK * LD;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = opaque(dP[qt][r] * s_gup);   // (not fused into the conversion: common.h opaque)
        const f16 vh = (f16)v;
        const int o = (qt * 32 + acc_row(r, hh)) * LD + l31;
        dsh[o] = vh;
        dsl[o] = (f16)(v - (float)vh);
      }
    wave_sync();   // (the wave reads back only its own tile)
    f32x16 aq[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) aq[qt][r] = 0.f;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const f16x8 kh = hrows_nat(sK[w][0], 0, s, lane), kl = hrows_nat(sK[w][1], 0, s, lane);
        const f16x8 dh = hcols(dsh, LD, qt * 32 + l31, s, lane), dl = hcols(dsl, LD, qt * 32 + l31, s, lane);
        aq[qt] = mfma32(kh, dh, aq[qt]);
        aq[qt] = mfma32(kh, dl, aq[qt]);
        aq[qt] = mfma32(kl, dh, aq[qt]);
      }
    }
    // the two key halves' partials: wave w finishes the queries of tile qt = w, the other tile's partial goes
    // to the partner through this wave's exchange slot (its k tile is no longer read)
    wave_sync();
    const f32x16 aqs = w ? aq[0] : aq[1], aqk = w ? aq[1] : aq[0];   // (selects, not a run-time register index)
    float* xo = (float*)&sK[w][0][0];
#pragma unroll
    for (int r = 0; r < 16; ++r) xo[r * 64 + lane] = aqs[r];
    __syncthreads();
    const float* xi = (const float*)&sK[1 - w][0][0];
    {
      const long qi = w * 32 + l31;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float qa[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) qa[j] = (aqk[4 * g + j] + xi[(4 * g + j) * 64 + lane]) * (scale * s_dk);
        if (dqkvl) {
          f16x4 qh, ql;
          pair4(qa, 1.f, qh, ql);
          *(f16x4*)(dq_out + qi * tstr + 8 * g + 4 * hh) = qh;
          *(f16x4*)(dql_out + qi * tstr + 8 * g + 4 * hh) = ql;
        } else {
          *(float4*)(dqf + qi * tstr + 8 * g + 4 * hh) = make_float4(qa[0] * s_g, qa[1] * s_g, qa[2] * s_g, qa[3] * s_g);
        }
      }
    }
  }
  // partial bias gradient of this (group, head), binned by wave 0 (its k tile is free scratch now)
  __syncthreads();
  if (w == 0) bin_dbias<true>(sDB, LDB, (float*)&sK[0][0][0], dB_part + (grp * nh + h) * NBIN, lane);
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

}  // namespace

// windows per backward wave: enough (group, head) waves for ONE round at the residency the backward's LDS
// allows (3 two-wave workgroups of ~50 KB per CU; kair_window_attn_bwd_groups / _ws size the partials from it)
long kair_attn_x3_wpg(long nWin, int nh) {
  // groups per head that fit one round of workgroups, then windows per group (as bwd_wpg_bf16: rounding the
  // windows per group up from nWin * nh / slots can leave a few workgroups for a second round)
  long per = 3L * x3_cus() / nh;
  if (per < 1) per = 1;
  const long w = (nWin + per - 1) / per;
  return w < 1 ? 1 : w;
}

extern "C" int kair_window_attn_fwd_x3(const void* qkv, const void* qkv_lo, const float* table, void* O, void* O_lo, long ldo,
                                       float* lse, long nWin, int nh, int hd, float scale, int H, int W, int shift,
                                       int ones_col, int e_in, int e_out, void* stream) {
  KAIR_CHECK_ARG(qkv && qkv_lo && table && O && lse, "window_attn_fwd_x3: null pointer");
  KAIR_CHECK_ARG(hd > 0 && hd <= HDP && nh > 0 && nWin > 0, "window_attn_fwd_x3: head_dim %d must be <= 32", hd);
  KAIR_CHECK_ARG(H % WS == 0 && W % WS == 0 && (shift == 0 || (shift > 0 && shift < WS)),
                 "window_attn_fwd_x3: grid %dx%d / shift %d", H, W, shift);
  KAIR_CHECK_ARG(ldo >= nh * HDP && ldo % 8 == 0, "window_attn_fwd_x3: ldo");
  KAIR_CHECK_ARG(ones_col < 0 || (ones_col < nh * HDP && ones_col % HDP >= hd), "window_attn_fwd_x3: ones column must be a pad column");
  KAIR_CHECK_ARG(((uintptr_t)qkv % 16) == 0 && ((uintptr_t)qkv_lo % 16) == 0 && ((uintptr_t)O % (O_lo ? 8 : 16)) == 0 &&
                     ((uintptr_t)O_lo % 8) == 0 && (O_lo || ldo % 4 == 0),
                 "window_attn_fwd_x3: alignment");
  const long tasks = nWin * nh;
  const long nb = (tasks + FWD_NW - 1) / FWD_NW;
  KAIR_CHECK_ARG(e_in > -60 && e_in < 60 && e_out > -60 && e_out < 60, "window_attn_fwd_x3: exponents");
  KAIR_LAUNCH(attn_fwd_x3_kernel, dim3((unsigned)nb), dim3(64 * FWD_NW), 0, (hipStream_t)stream, (const f16*)qkv,
                     (const f16*)qkv_lo, table, (f16*)O, (f16*)O_lo, ldo, lse, nWin, nh, scale, H, W, shift, ones_col, e_in,
                     e_out);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_window_attn_bwd_x3(const void* qkv, const void* qkv_lo, const void* O, const void* O_lo, long ldo,
                                       const void* dO, const void* dO_lo, long lddo, const float* table, const float* lse,
                                       void* dqkv, void* dqkv_lo, float* dtable, int dtable_accumulate, float* ws, long nWin,
                                       int nh, int hd, float scale, int H, int W, int shift, int e_act, int e_grad,
                                       void* stream) {
  KAIR_CHECK_ARG(qkv && qkv_lo && O && dO && dO_lo && table && lse && dqkv && ws, "window_attn_bwd_x3: null pointer");
  KAIR_CHECK_ARG((O_lo || (uintptr_t)O % 16 == 0) && (dqkv_lo || (uintptr_t)dqkv % 16 == 0), "window_attn_bwd_x3: alignment");
  KAIR_CHECK_ARG(hd > 0 && hd <= HDP && nh > 0 && nWin > 0, "window_attn_bwd_x3: head_dim");
  KAIR_CHECK_ARG(H % WS == 0 && W % WS == 0 && (shift == 0 || (shift > 0 && shift < WS)), "window_attn_bwd_x3: geometry");
  KAIR_CHECK_ARG(ldo % 8 == 0 && lddo % 8 == 0, "window_attn_bwd_x3: strides");
  const long wpg = kair_attn_x3_wpg(nWin, nh);
  const long ngroups = (nWin + wpg - 1) / wpg;
  hipStream_t s = (hipStream_t)stream;
  KAIR_CHECK_ARG(e_act > -60 && e_act < 60 && e_grad > -60 && e_grad < 60, "window_attn_bwd_x3: exponents");
  KAIR_LAUNCH(attn_bwd_x3_kernel, dim3((unsigned)(ngroups * nh)), dim3(64 * BWD_NW), 0, s, (const f16*)qkv, (const f16*)qkv_lo,
                     (const f16*)O, (const f16*)O_lo, ldo, (const f16*)dO, (const f16*)dO_lo, lddo, table, lse, (f16*)dqkv,
                     (f16*)dqkv_lo, ws, nWin, nh, (int)wpg, scale, H, W, shift, e_act, e_grad);
  KAIR_CHECK_LAUNCH();
  if (!dtable) return 0;   // deferred: the per-group partials stay in ws for kair_attn_dtable_grouped (dtype x3)
  kair_attn_dtable_sum(ws, ngroups, nh, dtable, dtable_accumulate, s);
  return 0;
}
