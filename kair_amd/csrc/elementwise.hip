// Memory-bound helpers around the KAIR training step on gfx950: weight packing into the padded
// MFMA layouts, deterministic weight-gradient finalisation, image <-> token layout, the L1 loss
// (nn.L1Loss mean, model_plain.py:183-188) and the fused Adam + EMA update (torch.optim.Adam maths,
// model_plain.py:210-222/302; ModelBase.update_E model_base.py:247-252).
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "common.h"

namespace {

// padded index -> reference index along one grouped dim (-1 for pad)
KAIR_DEV int unpad(int ip, int G, int Gr, int Gp) {
  const int g = ip / Gp, i = ip - g * Gp;
  return (g < G && i < Gr) ? g * Gr + i : -1;
}

// kair_wmap.n_perm: the out dim stored sub-pixel-major (packed s*nf + c <-> reference c*r2 + s)
KAIR_DEV int nperm_fwd(const kair_wmap& mp, int n) {   // packed (unpadded) -> reference
  if (mp.n_perm <= 1 || n < 0) return n;
  const int nf = mp.N / mp.n_perm;
  return (n % nf) * mp.n_perm + n / nf;
}
KAIR_DEV int nperm_inv(const kair_wmap& mp, int co) {  // reference -> packed (unpadded)
  if (mp.n_perm <= 1) return co;
  const int nf = mp.N / mp.n_perm;
  return (co % mp.n_perm) * nf + co / mp.n_perm;
}

// Row geometry of the split forms 17 / 18 / 19 (hi/lo pairs of kinds 0 / 2 / 3, kair_wmap): the plain
// form's row length and the kind it splits
__host__ __device__ inline void split_rows(const kair_wmap& mp, int* base, long* rowlen, long* rows) {
  const long Np = (long)mp.nG * mp.nGp, Kp = (long)mp.kG * mp.kGp;
  if (mp.kind == 17) { *base = 0; *rowlen = Kp; *rows = Np; }
  else if (mp.kind == 18) { *base = 2; *rowlen = 9 * Np; *rows = Kp; }
  else { *base = 3; *rowlen = Np; *rows = Kp; }
}

// Reference value of element t of a plain linear / conv-dgrad / transposed-linear form (kinds 0, 2, 3)
KAIR_DEV float pack_value(const float* __restrict__ src, const kair_wmap& mp, int kind, long t) {
  const int Np = mp.nG * mp.nGp, Kp = mp.kG * mp.kGp;
  if (kind == 2) {
    const int cip = (int)(t / (9 * Np));
    const int kk = (int)(t - (long)cip * 9 * Np);
    const int tap = kk / Np, cop = kk - tap * Np;
    const int n = nperm_fwd(mp, unpad(cop, mp.nG, mp.nGr, mp.nGp)), ci = unpad(cip, mp.kG, mp.kGr, mp.kGp);
    return (n >= 0 && ci >= 0) ? src[((long)n * mp.K + ci) * 9 + tap] : 0.f;
  }
  int np, kp;
  if (kind == 0) { np = (int)(t / Kp); kp = (int)(t - (long)np * Kp); }
  else { kp = (int)(t / Np); np = (int)(t - (long)kp * Np); }
  const int n = nperm_fwd(mp, unpad(np, mp.nG, mp.nGr, mp.nGp)), k = unpad(kp, mp.kG, mp.kGr, mp.kGp);
  return (n >= 0 && k >= 0) ? src[(long)n * mp.K + k] : 0.f;
}

KAIR_DEV void pack_element(const float* __restrict__ src, void* __restrict__ dst, int dt, const kair_wmap& mp, long t) {
  if (mp.kind >= 17 && mp.kind <= 19) {   // hi/lo split rows: 64-column chunks alternate hi / lo
    int base;
    long rowlen, rows;
    split_rows(mp, &base, &rowlen, &rows);
    const long KS = 2 * ((rowlen + 63) / 64) * 64;
    const long row = t / KS;
    const long kk = t - row * KS;
    const int half = (int)((kk >> 6) & 1);
    const long k = ((kk >> 7) << 6) + (kk & 63);
    const float v = k < rowlen ? pack_value(src, mp, base, row * rowlen + k) : 0.f;
    if (dt == KAIR_F16) {   // x3 weights: the fp16 pair of w * 2^KAIR_X3_WEXP
      const float w = ldexpf(v, KAIR_X3_WEXP);
      const f16 hi = (f16)w;
      ((f16*)dst)[t] = half ? (f16)(w - (float)hi) : hi;
      return;
    }
    const bf16 hi = (bf16)v;
    ((bf16*)dst)[t] = half ? (bf16)(v - (float)hi) : hi;
    return;
  }
  const int Np = mp.nG * mp.nGp, Kp = mp.kG * mp.kGp;
  float v = 0.f;
  if (mp.kind == 0 || mp.kind == 3) {  // linear [Np][Kp] (or transposed [Kp][Np])
    int np, kp;
    if (mp.kind == 0) { np = (int)(t / Kp); kp = (int)(t - (long)np * Kp); }
    else { kp = (int)(t / Np); np = (int)(t - (long)kp * Np); }
    const int n = nperm_fwd(mp, unpad(np, mp.nG, mp.nGr, mp.nGp)), k = unpad(kp, mp.kG, mp.kGr, mp.kGp);
    if (n >= 0 && k >= 0) v = src[(long)n * mp.K + k];
  } else if (mp.kind == 1) {  // conv [Cop][9*Cip], k = tap*Cip + ci
    const int np = (int)(t / (9 * Kp));
    const int kk = (int)(t - (long)np * 9 * Kp);
    const int tap = kk / Kp, cip = kk - tap * Kp;
    const int n = nperm_fwd(mp, unpad(np, mp.nG, mp.nGr, mp.nGp)), ci = unpad(cip, mp.kG, mp.kGr, mp.kGp);
    if (n >= 0 && ci >= 0) v = src[((long)n * mp.K + ci % mp.K) * 9 + tap];   // % K: tied in-dim copies
  } else if (mp.kind == 2) {  // conv dgrad form [Cip][9*Cop], k = tap*Cop + co (loader negates taps)
    const int cip = (int)(t / (9 * Np));
    const int kk = (int)(t - (long)cip * 9 * Np);
    const int tap = kk / Np, cop = kk - tap * Np;
    const int n = nperm_fwd(mp, unpad(cop, mp.nG, mp.nGr, mp.nGp)), ci = unpad(cip, mp.kG, mp.kGr, mp.kGp);
    if (n >= 0 && ci >= 0) v = src[((long)n * mp.K + ci) * 9 + tap];
  } else if (mp.kind == 7) {  // conv2x2 [Np][4*Kp], k = tap*Kp + kp (stride-2 conv fwd / transposed-conv dgrad)
    const int np = (int)(t / (4 * Kp));
    const int kk = (int)(t - (long)np * 4 * Kp);
    const int tap = kk / Kp, kp = kk - tap * Kp;
    const int n = nperm_fwd(mp, unpad(np, mp.nG, mp.nGr, mp.nGp)), k = unpad(kp, mp.kG, mp.kGr, mp.kGp);
    if (n >= 0 && k >= 0) v = src[((long)n * mp.K + k) * 4 + tap];
  } else if (mp.kind == 9) {  // conv3x3 forward, hi/lo split: [Cop][KS], 64-col chunks alternate hi / lo
    const int Kc = 9 * Kp, KS = 2 * ((Kc + 63) / 64) * 64;
    const int np = (int)(t / KS);
    const int kk = (int)(t - (long)np * KS);
    const int half = (kk >> 6) & 1, k = ((kk >> 7) << 6) + (kk & 63);
    if (k < Kc) {
      const int tap = k / Kp, cip = k - tap * Kp;
      const int n = nperm_fwd(mp, unpad(np, mp.nG, mp.nGr, mp.nGp)), ci = unpad(cip, mp.kG, mp.kGr, mp.kGp);
      if (n >= 0 && ci >= 0) v = src[((long)n * mp.K + ci % mp.K) * 9 + tap];   // % K: tied in-dim copies
    }
    if (dt == KAIR_F16) {   // x3 weights: the fp16 pair of w * 2^KAIR_X3_WEXP
      const float w = ldexpf(v, KAIR_X3_WEXP);
      const f16 hf = (f16)w;
      ((f16*)dst)[t] = half ? (f16)(w - (float)hf) : hf;
      return;
    }
    const bf16 hi = (bf16)v;
    ((bf16*)dst)[t] = half ? (bf16)(v - (float)hi) : hi;
    return;
  } else if (mp.kind == 10) {  // linear in MFMA-fragment order: [Np/32][Kp/16][64 lanes][8]
    const int KB = Kp / 16;
    const int j = (int)(t & 7), ln = (int)((t >> 3) & 63);
    const long blk = t >> 9;
    const int kb = (int)(blk % KB), nb = (int)(blk / KB);
    const int np = nb * 32 + (ln & 31), kp = kb * 16 + 8 * (ln >> 5) + j;
    const int n = nperm_fwd(mp, unpad(np, mp.nG, mp.nGr, mp.nGp)), k = unpad(kp, mp.kG, mp.kGr, mp.kGp);
    if (n >= 0 && k >= 0) v = src[(long)n * mp.K + k];
  } else if (mp.kind == 13) {  // transposed linear in fragment order: [Kp/32][Np/16][64 lanes][8] of W^T
    const int KB = Np / 16;
    const int j = (int)(t & 7), ln = (int)((t >> 3) & 63);
    const long blk = t >> 9;
    const int kb = (int)(blk % KB), ob = (int)(blk / KB);
    const int kp = ob * 32 + (ln & 31), np = kb * 16 + 8 * (ln >> 5) + j;
    const int n = nperm_fwd(mp, unpad(np, mp.nG, mp.nGr, mp.nGp)), k = unpad(kp, mp.kG, mp.kGr, mp.kGp);
    if (n >= 0 && k >= 0) v = src[(long)n * mp.K + k];
  } else if (mp.kind == 14) {  // linear in v_mfma_f32_16x16x32 fragment order: [Np/16][Kp/32][64 lanes][8]
    const int KB = Kp / 32;
    const int j = (int)(t & 7), ln = (int)((t >> 3) & 63);
    const long blk = t >> 9;
    const int kb = (int)(blk % KB), nb = (int)(blk / KB);
    const int np = nb * 16 + (ln & 15), kp = kb * 32 + 8 * (ln >> 4) + j;
    const int n = nperm_fwd(mp, unpad(np, mp.nG, mp.nGr, mp.nGp)), k = unpad(kp, mp.kG, mp.kGr, mp.kGp);
    if (n >= 0 && k >= 0) v = src[(long)n * mp.K + k];
  } else if (mp.kind == 12) {  // linear, fragment order with hi/lo halves: [Np/32][Kp/16][2][64 lanes][8]
    const int KB = Kp / 16;
    const int j = (int)(t & 7), ln = (int)((t >> 3) & 63), half = (int)((t >> 9) & 1);
    const long blk = t >> 10;
    const int kb = (int)(blk % KB), nb = (int)(blk / KB);
    const int np = nb * 32 + (ln & 31), kp = kb * 16 + 8 * (ln >> 5) + j;
    const int n = nperm_fwd(mp, unpad(np, mp.nG, mp.nGr, mp.nGp)), k = unpad(kp, mp.kG, mp.kGr, mp.kGp);
    if (n >= 0 && k >= 0) v = src[(long)n * mp.K + k];
    const bf16 hi = (bf16)v;
    ((bf16*)dst)[t] = half ? (bf16)(v - (float)hi) : hi;
    return;
  } else if (mp.kind == 15) {  // conv3x3 forward in 16x16x32 fragment order, hi/lo halves: [Np/16][9*Kp/32][2][64][8]
    const int KB = 9 * Kp / 32;
    const int j = (int)(t & 7), ln = (int)((t >> 3) & 63), half = (int)((t >> 9) & 1);
    const long blk = t >> 10;
    const int kb = (int)(blk % KB), nb = (int)(blk / KB);
    const int np = nb * 16 + (ln & 15), kk = kb * 32 + 8 * (ln >> 4) + j;   // kk = tap * Kp + cip
    const int tap = kk / Kp, cip = kk - tap * Kp;
    const int n = nperm_fwd(mp, unpad(np, mp.nG, mp.nGr, mp.nGp)), ci = unpad(cip, mp.kG, mp.kGr, mp.kGp);
    if (n >= 0 && ci >= 0) v = src[((long)n * mp.K + ci % mp.K) * 9 + tap];
    const bf16 hi = (bf16)v;
    ((bf16*)dst)[t] = half ? (bf16)(v - (float)hi) : hi;
    return;
  } else if (mp.kind == 16) {  // conv3x3 input-gradient form (kind 2) in 16x16x32 fragment order:
                               // [Kp/16][9*Np/32][64][8], rows = input channels cip, k = tap*Np + cop
    const int KB = 9 * Np / 32;
    const int j = (int)(t & 7), ln = (int)((t >> 3) & 63);
    const long blk = t >> 9;
    const int kb = (int)(blk % KB), cb = (int)(blk / KB);
    const int cip = cb * 16 + (ln & 15), kk = kb * 32 + 8 * (ln >> 4) + j;
    const int tap = kk / Np, cop = kk - tap * Np;
    const int n = nperm_fwd(mp, unpad(cop, mp.nG, mp.nGr, mp.nGp)), ci = unpad(cip, mp.kG, mp.kGr, mp.kGp);
    if (n >= 0 && ci >= 0) v = src[((long)n * mp.K + ci) * 9 + tap];
  } else if (mp.kind == 8) {  // conv2x2 [4*Kp][Np], row = kp*4 + tap (pixel-shuffle forms)
    const int row = (int)(t / Np), np = (int)(t - (long)row * Np);
    const int kp = row >> 2, tap = row & 3;
    const int n = nperm_fwd(mp, unpad(np, mp.nG, mp.nGr, mp.nGp)), k = unpad(kp, mp.kG, mp.kGr, mp.kGp);
    if (n >= 0 && k >= 0) v = src[((long)n * mp.K + k) * 4 + tap];
  } else {  // bias vector
    const int n = nperm_fwd(mp, unpad((int)t, mp.nG, mp.nGr, mp.nGp));
    if (n >= 0) v = src[n];
  }
  if (dt == KAIR_BF16) ((bf16*)dst)[t] = (bf16)v;
  else ((float*)dst)[t] = v;
}

__global__ void pack_kernel(const float* __restrict__ src, void* __restrict__ dst, int dt, kair_wmap mp, long total) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < total) pack_element(src, dst, dt, mp, t);
}

// Chunked packing of the bf16 linear forms (kinds 0, 10, 13, 14): one thread makes 8 consecutive
// packed elements (one 16-byte store) and the threads of a wave walk the SOURCE in row order, so the
// fp32 master rows are read once and coalesced (the per-element gather re-fetched each source line
// from a different packed position: ~3-4x the bytes).  A chunk never straddles a padded group
// (group widths are multiples of 8), so its 8 elements are 8 consecutive packed indices.
__host__ __device__ inline bool pack_vec(const kair_wmap& mp, int dt) {
  if (dt != KAIR_BF16) return false;
  if (mp.kind == 0 || mp.kind == 10 || mp.kind == 14) return mp.kGp % 8 == 0 && (mp.kG * mp.kGp) % 8 == 0;
  if (mp.kind == 13) return mp.nGp % 8 == 0 && (mp.nG * mp.nGp) % 8 == 0;
  return false;
}

KAIR_DEV void pack_chunk(const float* __restrict__ src, bf16* __restrict__ dst, const kair_wmap& mp, long u) {
  const int Np = mp.nG * mp.nGp, Kp = mp.kG * mp.kGp;
  float v[8];
  long t0;
  if (mp.kind == 13) {   // 8 consecutive contraction rows np0.. of one output column kp
    const int kp = (int)(u % Kp), np0 = (int)(u / Kp) * 8;
    const int k = unpad(kp, mp.kG, mp.kGr, mp.kGp);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = nperm_fwd(mp, unpad(np0 + j, mp.nG, mp.nGr, mp.nGp));
      v[j] = (n >= 0 && k >= 0) ? src[(long)n * mp.K + k] : 0.f;
    }
    t0 = (((long)(kp >> 5) * (Np / 16) + (np0 >> 4)) * 64 + (kp & 31) + 32 * ((np0 & 15) >> 3)) * 8;
  } else {               // 8 consecutive columns kp0.. of one row np
    const int kc = Kp / 8;
    const int np = (int)(u / kc), kp0 = (int)(u % kc) * 8;
    const int n = nperm_fwd(mp, unpad(np, mp.nG, mp.nGr, mp.nGp));
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = unpad(kp0 + j, mp.kG, mp.kGr, mp.kGp);
      v[j] = (n >= 0 && k >= 0) ? src[(long)n * mp.K + k] : 0.f;
    }
    if (mp.kind == 0) t0 = (long)np * Kp + kp0;
    else if (mp.kind == 10) t0 = (((long)(np >> 5) * (Kp / 16) + (kp0 >> 4)) * 64 + (np & 31) + 32 * ((kp0 & 15) >> 3)) * 8;
    else t0 = (((long)(np >> 4) * (Kp / 32) + (kp0 >> 5)) * 64 + (np & 15) + 16 * ((kp0 & 31) >> 3)) * 8;
  }
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
  *(bf16x8*)(dst + t0) = o;
}

// Chunked packing of the split pair forms (kinds 9, 17, 18, 19; x3 fp16 pairs of w 2^KAIR_X3_WEXP or bf16 hi / lo):
// one thread makes 8 consecutive columns of one packed row -- its hi and lo halves, two 16-byte stores -- with 32-bit
// index math and the row's output channel / tap resolved once (the per-element form re-derived both per element in
// 64-bit divides, ~300 us for the classical x4 network's 47 M packed elements per step).  Row geometry: kind 9 rows
// Np of 9 Kp (tap-major), 17 rows Np of Kp, 18 rows Kp of 9 Np (tap-major), 19 rows Kp of Np; a chunk never straddles
// a tap (Kp / Np % 8 == 0, pack_pair_vec).
__host__ __device__ inline bool pack_pair_vec(const kair_wmap& mp, int dt) {
  if (dt != KAIR_F16 && dt != KAIR_BF16) return false;
  const int Np = mp.nG * mp.nGp, Kp = mp.kG * mp.kGp;
  if (mp.kind == 9 || mp.kind == 17) return Kp % 8 == 0;
  if (mp.kind == 18 || mp.kind == 19) return Np % 8 == 0;
  return false;
}

KAIR_DEV void pack_pair_chunk(const float* __restrict__ src, void* __restrict__ dst, int dt, const kair_wmap& mp, int u) {
  const int Np = mp.nG * mp.nGp, Kp = mp.kG * mp.kGp;
  const bool rows_n = mp.kind == 9 || mp.kind == 17;   // rows are output channels (else input channels)
  const int rowlen = mp.kind == 9 ? 9 * Kp : mp.kind == 17 ? Kp : mp.kind == 18 ? 9 * Np : Np;
  const int rl64 = (rowlen + 63) / 64 * 64, cpr = rl64 / 8;
  const int row = u / cpr, k0 = (u - row * cpr) * 8;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = 0.f;
  if (k0 < rowlen) {
    const int rr = rows_n ? nperm_fwd(mp, unpad(row, mp.nG, mp.nGr, mp.nGp)) : unpad(row, mp.kG, mp.kGr, mp.kGp);
    const int seg = (mp.kind == 9) ? Kp : (mp.kind == 18) ? Np : rowlen;   // tap-major forms: one tap per segment
    const int tap = k0 / seg, c0 = k0 - tap * seg;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      int n, k;
      if (rows_n) { n = rr; k = unpad(c, mp.kG, mp.kGr, mp.kGp); }
      else { n = nperm_fwd(mp, unpad(c, mp.nG, mp.nGr, mp.nGp)); k = rr; }
      if (n < 0 || k < 0) continue;
      if (mp.kind == 9) v[j] = src[((long)n * mp.K + k % mp.K) * 9 + tap];   // % K: tied in-dim copies
      else if (mp.kind == 18) v[j] = src[((long)n * mp.K + k) * 9 + tap];
      else v[j] = src[(long)n * mp.K + k];
    }
  }
  const long o = (long)row * 2 * rl64 + ((k0 >> 6) << 7) + (k0 & 63);
  if (dt == KAIR_F16) {
    f16x8 hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float w = ldexpf(v[j], KAIR_X3_WEXP);
      hi[j] = (f16)w;
      lo[j] = (f16)(w - (float)hi[j]);
    }
    *(f16x8*)((f16*)dst + o) = hi;
    *(f16x8*)((f16*)dst + o + 64) = lo;
  } else {
    bf16x8 hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      hi[j] = (bf16)v[j];
      lo[j] = (bf16)(v[j] - (float)hi[j]);
    }
    *(bf16x8*)((bf16*)dst + o) = hi;
    *(bf16x8*)((bf16*)dst + o + 64) = lo;
  }
}

// All packs of a network in one launch: table = kair_pack_job[njobs] followed by the first block
// of every job (long[njobs + 1]); each block finds its job by binary search (uniform, scalar loads).
// A chunked job (pack_vec) has total / 8 work items, a pair-chunked one (pack_pair_vec) total / 16, any other job
// one per packed element.
__global__ __launch_bounds__(256) void pack_batched_kernel(const kair_pack_job* __restrict__ jobs, int njobs,
                                                           const long* __restrict__ first) {
  const long bid = blockIdx.x;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (first[mid] <= bid) lo = mid;
    else hi = mid - 1;
  }
  const kair_pack_job& j = jobs[lo];
  const long t = (bid - first[lo]) * 256 + threadIdx.x;
  if (pack_vec(j.map, j.dst_dtype)) {
    if (t < j.total / 8) pack_chunk(j.src, (bf16*)j.dst, j.map, t);
  } else if (pack_pair_vec(j.map, j.dst_dtype)) {
    if (t < j.total / 16) pack_pair_chunk(j.src, j.dst, j.dst_dtype, j.map, (int)t);
  } else if (t < j.total) {
    pack_element(j.src, j.dst, j.dst_dtype, j.map, t);
  }
}

// 64 reference weight elements (+ bias elements) per 1024-thread block; 16 split phases per
// element, fixed summation order (deterministic).
__global__ __launch_bounds__(1024) void wgrad_finalize_kernel(const float* __restrict__ part, int splits, kair_wmap mp,
                                                              float* grad, float* bias_grad, int ones_col, int acc,
                                                              long nw, long Kt, long plane, int taps) {
  const long t = (long)blockIdx.x * 64 + (threadIdx.x & 63);
  const long nb = bias_grad ? mp.N : 0;
  const bool valid = t < nw + nb;
  long off = 0;
  if (valid) {
    if (t < nw) {
      if (mp.kind == 0) {
        const int n = (int)(t / mp.K), k = (int)(t - (long)n * mp.K);
        const int np = (n / mp.nGr) * mp.nGp + n % mp.nGr, kp = (k / mp.kGr) * mp.kGp + k % mp.kGr;
        off = (long)np * Kt + kp;
      } else {  // conv: grad[co][ci][tap] (3x3: 9 taps; 2x2: 4 taps)
        const int co = (int)(t / ((long)mp.K * taps));
        const int rem = (int)(t - (long)co * mp.K * taps);
        const int ci = rem / taps, tap = rem - (rem / taps) * taps;
        const int cq = nperm_inv(mp, co);
        const int np = (cq / mp.nGr) * mp.nGp + cq % mp.nGr;
        const int cip = (ci / mp.kGr) * mp.kGp + ci % mp.kGr;
        const int Cip = mp.kG * mp.kGp;
        off = (long)np * Kt + (long)tap * Cip + cip;
      }
    } else {
      const int n = nperm_inv(mp, (int)(t - nw));
      const int np = (n / mp.nGr) * mp.nGp + n % mp.nGr;
      off = (long)np * Kt + ones_col;
    }
  }
  const float s = split_sum16(part, splits, plane, off, valid);
  if (valid && threadIdx.x < 64) {
    float* o = t < nw ? grad + t : bias_grad + (t - nw);
    *o = acc ? *o + s : s;
  }
}

// Vectorised form: each block sums 64 float4 of the PACKED partial planes with 4 split-phases
// (fixed order, deterministic), then scatters the 4 sums to the reference layout — pad entries are
// dropped, the fused ones column goes to the bias gradient.  Needs N*K rows of whole float4s.
KAIR_DEV void finalize4_body(const float* __restrict__ part, int splits, const kair_wmap& mp, float* grad,
                             float* bias_grad, int ones_col, int acc, long Kt, long plane, int taps, long blk) {
  __shared__ float4 red[4][64];
  const int q = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const long e4 = blk * 64 + q;
  const bool valid = e4 * 4 < plane;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (valid) {
    // the ring TN kernel leaves up to 256 split planes: issue 8 plane loads per phase before adding
    // (a load-add chain waits out one memory latency per split); the sum order is unchanged
    const float4* p = (const float4*)part + e4;
    const long st = plane / 4;
    // (the last, partial batch too: a phase with 7 of 28 splits used to run 7 dependent round trips)
    for (int sp = ph; sp < splits; sp += 32) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int spu = sp + 4 * u < splits ? sp + 4 * u : splits - 1;   // clamped: every load issues
        v[u] = p[(long)spu * st];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (sp + 4 * u < splits) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
    }
  }
  red[ph][q] = s;
  __syncthreads();
  if (ph != 0 || !valid) return;
  const float4 a = red[0][q], b = red[1][q], c = red[2][q], d = red[3][q];
  const float t4[4] = {((a.x + b.x) + c.x) + d.x, ((a.y + b.y) + c.y) + d.y, ((a.z + b.z) + c.z) + d.z,
                       ((a.w + b.w) + c.w) + d.w};
  const int Cip = mp.kG * mp.kGp;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long pe = e4 * 4 + j;
    const int np = (int)(pe / Kt);
    const int kk = (int)(pe - (long)np * Kt);
    const int n = nperm_fwd(mp, unpad(np, mp.nG, mp.nGr, mp.nGp));
    if (n < 0) continue;
    float* o = nullptr;
    if (bias_grad && kk == ones_col) {
      o = bias_grad + n;
    } else {
      const int tap = taps == 1 ? 0 : kk / Cip;
      const int k = unpad(taps == 1 ? kk : kk - tap * Cip, mp.kG, mp.kGr, mp.kGp);
      if (k < 0) continue;
      o = grad + ((long)n * mp.K + k) * taps + tap;
    }
    *o = acc ? *o + t4[j] : t4[j];
  }
}

__global__ __launch_bounds__(256) void wgrad_finalize4_kernel(const float* __restrict__ part, int splits, kair_wmap mp,
                                                              float* grad, float* bias_grad, int ones_col, int acc,
                                                              long Kt, long plane, int taps) {
  finalize4_body(part, splits, mp, grad, bias_grad, ones_col, acc, Kt, plane, taps, blockIdx.x);
}

// every job of a kair_wgrad_grouped launch: block -> job by a scalar scan of the first blocks
__global__ __launch_bounds__(256) void wgrad_finalize_grouped_kernel(const FinGroup g) {
  const long b = blockIdx.x;
  int ji = 0;
  for (int i = 1; i < g.njobs; ++i)
    if (g.j[i].blk0 <= b) ji = i;
  ji = __builtin_amdgcn_readfirstlane(ji);
  const FinJob& jb = g.j[ji];
  finalize4_body(jb.part, g.splits, jb.mp, jb.grad, jb.bias, jb.ones_col, 0, jb.Kt, jb.plane, 1, b - jb.blk0);
}

// dst[token_to_win(t)] = scale(t) * src[t] (cast), 4 columns per thread
template <typename T>
__global__ void row_copy_kernel(const float* __restrict__ src, long lds, T* __restrict__ dst, long ldd,
                                const float* __restrict__ scale, int rps, WinMap wm, long M, int C4) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C4) return;
  const long t = i / C4;
  const int c = (int)(i - t * C4) * 4;
  const float4 v = *(const float4*)(src + t * lds + c);
  const float sc = scale ? scale[t / rps] : 1.f;
  T* o = dst + token_to_win(t, wm) * ldd + c;
  if constexpr (sizeof(T) == 2) {
    bf16x4 q = {(bf16)(sc * v.x), (bf16)(sc * v.y), (bf16)(sc * v.z), (bf16)(sc * v.w)};
    *(bf16x4*)o = q;
  } else {
    *(float4*)o = make_float4(sc * v.x, sc * v.y, sc * v.z, sc * v.w);
  }
}

// the x3 fp16-pair form: hi / lo planes of scale(t) * src[t] * 2^e
__global__ void row_copy_pair_kernel(const float* __restrict__ src, long lds, f16* __restrict__ hi, f16* __restrict__ lo,
                                     long ldd, const float* __restrict__ scale, int rps, WinMap wm, long M, int C4, float es) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C4) return;
  const long t = i / C4;
  const int c = (int)(i - t * C4) * 4;
  const float4 v = *(const float4*)(src + t * lds + c);
  const float sc = (scale ? scale[t / rps] : 1.f) * es;
  const float w[4] = {opaque(sc * v.x), opaque(sc * v.y), opaque(sc * v.z), opaque(sc * v.w)};   // (common.h opaque)
  f16x4 h, l;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    h[j] = (f16)w[j];
    l[j] = (f16)(w[j] - (float)h[j]);
  }
  const long o = token_to_win(t, wm) * ldd + c;
  *(f16x4*)(hi + o) = h;
  *(f16x4*)(lo + o) = l;
}

template <typename T>
__global__ void colsum_partial(const T* __restrict__ g, long ld, long M, int Np, float* __restrict__ ws, long rows_per) {
  const int c = blockIdx.y * blockDim.x + threadIdx.x;
  if (c >= Np) return;
  const long r0 = (long)blockIdx.x * rows_per;
  long r1 = r0 + rows_per;
  if (r1 > M) r1 = M;
  float s = 0.f;
  for (long r = r0; r < r1; ++r) s += (float)g[r * ld + c];
  ws[(long)blockIdx.x * Np + c] = s;
}

// Vectorised partial column sums (Np % 8 == 0, Np <= 256, 16-byte aligned rows): Np/8 lanes cover
// a row with 16-byte loads, 256/(Np/8) row phases run in parallel (4 rows in flight per thread),
// then the phases are added in fixed order through LDS (deterministic).
template <typename T>
__global__ __launch_bounds__(256) void colsum_partial_v(const T* __restrict__ g, long ld, long M, int Np,
                                                        float* __restrict__ ws, long rows_per) {
  __shared__ float red[256 * 8];
  const int cpr = Np >> 3, rp = 256 / cpr;
  const int cg = threadIdx.x % cpr, ph = threadIdx.x / cpr;
  const long r0 = (long)blockIdx.x * rows_per;
  long r1 = r0 + rows_per;
  if (r1 > M) r1 = M;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto add = [&](long r) {
    if constexpr (sizeof(T) == 2) {
      const bf16x8 q = *(const bf16x8*)(g + r * ld + cg * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += (float)q[j];
    } else {
      const float4 a = *(const float4*)(g + r * ld + cg * 8), b = *(const float4*)(g + r * ld + cg * 8 + 4);
      s[0] += a.x; s[1] += a.y; s[2] += a.z; s[3] += a.w; s[4] += b.x; s[5] += b.y; s[6] += b.z; s[7] += b.w;
    }
  };
  if (ph < rp) {
    long r = r0 + ph;
    for (; r + 3 * rp < r1; r += 4 * rp) {   // four independent rows in flight, summed in row order
      add(r); add(r + rp); add(r + 2 * rp); add(r + 3 * rp);
    }
    for (; r < r1; r += rp) add(r);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = s[j];
  __syncthreads();
  if (threadIdx.x < Np) {
    const int c = threadIdx.x, cgc = c >> 3, j = c & 7;
    float t = 0.f;
    for (int p = 0; p < rp; ++p) t += red[(p * cpr + cgc) * 8 + j];
    ws[(long)blockIdx.x * Np + c] = t;
  }
}

// 8 columns per 256-thread block, 32 block-phases per column with 8 partial loads in flight per
// thread, phases combined in a fixed order (deterministic).  (A 4-phase form summed 128 partials
// per thread one dependent load at a time: 30 us per conv bias gradient, latency-bound.)
__global__ __launch_bounds__(256) void colsum_final(const float* __restrict__ ws, int nb, int Np, kair_wmap mp, float* out,
                                                    int acc) {
  __shared__ float red[32][8];
  const int tx = threadIdx.x & 7, ty = threadIdx.x >> 3;
  const int n = blockIdx.x * 8 + tx;
  const bool ok = n < mp.N;
  const int nq = ok ? nperm_inv(mp, n) : 0;
  const int np = ok ? (nq / mp.nGr) * mp.nGp + nq % mp.nGr : 0;
  float s = 0.f;
  if (ok) {
    int b = ty;
    for (; b + 7 * 32 < nb; b += 8 * 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ws[(long)(b + 32 * u) * Np + np];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; b < nb; b += 32) s += ws[(long)b * Np + np];
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && ok) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) t += red[k][tx];
    out[n] = acc ? out[n] + t : t;
  }
}

template <typename T>
__global__ void image_to_nhwc_kernel(const float* __restrict__ img, T* __restrict__ out, int ldc,
                                     const float* __restrict__ mean, float range, int C, long HW, long total) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const long pix = t / ldc;
  const int c = (int)(t - pix * ldc);
  float v = 0.f;
  if (c < C) {
    const long b = pix / HW, p = pix - b * HW;
    v = (img[(b * C + c) * HW + p] - (mean ? mean[c] : 0.f)) * range;
  }
  out[t] = (T)v;
}

// hi/lo input split: channel c < C holds bf16(v), channel ldc/2 + c holds bf16(v - bf16(v)) (the
// conv_first weights are packed tied over both halves, so the product sees v to ~16 bits)
__global__ void image_to_nhwc_hilo_kernel(const float* __restrict__ img, bf16* __restrict__ out, int ldc,
                                          const float* __restrict__ mean, float range, int C, long HW, long total) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const long pix = t / ldc;
  const int c = (int)(t - pix * ldc), half = ldc / 2;
  const int cc = c < half ? c : c - half;
  float v = 0.f;
  if (cc < C) {
    const long b = pix / HW, p = pix - b * HW;
    v = (img[(b * C + cc) * HW + p] - (mean ? mean[cc] : 0.f)) * range;
  }
  const bf16 hi = (bf16)v;
  out[t] = c < half ? hi : (bf16)(v - (float)hi);
}

// I: index type (int when every index fits: 32-bit divisions are a fraction of the 64-bit ones)
// CH: Charbonnier (models/loss.py:208-218) sqrt(d^2 + eps) with gradient d / sqrt(d^2 + eps), else L1
template <typename T, typename I, bool CH>
__global__ void l1_kernel(const float* __restrict__ E, const float* __restrict__ H, T* __restrict__ dE, int ldc, int r,
                          float gscale, int C, int Hh, int Ww, long npix, float* __restrict__ ws, float eps) {
  // dE element t = (pixel of the [Hh/r, Ww/r] grid, channel slot); slot -> (c, i, j) when r > 1
  __shared__ float red[256];
  float s = 0.f;
  const I total = (I)(npix * ldc);
  const int hs = Hh / r, wsm = Ww / r, r2 = r * r;
  const I HW = (I)Hh * Ww;
  for (I t = (I)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (I)gridDim.x * blockDim.x) {
    const I pix = t / ldc;
    const int slot = (int)(t - pix * ldc);
    const int c = slot / r2, ij = slot - c * r2;
    float g = 0.f;
    if (c < C) {
      const I b = pix / ((I)hs * wsm);
      const int pp = (int)(pix - b * hs * wsm);
      const int y = (pp / wsm) * r + ij / r, x = (pp % wsm) * r + ij % r;
      const I i = (b * C + c) * HW + (I)y * Ww + x;
      const float d = E[i] - H[i];
      if constexpr (CH) {
        const float q = sqrtf(d * d + eps);
        s += q;
        g = q > 0.f ? gscale * d / q : 0.f;
      } else {
        s += fabsf(d);
        g = d > 0.f ? gscale : (d < 0.f ? -gscale : 0.f);
      }
    }
    dE[t] = (T)g;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) ws[blockIdx.x] = red[0];
}

// the same loss and gradient for the usual layout (r = 1, 16 bf16 slots per pixel, C <= 4): one thread per
// pixel -- its C channel reads coalesced across the wave (NCHW planes), its 16 slots stored as two 16-byte
// pieces -- instead of one thread per slot (16 threads per pixel, plane-strided reads, 2-byte stores)
template <bool CH>
__global__ void l1_pix16_kernel(const float* __restrict__ E, const float* __restrict__ H, bf16* __restrict__ dE,
                                float gscale, int C, int HW, int npix, float* __restrict__ ws, float eps) {
  __shared__ float red[256];
  float s = 0.f;
  for (int pix = blockIdx.x * blockDim.x + threadIdx.x; pix < npix; pix += gridDim.x * blockDim.x) {
    const int b = pix / HW, pp = pix - b * HW;
    bf16x8 g0 = {}, g1 = {};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c >= C) break;
      const long i = ((long)b * C + c) * HW + pp;
      const float d = E[i] - H[i];
      float g;
      if constexpr (CH) {
        const float q = sqrtf(d * d + eps);
        s += q;
        g = q > 0.f ? gscale * d / q : 0.f;
      } else {
        s += fabsf(d);
        g = d > 0.f ? gscale : (d < 0.f ? -gscale : 0.f);
      }
      g0[c] = (bf16)g;
    }
    uint4* o = (uint4*)(dE + (long)pix * 16);
    o[0] = __builtin_bit_cast(uint4, g0);
    o[1] = __builtin_bit_cast(uint4, g1);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) ws[blockIdx.x] = red[0];
}

// fp32 gradient rows of 4 slots per pixel (C <= 4; the fp32x3 engine's conv_last narrow kernels read 4 channels):
// one thread per pixel, one 16-byte store
template <bool CH>
__global__ void l1_pix4f_kernel(const float* __restrict__ E, const float* __restrict__ H, float* __restrict__ dE,
                                float gscale, int C, int HW, int npix, float* __restrict__ ws, float eps) {
  __shared__ float red[256];
  float s = 0.f;
  for (int pix = blockIdx.x * blockDim.x + threadIdx.x; pix < npix; pix += gridDim.x * blockDim.x) {
    const int b = pix / HW, pp = pix - b * HW;
    float g4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c >= C) break;
      const long i = ((long)b * C + c) * HW + pp;
      const float d = E[i] - H[i];
      if constexpr (CH) {
        const float q = sqrtf(d * d + eps);
        s += q;
        g4[c] = q > 0.f ? gscale * d / q : 0.f;
      } else {
        s += fabsf(d);
        g4[c] = d > 0.f ? gscale : (d < 0.f ? -gscale : 0.f);
      }
    }
    *(float4*)(dE + (long)pix * 4) = make_float4(g4[0], g4[1], g4[2], g4[3]);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) ws[blockIdx.x] = red[0];
}

__global__ void l1_final(const float* __restrict__ ws, int nb, float scale, float* out) {
  __shared__ float red[256];
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += 256) s += ws[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0] * scale;
}

// fp32x3 range guard (kair_range_check): flag |= 1 for a non-finite gradient, 2 for a non-finite loss, 4 for a
// parameter outside [-p_limit, p_limit] (the fp16 window of the x3 weight packs) or non-finite.  A split operand
// that leaves fp16's range becomes inf in its hi half and NaN/inf in every product it enters, so one pass over the
// step's gradients sees it wherever it happened (forward activations reach the weight gradients through the wgrad
// products).  One atomic OR per workgroup that found something (vector atomic; none on a clean step).
__global__ void range_check_kernel(const float* __restrict__ g, const float* __restrict__ p, long n,
                                   const float* __restrict__ loss, float p_limit, unsigned* __restrict__ flag) {
  unsigned bits = 0;
  const long n4 = n / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 gv = ((const float4*)g)[i];
    const float4 pv = ((const float4*)p)[i];
    // (x - x) is 0 for finite x and NaN for inf / NaN: one test per four values
    const float gs = (gv.x - gv.x) + (gv.y - gv.y) + (gv.z - gv.z) + (gv.w - gv.w);
    if (gs != 0.f) bits |= 1u;
    const float pm = fmaxf(fmaxf(fabsf(pv.x), fabsf(pv.y)), fmaxf(fabsf(pv.z), fabsf(pv.w)));
    if (!(pm < p_limit)) bits |= 4u;   // (NaN compares false)
  }
  for (long i = n4 * 4 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    if (g[i] - g[i] != 0.f) bits |= 1u;
    if (!(fabsf(p[i]) < p_limit)) bits |= 4u;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && loss && loss[0] - loss[0] != 0.f) bits |= 2u;
  __shared__ unsigned red;
  if (threadIdx.x == 0) red = 0;
  __syncthreads();
  if (bits) atomicOr(&red, bits);
  __syncthreads();
  if (threadIdx.x == 0 && red) atomicOr(flag, red);
}

// lr_t[0] = step_size = lr / (1 - b1^t),  lr_t[1] = sqrt(1 - b2^t);  skip: a range-guard flag -- nonzero: the
// step is dropped (parameters, moments and EMA untouched), as torch's GradScaler skips an inf step
__global__ void adam_ema_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                float* __restrict__ v, float* __restrict__ ema, long n, const float* __restrict__ lr_t,
                                float b1, float b2, float eps, float wd, float decay, const unsigned* __restrict__ skip) {
  if (skip && *skip) return;
  const float step = lr_t[0], bc2s = lr_t[1];
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float gi = g[i];
    float pi = p[i];
    if (wd != 0.f) gi = gi + wd * pi;
    float mi = m[i];
    mi = mi + (1.f - b1) * (gi - mi);  // lerp_(g, 1-b1)
    float vi = v[i] * b2;
    vi = vi + (1.f - b2) * (gi * gi);   // mul_(b2).addcmul_(g, g, 1-b2)
    const float denom = sqrtf(vi) / bc2s + eps;
    pi = pi + (-step) * (mi / denom);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
    if (ema) ema[i] = ema[i] * decay + (1.f - decay) * pi;
  }
}

__global__ void axpy_kernel(float* __restrict__ y, const float* __restrict__ x, float a, long n) {
  const long n4 = n / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 yv = ((float4*)y)[i];
    const float4 xv = ((const float4*)x)[i];
    yv.x += a * xv.x; yv.y += a * xv.y; yv.z += a * xv.z; yv.w += a * xv.w;
    ((float4*)y)[i] = yv;
  }
  for (long i = n4 * 4 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] += a * x[i];
}

__global__ void axpby_kernel(float* __restrict__ y, const float* __restrict__ x, float a, float b, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = a * x[i] + b * y[i];
}

__global__ void axpby_rows_kernel(float* __restrict__ y, long ldy, const float* __restrict__ x, long ldx, long M, int C,
                                  float a, float b) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C) return;
  const long m = i / C;
  const int c = (int)(i - m * C);
  float* o = y + m * ldy + c;
  *o = a * x[m * ldx + c] + b * *o;
}

template <typename TX, typename TO>
__global__ void act_grad_cast_kernel(const float* __restrict__ G, long ldg, const TX* __restrict__ X, long ldx,
                                     TO* __restrict__ out, long ldo, long M, int C, int kind, float slope, float scale) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C) return;
  const long m = i / C;
  const int c = (int)(i - m * C);
  float g = G[m * ldg + c] * scale;
  if (kind == 3) {
    g *= gelu_erf_grad((float)X[m * ldx + c]);   // X = pre-activation (nn.GELU backward)
  } else if (kind) {
    const float xv = (float)X[m * ldx + c];
    g = xv > 0.f ? g : (kind == 2 ? g * slope : 0.f);
  }
  out[m * ldo + c] = (TO)g;
}

__global__ void sumpool2x_kernel(const float* __restrict__ src, long lds, float* __restrict__ dst, long ldd, int B, int H,
                                 int W, int C, int acc) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)B * H * W * C;
  if (i >= total) return;
  const int c = (int)(i % C);
  const long pix = i / C;
  const int x = (int)(pix % W);
  const long by = pix / W;
  const int y = (int)(by % H);
  const long b = by / H;
  const long r0 = (b * 2 * H + 2 * y) * (2L * W) + 2 * x;
  const float s = src[r0 * lds + c] + src[(r0 + 1) * lds + c] + src[(r0 + 2L * W) * lds + c] +
                  src[(r0 + 2L * W + 1) * lds + c];
  float* o = dst + pix * ldd + c;
  *o = acc ? *o + s : s;
}

inline unsigned nblk(long n, int bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

static int pack_total(const kair_wmap& mp, int dst_dtype, long* total) {
  KAIR_CHECK_ARG((mp.kind != 12 && mp.kind != 15) || dst_dtype == KAIR_BF16,
                 "pack_weight: the hi/lo split forms 12 / 15 are bf16 only");
  KAIR_CHECK_ARG(mp.kind != 9 || dst_dtype == KAIR_BF16 || dst_dtype == KAIR_F16,
                 "pack_weight: kind 9 is a bf16 or (x3) fp16 pair form");
  KAIR_CHECK_ARG(dst_dtype == KAIR_F32 || dst_dtype == KAIR_BF16 || ((mp.kind == 9 || (mp.kind >= 17 && mp.kind <= 19)) &&
                                                                     dst_dtype == KAIR_F16),
                 "pack_weight: fp16 destinations are the x3 pair forms (kinds 9, 17, 18, 19)");
  KAIR_CHECK_ARG(mp.nG > 0 && mp.nGr > 0 && mp.nGp >= mp.nGr && mp.nG * mp.nGr == mp.N, "pack_weight: bad N map");
  // kinds 1 / 9 (conv forward) may repeat the in dim (kG * kGr a multiple of K: tied copies, e.g. the
  // hi / lo halves of a split input image); every other kind maps it one to one
  KAIR_CHECK_ARG(mp.kind == 4 ||
                     (mp.kG > 0 && mp.kGr > 0 && mp.kGp >= mp.kGr &&
                      (mp.kG * mp.kGr == mp.K ||
                       ((mp.kind == 1 || mp.kind == 9 || mp.kind == 15) && mp.K > 0 && (mp.kG * mp.kGr) % mp.K == 0))),
                 "pack_weight: bad K map");
  KAIR_CHECK_ARG(mp.n_perm <= 1 || (mp.nG == 1 && mp.N % mp.n_perm == 0), "pack_weight: n_perm needs nG == 1, N %% n_perm == 0");
  const long Np = (long)mp.nG * mp.nGp, Kp = (long)mp.kG * mp.kGp;
  KAIR_CHECK_ARG((mp.kind != 10 && mp.kind != 12) || (Np % 32 == 0 && Kp % 16 == 0),
                 "pack_weight: fragment order needs Np %% 32 == 0, Kp %% 16 == 0");
  KAIR_CHECK_ARG(mp.kind != 13 || (Kp % 32 == 0 && Np % 16 == 0), "pack_weight: transposed fragment order needs Kp %% 32 == 0, Np %% 16 == 0");
  KAIR_CHECK_ARG(mp.kind != 14 || (Np % 16 == 0 && Kp % 32 == 0), "pack_weight: 16x16x32 fragment order needs Np %% 16 == 0, Kp %% 32 == 0");
  KAIR_CHECK_ARG(mp.kind != 15 || (Np % 16 == 0 && (9 * Kp) % 32 == 0), "pack_weight: kind 15 needs Np %% 16 == 0, 9 Kp %% 32 == 0");
  KAIR_CHECK_ARG(mp.kind != 16 || (Kp % 16 == 0 && (9 * Np) % 32 == 0), "pack_weight: kind 16 needs Kp %% 16 == 0, 9 Np %% 32 == 0");
  if (mp.kind >= 17 && mp.kind <= 19) {   // hi/lo split rows of kinds 0 / 2 / 3
    KAIR_CHECK_ARG(dst_dtype == KAIR_BF16 || dst_dtype == KAIR_F16, "pack_weight: kinds 17-19 are bf16 / fp16 pairs");
    int base;
    long rowlen, rows;
    split_rows(mp, &base, &rowlen, &rows);
    *total = rows * 2 * ((rowlen + 63) / 64) * 64;
    return 0;
  }
  if (mp.kind == 0 || mp.kind == 3 || mp.kind == 10 || mp.kind == 13 || mp.kind == 14) *total = Np * Kp;
  else if (mp.kind == 12) *total = 2 * Np * Kp;
  else if (mp.kind == 1 || mp.kind == 2 || mp.kind == 16) *total = Np * 9 * Kp;
  else if (mp.kind == 7 || mp.kind == 8) *total = Np * 4 * Kp;
  else if (mp.kind == 9) *total = Np * 2 * ((9L * Kp + 63) / 64) * 64;
  else if (mp.kind == 15) *total = 2 * Np * 9 * Kp;
  else if (mp.kind == 4) *total = Np;
  else return kair_set_error(KAIR_ERR_ARG, "pack_weight: bad kind %d", mp.kind);
  return 0;
}

extern "C" int kair_pack_weight(const float* src, void* dst, int dst_dtype, const kair_wmap* map, void* stream) {
  KAIR_CHECK_ARG(src && dst && map, "pack_weight: null pointer");
  long total;
  if (int rc = pack_total(*map, dst_dtype, &total)) return rc;
  KAIR_LAUNCH(pack_kernel, dim3(nblk(total, 256)), dim3(256), 0, (hipStream_t)stream, src, dst, dst_dtype, *map,
                     total);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" long kair_pack_table_bytes(int njobs) {
  return (long)njobs * (long)sizeof(kair_pack_job) + (long)(njobs + 1) * (long)sizeof(long);
}

extern "C" long kair_pack_table_build(kair_pack_job* jobs, int njobs, void* table_dev) {
  KAIR_CHECK_ARG(jobs && table_dev && njobs > 0, "pack_table_build: bad args");
  const size_t jb = (size_t)njobs * sizeof(kair_pack_job);
  char* host = (char*)malloc(jb + (size_t)(njobs + 1) * sizeof(long));
  if (!host) return kair_set_error(KAIR_ERR_ARG, "pack_table_build: out of host memory");
  long* first = (long*)(host + jb);
  long nb = 0;
  for (int i = 0; i < njobs; ++i) {
    long total;
    int rc = jobs[i].src && jobs[i].dst ? pack_total(jobs[i].map, jobs[i].dst_dtype, &total)
                                        : kair_set_error(KAIR_ERR_ARG, "pack_table_build: job %d null pointer", i);
    if (rc) { free(host); return rc; }
    jobs[i].total = total;
    first[i] = nb;
    const long items = pack_vec(jobs[i].map, jobs[i].dst_dtype) ? total / 8
                       : pack_pair_vec(jobs[i].map, jobs[i].dst_dtype) ? total / 16 : total;
    if (items >= (1L << 31)) { free(host); return kair_set_error(KAIR_ERR_ARG, "pack_table_build: job %d too large", i); }
    nb += (items + 255) / 256;
  }
  first[njobs] = nb;
  memcpy(host, jobs, jb);
  const hipError_t e = hipMemcpy(table_dev, host, jb + (size_t)(njobs + 1) * sizeof(long), hipMemcpyHostToDevice);
  free(host);
  if (e != hipSuccess) return kair_set_error(KAIR_ERR_HIP, "pack_table_build: %s", hipGetErrorString(e));
  return nb;
}

extern "C" int kair_pack_weights(const void* table_dev, int njobs, long nblocks, void* stream) {
  KAIR_CHECK_ARG(table_dev && njobs > 0 && nblocks > 0, "pack_weights: bad args");
  const kair_pack_job* jobs = (const kair_pack_job*)table_dev;
  const long* first = (const long*)((const char*)table_dev + (size_t)njobs * sizeof(kair_pack_job));
  KAIR_LAUNCH(pack_batched_kernel, dim3((unsigned)nblocks), dim3(256), 0, (hipStream_t)stream, jobs, njobs, first);
  KAIR_CHECK_LAUNCH();
  return 0;
}

int kair_launch_finalize_grouped(const FinGroup& g, hipStream_t s) {
  KAIR_LAUNCH(wgrad_finalize_grouped_kernel, dim3((unsigned)g.nblocks), dim3(256), 0, s, g);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_wgrad_finalize(const float* partial, int splits, const kair_wmap* map, float* grad_ref,
                                   float* bias_grad, int ones_col, int accumulate, void* stream) {
  KAIR_CHECK_ARG(partial && map && grad_ref && splits > 0, "wgrad_finalize: null pointer");
  const kair_wmap& mp = *map;
  KAIR_CHECK_ARG(mp.kind == 0 || mp.kind == 1 || mp.kind == 7,
                 "wgrad_finalize: kind must be 0 (linear), 1 (conv3x3) or 7 (conv2x2)");
  KAIR_CHECK_ARG(!bias_grad || ones_col >= 0, "wgrad_finalize: bias needs ones_col");
  KAIR_CHECK_ARG(mp.n_perm <= 1 || (mp.nG == 1 && mp.N % mp.n_perm == 0), "wgrad_finalize: n_perm needs nG == 1");
  const int taps = mp.kind == 0 ? 1 : (mp.kind == 1 ? 9 : 4);
  const long Np = (long)mp.nG * mp.nGp;
  const long Kt = (long)taps * mp.kG * mp.kGp;
  const long nw = (long)mp.N * mp.K * taps;
  const long tot = nw + (bias_grad ? mp.N : 0);
  if ((Np * Kt) % 4 == 0 && ((uintptr_t)partial % 16) == 0) {
    KAIR_LAUNCH(wgrad_finalize4_kernel, dim3(nblk(Np * Kt / 4, 64)), dim3(256), 0, (hipStream_t)stream, partial,
                       splits, mp, grad_ref, bias_grad, ones_col, accumulate, Kt, Np * Kt, taps);
  } else {
    KAIR_LAUNCH(wgrad_finalize_kernel, dim3(nblk(tot, 64)), dim3(1024), 0, (hipStream_t)stream, partial, splits, mp,
                       grad_ref, bias_grad, ones_col, accumulate, nw, Kt, Np * Kt, taps);
  }
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_row_copy(const float* src, long lds, long M, int C, const kair_copy_desc* copy, void* stream) {
  KAIR_CHECK_ARG(src && copy && copy->out && M > 0 && C > 0, "row_copy: bad args");
  KAIR_CHECK_ARG(C % 4 == 0 && lds % 4 == 0 && copy->ld % 4 == 0, "row_copy: widths must be multiples of 4");
  KAIR_CHECK_ARG(M < KAIR_MAX_MAPPED_ROWS, "row_copy: M must be < 2^24");
  KAIR_CHECK_ARG(copy->win_ws == 0 || (copy->win_H % copy->win_ws == 0 && copy->win_W % copy->win_ws == 0),
                 "row_copy: window geometry");
  const WinMap wm = make_winmap(copy->win_H, copy->win_W, copy->win_ws, copy->win_shift);
  const int rps = copy->rows_per_scale > 0 ? copy->rows_per_scale : 1;
  const long n = M * (C / 4);
  hipStream_t s = (hipStream_t)stream;
  if (copy->dtype == KAIR_F16) {
    KAIR_CHECK_ARG(copy->out_lo && ((uintptr_t)copy->out % 8) == 0 && ((uintptr_t)copy->out_lo % 8) == 0,
                   "row_copy: an fp16 pair copy needs its 8-byte aligned lo plane (out_lo)");
    KAIR_LAUNCH(row_copy_pair_kernel, dim3(nblk(n, 256)), dim3(256), 0, s, src, lds, (f16*)copy->out,
                       (f16*)copy->out_lo, copy->ld, copy->rowscale, rps, wm, M, C / 4, ldexpf(1.f, copy->x3_exp));
  } else if (copy->dtype == KAIR_BF16)
    KAIR_LAUNCH(row_copy_kernel<bf16>, dim3(nblk(n, 256)), dim3(256), 0, s, src, lds, (bf16*)copy->out, copy->ld,
                       copy->rowscale, rps, wm, M, C / 4);
  else
    KAIR_LAUNCH(row_copy_kernel<float>, dim3(nblk(n, 256)), dim3(256), 0, s, src, lds, (float*)copy->out, copy->ld,
                       copy->rowscale, rps, wm, M, C / 4);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_colsum(const kair_operand* G, long M, int Np, const kair_wmap* map, float* bias_grad, float* ws,
                           int accumulate, void* stream) {
  KAIR_CHECK_ARG(G && G->ptr && map && bias_grad && ws, "colsum: null pointer");
  KAIR_CHECK_ARG(G->mode == KAIR_LD_ROWS && G->win_ws == 0, "colsum: plain row operands only");
  const int nb = 512;
  const long rows_per = (M + nb - 1) / nb;
  dim3 grid(nb, (Np + 255) / 256);
  hipStream_t s = (hipStream_t)stream;
  const bool vec = Np % 8 == 0 && Np <= 256 && G->ld % 8 == 0 && ((uintptr_t)G->ptr & 15) == 0;
  if (vec && G->dtype == KAIR_BF16)
    KAIR_LAUNCH(colsum_partial_v<bf16>, dim3(nb), dim3(256), 0, s, (const bf16*)G->ptr, G->ld, M, Np, ws, rows_per);
  else if (vec)
    KAIR_LAUNCH(colsum_partial_v<float>, dim3(nb), dim3(256), 0, s, (const float*)G->ptr, G->ld, M, Np, ws, rows_per);
  else if (G->dtype == KAIR_BF16)
    KAIR_LAUNCH(colsum_partial<bf16>, grid, dim3(256), 0, s, (const bf16*)G->ptr, G->ld, M, Np, ws, rows_per);
  else
    KAIR_LAUNCH(colsum_partial<float>, grid, dim3(256), 0, s, (const float*)G->ptr, G->ld, M, Np, ws, rows_per);
  KAIR_CHECK_LAUNCH();
  KAIR_LAUNCH(colsum_final, dim3(nblk(map->N, 8)), dim3(256), 0, s, ws, nb, Np, *map, bias_grad, accumulate);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_image_to_nhwc(const float* img, void* out, int dtype, int ldc, const float* mean, float img_range,
                                  int B, int C, int H, int W, void* stream) {
  KAIR_CHECK_ARG(img && out && ldc >= C, "image_to_nhwc: bad args");
  const long total = (long)B * H * W * ldc;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == KAIR_BF16)
    KAIR_LAUNCH(image_to_nhwc_kernel<bf16>, dim3(nblk(total, 256)), dim3(256), 0, s, img, (bf16*)out, ldc, mean,
                       img_range, C, (long)H * W, total);
  else
    KAIR_LAUNCH(image_to_nhwc_kernel<float>, dim3(nblk(total, 256)), dim3(256), 0, s, img, (float*)out, ldc, mean,
                       img_range, C, (long)H * W, total);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_image_to_nhwc_hilo(const float* img, void* out, int ldc, const float* mean, float img_range, int B,
                                       int C, int H, int W, void* stream) {
  KAIR_CHECK_ARG(img && out && ldc % 2 == 0 && 2 * C <= ldc, "image_to_nhwc_hilo: needs 2 * C <= ldc (even)");
  const long total = (long)B * H * W * ldc;
  KAIR_LAUNCH(image_to_nhwc_hilo_kernel, dim3(nblk(total, 256)), dim3(256), 0, (hipStream_t)stream, img, (bf16*)out,
                     ldc, mean, img_range, C, (long)H * W, total);
  KAIR_CHECK_LAUNCH();
  return 0;
}

static int pixel_loss(const float* E, const float* H, float* loss_out, void* dE, int dtype, int ldc, int ps_r, float weight,
                      float eps, bool charb, int B, int C, int Hh, int Ww, float* ws, void* stream) {
  KAIR_CHECK_ARG(E && H && loss_out && dE && ws && ps_r >= 1 && ldc >= C * ps_r * ps_r, "pixel loss: bad args");
  KAIR_CHECK_ARG(Hh % ps_r == 0 && Ww % ps_r == 0, "pixel loss: image not divisible by r");
  const long npix = (long)B * (Hh / ps_r) * (Ww / ps_r);
  const double numel = (double)B * Hh * Ww * C;
  const int nb = 1024;
  hipStream_t s = (hipStream_t)stream;
  const float gs = (float)(weight / numel);
  // int indices when the largest index (dE element or image element) and the grid stride fit
  const bool i32 = (double)npix * ldc < 2.0e9 && numel < 2.0e9;
  const bool pix4f = ps_r == 1 && ldc == 4 && C <= 4 && dtype == KAIR_F32 && npix < (1L << 31) && ((uintptr_t)dE & 15) == 0;
  if (pix4f || (ps_r == 1 && ldc == 16 && C <= 4 && dtype == KAIR_BF16 && npix < (1L << 31) && ((uintptr_t)dE & 15) == 0)) {
    if (pix4f && charb) KAIR_LAUNCH(l1_pix4f_kernel<true>, dim3(nb), dim3(256), 0, s, E, H, (float*)dE, gs, C, Hh * Ww, (int)npix, ws, eps);
    else if (pix4f) KAIR_LAUNCH(l1_pix4f_kernel<false>, dim3(nb), dim3(256), 0, s, E, H, (float*)dE, gs, C, Hh * Ww, (int)npix, ws, eps);
    else if (charb) KAIR_LAUNCH(l1_pix16_kernel<true>, dim3(nb), dim3(256), 0, s, E, H, (bf16*)dE, gs, C, Hh * Ww, (int)npix, ws, eps);
    else KAIR_LAUNCH(l1_pix16_kernel<false>, dim3(nb), dim3(256), 0, s, E, H, (bf16*)dE, gs, C, Hh * Ww, (int)npix, ws, eps);
    KAIR_CHECK_LAUNCH();
    KAIR_LAUNCH(l1_final, dim3(1), dim3(256), 0, s, ws, nb, (float)(weight / numel), loss_out);
    KAIR_CHECK_LAUNCH();
    return 0;
  }
#define KAIR_PIXEL_LOSS(T, I, CHV)                                                                                       \
  KAIR_LAUNCH((l1_kernel<T, I, CHV>), dim3(nb), dim3(256), 0, s, E, H, (T*)dE, ldc, ps_r, gs, C, Hh, Ww, npix, ws, \
                     eps)
  if (charb) {
    if (dtype == KAIR_BF16 && i32) KAIR_PIXEL_LOSS(bf16, int, true);
    else if (dtype == KAIR_BF16) KAIR_PIXEL_LOSS(bf16, long, true);
    else if (i32) KAIR_PIXEL_LOSS(float, int, true);
    else KAIR_PIXEL_LOSS(float, long, true);
  } else {
    if (dtype == KAIR_BF16 && i32) KAIR_PIXEL_LOSS(bf16, int, false);
    else if (dtype == KAIR_BF16) KAIR_PIXEL_LOSS(bf16, long, false);
    else if (i32) KAIR_PIXEL_LOSS(float, int, false);
    else KAIR_PIXEL_LOSS(float, long, false);
  }
#undef KAIR_PIXEL_LOSS
  KAIR_CHECK_LAUNCH();
  KAIR_LAUNCH(l1_final, dim3(1), dim3(256), 0, s, ws, nb, (float)(weight / numel), loss_out);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_l1_loss(const float* E, const float* H, float* loss_out, void* dE, int dtype, int ldc, int ps_r,
                            float weight, int B, int C, int Hh, int Ww, float* ws, void* stream) {
  return pixel_loss(E, H, loss_out, dE, dtype, ldc, ps_r, weight, 0.f, false, B, C, Hh, Ww, ws, stream);
}

extern "C" int kair_charbonnier_loss(const float* E, const float* H, float* loss_out, void* dE, int dtype, int ldc,
                                     int ps_r, float weight, float eps, int B, int C, int Hh, int Ww, float* ws,
                                     void* stream) {
  KAIR_CHECK_ARG(eps >= 0.f, "charbonnier_loss: eps must be >= 0");
  return pixel_loss(E, H, loss_out, dE, dtype, ldc, ps_r, weight, eps, true, B, C, Hh, Ww, ws, stream);
}

extern "C" int kair_adam_ema(float* p, const float* g, float* m, float* v, float* ema, long n, const float* lr_t,
                             float beta1, float beta2, float eps, float weight_decay, float ema_decay, void* stream) {
  KAIR_CHECK_ARG(p && g && m && v && lr_t && n > 0, "adam_ema: bad args");
  long nb = (n + 255) / 256;
  if (nb > 8192) nb = 8192;
  KAIR_LAUNCH(adam_ema_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, p, g, m, v, ema, n, lr_t,
                     beta1, beta2, eps, weight_decay, ema_decay, (const unsigned*)nullptr);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_adam_ema_ex(float* p, const float* g, float* m, float* v, float* ema, long n, const float* lr_t,
                                float beta1, float beta2, float eps, float weight_decay, float ema_decay,
                                const unsigned* skip, void* stream) {
  KAIR_CHECK_ARG(p && g && m && v && lr_t && n > 0, "adam_ema_ex: bad args");
  long nb = (n + 255) / 256;
  if (nb > 8192) nb = 8192;
  KAIR_LAUNCH(adam_ema_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, p, g, m, v, ema, n, lr_t,
                     beta1, beta2, eps, weight_decay, ema_decay, skip);
  KAIR_CHECK_LAUNCH();
  return 0;
}

// Kernel timing window (bench.py's in-step kernel table): while open, every libkair launch (KAIR_LAUNCH) goes through
// hipExtLaunchKernel with an event pair that the runtime stamps with the dispatch packet's own start / end timestamps
// -- the times rocprofv3 --kernel-trace reports -- and the slot remembers the kernel's host symbol.  Host-side
// bookkeeping of the launching thread; launches into a capturing stream are never timed (events cannot be captured).
namespace {
struct KtSlot {
  hipEvent_t e0, e1;
  const void* fn;
};
std::vector<KtSlot> g_kt;
int g_kt_next = -1, g_kt_used = 0;   // next slot (-1: window closed), slots filled by the last window
}   // namespace

bool kair_ktime_take(const void* fn, hipStream_t s, hipEvent_t* e0, hipEvent_t* e1) {
  if (g_kt_next < 0 || g_kt_next >= (int)g_kt.size()) return false;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return false;
  KtSlot& k = g_kt[g_kt_next++];
  k.fn = fn;
  *e0 = k.e0;
  *e1 = k.e1;
  return true;
}

extern "C" int kair_ktime_begin(int n) {
  KAIR_CHECK_ARG(n > 0 && n <= (1 << 16), "ktime_begin: slot count out of range");
  while ((int)g_kt.size() < n) {
    KtSlot k{nullptr, nullptr, nullptr};
    if (hipEventCreate(&k.e0) != hipSuccess || hipEventCreate(&k.e1) != hipSuccess)
      return kair_set_error(KAIR_ERR_HIP, "ktime_begin: hipEventCreate failed");
    g_kt.push_back(k);
  }
  g_kt_next = 0;
  g_kt_used = 0;
  return 0;
}

extern "C" int kair_ktime_count(void) { return g_kt_next >= 0 ? g_kt_next : g_kt_used; }

extern "C" int kair_ktime_end(void) {
  if (g_kt_next >= 0) g_kt_used = g_kt_next;
  g_kt_next = -1;
  return g_kt_used;
}

extern "C" int kair_ktime_read(int i, float* ms, const char** name) {
  KAIR_CHECK_ARG(ms && name && i >= 0 && i < kair_ktime_count(), "ktime_read: slot out of range");
  const KtSlot& k = g_kt[i];
  if (hipEventSynchronize(k.e1) != hipSuccess || hipEventElapsedTime(ms, k.e0, k.e1) != hipSuccess)
    return kair_set_error(KAIR_ERR_HIP, "ktime_read: event query failed");
  *name = hipKernelNameRefByPtr(k.fn, nullptr);
  if (!*name) *name = "";
  return 0;
}

// Launch gate (bench.py's kernel table): one wave that holds its stream until the host releases it (or a time limit
// passes), so the host can queue a whole eager pass behind it and the pass then runs back to back, with the stream
// concurrency of the graph-replayed step instead of the host's launch pace.  The flag and status words live in
// host-mapped memory; the wave polls with system-scope vector loads and reports with a vector store.
namespace {
unsigned* g_gate_host = nullptr;   // [0] release flag (host writes), [1] status (kernel writes: 1 released, 2 timed out)
unsigned* g_gate_dev = nullptr;
}   // namespace

__global__ void gate_kernel(const unsigned* flag, unsigned* status, unsigned long long limit) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned seen = 0;
  while (!(seen = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) &&
         __builtin_amdgcn_s_memrealtime() - t0 < limit)
    __builtin_amdgcn_s_sleep(8);
  __hip_atomic_store(status, seen ? 1u : 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C" int kair_gate_hold(int timeout_ms, void* stream) {
  KAIR_CHECK_ARG(timeout_ms > 0 && timeout_ms <= 10000, "gate_hold: timeout out of range (1 .. 10000 ms)");
  if (!g_gate_host) {
    if (hipHostMalloc((void**)&g_gate_host, 2 * sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&g_gate_dev, g_gate_host, 0) != hipSuccess)
      return kair_set_error(KAIR_ERR_HIP, "gate_hold: host-mapped flag allocation failed");
  }
  __atomic_store_n(&g_gate_host[0], 0u, __ATOMIC_SEQ_CST);
  __atomic_store_n(&g_gate_host[1], 0u, __ATOMIC_SEQ_CST);
  KAIR_LAUNCH(gate_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, g_gate_dev, g_gate_dev + 1,
              (unsigned long long)timeout_ms * 100000ull);   // the 100 MHz real-time counter
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_gate_release(void) {
  KAIR_CHECK_ARG(g_gate_host != nullptr, "gate_release: no gate held");
  __atomic_store_n(&g_gate_host[0], 1u, __ATOMIC_SEQ_CST);
  return 0;
}

extern "C" int kair_gate_status(void) { return g_gate_host ? (int)__atomic_load_n(&g_gate_host[1], __ATOMIC_SEQ_CST) : 0; }

extern "C" int kair_range_check(const float* g, const float* p, long n, const float* loss, float p_limit, unsigned* flag,
                                void* stream) {
  KAIR_CHECK_ARG(g && p && flag && n > 0 && p_limit > 0.f, "range_check: bad args");
  if (hipMemsetAsync(flag, 0, sizeof(unsigned), (hipStream_t)stream) != hipSuccess) {
    KAIR_CHECK_ARG(false, "range_check: memset failed");
  }
  long nb = (n / 4 + 255) / 256;
  if (nb > 2048) nb = 2048;
  if (nb < 1) nb = 1;
  KAIR_LAUNCH(range_check_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, g, p, n, loss, p_limit,
                     flag);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_axpby(float* y, const float* x, float a, float b, long n, void* stream) {
  KAIR_CHECK_ARG(y && x && n >= 0, "axpby: bad args");
  long nb = (n + 255) / 256;
  if (nb > 8192) nb = 8192;
  if (nb < 1) nb = 1;
  KAIR_LAUNCH(axpby_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, y, x, a, b, n);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_axpby_rows(float* y, long ldy, const float* x, long ldx, long M, int C, float a, float b,
                                void* stream) {
  KAIR_CHECK_ARG(y && x && M > 0 && C > 0 && ldy >= C && ldx >= C, "axpby_rows: bad args");
  KAIR_LAUNCH(axpby_rows_kernel, dim3(nblk(M * C, 256)), dim3(256), 0, (hipStream_t)stream, y, ldy, x, ldx, M, C, a, b);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_act_grad_cast(const float* G, long ldg, const void* X, int x_dtype, long ldx, void* out, int out_dtype,
                                  long ldo, long M, int C, int kind, float slope, float scale, void* stream) {
  KAIR_CHECK_ARG(G && out && M > 0 && C > 0 && (kind == 0 || X), "act_grad_cast: bad args");
  const long n = M * C;
  hipStream_t s = (hipStream_t)stream;
  const dim3 g(nblk(n, 256)), b(256);
  if (x_dtype == KAIR_BF16) {
    if (out_dtype == KAIR_BF16)
      KAIR_LAUNCH((act_grad_cast_kernel<bf16, bf16>), g, b, 0, s, G, ldg, (const bf16*)X, ldx, (bf16*)out, ldo, M, C,
                         kind, slope, scale);
    else
      KAIR_LAUNCH((act_grad_cast_kernel<bf16, float>), g, b, 0, s, G, ldg, (const bf16*)X, ldx, (float*)out, ldo, M,
                         C, kind, slope, scale);
  } else {
    if (out_dtype == KAIR_BF16)
      KAIR_LAUNCH((act_grad_cast_kernel<float, bf16>), g, b, 0, s, G, ldg, (const float*)X, ldx, (bf16*)out, ldo, M,
                         C, kind, slope, scale);
    else
      KAIR_LAUNCH((act_grad_cast_kernel<float, float>), g, b, 0, s, G, ldg, (const float*)X, ldx, (float*)out, ldo,
                         M, C, kind, slope, scale);
  }
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_sumpool2x(const float* src, long lds, float* dst, long ldd, int B, int H, int W, int C, int accumulate,
                              void* stream) {
  KAIR_CHECK_ARG(src && dst && B > 0 && H > 0 && W > 0 && C > 0 && lds >= C && ldd >= C, "sumpool2x: bad args");
  const long n = (long)B * H * W * C;
  KAIR_LAUNCH(sumpool2x_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, src, lds, dst, ldd, B, H, W,
                     C, accumulate);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_axpy(float* y, const float* x, float a, long n, void* stream) {
  KAIR_CHECK_ARG(y && x && n >= 0 && ((uintptr_t)y % 16) == 0 && ((uintptr_t)x % 16) == 0, "axpy: bad args");
  long nb = (n / 4 + 255) / 256;
  if (nb > 4096) nb = 4096;
  if (nb < 1) nb = 1;
  KAIR_LAUNCH(axpy_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, y, x, a, n);
  KAIR_CHECK_LAUNCH();
  return 0;
}
