// Window-attention helpers shared by the bf16 / fp32 kernels (window_attn.hip) and the fp16-pair (fp32x3)
// ("x3") kernels (attn_x3.hip): Swin window geometry (ws = 8, 64 tokens, head dim padded to 32),
// the relative-position index and its binned gradient, the shifted-window region ids, and the
// MFMA-fragment reads of [64][32] bf16 LDS tiles.
#pragma once
#include "common.h"

namespace {

constexpr int ATT_LD = 40;   // LDS row stride (bf16 elements) of a [64][32] tile

constexpr int WS = 8, TOK = 64, HDP = 32;
// Each wave works only on its own LDS slice, so a wave-local fence replaces __syncthreads (waves of
// a block may run different trip counts).  LDS operations of one wave complete in issue order.
KAIR_DEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

KAIR_DEV int relidx(int q, int k) { return ((q >> 3) - (k >> 3) + WS - 1) * (2 * WS - 1) + ((q & 7) - (k & 7) + WS - 1); }

// The relative-position bias gradient of one (group, head) tile, binned inside the wave that made it:
// out[idx] = sum of db[q][k] over the window's (query, key) pairs with relidx(q, k) = idx (the
// backward of network_swinir.py:132-135's table gather).  The per-group output is 225 floats instead
// of the 64 x 64 tile (16 KB per (group, head) at B = 4's one window per wave).  Stage 1: lane
// (qy, ky) sums its 8 x 8 block of db along the 15 diagonals qx - kx; stage 2: lane = bin (dy, dx)
// sums the blocks with qy - ky = dy.  Fixed order (deterministic).  scr: 1024 floats of the wave's LDS.
constexpr int NBIN = (2 * WS - 1) * (2 * WS - 1);
template <bool VEC>
KAIR_DEV void bin_dbias(const float* db, int ldb, float* scr, float* __restrict__ out, int lane) {
  const int qy = lane >> 3, ky = lane & 7;
  float d[2 * WS - 1];
#pragma unroll
  for (int j = 0; j < 2 * WS - 1; ++j) d[j] = 0.f;
#pragma unroll
  for (int qx = 0; qx < WS; ++qx) {
    const float* row = db + (qy * WS + qx) * ldb + ky * WS;
    float v[WS];
    if constexpr (VEC) {
      const float4 a = *(const float4*)row, b = *(const float4*)(row + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
      for (int kx = 0; kx < WS; ++kx) v[kx] = row[kx];
    }
#pragma unroll
    for (int kx = 0; kx < WS; ++kx) d[qx - kx + WS - 1] += v[kx];
  }
#pragma unroll
  for (int j = 0; j < 2 * WS - 1; ++j) scr[lane * 16 + j] = d[j];
  wave_sync();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = lane + 64 * i;
    if (idx < NBIN) {
      const int dy = idx / (2 * WS - 1) - (WS - 1), j = idx % (2 * WS - 1);
      float s = 0.f;
#pragma unroll
      for (int y = 0; y < WS; ++y) {
        const int kyy = y - dy;
        if (kyy >= 0 && kyy < WS) s += scr[(y * WS + kyy) * 16 + j];
      }
      out[idx] = s;
    }
  }
}

KAIR_DEV int region(int coord, int n, int shift) { return coord < n - WS ? 0 : (coord < n - shift ? 1 : 2); }

// region id of token t of window `wi` (index within the image) on the shifted H x W grid
KAIR_DEV int token_region(int wi, int t, int H, int W, int shift) {
  const int nWw = W / WS;
  const int wy = wi / nWw, wx = wi - wy * nWw;
  return region(wy * WS + (t >> 3), H, shift) * 3 + region(wx * WS + (t & 7), W, shift);
}

typedef short __attribute__((ext_vector_type(8))) short8v;

KAIR_DEV bf16x8 tr_read8(const bf16* p0, const bf16* p1) {
  const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)p0);
  const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)p1);
  const short8v s = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, s);
}

// B fragment (32x32x16) of a row-major [64][32] LDS tile X, contraction over X's rows in the
// PERMUTED order produced by using a 32x32 accumulator as the other operand:
// element j of lane half h <-> row base + 16*s + 8*(j>>2) + 4*h + (j&3), column = lane&31.
KAIR_DEV bf16x8 frag_rows_perm(const bf16* X, int base, int s, int lane) {
  constexpr int LD = ATT_LD;
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int h = G >> 1, c0 = (G & 1) * 16;
  const bf16* a = X + (base + 16 * s + 4 * h + q) * LD + c0 + 4 * p;
  return tr_read8(a, a + 8 * LD);
}
// same, natural order: element j of lane half h <-> row base + 16*s + 8*h + j
KAIR_DEV bf16x8 frag_rows_nat(const bf16* X, int base, int s, int lane) {
  constexpr int LD = ATT_LD;
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int h = G >> 1, c0 = (G & 1) * 16;
  const bf16* a = X + (base + 16 * s + 8 * h + q) * LD + c0 + 4 * p;
  return tr_read8(a, a + 4 * LD);
}
// A/B fragment from a row-major tile where the lane's row is `row` and the 8 contiguous
// contraction elements start at column 16*s + 8*(lane>>5)
KAIR_DEV bf16x8 frag_cols(const bf16* X, int ld, int row, int s, int lane) {
  return *(const bf16x8*)(X + row * ld + 16 * s + 8 * (lane >> 5));
}

KAIR_DEV bf16x8 pack8(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)a[8 * s + j];
  return r;
}

// accumulator row (within a 32x32 tile) held by register r of lane half h
KAIR_DEV int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }


// the lo half of pack8: bf16(a - bf16(a)), the second term of a hi/lo split operand
KAIR_DEV bf16x8 pack8_lo(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float v = a[8 * s + j];
    r[j] = (bf16)(v - (float)(bf16)v);
  }
  return r;
}

}  // namespace
