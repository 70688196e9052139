// Row-streaming GEMM with full-row epilogues for gfx950 (bf16 MFMA, fp32 accumulation):
//
//   Y[m, :] = A[m, :] . W^T          A: bf16 rows [M][K] (K = 192 / 384 / 576), W: the linear's weight
//                                    in transposed MFMA-fragment order (pack kind 13)
//
// i.e. the INPUT gradient of one Swin-block linear (nn.Linear backward, network_swinir.py:19-20
// fc1 / fc2, :105 qkv, :107 proj), with the consumer of that gradient fused into the epilogue:
//
//   EPI_LN    Y = dL/d(LayerNorm output) -> the LayerNorm backward (nn.LayerNorm, network_swinir.py
//             :199 norm1 / :205 norm2) accumulated into the residual-stream gradient D, the row-scaled
//             bf16 copy of the finished D row that the next GEMMs read, and per-workgroup dgamma /
//             dbeta partials.  Y never leaves the registers (the unfused path rounded it to bf16 and
//             round-tripped it through HBM between a GEMM and a LayerNorm-backward launch);
//   EPI_GATE  Y * g (g = the stored GELU'(fc1 pre-activation)) -> bf16 rows   (fc2 input gradient);
//   EPI_STORE Y -> bf16 rows                                                  (proj input gradient).
//
// Layout of the work: a workgroup owns one 32-row tile at a time (persistent over tiles), NWC waves
// each computing 96 output columns of it (3 x v_mfma_f32_32x32x16_bf16 accumulators: lane = column,
// registers = rows).  One wave per SIMD (the kernel keeps ~350 VGPRs), so every wave streams:
//   * A fragments straight from HBM into registers, PD k-steps ahead, continuing into the NEXT tile's
//     first k-steps while this tile finishes (no LDS staging, no barrier in the k-loop);
//   * W fragments (1 KiB coalesced wave loads, L2-resident) at the SAME distance PD: vmcnt retires
//     loads in issue order, so a W stream prefetched less deeply than A would make every W wait
//     also wait for the younger A loads and cut A's latency budget down to W's;
//   * the epilogue's per-tile operands (x / the gate) at the tile start, landed by the epilogue.
// The LayerNorm row sums need the whole row: each wave reduces its 96 columns in registers
// (+ a 32-lane DPP / swizzle reduction) and the NWC waves exchange the per-row partials through
// LDS (fixed order, deterministic).
#include <string.h>

#include "common.h"

namespace {

constexpr int RT = 32;   // rows per tile
constexpr int NCT = 3;   // 32-column accumulator tiles per wave
enum { EPI_STORE = 0, EPI_GATE = 1, EPI_LN = 2 };

struct RgArgs {
  const bf16* A; long lda; long M; long ntiles;
  long xbytes, dbytes, cbytes;                // LN: buffer sizes of x, D and the copy (bounds of the resources)
  const bf16* W;                              // kind 13: [N/32][KB][64 lanes][8]
  bf16* out; long ldo;                        // STORE / GATE
  const bf16* gate; long ldg;                 // GATE
  const float* x; long ldx;                   // LN: LayerNorm input (fp32, token rows)
  const float* gamma; const float* mean; const float* rstd;
  int C; float inv_c;
  float* D; long ldD;                         // LN: dL/d(LN input) accumulated in place (token rows)
  bf16* cp; long ldc;                         // LN: bf16 copy of the finished D row (optional)
  const float* cp_scale; int cp_rps;          //     per-sample scale of the copy (DropPath), or NULL
  WinMap wm;                                  // LN: GEMM row -> token (Swin window order, or identity)
  WinMap cwm;                                 // LN: token -> copy row (token_to_win)
  float* part;                                // LN: [gridDim.x][2][C] dgamma / dbeta partials
};

KAIR_DEV int acc_row(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }

// buffer-resource access for the epilogue operands: one 32-bit byte offset per row (shared by x and
// D, which have the same row stride) instead of a 64-bit address per element
typedef __amdgpu_buffer_rsrc_t Rsrc;
KAIR_DEV Rsrc rsrc(const void* p, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)(bytes > 0x7fffffffL ? 0x7fffffffL : bytes),
                                           0x00020000);
}
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
// 16 bytes per lane at (lane offset voff) + (wave-uniform soff): the uniform part in an SGPR
KAIR_DEV bf16x8 bld16(Rsrc r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0));
}
KAIR_DEV float4 bld4(Rsrc r, unsigned off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
KAIR_DEV void bst4(Rsrc r, unsigned off, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)off, 0, 0);
}
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
KAIR_DEV void bst8(Rsrc r, unsigned off, bf16x4 v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, (int)off, 0, 0);
}
KAIR_DEV float bld(Rsrc r, unsigned off) { return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0)); }
KAIR_DEV void bst(Rsrc r, unsigned off, float v) { __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)off, 0, 0); }
KAIR_DEV void bst16(Rsrc r, unsigned off, bf16 v) {
  __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, v), r, (int)off, 0, 0);
}

// sum over the 32 lanes of each wave half (DPP within 16, then one swizzle across the 16-lane rows)
KAIR_DEV float half_sum32(float v) {
  v = dpp_sum16(v);
  return v + __shfl_xor(v, 16, 64);
}

template <int KB, int PD, int NWC, int EPI>
__global__ __launch_bounds__(64 * NWC, 2) void rowgemm_kernel(const RgArgs a) {
  static_assert(PD <= KB, "prefetch distance must not exceed the k-steps of a tile");
  static_assert(EPI != EPI_LN || NWC == 2, "the LayerNorm epilogue is laid out for 192 columns");
  constexpr int NT = 64 * NWC, N = 96 * NWC, LDY = N + 4;
  constexpr int NCH = N / 8, CPT = RT * NCH / NT;   // STORE / GATE: 8-column chunks per row / per thread
  static_assert(RT * NCH % NT == 0, "chunks per thread");
  const int tid = threadIdx.x, lane = tid & 63, cw = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l31 = lane & 31, hh = lane >> 5;
  // the tile's Y (fp32), written by the accumulators (lane = column) and read back row-contiguous
  __shared__ __attribute__((aligned(16))) float sY[RT * LDY];
  const long G = gridDim.x;
  long tile = blockIdx.x;
  if (tile >= a.ntiles) return;           // the host launches at most ntiles workgroups

  // W: a buffer resource over this wave's fragments (wave-uniform) + one 32-bit lane offset; the
  // per-fragment offsets are constants passed as the scalar offset (no per-load 64-bit address)
  const Rsrc rW = rsrc(a.W + (long)(NCT * cw) * KB * 512, (long)NCT * KB * 1024);
  const unsigned wl = lane * 16u;
  const int c0 = 96 * cw + l31;           // this lane's accumulator column of tile ct: c0 + 32 ct

  // LN row layout: 16 lanes per row (lane jl: columns 4 jl + 64 k, k < 3), 8 rows per pass, 4 passes
  constexpr int LPASS = RT / (NT / 16);
  const int lr = tid >> 4, jl = tid & 15;
  float4 gam4[3], pg[3], pb[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    pg[k] = pb[k] = gam4[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (EPI == EPI_LN) {
      const int c = 4 * jl + 64 * k;
      gam4[k] = make_float4(c < a.C ? a.gamma[c] : 0.f, c + 1 < a.C ? a.gamma[c + 1] : 0.f,
                            c + 2 < a.C ? a.gamma[c + 2] : 0.f, c + 3 < a.C ? a.gamma[c + 3] : 0.f);
    }
  }
  const Rsrc rx = rsrc(a.x, a.xbytes), rD = rsrc(a.D, a.dbytes), rC = rsrc(a.cp, a.cp ? a.cbytes : 0);

  for (; tile < a.ntiles; tile += G) {
    const long row0 = tile * RT;
    // ---- epilogue operands of this tile, issued before the k-loop (landed by the epilogue)
    unsigned tof[LPASS], cof[LPASS];   // LN: byte offsets of this lane's rows in x / D and in the copy
    float mu[LPASS], rs[LPASS], sc[LPASS];
    float4 xv[LPASS][3];
    uint4 gv[CPT];                      // GATE: 8 bf16 gate values per chunk
    if constexpr (EPI == EPI_LN) {
#pragma unroll
      for (int p = 0; p < LPASS; ++p) {
        const long row = row0 + (NT / 16) * p + lr;
        const bool ok = row < a.M;
        const int t = win_to_token32((int)(ok ? row : a.M - 1), a.wm);
        mu[p] = a.mean[t];
        rs[p] = a.rstd[t];
        sc[p] = a.cp_scale ? a.cp_scale[t / a.cp_rps] : 1.f;
        // rows past M: offsets outside the resources (the range check drops those loads and stores)
        tof[p] = ok ? ((unsigned)t * (unsigned)a.ldx + 4u * jl) * 4u : 0x80000000u;
        cof[p] = ok ? ((unsigned)token_to_win(t, a.cwm) * (unsigned)a.ldc + 4u * jl) * 2u : 0x80000000u;
#pragma unroll
        for (int k = 0; k < 3; ++k) xv[p][k] = bld4(rx, tof[p] + 256u * k);
      }
    } else if constexpr (EPI == EPI_GATE) {
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const int q = tid + NT * i, r = q / NCH, c8 = (q - r * NCH) * 8;
        const long row = row0 + r < a.M ? row0 + r : a.M - 1;
        gv[i] = *(const uint4*)(a.gate + row * a.ldg + c8);
      }
    }

    // ---- k-loop.  Issue order: the first PD W k-steps, then the whole A tile, W refills after.
    // vmcnt retires in issue order: the first MFMA waits for A[0] (and the epilogue operands) only,
    // the refill of W[PD] is the first point at which the whole A tile must have landed.
    bf16x8 rw[PD][NCT], ra[KB];
#pragma unroll
    for (int i = 0; i < PD; ++i)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) rw[i][ct] = bld16(rW, wl, (ct * KB + i) * 1024u);
    {
      long r = row0 + l31;
      if (r >= a.M) r = a.M - 1;
      const bf16* ap = a.A + r * a.lda + 8 * hh;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) ra[kb] = *(const bf16x8*)(ap + 16 * kb);
    }
    f32x16 acc[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[ct][r] = 0.f;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const int s = kb % PD;
      bf16x8 fw[NCT];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) fw[ct] = rw[s][ct];
      if (kb + PD < KB) {
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) rw[s][ct] = bld16(rW, wl, (ct * KB + kb + PD) * 1024u);
      }
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra[kb], fw[ct], acc[ct], 0, 0, 0);
    }

    // ---- Y -> LDS (lane = column, register = row), then every epilogue reads whole rows
    __builtin_amdgcn_sched_barrier(0);
    float4 dv[LPASS][3];
    if constexpr (EPI == EPI_LN) {   // D of this lane's rows: in flight across the transpose
#pragma unroll
      for (int p = 0; p < LPASS; ++p)
#pragma unroll
        for (int k = 0; k < 3; ++k) dv[p][k] = bld4(rD, tof[p] + 256u * k);
    }
    __syncthreads();   // the previous tile's epilogue has read sY
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) sY[acc_row(r, hh) * LDY + c0 + 32 * ct] = acc[ct][r];
    __syncthreads();

    if constexpr (EPI == EPI_STORE || EPI == EPI_GATE) {
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const int q = tid + NT * i, r = q / NCH, c8 = (q - r * NCH) * 8;
        const float4 y0 = *(const float4*)(sY + r * LDY + c8), y1 = *(const float4*)(sY + r * LDY + c8 + 4);
        float v[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
        if constexpr (EPI == EPI_GATE) {
          const bf16x8 g = __builtin_bit_cast(bf16x8, gv[i]);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] *= (float)g[j];
        }
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
        if (row0 + r < a.M) *(bf16x8*)(a.out + (row0 + r) * a.ldo + c8) = o;
      }
    } else {
      // LayerNorm backward (ln_bwd_kernel maths, layernorm.hip), one row per 16 lanes: with
      // xh = (x - mu) rstd, gy = dy gamma:  dx = rstd (gy - mean_c(gy) - xh mean_c(gy xh)),
      // dgamma += dy xh, dbeta += dy (rows past M contribute 0: their dy is read as 0 below)
#pragma unroll
      for (int p = 0; p < LPASS; ++p) {
        const int tr = (NT / 16) * p + lr;
        const float live = row0 + tr < a.M ? 1.f : 0.f;
        float dy[3][4], xh[3][4];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float4 d4 = *(const float4*)(sY + tr * LDY + 4 * jl + 64 * k);
          const float da[4] = {d4.x, d4.y, d4.z, d4.w}, xa[4] = {xv[p][k].x, xv[p][k].y, xv[p][k].z, xv[p][k].w};
          const float ga[4] = {gam4[k].x, gam4[k].y, gam4[k].z, gam4[k].w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const bool in = 4 * jl + 64 * k + j < a.C;
            dy[k][j] = live * da[j];   // 0 past C: the packed weight rows are 0 there
            xh[k][j] = in ? (xa[j] - mu[p]) * rs[p] : 0.f;
            const float gy = dy[k][j] * ga[j];
            s1 += gy;
            s2 += gy * xh[k][j];
          }
          pg[k].x += dy[k][0] * xh[k][0]; pg[k].y += dy[k][1] * xh[k][1];
          pg[k].z += dy[k][2] * xh[k][2]; pg[k].w += dy[k][3] * xh[k][3];
          pb[k].x += dy[k][0]; pb[k].y += dy[k][1]; pb[k].z += dy[k][2]; pb[k].w += dy[k][3];
        }
        s1 = dpp_sum16(s1) * a.inv_c;
        s2 = dpp_sum16(s2) * a.inv_c;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float ga[4] = {gam4[k].x, gam4[k].y, gam4[k].z, gam4[k].w};
          const float cu[4] = {dv[p][k].x, dv[p][k].y, dv[p][k].z, dv[p][k].w};
          float o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)   // columns past C keep their value
            o[j] = 4 * jl + 64 * k + j < a.C ? cu[j] + rs[p] * (dy[k][j] * ga[j] - s1 - xh[k][j] * s2) : cu[j];
          bst4(rD, tof[p] + 256u * k, make_float4(o[0], o[1], o[2], o[3]));
          const bf16x4 cb = {(bf16)(sc[p] * o[0]), (bf16)(sc[p] * o[1]), (bf16)(sc[p] * o[2]), (bf16)(sc[p] * o[3])};
          bst8(rC, cof[p] + 128u * k, cb);
        }
      }
    }
  }

  if constexpr (EPI == EPI_LN) {   // this workgroup's dgamma / dbeta partials: the 8 row groups summed
    __syncthreads();               // in fixed order (deterministic) through sY
    constexpr int NG = NT / 16;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      *(float4*)(sY + lr * 2 * 192 + 4 * jl + 64 * k) = pg[k];
      *(float4*)(sY + lr * 2 * 192 + 192 + 4 * jl + 64 * k) = pb[k];
    }
    __syncthreads();
    for (int c = tid; c < 2 * 192; c += NT) {
      float t = 0.f;
#pragma unroll
      for (int g = 0; g < NG; ++g) t += sY[g * 2 * 192 + c];
      const int w = c / 192, cc = c - w * 192;
      if (cc < a.C) a.part[(long)blockIdx.x * 2 * a.C + w * a.C + cc] = t;
    }
  }
}

int g_rg_cus = 0;
int rg_cus() {
  if (g_rg_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      g_rg_cus = n;
    if (g_rg_cus <= 0) g_rg_cus = 256;
  }
  return g_rg_cus;
}

// persistent grid: as many workgroups as the CUs hold at the kernel's occupancy (registers), at most
// one per tile
template <int KB, int PD, int NWC, int EPI>
int rg_launch(const RgArgs& a, hipStream_t s, long* grid_out) {
  auto kern = rowgemm_kernel<KB, PD, NWC, EPI>;
  static int per_cu = 0;   // workgroups per CU at this instantiation's occupancy (one cache each)
  if (per_cu == 0) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, 64 * NWC, 0) != hipSuccess || n <= 0) n = 4 / NWC;
    per_cu = n;
  }
  const long tiles = (a.M + RT - 1) / RT, slots = (long)rg_cus() * per_cu;
  const long grid = tiles < slots ? tiles : slots;
  if (grid_out) { *grid_out = grid; return 0; }
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * NWC), 0, s, a);
  KAIR_CHECK_LAUNCH();
  return 0;
}

// grid_out != NULL: report the grid (the LN partial count) without launching
template <int EPI, int NWC>
int rg_dispatch(int K, const RgArgs& a, hipStream_t s, long* grid_out = nullptr) {
  switch (K) {
    case 192: return rg_launch<12, 4, NWC, EPI>(a, s, grid_out);
    case 384: return rg_launch<24, 4, NWC, EPI>(a, s, grid_out);
    case 576: return rg_launch<36, 2, NWC, EPI>(a, s, grid_out);
    default: return kair_set_error(KAIR_ERR_ARG, "rowgemm: K must be 192, 384 or 576 (got %d)", K);
  }
}

int rg_common(const void* A, long lda, long M, int K, const void* W, int N, RgArgs& a) {
  KAIR_CHECK_ARG(A && W, "rowgemm: null operand");
  KAIR_CHECK_ARG(M > 0 && M < KAIR_MAX_MAPPED_ROWS, "rowgemm: M out of range");
  KAIR_CHECK_ARG(lda >= K && lda % 8 == 0 && ((uintptr_t)A % 16) == 0 && ((uintptr_t)W % 16) == 0,
                 "rowgemm: A rows must be 16-byte aligned with lda >= K, lda %% 8 == 0");
  KAIR_CHECK_ARG(N == 192 || N == 384, "rowgemm: N must be 192 or 384 (got %d)", N);
  memset(&a, 0, sizeof(a));
  a.A = (const bf16*)A; a.lda = lda; a.M = M; a.ntiles = (M + RT - 1) / RT;
  a.W = (const bf16*)W;
  a.wm = make_winmap(0, 0, 0, 0);
  a.cwm = make_winmap(0, 0, 0, 0);
  return 0;
}

}  // namespace

/* Number of dgamma / dbeta partial rows kair_rowgemm_lnbwd leaves in `part` for (M, K). */
extern "C" long kair_rowgemm_ln_blocks(long M, int K) {
  if (M <= 0) return 0;
  RgArgs a;
  memset(&a, 0, sizeof(a));
  a.M = M;
  long g = 0;
  if (rg_dispatch<EPI_LN, 2>(K, a, nullptr, &g) != 0) return -1;
  return g;
}

extern "C" int kair_rowgemm_store(const void* A, long lda, long M, int K, const void* W, int N, void* out, long ldo,
                                  void* stream) {
  RgArgs a;
  if (int rc = rg_common(A, lda, M, K, W, N, a)) return rc;
  KAIR_CHECK_ARG(out && ldo >= N, "rowgemm_store: out");
  a.out = (bf16*)out; a.ldo = ldo;
  hipStream_t s = (hipStream_t)stream;
  return N == 192 ? rg_dispatch<EPI_STORE, 2>(K, a, s) : rg_dispatch<EPI_STORE, 4>(K, a, s);
}

extern "C" int kair_rowgemm_gate(const void* A, long lda, long M, int K, const void* W, int N, const void* gate, long ldg,
                                 void* out, long ldo, void* stream) {
  RgArgs a;
  if (int rc = rg_common(A, lda, M, K, W, N, a)) return rc;
  KAIR_CHECK_ARG(out && ldo >= N && gate && ldg >= N, "rowgemm_gate: out / gate");
  a.out = (bf16*)out; a.ldo = ldo; a.gate = (const bf16*)gate; a.ldg = ldg;
  hipStream_t s = (hipStream_t)stream;
  return N == 192 ? rg_dispatch<EPI_GATE, 2>(K, a, s) : rg_dispatch<EPI_GATE, 4>(K, a, s);
}

extern "C" int kair_rowgemm_lnbwd(const void* A, long lda, long M, int K, const void* W, const float* x, long ldx,
                                  const float* gamma, const float* mean, const float* rstd, int C, float* D, long ldD,
                                  int win_H, int win_W, int win_ws, int win_shift, const kair_copy_desc* copy, float* part,
                                  void* stream) {
  RgArgs a;
  if (int rc = rg_common(A, lda, M, K, W, 192, a)) return rc;
  KAIR_CHECK_ARG(x && gamma && mean && rstd && D && part, "rowgemm_lnbwd: null pointer");
  KAIR_CHECK_ARG(C > 0 && C <= 192 && ldx >= C && ldD >= C, "rowgemm_lnbwd: C %d must be <= 192", C);
  KAIR_CHECK_ARG(M * ldx * 4 < 0x7fffffffL && M * 192 * 2 < 0x7fffffffL, "rowgemm_lnbwd: operands past 2 GiB");
  KAIR_CHECK_ARG(win_ws == 0 || (win_H % win_ws == 0 && win_W % win_ws == 0 && (long)win_H * win_W > 0 &&
                                 M % ((long)win_H * win_W) == 0),
                 "rowgemm_lnbwd: window geometry");
  a.x = x; a.ldx = ldx; a.gamma = gamma; a.mean = mean; a.rstd = rstd; a.C = C; a.inv_c = 1.0f / (float)C;
  KAIR_CHECK_ARG(ldx == ldD, "rowgemm_lnbwd: x and D must share the row stride");
  a.D = D; a.ldD = ldD; a.part = part;
  // buffer bounds: the largest token index any GEMM row maps to is M - 1 (the window map permutes)
  a.xbytes = M * ldx * 4; a.dbytes = M * ldD * 4;
  a.wm = make_winmap(win_H, win_W, win_ws, win_shift);
  if (copy && copy->out) {
    KAIR_CHECK_ARG(copy->dtype == KAIR_BF16 && copy->ld >= C, "rowgemm_lnbwd: the copy is bf16 rows, ld >= C");
    KAIR_CHECK_ARG(copy->win_ws == 0 || (copy->win_H % copy->win_ws == 0 && copy->win_W % copy->win_ws == 0),
                   "rowgemm_lnbwd: copy window geometry");
    a.cp = (bf16*)copy->out; a.ldc = copy->ld; a.cp_scale = copy->rowscale;
    a.cbytes = M * copy->ld * 2;
    a.cp_rps = copy->rows_per_scale > 0 ? copy->rows_per_scale : 1;
    a.cwm = make_winmap(copy->win_H, copy->win_W, copy->win_ws, copy->win_shift);
  }
  return rg_dispatch<EPI_LN, 2>(K, a, (hipStream_t)stream);
}
