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
// Layout of the work: a workgroup (one per CU, persistent over 32-row tiles) splits the K = 16 KB
// contraction over KS groups of NWC waves; wave (group g, column block c) computes 96 output columns
// (3 x v_mfma_f32_32x32x16_bf16 accumulators: lane = column, registers = rows) over k-steps
// [g KB/KS, (g+1) KB/KS).  Short per-wave k-loops are what the small per-GPU batch needs (B = 4:
// 288 tiles for 256 CUs, so a tile's dependent chain IS the kernel time):
//   * the wave's weight fragments are loaded ONCE and held in registers for every tile (HOLD of its
//     k-steps; the rest re-read from L2 under the held steps' MFMAs where registers run out);
//   * the next tile's A rows and epilogue operands are issued right after this tile's MFMAs, so they
//     land under the partial-sum exchange and the epilogue; no LDS staging, no barrier in the k-loop.
// The KS partial products meet in LDS (one fp32 plane per group), summed in fixed order by the
// epilogue, which reads whole rows (deterministic).  The LayerNorm epilogue runs 16 lanes per row.
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

// Per-tile epilogue operands (double-buffered across the persistent loop: tile t's are in use while
// tile t + G's land)
template <int LPASS, int CPT>
struct EpiOps {
  unsigned tof[LPASS], cof[LPASS];   // LN: byte offsets of this lane's rows in x / D and in the copy
  float mu[LPASS], rs[LPASS], sc[LPASS];
  float4 xv[LPASS][3];
  uint4 gv[CPT];                      // GATE: 8 bf16 gate values per chunk
};

// KB k-steps of 16 split over KS wave groups (KBW each); NWC waves per group, 96 columns per wave.
// Every wave holds ITS weight fragments (KBW x 3) in registers for the whole launch (loaded once),
// so a tile's k-loop waits for nothing but its own A rows, which were prefetched during the previous
// tile's epilogue.  The KS partial products meet in LDS (one fp32 plane per group) and the epilogue
// sums them in fixed order (deterministic).
// HOLD < KBW: only the first HOLD k-steps' fragments stay resident, the rest are re-read from L2 at
// each tile's start (in flight under the resident steps' MFMAs) -- the register budget of the
// LayerNorm epilogue at K = 576.
template <int KB, int KS, int NWC, int EPI, int HOLD>
__global__ __launch_bounds__(64 * NWC * KS, 1) void rowgemm_kernel(const RgArgs a) {
  static_assert(KB % KS == 0, "k-steps per group");
  constexpr int KBW = KB / KS, NSTR = KBW - HOLD;
  static_assert(HOLD >= 1 && HOLD <= KBW && HOLD * NCT <= 27, "weight fragments held in registers");
  static_assert(EPI != EPI_LN || NWC == 2, "the LayerNorm epilogue is laid out for 192 columns");
  constexpr int NT = 64 * NWC * KS, N = 96 * NWC, LDY = N + 4, PLANE = RT * LDY;
  constexpr int NCH = N / 8, NCHUNK = RT * NCH, CPT = (NCHUNK + NT - 1) / NT;   // STORE / GATE chunks
  constexpr int RPP = NT / 16, LPASS = RT / RPP;                                   // LN: rows per pass
  static_assert(RT % RPP == 0, "LayerNorm passes");
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cw = wave % NWC, ks = wave / NWC;
  const int l31 = lane & 31, hh = lane >> 5;
  __shared__ __attribute__((aligned(16))) float sY[KS * PLANE];
  const long G = gridDim.x;
  long tile = blockIdx.x;
  if (tile >= a.ntiles) return;           // the host launches at most ntiles workgroups

  // this wave's weight fragments, once: kind 13 [N/32][KB][64 lanes][8], 1 KiB coalesced wave loads
  const Rsrc rW = rsrc(a.W + (long)(NCT * cw) * KB * 512, (long)NCT * KB * 1024);
  const unsigned wl = lane * 16u;
  bf16x8 rw[HOLD][NCT];
#pragma unroll
  for (int i = 0; i < HOLD; ++i)
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) rw[i][ct] = bld16(rW, wl, (ct * KB + ks * KBW + i) * 1024u);
  const int c0 = 96 * cw + l31;           // this lane's accumulator column of tile ct: c0 + 32 ct

  // LN row layout: 16 lanes per row (lane jl: columns 4 jl + 64 k, k < 3), RPP rows per pass.
  // The dgamma / dbeta partials of a lane's columns live in LDS slots only that lane touches (registers
  // are the K=576 launch's limit), summed over the RPP row groups in fixed order at the end.
  const int lr = tid >> 4, jl = tid & 15;
  __shared__ __attribute__((aligned(16))) float sP[EPI == EPI_LN ? RPP * 2 * 192 : 4];
  __shared__ __attribute__((aligned(16))) float sGam[EPI == EPI_LN ? 192 : 4];   // gamma, 0 past C
  if constexpr (EPI == EPI_LN) {
    for (int c = tid; c < 192; c += NT) sGam[c] = c < a.C ? a.gamma[c] : 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      *(float4*)(sP + lr * 2 * 192 + 4 * jl + 64 * k) = make_float4(0.f, 0.f, 0.f, 0.f);
      *(float4*)(sP + lr * 2 * 192 + 192 + 4 * jl + 64 * k) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  const Rsrc rx = rsrc(a.x, a.xbytes), rD = rsrc(a.D, a.dbytes), rC = rsrc(a.cp, a.cp ? a.cbytes : 0);

  typedef EpiOps<LPASS, CPT> E;
  auto load_epi = [&](long t, E& e) {
    const long row0 = t * RT;
    if constexpr (EPI == EPI_LN) {
#pragma unroll
      for (int p = 0; p < LPASS; ++p) {
        const long row = row0 + RPP * p + lr;
        const bool ok = row < a.M;
        const int tk = win_to_token32((int)(ok ? row : a.M - 1), a.wm);
        e.mu[p] = a.mean[tk];
        e.rs[p] = a.rstd[tk];
        e.sc[p] = a.cp_scale ? a.cp_scale[tk / a.cp_rps] : 1.f;
        // rows past M: offsets outside the resources (the range check drops those loads and stores)
        e.tof[p] = ok ? ((unsigned)tk * (unsigned)a.ldx + 4u * jl) * 4u : 0x80000000u;
        e.cof[p] = ok ? ((unsigned)token_to_win(tk, a.cwm) * (unsigned)a.ldc + 4u * jl) * 2u : 0x80000000u;
#pragma unroll
        for (int k = 0; k < 3; ++k) e.xv[p][k] = bld4(rx, e.tof[p] + 256u * k);
      }
    } else if constexpr (EPI == EPI_GATE) {
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const int q = tid + NT * i, r = q / NCH, c8 = (q - r * NCH) * 8;
        const long row = row0 + r < a.M ? row0 + r : a.M - 1;
        if (q < NCHUNK) e.gv[i] = *(const uint4*)(a.gate + row * a.ldg + c8);
      }
    }
  };
  bf16x8 ra[KBW];
  auto load_a = [&](long t) {
    long r = t * RT + l31;
    if (r >= a.M) r = a.M - 1;
    const bf16* ap = a.A + r * a.lda + 8 * hh + 16 * KBW * ks;
#pragma unroll
    for (int i = 0; i < KBW; ++i) ra[i] = *(const bf16x8*)(ap + 16 * i);
  };

  // one tile: k-loop on the landed A rows, prefetch of the next tile (A, epilogue operands) under the
  // partial-sum exchange and the epilogue
  auto run_tile = [&](long t, E& cur, E& nxt) {
    const long row0 = t * RT;
    f32x16 acc[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[ct][r] = 0.f;
    // streamed fragments f = NCT i + ct through a ring of SD registers: the first SD in flight under
    // the resident steps' MFMAs, each slot refilled right after the MFMA that read it (left to itself
    // the scheduler sinks every load to its use under the register budget: 12 serial L2 round trips)
    constexpr int NF = NSTR * NCT, SDM = EPI == EPI_GATE ? 2 : 4, SD = NF < SDM ? (NF > 0 ? NF : 1) : SDM;
    auto sfrag = [&](int f) { return bld16(rW, wl, ((f % NCT) * KB + ks * KBW + HOLD + f / NCT) * 1024u); };
    bf16x8 rs_[SD];
#pragma unroll
    for (int f = 0; f < SD && f < NF; ++f) rs_[f] = sfrag(f);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < HOLD; ++i)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra[i], rw[i][ct], acc[ct], 0, 0, 0);
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      acc[f % NCT] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra[HOLD + f / NCT], rs_[f % SD], acc[f % NCT], 0, 0, 0);
      if (f + SD < NF) rs_[f % SD] = sfrag(f + SD);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_sched_barrier(0);
    float4 dv[LPASS][3];
    if constexpr (EPI == EPI_LN) {   // D of this lane's rows: in flight across the exchange
#pragma unroll
      for (int p = 0; p < LPASS; ++p)
#pragma unroll
        for (int k = 0; k < 3; ++k) dv[p][k] = bld4(rD, cur.tof[p] + 256u * k);
    }
    const long tn = t + G;
    if (tn < a.ntiles) {
      load_epi(tn, nxt);
      load_a(tn);
    }
    __syncthreads();   // the previous tile's epilogue has read sY
    float* pl = sY + ks * PLANE;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) pl[acc_row(r, hh) * LDY + c0 + 32 * ct] = acc[ct][r];
    __syncthreads();

    if constexpr (EPI == EPI_STORE || EPI == EPI_GATE) {
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const int q = tid + NT * i, r = q / NCH, c8 = (q - r * NCH) * 8;
        if (q >= NCHUNK) break;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int g = 0; g < KS; ++g) {
          const float4 y0 = *(const float4*)(sY + g * PLANE + r * LDY + c8);
          const float4 y1 = *(const float4*)(sY + g * PLANE + r * LDY + c8 + 4);
          v[0] += y0.x; v[1] += y0.y; v[2] += y0.z; v[3] += y0.w;
          v[4] += y1.x; v[5] += y1.y; v[6] += y1.z; v[7] += y1.w;
        }
        if constexpr (EPI == EPI_GATE) {
          const bf16x8 gg = __builtin_bit_cast(bf16x8, cur.gv[i]);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] *= (float)gg[j];
        }
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
        if (row0 + r < a.M) *(bf16x8*)(a.out + (row0 + r) * a.ldo + c8) = o;
      }
    } else {
      // LayerNorm backward (ln_bwd_kernel maths, layernorm.hip), one row per 16 lanes: with
      // xh = (x - mu) rstd, gy = dy gamma:  dx = rstd (gy - mean_c(gy) - xh mean_c(gy xh)),
      // dgamma += dy xh, dbeta += dy (rows past M contribute 0: their dy is read as 0 below).
      // dy and xh are formed twice (row sums, then the outputs) instead of being held in registers.
#pragma unroll
      for (int p = 0; p < LPASS; ++p) {
        const int tr = RPP * p + lr;
        const float live = row0 + tr < a.M ? 1.f : 0.f;
        auto dyxh = [&](int k, float* dy, float* xh) {
          float4 d4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int g = 0; g < KS; ++g) {
            const float4 y = *(const float4*)(sY + g * PLANE + tr * LDY + 4 * jl + 64 * k);
            d4.x += y.x; d4.y += y.y; d4.z += y.z; d4.w += y.w;
          }
          const float da[4] = {d4.x, d4.y, d4.z, d4.w};
          const float xa[4] = {cur.xv[p][k].x, cur.xv[p][k].y, cur.xv[p][k].z, cur.xv[p][k].w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const bool in = 4 * jl + 64 * k + j < a.C;
            dy[j] = live * da[j];   // 0 past C: the packed weight rows are 0 there
            xh[j] = in ? (xa[j] - cur.mu[p]) * cur.rs[p] : 0.f;
          }
        };
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          float dy[4], xh[4];
          dyxh(k, dy, xh);
          const float4 g4k = *(const float4*)(sGam + 4 * jl + 64 * k);
          const float ga[4] = {g4k.x, g4k.y, g4k.z, g4k.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float gy = dy[j] * ga[j];
            s1 += gy;
            s2 += gy * xh[j];
          }
        }
        s1 = dpp_sum16(s1) * a.inv_c;
        s2 = dpp_sum16(s2) * a.inv_c;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          float dy[4], xh[4];
          dyxh(k, dy, xh);
          const float4 g4k = *(const float4*)(sGam + 4 * jl + 64 * k);
          const float ga[4] = {g4k.x, g4k.y, g4k.z, g4k.w};
          const float cu[4] = {dv[p][k].x, dv[p][k].y, dv[p][k].z, dv[p][k].w};
          float o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)   // columns past C keep their value
            o[j] = 4 * jl + 64 * k + j < a.C ? cu[j] + cur.rs[p] * (dy[j] * ga[j] - s1 - xh[j] * s2) : cu[j];
          bst4(rD, cur.tof[p] + 256u * k, make_float4(o[0], o[1], o[2], o[3]));
          const float sc = cur.sc[p];
          const bf16x4 cb = {(bf16)(sc * o[0]), (bf16)(sc * o[1]), (bf16)(sc * o[2]), (bf16)(sc * o[3])};
          bst8(rC, cur.cof[p] + 128u * k, cb);
          float4* sg = (float4*)(sP + lr * 2 * 192 + 4 * jl + 64 * k);
          float4* sb = (float4*)(sP + lr * 2 * 192 + 192 + 4 * jl + 64 * k);
          float4 g4 = *sg, b4 = *sb;
          g4.x += dy[0] * xh[0]; g4.y += dy[1] * xh[1]; g4.z += dy[2] * xh[2]; g4.w += dy[3] * xh[3];
          b4.x += dy[0]; b4.y += dy[1]; b4.z += dy[2]; b4.w += dy[3];
          *sg = g4;
          *sb = b4;
        }
      }
    }
  };

  E e0, e1;
  load_epi(tile, e0);
  load_a(tile);
  for (;;) {   // unrolled by two so the double-buffered operands stay in fixed registers
    run_tile(tile, e0, e1);
    tile += G;
    if (tile >= a.ntiles) break;
    run_tile(tile, e1, e0);
    tile += G;
    if (tile >= a.ntiles) break;
  }

  if constexpr (EPI == EPI_LN) {   // this workgroup's dgamma / dbeta partials: the row groups' LDS slots
    __syncthreads();               // summed in fixed order (deterministic)
    for (int c = tid; c < 2 * 192; c += NT) {
      float t = 0.f;
#pragma unroll
      for (int g = 0; g < RPP; ++g) t += sP[g * 2 * 192 + c];
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

// persistent grid: one workgroup per CU (the K-split planes take ~100 KB of LDS), at most one per tile
template <int KB, int KS, int NWC, int EPI, int HOLD = KB / KS>
int rg_launch(const RgArgs& a, hipStream_t s, long* grid_out) {
  auto kern = rowgemm_kernel<KB, KS, NWC, EPI, HOLD>;
  static int per_cu = 0;   // workgroups per CU at this instantiation's occupancy (one cache each)
  if (per_cu == 0) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, 64 * NWC * KS, 0) != hipSuccess || n <= 0) n = 1;
    per_cu = n;
  }
  const long tiles = (a.M + RT - 1) / RT, slots = (long)rg_cus() * per_cu;
  const long grid = tiles < slots ? tiles : slots;
  if (grid_out) { *grid_out = grid; return 0; }
  KAIR_LAUNCH(kern, dim3((unsigned)grid), dim3(64 * NWC * KS), 0, s, a);
  KAIR_CHECK_LAUNCH();
  return 0;
}

// grid_out != NULL: report the grid (the LN partial count) without launching.  N = 192: K in
// {192, 384, 576}; N = 384 (the fc2 input gradient): K = 192.  HOLD (weight k-steps held in registers)
// measured: fc1 + LN2 all 6 (a 12-byte spill) and q/k/v + LN1 5 of 9 (20 bytes) beat 5 / 4 with no spill
// (B = 32 1291 -> 1300, B = 4 558 -> 569); 6 of 9 spills 64 bytes and loses.
template <int EPI>
int rg_dispatch(int K, int N, const RgArgs& a, hipStream_t s, long* grid_out = nullptr) {
  if (N == 384) {
    if constexpr (EPI != EPI_LN)
      if (K == 192) return rg_launch<12, 2, 4, EPI>(a, s, grid_out);
    return kair_set_error(KAIR_ERR_ARG, "rowgemm: N = 384 needs K = 192 (got %d)", K);
  }
  switch (K) {
    case 192: return rg_launch<12, 4, 2, EPI>(a, s, grid_out);
    case 384: return rg_launch<24, 4, 2, EPI, 6>(a, s, grid_out);
    case 576: return rg_launch<36, 4, 2, EPI, EPI == EPI_LN ? 5 : EPI == EPI_GATE ? 7 : 9>(a, s, grid_out);
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
  if (rg_dispatch<EPI_LN>(K, 192, a, nullptr, &g) != 0) return -1;
  return g;
}

extern "C" int kair_rowgemm_store(const void* A, long lda, long M, int K, const void* W, int N, void* out, long ldo,
                                  void* stream) {
  RgArgs a;
  if (int rc = rg_common(A, lda, M, K, W, N, a)) return rc;
  KAIR_CHECK_ARG(out && ldo >= N, "rowgemm_store: out");
  a.out = (bf16*)out; a.ldo = ldo;
  hipStream_t s = (hipStream_t)stream;
  return rg_dispatch<EPI_STORE>(K, N, a, s);
}

extern "C" int kair_rowgemm_gate(const void* A, long lda, long M, int K, const void* W, int N, const void* gate, long ldg,
                                 void* out, long ldo, void* stream) {
  RgArgs a;
  if (int rc = rg_common(A, lda, M, K, W, N, a)) return rc;
  KAIR_CHECK_ARG(out && ldo >= N && gate && ldg >= N, "rowgemm_gate: out / gate");
  a.out = (bf16*)out; a.ldo = ldo; a.gate = (const bf16*)gate; a.ldg = ldg;
  hipStream_t s = (hipStream_t)stream;
  return rg_dispatch<EPI_GATE>(K, N, a, s);
}

extern "C" int kair_rowgemm_lnbwd(const void* A, long lda, long M, int K, const void* W, const float* x, long ldx,
                                  const float* gamma, const float* mean, const float* rstd, int C, float* D, long ldD,
                                  int win_H, int win_W, int win_ws, int win_shift, const kair_copy_desc* copy, float* part,
                                  void* stream) {
  RgArgs a;
  if (int rc = rg_common(A, lda, M, K, W, 192, a)) return rc;
  KAIR_CHECK_ARG(x && gamma && mean && rstd && D && part, "rowgemm_lnbwd: null pointer");
  // the LN epilogue reads and writes all 192 columns of every x / D row (and of every copy row): a
  // shorter stride would overlap neighbouring rows
  KAIR_CHECK_ARG(C > 0 && C <= 192 && ldx >= 192 && ldD >= 192, "rowgemm_lnbwd: C %d must be <= 192, ldx / ldD >= 192", C);
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
    KAIR_CHECK_ARG(copy->dtype == KAIR_BF16 && copy->ld >= 192, "rowgemm_lnbwd: the copy is bf16 rows, ld >= 192");
    KAIR_CHECK_ARG(copy->win_ws == 0 || (copy->win_H % copy->win_ws == 0 && copy->win_W % copy->win_ws == 0),
                   "rowgemm_lnbwd: copy window geometry");
    a.cp = (bf16*)copy->out; a.ldc = copy->ld; a.cp_scale = copy->rowscale;
    a.cbytes = M * copy->ld * 2;
    a.cp_rps = copy->rows_per_scale > 0 ? copy->rows_per_scale : 1;
    a.cwm = make_winmap(copy->win_H, copy->win_W, copy->win_ws, copy->win_shift);
  }
  return rg_dispatch<EPI_LN>(K, 192, a, (hipStream_t)stream);
}
