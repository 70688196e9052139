// LayerNorm over the channel dim of token matrices (nn.LayerNorm(C), eps 1e-5:
// network_swinir.py:199,205,520,725).  16 lanes own one token row (4 rows per wave64), each lane
// holding float4 column groups, so a wave keeps four independent rows in flight and the row
// reductions are 4 shuffle steps.  The forward can write its output straight into Swin window
// order (the gather that torch.roll + window_partition perform in network_swinir.py:250-256), so the
// QKV GEMM reads a plain row-major operand.  Backward accumulates into the fp32 residual-stream
// gradient and produces deterministic per-block partial sums for dgamma / dbeta.
#include <stdlib.h>

#include <string.h>

#include <type_traits>

#include "common.h"

namespace {

constexpr int LPR = 16;              // lanes per row
constexpr int NV = 4;                // float4 groups per lane: C <= 16 * 4 * 4 = 256
constexpr int ROWS_PER_BLOCK_ITER = 16;  // 4 waves x 4 rows

KAIR_DEV float group_sum16(float v) {
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T> KAIR_DEV void store4(T* p, float a, float b, float c, float d);
template <> KAIR_DEV void store4<float>(float* p, float a, float b, float c, float d) {
  *(float4*)p = make_float4(a, b, c, d);
}
template <> KAIR_DEV void store4<bf16>(bf16* p, float a, float b, float c, float d) {
  bf16x4 q = {(bf16)a, (bf16)b, (bf16)c, (bf16)d};
  *(bf16x4*)p = q;
}
// x3 fp16 pair of 4 values: hi = f16(v s), lo = f16(v s - hi) (the fp32x3 engine's GEMM operand format)
KAIR_DEV void store4_pair(f16* hi, f16* lo, long off, float a, float b, float c, float d, float s) {
  const float w[4] = {a * s, b * s, c * s, d * s};
  f16x4 h, l;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    h[j] = (f16)w[j];
    l[j] = (f16)(w[j] - (float)h[j]);
  }
  *(f16x4*)(hi + off) = h;
  *(f16x4*)(lo + off) = l;
}
template <typename T> KAIR_DEV float4 load4(const T* p);
template <> KAIR_DEV float4 load4<float>(const float* p) { return *(const float4*)p; }
template <> KAIR_DEV float4 load4<bf16>(const bf16* p) {
  const bf16x4 q = *(const bf16x4*)p;
  return make_float4((float)q[0], (float)q[1], (float)q[2], (float)q[3]);
}

// T = f16: y / y_lo are the hi / lo planes of the x3 pair of y 2^e (ys = 2^e)
template <typename T>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, long ldx, T* __restrict__ y, long ldy,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      float* __restrict__ mean_out, float* __restrict__ rstd_out, long M,
                                                      int C, float eps, WinMap wm, int one_col, f16* __restrict__ y_lo,
                                                      float ys) {
  const int sub = threadIdx.x & (LPR - 1);
  const long grp = (long)blockIdx.x * ROWS_PER_BLOCK_ITER + (threadIdx.x >> 4);
  const long ng = (long)gridDim.x * ROWS_PER_BLOCK_ITER;
  // this lane's affine parameters, loaded once (not per row and element)
  float ga[NV][4], be[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = (sub + LPR * i) * 4 + j;
      ga[i][j] = c < C ? gamma[c] : 0.f;
      be[i][j] = c < C ? beta[c] : (c == one_col ? 1.f : 0.f);   // ones column for the weight-gradient GEMM
    }
  // two rows per iteration, both rows' loads issued before either is reduced: one dependent load per row left each
  // 16-lane group latency-bound on its rows (C <= 64: a single float4 per lane and row)
  auto load_row = [&](long r, float4 (&v)[NV]) {
    const long t = win_to_token(r, wm);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (sub + LPR * i) * 4;
      v[i] = c < C ? *(const float4*)(x + t * ldx + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    return t;
  };
  auto finish_row = [&](long r, long t, float4 (&v)[NV]) {   // r = output row (window order if wm.ws > 0)
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (sub + LPR * i) * 4;
      if (c + 4 > C) {  // column group straddling C: pad lanes do not count
        if (c + 1 >= C) v[i].y = 0.f;
        if (c + 2 >= C) v[i].z = 0.f;
        if (c + 3 >= C) v[i].w = 0.f;
      }
      s += v[i].x + v[i].y + v[i].z + v[i].w;
    }
    const float mu = group_sum16(s) / C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (sub + LPR * i) * 4;
      if (c < C) {
        const float a = v[i].x - mu, b = v[i].y - mu, cc = v[i].z - mu, d = v[i].w - mu;
        // the column group straddling C (C % 4 != 0) must not count pad lanes
        q += a * a + (c + 1 < C ? b * b : 0.f) + (c + 2 < C ? cc * cc : 0.f) + (c + 3 < C ? d * d : 0.f);
      }
    }
    const float rs = rsqrtf(group_sum16(q) / C + eps);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (sub + LPR * i) * 4;
      if (c < ldy) {
        float o[4];
        const float xv[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (xv[j] - mu) * rs * ga[i][j] + be[i][j];   // pad columns: 0 (or the ones column)
        if constexpr (sizeof(T) == 2 && !std::is_same_v<T, bf16>) store4_pair(y, y_lo, r * ldy + c, o[0], o[1], o[2], o[3], ys);
        else store4<T>(y + r * ldy + c, o[0], o[1], o[2], o[3]);
      }
    }
    if (sub == 0) {
      mean_out[t] = mu;
      rstd_out[t] = rs;
    }
  };
  long r = grp;
  for (; r + ng < M; r += 2 * ng) {
    float4 va[NV], vb[NV];
    const long ta = load_row(r, va), tb = load_row(r + ng, vb);
    finish_row(r, ta, va);
    finish_row(r + ng, tb, vb);
  }
  if (r < M) {
    float4 va[NV];
    const long ta = load_row(r, va);
    finish_row(r, ta, va);
  }
}

// NVK: float4 groups per lane (NV; 1 for C <= 64 -- SwinIR-lightweight's 60 -- where the narrow form keeps two rows
// in flight per 16-lane group: both rows' x / dy / mean / rstd / accumulated-gradient loads before either reduction)
template <typename T, int NVK>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ x, long ldx, const T* __restrict__ dy,
                                                      long ldy, const float* __restrict__ gamma,
                                                      const float* __restrict__ mean, const float* __restrict__ rstd,
                                                      float* dx, long ld_dx, int dx_acc, float* __restrict__ part,
                                                      long M, int C, WinMap wm, void* cp, int cp_dt, long ldc,
                                                      const float* __restrict__ cp_scale, int cp_rps, WinMap cwm,
                                                      f16* __restrict__ cp_lo, float cp_s) {
  const int sub = threadIdx.x & (LPR - 1);
  const long grp = (long)blockIdx.x * ROWS_PER_BLOCK_ITER + (threadIdx.x >> 4);
  const long ng = (long)gridDim.x * ROWS_PER_BLOCK_ITER;
  float dg[NV][4], db[NV][4], g[NVK][4];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = (sub + LPR * i) * 4 + j;
      dg[i][j] = db[i][j] = 0.f;
      if (i < NVK) g[i < NVK ? i : 0][j] = c < C ? gamma[c] : 0.f;
    }
  struct RowIn { long t; float mu, rs; float4 xv[NVK], dv[NVK], cur[NVK]; };
  auto load_row = [&](long r, RowIn& in) {
    const long t = win_to_token(r, wm);
    in.t = t;
    in.mu = mean[t];
    in.rs = rstd[t];
#pragma unroll
    for (int i = 0; i < NVK; ++i) {
      const int c = (sub + LPR * i) * 4;
      float4 xv = make_float4(0.f, 0.f, 0.f, 0.f), dv = xv, cu = xv;
      if (c < C) {
        xv = *(const float4*)(x + t * ldx + c);
        dv = load4<T>(dy + r * ldy + c);
        if (dx_acc) cu = *(const float4*)(dx + t * ld_dx + c);
      }
      in.xv[i] = xv; in.dv[i] = dv; in.cur[i] = cu;
    }
  };
  auto finish_row = [&](RowIn& in) {
    const long t = in.t;
    const float mu = in.mu, rs = in.rs;
    float xh[NVK][4], gy[NVK][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NVK; ++i) {
      const int c = (sub + LPR * i) * 4;
      const float4 xv = in.xv[i], dv = in.dv[i];
      const float xa[4] = {xv.x, xv.y, xv.z, xv.w}, da[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool ok = c + j < C;
        xh[i][j] = ok ? (xa[j] - mu) * rs : 0.f;
        const float d = ok ? da[j] : 0.f;
        gy[i][j] = d * g[i][j];
        dg[i][j] += d * xh[i][j];
        db[i][j] += d;
        s1 += gy[i][j];
        s2 += gy[i][j] * xh[i][j];
      }
    }
    s1 = group_sum16(s1) / C;
    s2 = group_sum16(s2) / C;
    // GEMM-operand copy row and scale: once per row
    const float sc = cp && cp_scale ? cp_scale[(int)t / cp_rps] : 1.f;
    const long cr = cp ? token_to_win(t, cwm) : 0;
#pragma unroll
    for (int i = 0; i < NVK; ++i) {
      const int c = (sub + LPR * i) * 4;
      if (c < C) {
        float* o = dx + t * ld_dx + c;
        float4 cu = in.cur[i];
        float d[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = (c + j < C) ? rs * (gy[i][j] - s1 - xh[i][j] * s2) : 0.f;
        cu.x += d[0]; cu.y += d[1]; cu.z += d[2]; cu.w += d[3];
        *(float4*)o = cu;
        if (cp) {   // GEMM-operand copy of the finished gradient row: scaled, cast, optionally window-ordered
          if (cp_dt == KAIR_BF16) store4<bf16>((bf16*)cp + cr * ldc + c, sc * cu.x, sc * cu.y, sc * cu.z, sc * cu.w);
          else if (cp_dt == KAIR_F16)   // (opaque products: the pair splits the fp32-rounded value, common.h)
            store4_pair((f16*)cp, cp_lo, cr * ldc + c, opaque(sc * cu.x), opaque(sc * cu.y), opaque(sc * cu.z),
                        opaque(sc * cu.w), cp_s);
          else store4<float>((float*)cp + cr * ldc + c, sc * cu.x, sc * cu.y, sc * cu.z, sc * cu.w);
        }
      }
    }
  };
  if constexpr (NVK == 1) {
    long r = grp;
    for (; r + ng < M; r += 2 * ng) {
      RowIn ra, rb;
      load_row(r, ra);
      load_row(r + ng, rb);
      finish_row(ra);
      finish_row(rb);
    }
    if (r < M) {
      RowIn ra;
      load_row(r, ra);
      finish_row(ra);
    }
  } else {   // (the wide form: one row per iteration, as measured for the classical geometry)
    for (long r = grp; r < M; r += ng) {
      const long t = win_to_token(r, wm);
      const float mu = mean[t], rs = rstd[t];
      float xh[NV][4], gy[NV][4];
      float4 cur[NV];   // the accumulated gradient row, loaded together with x and dy (one round trip)
      float s1 = 0.f, s2 = 0.f;
  #pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = (sub + LPR * i) * 4;
        float4 xv = make_float4(0.f, 0.f, 0.f, 0.f), dv = xv;
        cur[i] = xv;
        if (c < C) {
          xv = *(const float4*)(x + t * ldx + c);
          dv = load4<T>(dy + r * ldy + c);
          if (dx_acc) cur[i] = *(const float4*)(dx + t * ld_dx + c);
        }
        const float xa[4] = {xv.x, xv.y, xv.z, xv.w}, da[4] = {dv.x, dv.y, dv.z, dv.w};
  #pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool ok = c + j < C;
          xh[i][j] = ok ? (xa[j] - mu) * rs : 0.f;
          const float d = ok ? da[j] : 0.f;
          gy[i][j] = d * g[i][j];
          dg[i][j] += d * xh[i][j];
          db[i][j] += d;
          s1 += gy[i][j];
          s2 += gy[i][j] * xh[i][j];
        }
      }
      s1 = group_sum16(s1) / C;
      s2 = group_sum16(s2) / C;
      // GEMM-operand copy row and scale: once per row
      const float sc = cp && cp_scale ? cp_scale[(int)t / cp_rps] : 1.f;
      const long cr = cp ? token_to_win(t, cwm) : 0;
  #pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = (sub + LPR * i) * 4;
        if (c < C) {
          float* o = dx + t * ld_dx + c;
          float4 cu = cur[i];
          float d[4];
  #pragma unroll
          for (int j = 0; j < 4; ++j) d[j] = (c + j < C) ? rs * (gy[i][j] - s1 - xh[i][j] * s2) : 0.f;
          cu.x += d[0]; cu.y += d[1]; cu.z += d[2]; cu.w += d[3];
          *(float4*)o = cu;
          if (cp) {   // GEMM-operand copy of the finished gradient row: scaled, cast, optionally window-ordered
            if (cp_dt == KAIR_BF16) store4<bf16>((bf16*)cp + cr * ldc + c, sc * cu.x, sc * cu.y, sc * cu.z, sc * cu.w);
            else if (cp_dt == KAIR_F16)   // (opaque products: the pair splits the fp32-rounded value, common.h)
              store4_pair((f16*)cp, cp_lo, cr * ldc + c, opaque(sc * cu.x), opaque(sc * cu.y), opaque(sc * cu.z),
                          opaque(sc * cu.w), cp_s);
            else store4<float>((float*)cp + cr * ldc + c, sc * cu.x, sc * cu.y, sc * cu.z, sc * cu.w);
          }
        }
      }
    }
  }
  // block reduction of dgamma/dbeta partials: 16 row-groups share each column (fixed order); one
  // 16.6 KB buffer used twice (dgamma, then dbeta) so LDS admits more resident blocks per CU
  __shared__ float red[16][260];
  const int rg = threadIdx.x >> 4;
  for (int w = 0; w < 2; ++w) {
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[rg][(sub + LPR * i) * 4 + j] = w == 0 ? dg[i][j] : db[i][j];
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) s += red[k][c];
      part[(long)blockIdx.x * 2 * C + w * C + c] = s;
    }
    __syncthreads();
  }
}

// 8 columns per 256-thread block, 32 row-phases per column, fixed summation order (deterministic).
// Many small blocks: the reduction reads an L2-resident [nb][2C] partial array and is latency-bound,
// so it wants every CU issuing loads rather than a handful of wide blocks.
__global__ __launch_bounds__(256) void ln_param_reduce(const float* __restrict__ part, int nb, int C, float* dgamma,
                                                       float* dbeta, int acc) {
  __shared__ float red[32][8];
  const int tx = threadIdx.x & 7, ty = threadIdx.x >> 3;
  const int c = blockIdx.x * 8 + tx;
  float s0 = 0.f, s1 = 0.f;
  if (c < 2 * C) {
    int b = ty;
    // 8 loads in flight per thread, then the same alternating s0/s1 order as the pair loop below
    for (; b + 224 < nb; b += 256) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(long)(b + 32 * u) * 2 * C + c];
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        s0 += v[u];
        s1 += v[u + 1];
      }
    }
    for (; b + 32 < nb; b += 64) {
      s0 += part[(long)b * 2 * C + c];
      s1 += part[(long)(b + 32) * 2 * C + c];
    }
    if (b < nb) s0 += part[(long)b * 2 * C + c];
  }
  red[ty][tx] = s0 + s1;
  __syncthreads();
  if (ty == 0 && c < 2 * C) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) s += red[k][tx];
    float* o = c < C ? dgamma + c : dbeta + (c - C);
    *o = acc ? *o + s : s;
  }
}

// every deferred LayerNorm parameter reduction of a group (kair_ln_param_reduce_grouped): block ->
// job by a scalar scan; the same fixed-order sums as ln_param_reduce
struct LnParamJob { const float* part; float* dgamma; float* dbeta; int nb, C, acc, blk0; };
constexpr int LNP_MAX = 32;
struct LnParamGroup { LnParamJob j[LNP_MAX]; int njobs; };

__global__ __launch_bounds__(256) void ln_param_reduce_grouped(const LnParamGroup g) {
  int ji = 0;
  for (int i = 1; i < g.njobs; ++i)
    if (g.j[i].blk0 <= (int)blockIdx.x) ji = i;
  ji = __builtin_amdgcn_readfirstlane(ji);
  const LnParamJob& jb = g.j[ji];
  const int C = jb.C, nb = jb.nb;
  const float* part = jb.part;
  __shared__ float red[32][8];
  const int tx = threadIdx.x & 7, ty = threadIdx.x >> 3;
  const int c = ((int)blockIdx.x - jb.blk0) * 8 + tx;
  float s0 = 0.f, s1 = 0.f;
  if (c < 2 * C) {
    int b = ty;
    for (; b + 224 < nb; b += 256) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(long)(b + 32 * u) * 2 * C + c];
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        s0 += v[u];
        s1 += v[u + 1];
      }
    }
    for (; b + 32 < nb; b += 64) {
      s0 += part[(long)b * 2 * C + c];
      s1 += part[(long)(b + 32) * 2 * C + c];
    }
    if (b < nb) s0 += part[(long)b * 2 * C + c];
  }
  red[ty][tx] = s0 + s1;
  __syncthreads();
  if (ty == 0 && c < 2 * C) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) s += red[k][tx];
    float* o = c < C ? jb.dgamma + c : jb.dbeta + (c - C);
    *o = jb.acc ? *o + s : s;
  }
}

}  // namespace

constexpr int LN_BLOCKS = 2048;

static long ln_bwd_blocks(long M) {
  long nb = (M + ROWS_PER_BLOCK_ITER - 1) / ROWS_PER_BLOCK_ITER;
  return nb > LN_BLOCKS ? LN_BLOCKS : nb;
}

extern "C" long kair_layernorm_bwd_blocks(long M) { return M > 0 ? ln_bwd_blocks(M) : 0; }

extern "C" int kair_ln_param_reduce_grouped(const kair_ln_param_job* jobs, int njobs, void* stream) {
  KAIR_CHECK_ARG(jobs && njobs > 0 && njobs <= LNP_MAX, "ln_param_reduce_grouped: 1..%d jobs", LNP_MAX);
  LnParamGroup g;
  memset(&g, 0, sizeof(g));
  int blk = 0;
  for (int i = 0; i < njobs; ++i) {
    const kair_ln_param_job& J = jobs[i];
    KAIR_CHECK_ARG(J.part && J.dgamma && J.dbeta && J.C > 0 && J.C <= 256 && J.nb > 0,
                   "ln_param_reduce_grouped: job %d", i);
    g.j[i] = LnParamJob{J.part, J.dgamma, J.dbeta, (int)J.nb, J.C, J.accumulate ? 1 : 0, blk};
    blk += (2 * J.C + 7) / 8;
  }
  g.njobs = njobs;
  KAIR_LAUNCH(ln_param_reduce_grouped, dim3(blk), dim3(256), 0, (hipStream_t)stream, g);
  KAIR_CHECK_LAUNCH();
  return 0;
}  // ws holds LN_BLOCKS * 2 * C floats (kair_hip.h)

extern "C" int kair_layernorm_fwd(const float* x, long ldx, void* y, int y_dtype, long ldy, const float* gamma,
                                  const float* beta, float* mean, float* rstd, long M, int C, float eps, int win_H,
                                  int win_W, int win_ws, int win_shift, int one_col, void* stream) {
  KAIR_CHECK_ARG(x && y && gamma && beta && mean && rstd, "layernorm_fwd: null pointer");
  KAIR_CHECK_ARG(C > 0 && C <= 256 && ldx >= C && ldy >= C && ldy <= 256 && M > 0 && M < KAIR_MAX_MAPPED_ROWS,
                 "layernorm_fwd: bad sizes");
  KAIR_CHECK_ARG(ldx % 4 == 0 && ldy % 4 == 0 && ((uintptr_t)x % 16) == 0, "layernorm_fwd: strides must be multiples of 4");
  KAIR_CHECK_ARG(win_ws == 0 || (win_H % win_ws == 0 && win_W % win_ws == 0), "layernorm_fwd: window geometry");
  KAIR_CHECK_ARG(one_col < 0 || (one_col >= C && one_col < ldy), "layernorm_fwd: ones column must be a pad column");
  const WinMap wm = make_winmap(win_H, win_W, win_ws, win_shift);
  long nb = (M + ROWS_PER_BLOCK_ITER - 1) / ROWS_PER_BLOCK_ITER;
  // 1024 blocks (4 per CU): each 16-lane row group normalises several rows on the affine
  // parameters it loaded once (measured at B = 32: 8192 blocks 28.5 us -> 1024 blocks 18.3 us)
  constexpr long max_nb = 1024;
  if (nb > max_nb) nb = max_nb;
  hipStream_t s = (hipStream_t)stream;
  if (y_dtype == KAIR_BF16)
    KAIR_LAUNCH(ln_fwd_kernel<bf16>, dim3((unsigned)nb), dim3(256), 0, s, x, ldx, (bf16*)y, ldy, gamma, beta,
                       mean, rstd, M, C, eps, wm, one_col, (f16*)nullptr, 1.f);
  else
    KAIR_LAUNCH(ln_fwd_kernel<float>, dim3((unsigned)nb), dim3(256), 0, s, x, ldx, (float*)y, ldy, gamma, beta,
                       mean, rstd, M, C, eps, wm, one_col, (f16*)nullptr, 1.f);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_layernorm_fwd_x3(const float* x, long ldx, void* y_hi, void* y_lo, long ldy, const float* gamma,
                                     const float* beta, float* mean, float* rstd, long M, int C, float eps, int win_H,
                                     int win_W, int win_ws, int win_shift, int one_col, int x3_exp, void* stream) {
  KAIR_CHECK_ARG(x && y_hi && y_lo && gamma && beta && mean && rstd, "layernorm_fwd_x3: null pointer");
  KAIR_CHECK_ARG(C > 0 && C <= 256 && ldx >= C && ldy >= C && ldy <= 256 && M > 0 && M < KAIR_MAX_MAPPED_ROWS,
                 "layernorm_fwd_x3: bad sizes");
  KAIR_CHECK_ARG(ldx % 4 == 0 && ldy % 4 == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)y_hi % 8) == 0 &&
                     ((uintptr_t)y_lo % 8) == 0,
                 "layernorm_fwd_x3: strides / alignment");
  KAIR_CHECK_ARG(win_ws == 0 || (win_H % win_ws == 0 && win_W % win_ws == 0), "layernorm_fwd_x3: window geometry");
  KAIR_CHECK_ARG(one_col < 0 || (one_col >= C && one_col < ldy), "layernorm_fwd_x3: ones column must be a pad column");
  KAIR_CHECK_ARG(x3_exp > -100 && x3_exp < 100, "layernorm_fwd_x3: exponent");
  const WinMap wm = make_winmap(win_H, win_W, win_ws, win_shift);
  long nb = (M + ROWS_PER_BLOCK_ITER - 1) / ROWS_PER_BLOCK_ITER;
  if (nb > 1024) nb = 1024;
  KAIR_LAUNCH(ln_fwd_kernel<f16>, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, x, ldx, (f16*)y_hi, ldy,
                     gamma, beta, mean, rstd, M, C, eps, wm, one_col, (f16*)y_lo, ldexpf(1.f, x3_exp));
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_layernorm_bwd(const float* x, long ldx, const void* dy, int dy_dtype, long ldy, const float* gamma,
                                  const float* mean, const float* rstd, float* dx_acc, long ld_dx, int dx_accumulate,
                                  float* dgamma, float* dbeta, int dparam_accumulate, float* ws, long M, int C,
                                  int win_H, int win_W, int win_ws, int win_shift, const kair_copy_desc* copy,
                                  void* stream) {
  KAIR_CHECK_ARG(x && dy && gamma && mean && rstd && dx_acc && ws && (dgamma != nullptr) == (dbeta != nullptr),
                 "layernorm_bwd: null pointer");
  KAIR_CHECK_ARG(C > 0 && C <= 256 && M > 0 && M < KAIR_MAX_MAPPED_ROWS, "layernorm_bwd: bad sizes");
  KAIR_CHECK_ARG(ldx % 4 == 0 && ldy % 4 == 0 && ld_dx % 4 == 0, "layernorm_bwd: strides must be multiples of 4");
  const WinMap wm = make_winmap(win_H, win_W, win_ws, win_shift);
  void* cp = nullptr;
  f16* cp_lo = nullptr;
  float cp_s = 1.f;
  int cp_dt = KAIR_F32, cp_rps = 1;
  long ldc = 0;
  const float* cp_scale = nullptr;
  WinMap cwm = make_winmap(0, 0, 0, 0);
  if (copy && copy->out) {
    KAIR_CHECK_ARG(copy->ld % 4 == 0 && copy->ld >= C, "layernorm_bwd: copy stride");
    KAIR_CHECK_ARG(copy->win_ws == 0 || (copy->win_H % copy->win_ws == 0 && copy->win_W % copy->win_ws == 0),
                   "layernorm_bwd: copy window geometry");
    cp = copy->out; cp_dt = copy->dtype; ldc = copy->ld; cp_scale = copy->rowscale;
    cp_rps = copy->rows_per_scale > 0 ? copy->rows_per_scale : 1;
    cwm = make_winmap(copy->win_H, copy->win_W, copy->win_ws, copy->win_shift);
    if (cp_dt == KAIR_F16) {
      KAIR_CHECK_ARG(copy->out_lo && ((uintptr_t)copy->out % 8) == 0 && ((uintptr_t)copy->out_lo % 8) == 0,
                     "layernorm_bwd: an fp16 pair copy needs its 8-byte aligned lo plane (out_lo)");
      cp_lo = (f16*)copy->out_lo;
      cp_s = ldexpf(1.f, copy->x3_exp);
    }
  }
  hipStream_t s = (hipStream_t)stream;
  const long nb = ln_bwd_blocks(M);
#define KAIR_LNB(TT, NVV)                                                                                            \
  KAIR_LAUNCH((ln_bwd_kernel<TT, NVV>), dim3((unsigned)nb), dim3(256), 0, s, x, ldx, (const TT*)dy, ldy, gamma, mean, rstd, \
              dx_acc, ld_dx, dx_accumulate, ws, M, C, wm, cp, cp_dt, ldc, cp_scale, cp_rps, cwm, cp_lo, cp_s)
  if (dy_dtype == KAIR_BF16) {
    if (C <= 64) KAIR_LNB(bf16, 1);
    else KAIR_LNB(bf16, NV);
  } else {
    if (C <= 64) KAIR_LNB(float, 1);
    else KAIR_LNB(float, NV);
  }
#undef KAIR_LNB
  KAIR_CHECK_LAUNCH();
  if (!dgamma) return 0;   // deferred: the [nb][2C] partials stay in ws for kair_ln_param_reduce_grouped
  KAIR_LAUNCH(ln_param_reduce, dim3((2 * C + 7) / 8), dim3(256), 0, s, ws, (int)nb, C, dgamma, dbeta,
                     dparam_accumulate);
  KAIR_CHECK_LAUNCH();
  return 0;
}
