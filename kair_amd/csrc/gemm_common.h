// Operand addressing and epilogues shared by the GEMM kernels (gemm.hip: bf16 / fp32; gemm_x3.hip: the
// split-fp16 "x3" arithmetic): the kair_operand / kair_epilogue descriptors resolved for the device, the
// per-row address state, the two-phase chunk loads (issue under the MFMAs, commit to LDS after them) and the
// 8-column epilogue.
#pragma once
#include "common.h"

namespace {

constexpr int NT = 256;
enum { AM_ROWS = 0, AM_IM2COL = 1, AM_QKV = 2, AM_S2D = 3 };

template <typename CT> struct KStep { static constexpr int BK = sizeof(CT) == 2 ? 64 : 32; };

// ------------------------------------------------------------------------------------------
// operand description (trimmed copy of kair_operand, passed by value)
// ------------------------------------------------------------------------------------------
struct Op {
  const void* ptr;
  long ld;
  WinMap win;
  int imH, imW, imC, flip;
  int up_sh;   // IM2COL: log2 of the nearest-upsample factor (source image imH>>up_sh x imW>>up_sh)
  int nh, hdp, tok;
  const float* rowscale;
  int rps;
  int ones_col;
  int ones_in_data;
  long M;  // rows of this operand
  int wsplit;  // B only: hi/lo bf16 weight pairs interleaved per 64 columns (kair_operand.w_split)
  int asplit;  // A only: the activation as a hi/lo bf16 pair (kair_operand.a_split)
  const void* lo_ptr;   // bf16 A with asplit: the lo plane; x3: the fp16 lo plane
  int x3_exp;           // x3: power-of-2 exponent (kair_operand.x3_exp)
  float x3s;            // x3, fp32 operand: 2^x3_exp, applied before the fp16 split (1 for fp16 planes)
  FDiv d_rps, d_imC, d_imW, d_hw, d_tok, d_hdp, d_pw;
};

Op make_op(const kair_operand& o, long M) {
  Op op;
  op.ptr = o.ptr; op.ld = o.ld;
  op.win = make_winmap(o.win_H, o.win_W, o.win_ws, o.win_shift);
  op.imH = o.im_H; op.imW = o.im_W; op.imC = o.im_C; op.flip = o.im_flip;
  op.up_sh = o.im_up == 2 ? 1 : 0;
  if ((o.mode == KAIR_LD_IM2COL3 || o.mode == KAIR_LD_S2D) && op.ld == 0) op.ld = o.im_C;
  op.nh = o.qkv_nh; op.hdp = o.qkv_hdp; op.tok = o.qkv_tok;
  op.rowscale = o.rowscale; op.rps = o.rows_per_scale > 0 ? o.rows_per_scale : 1;
  op.ones_col = o.ones_col;
  op.ones_in_data = o.ones_in_data;
  op.M = M;
  op.wsplit = o.w_split ? 1 : 0;
  op.asplit = o.a_split;   // 0, 1 or 2 (kair_operand.a_split)
  op.lo_ptr = o.lo_ptr;
  op.x3_exp = o.x3_exp;
  op.x3s = o.dtype == KAIR_F32 ? ldexpf(1.f, o.x3_exp) : 1.f;
  op.d_rps = make_fdiv(op.rps);
  op.d_imC = make_fdiv(op.imC); op.d_imW = make_fdiv(op.imW); op.d_hw = make_fdiv(op.imH * op.imW);
  op.d_tok = make_fdiv(op.tok); op.d_hdp = make_fdiv(op.hdp); op.d_pw = make_fdiv(op.nh * op.hdp);
  return op;
}

KAIR_DEV void zero8(float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = 0.f;
}

template <typename T>
KAIR_DEV void gload8(const T* p, float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    const typename V8<T>::t q = *(const typename V8<T>::t*)p;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)q[j];
  } else {
    const float4 a = *(const float4*)p;
    const float4 b = *(const float4*)(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}

// Per-chunk row state: resolved once before the K loop.
struct RowState {
  long base;   // element offset of the row start (ROWS) / pixel index (IM2COL) / token offset (QKV)
  int y, x;    // IM2COL pixel coordinates
  float scale;
  bool valid;
};

template <int AM, typename T>
KAIR_DEV RowState row_state(const Op& op, long m) {
  RowState r;
  r.valid = m < op.M;
  r.scale = 1.f;
  r.y = r.x = 0;
  r.base = 0;
  if (!r.valid) return r;
  if constexpr (AM == AM_ROWS) {
    const long t = win_to_token(m, op.win);
    r.base = t * op.ld;
    if (op.rowscale) r.scale = op.rowscale[fdiv((int)t, op.d_rps)];
  } else if constexpr (AM == AM_IM2COL) {
    const int hw = op.d_hw.d;
    const int b = fdiv((int)m, op.d_hw);
    const int p = (int)m - b * hw;
    r.y = fdiv(p, op.d_imW);
    r.x = p - r.y * op.imW;
    r.base = (long)b * (hw >> (2 * op.up_sh));   // first pixel of image b in the SOURCE image
  } else if constexpr (AM == AM_S2D) {
    const int hw = op.d_hw.d;
    const int b = fdiv((int)m, op.d_hw);
    const int p = (int)m - b * hw;
    r.y = fdiv(p, op.d_imW);
    r.x = p - r.y * op.imW;
    r.base = (long)b * (4L * hw);                // the source image is 2H x 2W
  } else {
    const int win = fdiv((int)m, op.d_tok);
    const int t = (int)m - win * op.tok;
    r.base = ((long)win * op.nh * op.tok + t) * op.hdp;
    if (op.rowscale) r.scale = op.rowscale[fdiv((int)m, op.d_rps)];
  }
  return r;
}

// Two-phase chunk loads: issue() computes the address of 8 consecutive columns [k, k+8) of a
// resolved row and starts the global load into raw registers WITHOUT consuming it (invalid chunks
// load from the buffer start and are masked later); commit() converts / masks / scales and writes
// LDS after the MFMAs of the current step, so the load latency overlaps them.
template <typename T> struct Raw;
template <> struct Raw<bf16> { uint4 a; };
template <> struct Raw<f16> { uint4 a; };
template <> struct Raw<float> { uint4 a, b; };

struct Pend {
  float scale;   // 0 => masked chunk
  int ones;      // index in [0, 8) of the fused ones column, else -1
};

template <typename T>
KAIR_DEV void raw_load(const T* p, Raw<T>& r) {
  if constexpr (sizeof(T) == 2) {
    r.a = *(const uint4*)p;
  } else {
    r.a = *(const uint4*)p;
    r.b = *(const uint4*)(p + 4);
  }
}

template <int AM, typename T>
KAIR_DEV void issue_chunk(const Op& op, const RowState& r, int k, int K, Raw<T>& raw, Pend& pd,
                          const void* base = nullptr) {
  bool ok = r.valid && k < K;
  long off = 0;
  if constexpr (AM == AM_ROWS) {
    off = r.base + k;
  } else if constexpr (AM == AM_IM2COL) {
    const int tap = fdiv(k, op.d_imC);
    const int c = k - tap * op.imC;
    int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
    if (op.flip) { dy = -dy; dx = -dx; }
    const int y = r.y + dy, x = r.x + dx;
    ok = ok && y >= 0 && y < op.imH && x >= 0 && x < op.imW;
    off = (r.base + (long)(y >> op.up_sh) * (op.imW >> op.up_sh) + (x >> op.up_sh)) * op.ld + c;
  } else if constexpr (AM == AM_S2D) {
    const int tap = fdiv(k, op.d_imC);
    const int c = k - tap * op.imC;
    const int y = 2 * r.y + (tap >> 1), x = 2 * r.x + (tap & 1);
    off = (r.base + (long)y * (2 * op.imW) + x) * op.ld + c;
  } else {
    const int pw = op.d_pw.d;
    const int part = fdiv(k, op.d_pw);
    const int rr = k - part * pw;
    const int h = fdiv(rr, op.d_hdp), d = rr - h * op.hdp;
    off = (long)part * op.M * pw + r.base + (long)h * op.tok * op.hdp + d;
  }
  raw_load<T>((const T*)(base ? base : op.ptr) + (ok ? off : 0), raw);
  pd.scale = ok ? r.scale : 0.f;
  pd.ones = (r.valid && op.ones_col >= k && op.ones_col < k + 8) ? op.ones_col - k : -1;
}

template <typename T>
KAIR_DEV void raw_to_f32(const Raw<T>& r, float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    const typename V8<T>::t q = __builtin_bit_cast(typename V8<T>::t, r.a);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)q[j];
  } else {
    const float4 a = __builtin_bit_cast(float4, r.a), b = __builtin_bit_cast(float4, r.b);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}

// lo (fp32 source, bf16 compute): store the lo half bf16(x - bf16(x)) of the (scaled) value instead
// onev: the value of an injected ones column (x3: 2^e, the operand's own scale)
template <typename CT, typename T>
KAIR_DEV void commit_chunk(CT* dst, const Raw<T>& raw, const Pend& pd, bool lo = false, float onev = 1.f) {
  if constexpr (sizeof(CT) == 2 && sizeof(T) == 2) {
    if (pd.scale == 1.f && pd.ones < 0) {          // common case: raw bf16 straight to LDS
      *(uint4*)dst = raw.a;
      return;
    }
    if (pd.scale == 0.f && pd.ones < 0) {
      *(uint4*)dst = make_uint4(0, 0, 0, 0);
      return;
    }
  }
  float v[8];
  raw_to_f32<T>(raw, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (j == pd.ones) ? onev : (pd.scale == 0.f ? 0.f : v[j] * pd.scale);
  if constexpr (sizeof(CT) == 2) {
    typename V8<CT>::t q;
#pragma unroll
    for (int j = 0; j < 8; ++j) q[j] = lo ? (CT)(v[j] - (float)(CT)v[j]) : (CT)v[j];
    *(typename V8<CT>::t*)dst = q;
  } else {
#pragma unroll
    for (int j = 0; j < 8; j += 2) *(float2*)(dst + j) = make_float2(v[j], v[j + 1]);
  }
}

// ------------------------------------------------------------------------------------------
// epilogue
// ------------------------------------------------------------------------------------------
struct Epi {
  void* out; int odt, omode; long ldo;
  WinMap win;
  const float* bias;
  int act; float slope;
  void* pre; int pdt; long ldp;
  const float* resid; long ldr;
  const float* rowscale; int rps;
  const void* gate; int gdt; long ldg; int gkind;
  int prek;   // 1: pre receives act'(x) (GELU)
  int r, psH, psW;
  int nh, hdp, tok;
  const float* mean; float range; int imgC, imgH, imgW;
  int ones_col;   // -1 none
  const float* resid2; long ldr2;
  bf16* acopy; long ldac; int acones;   // halo conv: bf16 copy of the A image (acones: 1.0 channel, -1 none)
  bf16* out_lo;                         // bf16 ROWS / PSHUF_SPM out: lo plane bf16(v - bf16(v))
  long M; int N;
  float acc_scale;   // x3: 2^-(eA + eB), the accumulator back to natural units (1 otherwise)
  float oscale;      // x3, fp16 out: 2^x3_out_exp
  FDiv d_rps, d_tok, d_hdp, d_pw;
  int dbg;   // ring-kernel ablation bits (KAIR_RING_DBG, perf investigation only): 1 no stores, 2 no MFMA, 4 no A loads
  // EX_LNB (x3 NT ring, kair_gemm_nt_x3_lnbwd): the GEMM is the LayerNorm's input-gradient producer; out is the
  // accumulated fp32 gradient D (token rows, read-modify-write), bias the LayerNorm weight gamma
  const float* lnx; long lnldx;             // the LayerNorm input rows (token order)
  const float* lnmu; const float* lnrs;     // its saved row mean / rstd
  float* lnpart; int lnC;                   // dgamma / dbeta partial rows [tile * 4 + row wave][2 C]; real channels
  void* cpo; void* cplo; long cpld;         // optional fp16-pair operand copy of the finished D rows
  const float* cprs; FDiv d_cprps; WinMap cpwin; float cps;
};

Epi make_epi(const kair_epilogue& o, long M, int N) {
  Epi e;
  e.out = o.out; e.odt = o.out_dtype; e.omode = o.out_mode; e.ldo = o.ldo;
  e.win = make_winmap(o.win_H, o.win_W, o.win_ws, o.win_shift);
  e.bias = o.bias; e.act = o.act; e.slope = o.slope;
  e.pre = o.out_pre; e.pdt = o.pre_dtype; e.ldp = o.ldp;
  e.resid = o.resid; e.ldr = o.ldr;
  e.rowscale = o.rowscale; e.rps = o.rows_per_scale > 0 ? o.rows_per_scale : 1;
  e.gate = o.gate; e.gdt = o.gate_dtype; e.ldg = o.ldg; e.gkind = o.gate_kind;
  e.prek = o.pre_kind;
  e.r = o.ps_r; e.psH = o.ps_H; e.psW = o.ps_W;
  e.nh = o.qkv_nh; e.hdp = o.qkv_hdp; e.tok = o.qkv_tok;
  e.mean = o.img_mean; e.range = o.img_range; e.imgC = o.img_C; e.imgH = o.img_H; e.imgW = o.img_W;
  e.ones_col = o.out_ones_col_p1 - 1;
  e.resid2 = o.resid2; e.ldr2 = o.ldr2;
  e.acopy = (bf16*)o.a_copy; e.ldac = o.ld_acopy; e.acones = o.acopy_ones_col_p1 - 1;
  e.out_lo = (bf16*)o.out_lo;
  e.M = M; e.N = N;
  e.acc_scale = 1.f;
  e.oscale = ldexpf(1.f, o.x3_out_exp);
  e.d_rps = make_fdiv(e.rps); e.d_tok = make_fdiv(e.tok); e.d_hdp = make_fdiv(e.hdp); e.d_pw = make_fdiv(e.nh * e.hdp);
  static const int dbg = kair_dbg_env("KAIR_RING_DBG");
  e.dbg = dbg;
  e.lnx = nullptr; e.lnldx = 0; e.lnmu = e.lnrs = nullptr; e.lnpart = nullptr; e.lnC = 0;
  e.cpo = e.cplo = nullptr; e.cpld = 0; e.cprs = nullptr; e.d_cprps = make_fdiv(1); e.cpwin = make_winmap(0, 0, 0, 0);
  e.cps = 1.f;
  return e;
}

KAIR_DEV void load8_any(const void* p, int dt, long off, float (&v)[8]) {
  if (dt == KAIR_BF16) gload8<bf16>((const bf16*)p + off, v);
  else gload8<float>((const float*)p + off, v);
}
// x3 fp16 pair output: hi = f16(v s), lo = f16(v s - hi) at the same offsets of out / out_lo
KAIR_DEV void store8_f16pair(void* p, void* plo, long off, const float (&v)[8], float s) {
  f16x8 h, l;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float w = v[j] * s;
    h[j] = (f16)w;
    l[j] = (f16)(w - (float)h[j]);
  }
  *(f16x8*)((f16*)p + off) = h;
  if (plo) *(f16x8*)((f16*)plo + off) = l;
}
KAIR_DEV void st1_f16pair(void* p, void* plo, long off, float v, float s) {
  const float w = v * s;
  const f16 h = (f16)w;
  ((f16*)p)[off] = h;
  if (plo) ((f16*)plo)[off] = (f16)(w - (float)h);
}

KAIR_DEV void store8_any(void* p, int dt, long off, const float (&v)[8]) {
  if (dt == KAIR_BF16) {
    bf16x8 q;
#pragma unroll
    for (int j = 0; j < 8; ++j) q[j] = (bf16)v[j];
    *(bf16x8*)((bf16*)p + off) = q;
  } else {
    float* d = (float*)p + off;
    *(float4*)d = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)(d + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}
// the lo plane of 8 values stored as bf16 hi: bf16(v - bf16(v))
KAIR_DEV void store8_lo(bf16* p, long off, const float (&v)[8]) {
  bf16x8 q;
#pragma unroll
  for (int j = 0; j < 8; ++j) q[j] = (bf16)(v[j] - (float)(bf16)v[j]);
  *(bf16x8*)(p + off) = q;
}
KAIR_DEV void st1(void* p, int dt, long off, float v) {
  if (dt == KAIR_BF16) ((bf16*)p)[off] = (bf16)v;
  else ((float*)p)[off] = v;
}

// finish 8 consecutive columns [n, n+8) of GEMM row m (n % 8 == 0)
KAIR_DEV void epi_chunk(const Epi& e, long m, int n, float (&v)[8]) {
  if (m >= e.M || n >= e.N) return;
  const bool full = n + 8 <= e.N;
  if (e.bias) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += (n + j < e.N) ? e.bias[n + j] : 0.f;
  }
  float pre[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    pre[j] = (e.prek && e.act == KAIR_ACT_GELU) ? gelu_erf_grad(v[j]) : v[j];
    if (e.act == KAIR_ACT_GELU) v[j] = gelu_erf(v[j]);
    else if (e.act == KAIR_ACT_LEAKY) v[j] = v[j] > 0.f ? v[j] : v[j] * e.slope;
    else if (e.act == KAIR_ACT_RELU) v[j] = fmaxf(v[j], 0.f);
  }
  if (e.omode == KAIR_OUT_ROWS) {
    const long row = win_to_token(m, e.win);
    if (e.gate) {
      float g[8];
      if (full) load8_any(e.gate, e.gdt, row * e.ldg + n, g);
      else
        for (int j = 0; j < 8; ++j)
          g[j] = n + j < e.N ? (e.gdt == KAIR_BF16 ? (float)((const bf16*)e.gate)[row * e.ldg + n + j]
                                                    : ((const float*)e.gate)[row * e.ldg + n + j]) : 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (e.gkind == 1) v[j] *= gelu_erf_grad(g[j]);
        else if (e.gkind == 2) v[j] *= (g[j] > 0.f ? 1.f : e.slope);
        else if (e.gkind == 4) v[j] *= g[j];
        else v[j] *= (g[j] > 0.f ? 1.f : 0.f);
      }
    }
    if (e.resid) {
      const float s = e.rowscale ? e.rowscale[fdiv((int)row, e.d_rps)] : 1.f;
      for (int j = 0; j < 8; ++j)
        if (n + j < e.N) v[j] = e.resid[row * e.ldr + n + j] + s * v[j];
    }
    if (e.resid2) {
      for (int j = 0; j < 8; ++j)
        if (n + j < e.N) v[j] += e.resid2[row * e.ldr2 + n + j];
    }
    if (e.ones_col >= n && e.ones_col < n + 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (n + j == e.ones_col) v[j] = 1.f;
    }
    if (e.odt == KAIR_F16) {   // x3: the fp16 pair of v * 2^x3_out_exp
      if (full && (e.ldo % 8) == 0) store8_f16pair(e.out, e.out_lo, row * e.ldo + n, v, e.oscale);
      else
        for (int j = 0; j < 8 && n + j < e.N; ++j) st1_f16pair(e.out, e.out_lo, row * e.ldo + n + j, v[j], e.oscale);
      if (e.pre) {
        if (full && (e.ldp % 8) == 0) store8_any(e.pre, e.pdt, row * e.ldp + n, pre);
        else
          for (int j = 0; j < 8 && n + j < e.N; ++j) st1(e.pre, e.pdt, row * e.ldp + n + j, pre[j]);
      }
    } else if (full && (e.ldo % 8) == 0) {
      store8_any(e.out, e.odt, row * e.ldo + n, v);
      if (e.pre) store8_any(e.pre, e.pdt, row * e.ldp + n, pre);
      if (e.out_lo) store8_lo(e.out_lo, row * e.ldo + n, v);
    } else {
      for (int j = 0; j < 8 && n + j < e.N; ++j) {
        st1(e.out, e.odt, row * e.ldo + n + j, v[j]);
        if (e.pre) st1(e.pre, e.pdt, row * e.ldp + n + j, pre[j]);
        if (e.out_lo) e.out_lo[row * e.ldo + n + j] = (bf16)(v[j] - (float)(bf16)v[j]);
      }
    }
  } else if (e.omode == KAIR_OUT_QKVBLK) {
    const int pw = e.nh * e.hdp;
    const int part = fdiv(n, e.d_pw), rr = n - part * pw;
    const int h = fdiv(rr, e.d_hdp), d = rr - h * e.hdp;
    const long win = fdiv((int)m, e.d_tok);
    const int t = (int)(m - win * e.tok);
    const long o = (long)part * e.M * pw + ((win * e.nh + h) * e.tok + t) * e.hdp + d;
    if (e.odt == KAIR_F16) {
      store8_f16pair(e.out, e.out_lo, o, v, e.oscale);
    } else {
      store8_any(e.out, e.odt, o, v);
      if (e.out_lo) store8_lo(e.out_lo, o, v);
    }
  } else if (e.omode == KAIR_OUT_PSHUF || e.omode == KAIR_OUT_PSHUF_NCHW) {
    const int r = e.r, r2 = r * r;
    const long hw = (long)e.psH * e.psW;
    const long b = m / hw;
    const int p = (int)(m - b * hw), y = p / e.psW, x = p - (p / e.psW) * e.psW;
    for (int j = 0; j < 8 && n + j < e.N; ++j) {
      const int nn = n + j;
      const int c = nn / r2, ij = nn - c * r2, i = ij / r, jj = ij - i * r;
      if (e.omode == KAIR_OUT_PSHUF) {
        const long orow = (b * e.psH * r + (long)y * r + i) * ((long)e.psW * r) + (long)x * r + jj;
        st1(e.out, e.odt, orow * e.ldo + c, v[j]);
        if (e.pre) st1(e.pre, e.pdt, orow * e.ldp + c, pre[j]);
      } else if (c < e.imgC) {
        const float o = v[j] / e.range + (e.mean ? e.mean[c] : 0.f);
        ((float*)e.out)[((b * e.imgC + c) * e.psH * r + (long)y * r + i) * ((long)e.psW * r) + (long)x * r + jj] = o;
      }
    }
  } else if (e.omode == KAIR_OUT_PSHUF_SPM) {
    // columns sub-pixel-major: n = (i*r + j)*nf + c, so a chunk of 8 is 8 channels of one pixel
    const int r = e.r, nf = e.N / (r * r);
    const long hw = (long)e.psH * e.psW;
    const long b = m / hw;
    const int p = (int)(m - b * hw), y = p / e.psW, x = p - (p / e.psW) * e.psW;
    const int sp = n / nf, c = n - sp * nf, i = sp / r, jj = sp - i * r;
    const long orow = (b * e.psH * r + (long)y * r + i) * ((long)e.psW * r) + (long)x * r + jj;
    if (full && c + 8 <= nf && (e.ldo % 8) == 0 && (c % 8) == 0) {
      store8_any(e.out, e.odt, orow * e.ldo + c, v);
      if (e.pre) store8_any(e.pre, e.pdt, orow * e.ldp + c, pre);
      if (e.out_lo) store8_lo(e.out_lo, orow * e.ldo + c, v);
    } else {
      for (int j = 0; j < 8 && n + j < e.N; ++j) {
        const int nn = n + j, s2 = nn / nf, c2 = nn - s2 * nf, i2 = s2 / r, j2 = s2 - i2 * r;
        const long orow2 = (b * e.psH * r + (long)y * r + i2) * ((long)e.psW * r) + (long)x * r + j2;
        st1(e.out, e.odt, orow2 * e.ldo + c2, v[j]);
        if (e.pre) st1(e.pre, e.pdt, orow2 * e.ldp + c2, pre[j]);
        if (e.out_lo) e.out_lo[orow2 * e.ldo + c2] = (bf16)(v[j] - (float)(bf16)v[j]);
      }
    }
  } else if (e.omode == KAIR_OUT_PUNSHUF_SPM) {
    // pixel (b, Y, X) of the shuffled image, column c -> pre-shuffle row (b, Y/r, X/r), column
    // (i*r + j)*N + c: a chunk of 8 columns is 8 contiguous pre-shuffle channels
    const int r = e.r;
    const long HW = (long)e.psH * r * e.psW * r;
    const long b = m / HW;
    const long p = m - b * HW;
    const int Y = (int)(p / (e.psW * r)), X = (int)(p - (long)Y * e.psW * r);
    const int y = Y / r, i = Y - y * r, x = X / r, jj = X - x * r;
    const long orow = (b * e.psH + y) * e.psW + x;
    const long o0 = orow * e.ldo + (long)(i * r + jj) * e.N + n;
    if (e.gate) {
      float g[8];
      if (full) load8_any(e.gate, e.gdt, orow * e.ldg + (long)(i * r + jj) * e.N + n, g);
      else
        for (int j = 0; j < 8; ++j)
          g[j] = n + j < e.N ? (e.gdt == KAIR_BF16 ? (float)((const bf16*)e.gate)[orow * e.ldg + (long)(i * r + jj) * e.N + n + j]
                                                    : ((const float*)e.gate)[orow * e.ldg + (long)(i * r + jj) * e.N + n + j]) : 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[j] *= (e.gkind == 2) ? (g[j] > 0.f ? 1.f : e.slope) : (e.gkind == 4 ? g[j] : (g[j] > 0.f ? 1.f : 0.f));
    }
    if (full && (e.ldo % 8) == 0 && (e.N % 8) == 0) {
      store8_any(e.out, e.odt, o0, v);
    } else {
      for (int j = 0; j < 8 && n + j < e.N; ++j) st1(e.out, e.odt, o0 + j, v[j]);
    }
  } else if (e.omode == KAIR_OUT_PUNSHUF) {
    const int r = e.r;
    const long HW = (long)e.psH * r * e.psW * r;
    const long b = m / HW;
    const long p = m - b * HW;
    const int Y = (int)(p / (e.psW * r)), X = (int)(p - (long)Y * e.psW * r);
    const int y = Y / r, i = Y - y * r, x = X / r, jj = X - x * r;
    const long orow = (b * e.psH + y) * e.psW + x;
    for (int j = 0; j < 8 && n + j < e.N; ++j) {
      const int oc = (n + j) * r * r + i * r + jj;
      float val = v[j];
      if (e.gate) {
        const float g = e.gdt == KAIR_BF16 ? (float)((const bf16*)e.gate)[orow * e.ldg + oc]
                                            : ((const float*)e.gate)[orow * e.ldg + oc];
        val *= (e.gkind == 2) ? (g > 0.f ? 1.f : e.slope) : (e.gkind == 4 ? g : (g > 0.f ? 1.f : 0.f));
      }
      st1(e.out, e.odt, orow * e.ldo + oc, val);
    }
  } else {  // NCHW image; resid (optional): an NCHW image of the same shape added after the range
    const long hw = (long)e.imgH * e.imgW;
    const long b = m / hw;
    const long p = m - b * hw;
    for (int j = 0; j < 8 && n + j < e.imgC && n + j < e.N; ++j) {
      const long o = (b * e.imgC + n + j) * hw + p;
      ((float*)e.out)[o] = v[j] / e.range + (e.mean ? e.mean[n + j] : 0.f) + (e.resid ? e.resid[o] : 0.f);
    }
  }
}

// ------------------------------------------------------------------------------------------
// LDS-DMA ring plumbing (the persistent ring kernels of gemm.hip and gemm_x3.hip)
// ------------------------------------------------------------------------------------------
KAIR_DEV void ring_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// LDS-DMA of 16 bytes per lane (global_load_lds_dwordx4 into lds_base + 16 * lane) issued from
// inline asm.  hipcc treats the builtin form as a pending LDS write and emits s_waitcnt vmcnt(0)
// before the next ds_read of the shared array -- every chunk of a ring would drain all the DMA (and
// stores) in flight.  Hidden in asm, the DMA is waited for only by the ring's own counted vmcnt.
KAIR_DEV void glds16(const void* src, const char* lds_base) {
  const unsigned la = __builtin_amdgcn_readfirstlane(
      (unsigned)(unsigned long)(__attribute__((address_space(3))) const char*)lds_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(la) : "memory", "m0");
}

// Wait for an ordinary (compiler-visible) load's result HERE, on every path: a load still pending
// at a loop back-edge on any path makes hipcc wait vmcnt(0) at the next write of its register.
KAIR_DEV void land(float& v) { asm volatile("" : "+v"(v)); }
KAIR_DEV void land(float4& v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }

// ring epilogue operand kinds (compile-time, so the plain kernels carry no epilogue loads at all)
enum { EX_NONE = 0, EX_RESID = 1, EX_GATE_BF16 = 2, EX_GATE_F32 = 3, EX_LNB = 4 };   // EX_LNB: x3 NT ring only

// a zero line for masked loads (read-only; zero-initialised device memory)
__device__ __attribute__((aligned(64))) unsigned char g_kair_zero_line[64];

// s_waitcnt vmcnt(n) for a wave-uniform run-time n (clamped to the 6-bit field: waiting for more
// than asked is always safe)
#define KAIR_VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
KAIR_DEV void vm_wait(int n) {
  n = __builtin_amdgcn_readfirstlane(n);   // scalar branch tree, not exec-masked
  switch (n < 63 ? n : 63) {
    KAIR_VMW(0) KAIR_VMW(1) KAIR_VMW(2) KAIR_VMW(3) KAIR_VMW(4) KAIR_VMW(5) KAIR_VMW(6) KAIR_VMW(7)
    KAIR_VMW(8) KAIR_VMW(9) KAIR_VMW(10) KAIR_VMW(11) KAIR_VMW(12) KAIR_VMW(13) KAIR_VMW(14) KAIR_VMW(15)
    KAIR_VMW(16) KAIR_VMW(17) KAIR_VMW(18) KAIR_VMW(19) KAIR_VMW(20) KAIR_VMW(21) KAIR_VMW(22) KAIR_VMW(23)
    KAIR_VMW(24) KAIR_VMW(25) KAIR_VMW(26) KAIR_VMW(27) KAIR_VMW(28) KAIR_VMW(29) KAIR_VMW(30) KAIR_VMW(31)
    KAIR_VMW(32) KAIR_VMW(33) KAIR_VMW(34) KAIR_VMW(35) KAIR_VMW(36) KAIR_VMW(37) KAIR_VMW(38) KAIR_VMW(39)
    KAIR_VMW(40) KAIR_VMW(41) KAIR_VMW(42) KAIR_VMW(43) KAIR_VMW(44) KAIR_VMW(45) KAIR_VMW(46) KAIR_VMW(47)
    KAIR_VMW(48) KAIR_VMW(49) KAIR_VMW(50) KAIR_VMW(51) KAIR_VMW(52) KAIR_VMW(53) KAIR_VMW(54) KAIR_VMW(55)
    KAIR_VMW(56) KAIR_VMW(57) KAIR_VMW(58) KAIR_VMW(59) KAIR_VMW(60) KAIR_VMW(61) KAIR_VMW(62)
    default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
  }
}
#undef KAIR_VMW

// sum over the 16 lanes of a DPP row, every lane gets the same bits (quad swaps, then the half-row and row mirrors)
KAIR_DEV float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));    // quad_perm 1,0,3,2
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));    // quad_perm 2,3,0,1
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));   // row_half_mirror
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false));   // row_mirror
  return v;
}

// bijective XCD-aware remap: consecutive logical tiles share an XCD (L2)
KAIR_DEV int xcd_remap(int hw, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int x = hw % 8, pos = hw / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + pos;
}


}  // namespace
