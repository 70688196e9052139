// Narrow-output 3x3 convolutions for gfx950: the last conv of an image-restoration network maps a
// 64-channel feature image to the NR <= 4 channels of the output image (SwinIR conv_last,
// network_swinir.py:745 / :817).  As a generic implicit GEMM its N = NR padded to 16 wastes the MFMA
// tile and its im2col re-reads the 64-channel image once per K tile; here each of the three products
// of the training step gets its own kernel, all three built on one access pattern:
//
//   Rolling row window.  The image is cut into 64-pixel row segments; a persistent workgroup owns a
//   contiguous run of output rows of one column strip (a 64-pixel-wide strip of one image) and keeps
//   the input rows y-1, y, y+1 of its segment (+1 halo pixel each side) in an LDS ring, loading row
//   y+2 with bulk 16-byte loads while it computes row y.  Every input pixel is fetched from HBM once
//   (plus two halo rows per run); the nine taps read LDS.
//
//   kair_conv3x3_narrow_fwd    E = conv(X) -> NCHW image (v / range + mean): v_mfma_f32_16x16x32_bf16
//                              with D = W . X^T (a lane ends with 4 output channels of one pixel), the
//                              hi/lo split weights (pack kind 15) resident in VGPRs for the launch, the
//                              image a [hi | lo] pair (split activations: 3 products per k-step);
//   kair_conv3x3_narrow_dgrad  dX = conv^T(dE): MFMA with D = W'^T . dE_im2col^T over k = (tap, n) (36
//                              -> 2 k-steps), the dE rows staged as 4 channels per pixel; rows or
//                              PixelUnshuffle sub-pixel-major store (the previous upsampling conv's
//                              pre-shuffle gradient);
//   kair_conv3x3_narrow_wgrad  dW = sum_p dE[p] x X[p + tap]: MFMA over the pixels (32 per k-step), both
//                              operands read with transposing LDS reads (ds_read_b64_tr_b16), the dE rows
//                              staged with a halo; per-workgroup partials summed in fixed order.
#include <stdlib.h>

#include "common.h"

namespace {

constexpr int NF = 64;      // feature channels of the image side
constexpr int SEG = 64;     // output pixels per row segment
constexpr int PXS = SEG + 2;

// A run of output rows: rows [g0, g1) of the global (strip, y) order, strip = b * nseg + segment.
struct RowRun {
  long g0, g1;
};
KAIR_DEV RowRun row_run(long total, int nblk, int blk) {
  const long per = (total + nblk - 1) / nblk;
  RowRun r;
  r.g0 = (long)blk * per;
  r.g1 = r.g0 + per < total ? r.g0 + per : total;
  return r;
}

int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}

// ---------------------------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------------------------
struct NarrowFwdArgs {
  const bf16* x; long ldx; int lo_off;   // [B*H*W][ldx] bf16: hi channels [0, 64), lo [lo_off, lo_off + 64) (0: none)
  const bf16* w;                        // pack kind 15: [1][18][2][64][8]
  const float* bias;                    // [16] (>= NR real)
  const float* mean; float range; int NR;
  const float* resid;                   // optional NCHW image added after the range (denoising head)
  float* out;                           // NCHW [B][NR][H][W]
  int B, H, W;
};

constexpr int FPST = 136;               // LDS pixel stride (bf16): 128 channels + 8 (272 B: 16 lanes conflict-free)
constexpr int FROW = PXS * FPST;        // one staged row
constexpr int FCH = PXS * 16;           // 16-byte chunks per staged row (hi + lo: 16 per pixel)
constexpr int FPER = (FCH + 255) / 256; // chunks per thread

__global__ __launch_bounds__(256, 2) void conv3x3_narrow_fwd_kernel(const NarrowFwdArgs a) {
  constexpr int KS = 9 * NF / 32;   // 18 k-steps of 32: (tap, channel half)
  __shared__ __attribute__((aligned(16))) bf16 sRow[4 * FROW];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  bf16x8 wh[KS], wl[KS];
#pragma unroll
  for (int kb = 0; kb < KS; ++kb) {
    wh[kb] = *(const bf16x8*)(a.w + ((long)kb * 2 + 0) * 512 + lane * 8);
    wl[kb] = *(const bf16x8*)(a.w + ((long)kb * 2 + 1) * 512 + lane * 8);
  }
  float bias4[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) bias4[n] = n < a.NR ? a.bias[n] : 0.f;
  const int nseg = a.W / SEG;
  const long total = (long)a.B * nseg * a.H;
  const RowRun run = row_run(total, gridDim.x, blockIdx.x);
  const bool split = a.lo_off > 0;
  uint4 pre[FPER];
  // issue the loads of input row yy of strip st (zeros outside the image): chunk c = pixel c / 16, part c % 16
  auto load_row = [&](long st, int yy) {
    const int b = (int)(st / nseg), x0 = (int)(st - (long)b * nseg) * SEG;
#pragma unroll
    for (int i = 0; i < FPER; ++i) {
      const int c = tid + 256 * i;
      const int px = c >> 4, part = c & 15;
      const int xx = x0 - 1 + px;
      const bool ok = c < FCH && (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W && (split || part < 8);
      const long off = ok ? ((long)(b * a.H + yy) * a.W + xx) * a.ldx + (part < 8 ? part * 8 : a.lo_off + (part - 8) * 8) : 0;
      pre[i] = *(const uint4*)(a.x + off);
      if (!ok) pre[i] = make_uint4(0, 0, 0, 0);
    }
  };
  auto store_row = [&](int yy) {
    bf16* dst = sRow + (yy & 3) * FROW;
#pragma unroll
    for (int i = 0; i < FPER; ++i) {
      const int c = tid + 256 * i;
      if (c < FCH) *(uint4*)(dst + (c >> 4) * FPST + (c & 15) * 8) = pre[i];
    }
  };
  const int pl = lane & 15, cq = 8 * (lane >> 4);
  long cur_strip = -1;
  for (long g = run.g0; g < run.g1; ++g) {
    const long st = g / a.H;
    const int y = (int)(g - st * a.H);
    if (st != cur_strip) {   // (re)start the window: rows y-1, y, y+1
      __syncthreads();
      for (int d = -1; d <= 1; ++d) {
        load_row(st, y + d);
        store_row(y + d + 4);   // + 4: slot of a negative row index stays in [0, 4)
      }
      cur_strip = st;
      __syncthreads();
    }
    const bool more = g + 1 < run.g1 && (g + 1) / a.H == st;
    if (more) load_row(st, y + 2);   // in flight during this row's MFMAs
    // wave w: output pixels x0 + 16 w + pl
    // three independent accumulator chains (hi.w_hi, hi.w_lo, lo.w_hi), summed at the end
    f32x4 acc = {0.f, 0.f, 0.f, 0.f}, acc1 = acc, acc2 = acc;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int dy = tap / 3 - 1, dx = tap % 3 - 1;
      const bf16* src = sRow + ((y + dy + 4) & 3) * FROW + (1 + 16 * wave + pl + dx) * FPST + cq;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 xh = *(const bf16x8*)(src + 32 * ks);
        const int kb = tap * 2 + ks;
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[kb], xh, acc, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl[kb], xh, acc1, 0, 0, 0);
        if (split) {
          const bf16x8 xl = *(const bf16x8*)(src + 64 + 32 * ks);
          acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[kb], xl, acc2, 0, 0, 0);
        }
      }
    }
    acc += acc1 + acc2;
    if (lane < 16) {   // D[n][px]: lanes 0..15 hold n = 0..3 of pixel pl
      const int b = (int)(st / nseg), x0 = (int)(st - (long)b * nseg) * SEG;
      const long HW = (long)a.H * a.W;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        if (n < a.NR) {
          const long o = ((long)b * a.NR + n) * HW + (long)y * a.W + x0 + 16 * wave + pl;
          float v = (acc[n] + bias4[n]) / a.range + (a.mean ? a.mean[n] : 0.f);
          if (a.resid) v += a.resid[o];
          a.out[o] = v;
        }
      }
    }
    __syncthreads();   // every wave is done with row y - 1's slot
    if (more) store_row(y + 2);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------------
// input gradient
// ---------------------------------------------------------------------------------------------------
struct NarrowDgradArgs {
  const bf16* dE; long lde;             // [B*H*W][lde] bf16, channels [0, NR) (NR <= 4; the rest ignored)
  const bf16* w;                        // [4 c-blocks][2 k-steps][64][8]: W'[c][k = tap*4 + n] in fragment order
  void* out; int odt; long ldo;         // rows [B*H*W][ldo] (ps_r <= 1) or PixelUnshuffle SPM (ps_r > 1)
  int ps_r;
  int B, H, W;
};

constexpr int DPST = 4;                 // staged dE: 4 channels (8 B) per pixel
constexpr int DROW = PXS * DPST;

__global__ __launch_bounds__(256) void conv3x3_narrow_dgrad_kernel(const NarrowDgradArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 sE[4 * DROW];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // weight fragments: A operand rows = output channel (16 per block), k = 8 (l / 16) + j
  bf16x8 wf[4][2];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) wf[cb][ks] = *(const bf16x8*)(a.w + ((cb * 2 + ks) * 64 + lane) * 8);
  const int nseg = a.W / SEG;
  const long total = (long)a.B * nseg * a.H;
  const RowRun run = row_run(total, gridDim.x, blockIdx.x);
  uint2 pre = make_uint2(0, 0);
  auto load_row = [&](long st, int yy) {   // 66 pixels x 8 B: one per thread (threads >= 66 idle)
    const int b = (int)(st / nseg), x0 = (int)(st - (long)b * nseg) * SEG;
    const int xx = x0 - 1 + tid;
    const bool ok = tid < PXS && (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W;
    pre = *(const uint2*)(a.dE + (ok ? ((long)(b * a.H + yy) * a.W + xx) * a.lde : 0));
    if (!ok) pre = make_uint2(0, 0);
  };
  auto store_row = [&](int yy) {
    if (tid < PXS) *(uint2*)(sE + (yy & 3) * DROW + tid * DPST) = pre;
  };
  const int pl = lane & 15, kq = lane >> 4;   // B fragment: pixel pl, k = 8 kq + j -> taps 2 kq, 2 kq + 1 (x 4 n)
  long cur_strip = -1;
  for (long g = run.g0; g < run.g1; ++g) {
    const long st = g / a.H;
    const int y = (int)(g - st * a.H);
    if (st != cur_strip) {
      __syncthreads();
      for (int d = -1; d <= 1; ++d) {
        load_row(st, y + d);
        store_row(y + d + 4);
      }
      cur_strip = st;
      __syncthreads();
    }
    const bool more = g + 1 < run.g1 && (g + 1) / a.H == st;
    if (more) load_row(st, y + 2);
    // dX[q] = sum_tap sum_n dE[q - (dy, dx)][n] W[n][c][tap]: B fragment of pixel q = x0 + 16 wave + pl
    bf16x8 bfr[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x4 e2[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int tap = 8 * ks + 2 * kq + h;   // k = tap * 4 + n
        if (tap < 9) {
          const int dy = tap / 3 - 1, dx = tap % 3 - 1;
          e2[h] = *(const bf16x4*)(sE + ((y - dy + 4) & 3) * DROW + (1 + 16 * wave + pl - dx) * DPST);
        } else {
          e2[h] = bf16x4{};
        }
      }
      bfr[ks] = bf16x8{e2[0][0], e2[0][1], e2[0][2], e2[0][3], e2[1][0], e2[1][1], e2[1][2], e2[1][3]};
    }
    const int b = (int)(st / nseg), x0 = (int)(st - (long)b * nseg) * SEG;
    const int x = x0 + 16 * wave + pl;
    long o;
    if (a.ps_r > 1) {   // pixel (b, y, x) of the r-times image -> pre-shuffle row (b, y/r, x/r), column (i r + j) 64 + c
      const int r = a.ps_r, yl = y / r, xl = x / r;
      o = ((long)(b * (a.H / r) + yl) * (a.W / r) + xl) * a.ldo + ((y - yl * r) * r + (x - xl * r)) * NF;
    } else {
      o = ((long)(b * a.H + y) * a.W + x) * a.ldo;
    }
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cb][0], bfr[0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cb][1], bfr[1], acc, 0, 0, 0);
      // D[c][q]: lane holds channels 16 cb + 4 kq .. +3 of pixel pl
      const long oc = o + 16 * cb + 4 * kq;
      if (a.odt == KAIR_BF16) *(bf16x4*)((bf16*)a.out + oc) = bf16x4{(bf16)acc[0], (bf16)acc[1], (bf16)acc[2], (bf16)acc[3]};
      else *(float4*)((float*)a.out + oc) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    }
    __syncthreads();
    if (more) store_row(y + 2);
    __syncthreads();
  }
}

// W'[c][k] fragment order for the dgrad kernel from the fp32 weight [NR][64][3][3]: k = tap * 4 + n
__global__ void narrow_dgrad_pack_kernel(const float* __restrict__ w, int NR, bf16* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;   // [4][2][64][8]
  if (t >= 4 * 2 * 64 * 8) return;
  const int j = t & 7, ln = (t >> 3) & 63, ks = (t >> 9) & 1, cb = t >> 10;
  const int c = 16 * cb + (ln & 15), k = 32 * ks + 8 * (ln >> 4) + j;
  const int tap = k >> 2, n = k & 3;
  out[t] = (bf16)(tap < 9 && n < NR ? w[((long)n * NF + c) * 9 + tap] : 0.f);
}

// ---------------------------------------------------------------------------------------------------
// weight gradient
// ---------------------------------------------------------------------------------------------------
struct NarrowWgradArgs {
  const bf16* dE; long lde;             // [M][lde] bf16, channels [0, NR)
  const bf16* x; long ldx;              // [M][ldx] bf16 image, channels [0, 64)
  int NR;
  int B, H, W;
  float* part;                          // [gridDim.x][NR * 64 * 9 + NR]
};

constexpr int XS = NF + 8;               // staged X row: [64 px][64 + 8] bf16
constexpr int EPX = PXS * 4;             // staged dE row: [66 px][4] bf16

// MFMA over the pixels: D[c][(tap, n)] = sum_p X[p][c] dE[p - (dy, dx)][n] (p a pixel of X row Y, the
// dE rows Y - dy staged with a halo), v_mfma_f32_16x16x32_bf16 with 32 pixels per k-step.  Both operands
// are pixel-major in LDS and read with ds_read_b64_tr_b16 (8 consecutive pixels per lane): A = X^T
// (16 channels per wave), B = 4 taps x 4 channels of dE per 16 columns, each lane's 4-column group
// addressing its own tap's shifted row -- 3 tap groups (taps 0-3, 4-7, 8).  Wave w owns channels
// 16 w .. 16 w + 15; per X row a wave issues 6 MFMAs, so the kernel runs at the rate its rows stream in.
__global__ __launch_bounds__(256) void conv3x3_narrow_wgrad_kernel(const NarrowWgradArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 sXr[2][SEG * XS];
  __shared__ __attribute__((aligned(16))) bf16 sEr[4][EPX + 8];   // + a zero tail for tap >= 9 lanes
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = (lane & 15) >> 2, p4 = (lane & 3) * 4, g8 = (lane >> 4) * 8;
  const int tl = p4 >> 2;   // this lane's tap within a group (its 4-column block)
  f32x4 acc[3];
#pragma unroll
  for (int tg = 0; tg < 3; ++tg) acc[tg] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc[4] = {0.f, 0.f, 0.f, 0.f};
  const int nseg = a.W / SEG;
  const long total = (long)a.B * nseg * a.H;
  const RowRun run = row_run(total, gridDim.x, blockIdx.x);
  uint4 px_[2];
  uint2 pe = make_uint2(0, 0);
  auto load_x = [&](long st, int yy) {   // X row yy (inside the image): 64 px x 8 chunks of 16 B
    const int b = (int)(st / nseg), x0 = (int)(st - (long)b * nseg) * SEG;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int cidx = tid + 256 * i, p = cidx >> 3, part = cidx & 7;
      px_[i] = *(const uint4*)(a.x + ((long)(b * a.H + yy) * a.W + x0 + p) * a.ldx + part * 8);
    }
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int cidx = tid + 256 * i;
      *(uint4*)(&sXr[buf][(cidx >> 3) * XS + (cidx & 7) * 8]) = px_[i];
    }
  };
  auto load_e = [&](long st, int yy) {   // dE row yy with a one-pixel halo (zeros outside the image)
    const int b = (int)(st / nseg), x0 = (int)(st - (long)b * nseg) * SEG;
    const int xx = x0 - 1 + tid;
    const bool ok = tid < PXS && (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W;
    pe = *(const uint2*)(a.dE + (ok ? ((long)(b * a.H + yy) * a.W + xx) * a.lde : 0));
    if (!ok) pe = make_uint2(0, 0);
  };
  auto store_e = [&](int yy) {
    if (tid < PXS) *(uint2*)(&sEr[yy & 3][tid * 4]) = pe;
    if (tid >= PXS && tid < PXS + 2) *(uint2*)(&sEr[yy & 3][EPX + (tid - PXS) * 4]) = make_uint2(0, 0);
  };
  // the zero tails of all four dE slots (taps >= 9 read slot 0's): set once here, and store_e only ever
  // rewrites a tail with zeros, so every slot's tail is zero whichever slots a strip restart fills
  if (tid < 8) *(uint2*)(&sEr[tid >> 1][EPX + (tid & 1) * 4]) = make_uint2(0, 0);
  long cur_strip = -1;
  int xb = 0;
  for (long g = run.g0; g < run.g1; ++g) {
    const long st = g / a.H;
    const int y = (int)(g - st * a.H);
    if (st != cur_strip) {   // (re)start: dE rows y-1 .. y+1, X row y
      __syncthreads();
      for (int d = -1; d <= 1; ++d) {
        load_e(st, y + d);
        store_e(y + d + 4);
      }
      load_x(st, y);
      store_x(xb);
      cur_strip = st;
      __syncthreads();
    }
    const bool more = g + 1 < run.g1 && (g + 1) / a.H == st;
    if (more) {   // the next row's operands in flight during this row's MFMAs
      load_x(st, y + 1);
      load_e(st, y + 2);
    }
    const bf16* xr = sXr[xb];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int r0 = 32 * ks + g8 + q;   // rows (pixels) r0 and r0 + 4 of this lane's transposed reads
      bf16x8 af;
      {
        const bf16* base = xr + r0 * XS + 16 * wave + p4;
        const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)base);
        const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)(base + 4 * XS));
        short __attribute__((ext_vector_type(8))) s8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af = __builtin_bit_cast(bf16x8, s8);
      }
#pragma unroll
      for (int tg = 0; tg < 3; ++tg) {
        const int tap = 4 * tg + tl;
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
        // dE[p - (dy, dx)]: staged row y - dy, pixel index 1 + p - dx; taps >= 9 read the zero tail
        const bf16* base = tap < 9 ? &sEr[(y - dy + 4) & 3][(1 + r0 - dx) * 4] : &sEr[0][EPX];
        const int step = tap < 9 ? 16 : 0;   // rows r0 + 4: 4 pixels on (the zero tail stays put)
        const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)base);
        const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)(base + step));
        short __attribute__((ext_vector_type(8))) s8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        acc[tg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, __builtin_bit_cast(bf16x8, s8), acc[tg], 0, 0, 0);
      }
    }
    if (tid < SEG) {   // bias: every pixel of dE row y once
      const bf16x4 e = *(const bf16x4*)(&sEr[y & 3][(1 + tid) * 4]);
#pragma unroll
      for (int n = 0; n < 4; ++n) bacc[n] += (float)e[n];
    }
    __syncthreads();   // this row's X buffer and dE row y - 1's slot are free
    if (more) {
      xb ^= 1;
      store_x(xb);
      store_e(y + 2);
    }
    __syncthreads();
  }
  // D[c][(tap, n)]: lane holds c = 16 w + 4 (l / 16) + i, tap = 4 tg + (l % 16) / 4, n = l % 4
  const int stride = a.NR * NF * 9 + a.NR;
  float* dst = a.part + (long)blockIdx.x * stride;
  const int n = lane & 3;
#pragma unroll
  for (int tg = 0; tg < 3; ++tg) {
    const int tap = 4 * tg + q;   // D column l % 16 = 4 (tap - 4 tg) + n
    if (tap < 9 && n < a.NR)
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[(n * NF + 16 * wave + 4 * (lane >> 4) + i) * 9 + tap] = acc[tg][i];
  }
  if (wave == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) bacc[k] = wave_sum(bacc[k]);
    if (lane == 0)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k < a.NR) dst[a.NR * NF * 9 + k] = bacc[k];
  }
}

// grad[e] (+)= sum over workgroups, in fixed order: 16 elements x 16 partial ranges per 256-thread
// workgroup (each thread sums its range's partials; the 16 range sums then added in range order), so the
// ~1,700 outputs x 1,024 partials spread over ~110 workgroups instead of one thread per output
constexpr int FIN_E = 16, FIN_R = 16;
__global__ __launch_bounds__(256) void narrow_wgrad_finalize_kernel(const float* __restrict__ part, int nblk, int NR,
                                                                    float* __restrict__ gw, float* __restrict__ gb,
                                                                    int accumulate) {
  __shared__ float sp[FIN_R][FIN_E];
  const int nw = NR * NF * 9, stride = nw + NR;
  const int el = threadIdx.x % FIN_E, rg = threadIdx.x / FIN_E;
  const int e = blockIdx.x * FIN_E + el;
  const int per = (nblk + FIN_R - 1) / FIN_R, k0 = rg * per, k1 = k0 + per < nblk ? k0 + per : nblk;
  float s = 0.f;
  if (e < stride) {
#pragma unroll 8
    for (int k = k0; k < k1; ++k) s += part[(long)k * stride + e];
  }
  sp[rg][el] = s;
  __syncthreads();
  if (rg == 0 && e < stride) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < FIN_R; ++r) t += sp[r][el];
    if (e < nw) gw[e] = accumulate ? gw[e] + t : t;
    else if (gb) gb[e - nw] = accumulate ? gb[e - nw] + t : t;
  }
}

// persistent workgroups: `per_cu` per CU (row runs of equal length)
int grid_rows(long total, int per_cu) {
  const long g = (long)num_cus() * per_cu;
  return (int)(total < g ? total : g);
}

// ---------------------------------------------------------------------------------------------------
// fp32x3 forms (the fp32 engine's arithmetic, gemm_x3.hip): fp32 operands, each staged into LDS as the fp16
// pair of v 2^e (hi = f16(v 2^e), lo = f16(v 2^e - hi)), every product hi.hi + lo.hi + hi.lo on
// v_mfma_f32_16x16x32_f16, fp32 accumulation rescaled by 2^-(eA + eB).  Same row windows, fragment orders
// and MFMA shapes as the bf16 kernels above; the weights come from the fp32 master weight [NR][64][3][3]
// (x 2^KAIR_X3_WEXP) through a pack launch into ws.
// ---------------------------------------------------------------------------------------------------
KAIR_DEV void split4(const float4 v, float s, f16x4& h, f16x4& l) {
  const float a[4] = {v.x * s, v.y * s, v.z * s, v.w * s};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    h[j] = (f16)a[j];
    l[j] = (f16)(a[j] - (float)h[j]);
  }
}

KAIR_DEV f16x8 cat8(const f16x4& a, const f16x4& b) { return f16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]}; }

// 8 consecutive rows (pixels) of one column of a 16-bit LDS plane: two ds_read_b64_tr_b16, the second at + d
KAIR_DEV f16x8 tr8(const f16* p, int d) {
  typedef __attribute__((address_space(3))) short4v* lp;
  const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)p), hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(p + d));
  short __attribute__((ext_vector_type(8))) s8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(f16x8, s8);
}

KAIR_DEV f32x4 mfma_h(const f16x8& a, const f16x8& b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }

// fp16 pair of w 2^KAIR_X3_WEXP
KAIR_DEV f16 wsplit(float w, int half) {
  const float v = ldexpf(w, KAIR_X3_WEXP);
  const f16 h = (f16)v;
  return half ? (f16)(v - (float)h) : h;
}

// forward fragments [18 kb][hi, lo][64][8]: A row n = lane % 16, k = 8 (lane / 16) + j of k-step kb
// (tap = kb / 2, channel 32 (kb % 2) + k) -- the kind-15 order
__global__ void narrow_fwd_x3_pack_kernel(const float* __restrict__ w, int NR, f16* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 18 * 2 * 64 * 8) return;
  const int j = t & 7, ln = (t >> 3) & 63, half = (t >> 9) & 1, kb = t >> 10;
  const int n = ln & 15, c = 32 * (kb & 1) + 8 * (ln >> 4) + j, tap = kb >> 1;
  out[t] = wsplit(n < NR ? w[((long)n * NF + c) * 9 + tap] : 0.f, half);
}

// input-gradient fragments [4 cb][2 ks][hi, lo][64][8]: row c = 16 cb + lane % 16, k = tap * 4 + n
__global__ void narrow_dgrad_x3_pack_kernel(const float* __restrict__ w, int NR, f16* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 4 * 2 * 2 * 64 * 8) return;
  const int j = t & 7, ln = (t >> 3) & 63, half = (t >> 9) & 1, ks = (t >> 10) & 1, cb = t >> 11;
  const int c = 16 * cb + (ln & 15), k = 32 * ks + 8 * (ln >> 4) + j;
  const int tap = k >> 2, n = k & 3;
  out[t] = wsplit(tap < 9 && n < NR ? w[((long)n * NF + c) * 9 + tap] : 0.f, half);
}

struct NarrowFwdX3Args {
  const float* x; long ldx;             // [B*H*W][ldx] fp32, channels [0, 64)
  const f16* w;                         // narrow_fwd_x3_pack_kernel fragments
  const float* bias; const float* mean; float range; int NR;
  const float* resid; float* out;       // as NarrowFwdArgs
  int B, H, W;
  float sx, oscale;                     // 2^ex, 2^-(ex + KAIR_X3_WEXP)
};

// the staged row as kair_conv3x3_narrow_fwd's pair layout (FPST halves per pixel: hi [0, 64), lo [64, 128));
// a 16-byte chunk c of the fp32 row is pixel c / 16, channels 4 (c % 16) .. + 3
__global__ __launch_bounds__(256, 2) void conv3x3_narrow_fwd_x3_kernel(const NarrowFwdX3Args a) {
  constexpr int KS = 9 * NF / 32;
  __shared__ __attribute__((aligned(16))) f16 sRow[4 * FROW];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  f16x8 wh[KS], wl[KS];
#pragma unroll
  for (int kb = 0; kb < KS; ++kb) {
    wh[kb] = *(const f16x8*)(a.w + ((long)kb * 2 + 0) * 512 + lane * 8);
    wl[kb] = *(const f16x8*)(a.w + ((long)kb * 2 + 1) * 512 + lane * 8);
  }
  float bias4[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) bias4[n] = n < a.NR ? a.bias[n] : 0.f;
  const int nseg = a.W / SEG;
  const long total = (long)a.B * nseg * a.H;
  const RowRun run = row_run(total, gridDim.x, blockIdx.x);
  float4 pre[FPER];
  auto load_row = [&](long st, int yy) {
    const int b = (int)(st / nseg), x0 = (int)(st - (long)b * nseg) * SEG;
#pragma unroll
    for (int i = 0; i < FPER; ++i) {
      const int c = tid + 256 * i;
      const int xx = x0 - 1 + (c >> 4);
      const bool ok = c < FCH && (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W;
      pre[i] = *(const float4*)(a.x + (ok ? ((long)(b * a.H + yy) * a.W + xx) * a.ldx + (c & 15) * 4 : 0));
      if (!ok) pre[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_row = [&](int yy) {
    f16* dst = sRow + (yy & 3) * FROW;
#pragma unroll
    for (int i = 0; i < FPER; ++i) {
      const int c = tid + 256 * i;
      if (c < FCH) {
        f16x4 h, l;
        split4(pre[i], a.sx, h, l);
        f16* p = dst + (c >> 4) * FPST + (c & 15) * 4;
        *(f16x4*)p = h;
        *(f16x4*)(p + NF) = l;
      }
    }
  };
  const int pl = lane & 15, cq = 8 * (lane >> 4);
  long cur_strip = -1;
  for (long g = run.g0; g < run.g1; ++g) {
    const long st = g / a.H;
    const int y = (int)(g - st * a.H);
    if (st != cur_strip) {
      __syncthreads();
      for (int d = -1; d <= 1; ++d) {
        load_row(st, y + d);
        store_row(y + d + 4);
      }
      cur_strip = st;
      __syncthreads();
    }
    const bool more = g + 1 < run.g1 && (g + 1) / a.H == st;
    if (more) load_row(st, y + 2);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f}, acc1 = acc, acc2 = acc;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int dy = tap / 3 - 1, dx = tap % 3 - 1;
      const f16* src = sRow + ((y + dy + 4) & 3) * FROW + (1 + 16 * wave + pl + dx) * FPST + cq;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const f16x8 xh = *(const f16x8*)(src + 32 * ks), xl = *(const f16x8*)(src + NF + 32 * ks);
        const int kb = tap * 2 + ks;
        acc = mfma_h(wh[kb], xh, acc);
        acc1 = mfma_h(wl[kb], xh, acc1);
        acc2 = mfma_h(wh[kb], xl, acc2);
      }
    }
    acc += acc1 + acc2;
    if (lane < 16) {
      const int b = (int)(st / nseg), x0 = (int)(st - (long)b * nseg) * SEG;
      const long HW = (long)a.H * a.W;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        if (n < a.NR) {
          const long o = ((long)b * a.NR + n) * HW + (long)y * a.W + x0 + 16 * wave + pl;
          float v = (acc[n] * a.oscale + bias4[n]) / a.range + (a.mean ? a.mean[n] : 0.f);
          if (a.resid) v += a.resid[o];
          a.out[o] = v;
        }
      }
    }
    __syncthreads();
    if (more) store_row(y + 2);
    __syncthreads();
  }
}

struct NarrowDgradX3Args {
  const float* dE; long lde;            // [B*H*W][lde] fp32, channels [0, 4) read (weights 0 for n >= NR)
  const f16* w;                         // narrow_dgrad_x3_pack_kernel fragments
  float* out; long ldo; int ps_r;       // fp32 rows or PixelUnshuffle SPM, as NarrowDgradArgs
  int B, H, W;
  float se, oscale;                     // 2^eg, 2^-(eg + KAIR_X3_WEXP)
};

__global__ __launch_bounds__(256) void conv3x3_narrow_dgrad_x3_kernel(const NarrowDgradX3Args a) {
  __shared__ __attribute__((aligned(16))) f16 sEh[4 * DROW], sEl[4 * DROW];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  f16x8 wf[4][2][2];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int h = 0; h < 2; ++h) wf[cb][ks][h] = *(const f16x8*)(a.w + (((cb * 2 + ks) * 2 + h) * 64 + lane) * 8);
  const int nseg = a.W / SEG;
  const long total = (long)a.B * nseg * a.H;
  const RowRun run = row_run(total, gridDim.x, blockIdx.x);
  float4 pre = make_float4(0.f, 0.f, 0.f, 0.f);
  auto load_row = [&](long st, int yy) {
    const int b = (int)(st / nseg), x0 = (int)(st - (long)b * nseg) * SEG;
    const int xx = x0 - 1 + tid;
    const bool ok = tid < PXS && (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W;
    pre = *(const float4*)(a.dE + (ok ? ((long)(b * a.H + yy) * a.W + xx) * a.lde : 0));
    if (!ok) pre = make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto store_row = [&](int yy) {
    if (tid < PXS) {
      f16x4 h, l;
      split4(pre, a.se, h, l);
      *(f16x4*)(sEh + (yy & 3) * DROW + tid * DPST) = h;
      *(f16x4*)(sEl + (yy & 3) * DROW + tid * DPST) = l;
    }
  };
  const int pl = lane & 15, kq = lane >> 4;
  long cur_strip = -1;
  for (long g = run.g0; g < run.g1; ++g) {
    const long st = g / a.H;
    const int y = (int)(g - st * a.H);
    if (st != cur_strip) {
      __syncthreads();
      for (int d = -1; d <= 1; ++d) {
        load_row(st, y + d);
        store_row(y + d + 4);
      }
      cur_strip = st;
      __syncthreads();
    }
    const bool more = g + 1 < run.g1 && (g + 1) / a.H == st;
    if (more) load_row(st, y + 2);
    f16x8 bh[2], bl[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f16x4 eh[2], el[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int tap = 8 * ks + 2 * kq + h;
        if (tap < 9) {
          const int dy = tap / 3 - 1, dx = tap % 3 - 1;
          const int o = ((y - dy + 4) & 3) * DROW + (1 + 16 * wave + pl - dx) * DPST;
          eh[h] = *(const f16x4*)(sEh + o);
          el[h] = *(const f16x4*)(sEl + o);
        } else {
          eh[h] = f16x4{};
          el[h] = f16x4{};
        }
      }
      bh[ks] = cat8(eh[0], eh[1]);
      bl[ks] = cat8(el[0], el[1]);
    }
    const int b = (int)(st / nseg), x0 = (int)(st - (long)b * nseg) * SEG;
    const int x = x0 + 16 * wave + pl;
    long o;
    if (a.ps_r > 1) {
      const int r = a.ps_r, yl = y / r, xl = x / r;
      o = ((long)(b * (a.H / r) + yl) * (a.W / r) + xl) * a.ldo + ((y - yl * r) * r + (x - xl * r)) * NF;
    } else {
      o = ((long)(b * a.H + y) * a.W + x) * a.ldo;
    }
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f}, acc1 = acc;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        acc = mfma_h(wf[cb][ks][0], bh[ks], acc);
        acc1 = mfma_h(wf[cb][ks][1], bh[ks], acc1);
        acc1 = mfma_h(wf[cb][ks][0], bl[ks], acc1);
      }
      acc += acc1;
      *(float4*)(a.out + o + 16 * cb + 4 * kq) =
          make_float4(acc[0] * a.oscale, acc[1] * a.oscale, acc[2] * a.oscale, acc[3] * a.oscale);
    }
    __syncthreads();
    if (more) store_row(y + 2);
    __syncthreads();
  }
}

struct NarrowWgradX3Args {
  const float* dE; long lde;            // [M][lde] fp32, channels [0, 4)
  const float* x; long ldx;             // [M][ldx] fp32 image, channels [0, 64)
  int NR;
  int B, H, W;
  float* part;                          // [gridDim.x][NR * 64 * 9 + NR]
  float se, sx, oscale, bscale;         // 2^eg, 2^ex, 2^-(eg + ex), 2^-eg
};

// conv3x3_narrow_wgrad_kernel's MFMA over the pixels with both operands as fp16 pairs: an X row is 64 px x 16
// chunks of 4 fp32 channels (4 per thread), split into its hi and lo planes
__global__ __launch_bounds__(256) void conv3x3_narrow_wgrad_x3_kernel(const NarrowWgradX3Args a) {
  __shared__ __attribute__((aligned(16))) f16 sXh[2][SEG * XS], sXl[2][SEG * XS];
  __shared__ __attribute__((aligned(16))) f16 sEh[4][EPX + 8], sEl[4][EPX + 8];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = (lane & 15) >> 2, p4 = (lane & 3) * 4, g8 = (lane >> 4) * 8;
  const int tl = p4 >> 2;
  f32x4 acc[3];
#pragma unroll
  for (int tg = 0; tg < 3; ++tg) acc[tg] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc[4] = {0.f, 0.f, 0.f, 0.f};
  const int nseg = a.W / SEG;
  const long total = (long)a.B * nseg * a.H;
  const RowRun run = row_run(total, gridDim.x, blockIdx.x);
  float4 px_[4];
  float4 pe = make_float4(0.f, 0.f, 0.f, 0.f);
  auto load_x = [&](long st, int yy) {
    const int b = (int)(st / nseg), x0 = (int)(st - (long)b * nseg) * SEG;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cidx = tid + 256 * i;
      px_[i] = *(const float4*)(a.x + ((long)(b * a.H + yy) * a.W + x0 + (cidx >> 4)) * a.ldx + (cidx & 15) * 4);
    }
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cidx = tid + 256 * i, o = (cidx >> 4) * XS + (cidx & 15) * 4;
      f16x4 h, l;
      split4(px_[i], a.sx, h, l);
      *(f16x4*)(&sXh[buf][o]) = h;
      *(f16x4*)(&sXl[buf][o]) = l;
    }
  };
  auto load_e = [&](long st, int yy) {
    const int b = (int)(st / nseg), x0 = (int)(st - (long)b * nseg) * SEG;
    const int xx = x0 - 1 + tid;
    const bool ok = tid < PXS && (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W;
    pe = *(const float4*)(a.dE + (ok ? ((long)(b * a.H + yy) * a.W + xx) * a.lde : 0));
    if (!ok) pe = make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto store_e = [&](int yy) {
    if (tid < PXS) {
      f16x4 h, l;
      split4(pe, a.se, h, l);
      *(f16x4*)(&sEh[yy & 3][tid * 4]) = h;
      *(f16x4*)(&sEl[yy & 3][tid * 4]) = l;
    }
  };
  // zero tails of every slot of both planes (taps >= 9 read slot 0's; store_e never writes them)
  if (tid < 16) {
    f16* t = (tid & 8 ? &sEl[0][0] : &sEh[0][0]) + ((tid >> 1) & 3) * (EPX + 8) + EPX + (tid & 1) * 4;
    *(f16x4*)t = f16x4{};
  }
  long cur_strip = -1;
  int xb = 0;
  for (long g = run.g0; g < run.g1; ++g) {
    const long st = g / a.H;
    const int y = (int)(g - st * a.H);
    if (st != cur_strip) {
      __syncthreads();
      for (int d = -1; d <= 1; ++d) {
        load_e(st, y + d);
        store_e(y + d + 4);
      }
      load_x(st, y);
      store_x(xb);
      cur_strip = st;
      __syncthreads();
    }
    const bool more = g + 1 < run.g1 && (g + 1) / a.H == st;
    if (more) {
      load_x(st, y + 1);
      load_e(st, y + 2);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int r0 = 32 * ks + g8 + q;
      const int xo = r0 * XS + 16 * wave + p4;
      const f16x8 ah = tr8(&sXh[xb][xo], 4 * XS), al = tr8(&sXl[xb][xo], 4 * XS);
#pragma unroll
      for (int tg = 0; tg < 3; ++tg) {
        const int tap = 4 * tg + tl;
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
        const int eo = tap < 9 ? ((y - dy + 4) & 3) * (EPX + 8) + (1 + r0 - dx) * 4 : EPX;
        const int step = tap < 9 ? 16 : 0;   // rows r0 + 4: 4 pixels on (the zero tail stays put)
        const f16x8 eh = tr8(&sEh[0][0] + eo, step), el = tr8(&sEl[0][0] + eo, step);
        acc[tg] = mfma_h(ah, eh, acc[tg]);
        acc[tg] = mfma_h(al, eh, acc[tg]);
        acc[tg] = mfma_h(ah, el, acc[tg]);
      }
    }
    if (tid < SEG) {
      const f16x4 h = *(const f16x4*)(&sEh[y & 3][(1 + tid) * 4]), l = *(const f16x4*)(&sEl[y & 3][(1 + tid) * 4]);
#pragma unroll
      for (int n = 0; n < 4; ++n) bacc[n] += (float)h[n] + (float)l[n];
    }
    __syncthreads();
    if (more) {
      xb ^= 1;
      store_x(xb);
      store_e(y + 2);
    }
    __syncthreads();
  }
  const int stride = a.NR * NF * 9 + a.NR;
  float* dst = a.part + (long)blockIdx.x * stride;
  const int n = lane & 3;
#pragma unroll
  for (int tg = 0; tg < 3; ++tg) {
    const int tap = 4 * tg + q;
    if (tap < 9 && n < a.NR)
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[(n * NF + 16 * wave + 4 * (lane >> 4) + i) * 9 + tap] = acc[tg][i] * a.oscale;
  }
  if (wave == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) bacc[k] = wave_sum(bacc[k]);
    if (lane == 0)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k < a.NR) dst[a.NR * NF * 9 + k] = bacc[k] * a.bscale;
  }
}

}  // namespace

extern "C" int kair_conv3x3_narrow_fwd(const void* x, long ldx, int lo_off, const void* w, const float* bias, int NR,
                                       const float* mean, float img_range, const float* resid, float* out, int B, int H,
                                       int W, void* stream) {
  KAIR_CHECK_ARG(x && w && bias && out && NR >= 1 && NR <= 4 && B > 0 && H > 0 && W > 0, "conv3x3_narrow_fwd: bad args");
  KAIR_CHECK_ARG(W % SEG == 0, "conv3x3_narrow_fwd: W must be a multiple of 64 (row segments)");
  KAIR_CHECK_ARG(ldx % 8 == 0 && ldx >= NF && (lo_off == 0 || (lo_off % 8 == 0 && lo_off + NF <= ldx)) &&
                     ((uintptr_t)x & 15) == 0 && ((uintptr_t)w & 15) == 0,
                 "conv3x3_narrow_fwd: x rows of >= 64 bf16 channels (lo half at lo_off), 16-byte aligned");
  KAIR_CHECK_ARG((long)B * H * W < (1L << 31), "conv3x3_narrow_fwd: too many pixels");
  NarrowFwdArgs a;
  a.x = (const bf16*)x; a.ldx = ldx; a.lo_off = lo_off; a.w = (const bf16*)w; a.bias = bias;
  a.mean = mean; a.range = img_range; a.NR = NR; a.resid = resid; a.out = out;
  a.B = B; a.H = H; a.W = W;
  // two workgroups per CU (72 KB LDS, <= 256 VGPRs each): one computes while the other waits on its rows
  KAIR_LAUNCH(conv3x3_narrow_fwd_kernel, dim3(grid_rows((long)B * (W / SEG) * H, 2)), dim3(256), 0,
                     (hipStream_t)stream, a);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" long kair_conv3x3_narrow_dgrad_ws(void) { return 4 * 2 * 64 * 8 / 2; }   // floats (bf16 fragments)

extern "C" int kair_conv3x3_narrow_dgrad(const void* dE, long lde, const float* w, int NR, void* ws, void* out, int out_dtype,
                                         long ldo, int ps_r, int B, int H, int W, void* stream) {
  KAIR_CHECK_ARG(dE && w && ws && out && NR >= 1 && NR <= 4 && lde >= 4 && lde % 4 == 0 && ((uintptr_t)dE & 7) == 0 &&
                     ((uintptr_t)ws & 15) == 0,
                 "conv3x3_narrow_dgrad: dE rows of >= 4 bf16 channels, 8-byte aligned; 16-byte aligned ws");
  KAIR_CHECK_ARG(out_dtype == KAIR_BF16 || out_dtype == KAIR_F32, "conv3x3_narrow_dgrad: out dtype");
  KAIR_CHECK_ARG(W % SEG == 0, "conv3x3_narrow_dgrad: W must be a multiple of 64 (row segments)");
  KAIR_CHECK_ARG(ps_r <= 1 ? ldo >= NF : (H % ps_r == 0 && W % ps_r == 0 && ldo >= (long)ps_r * ps_r * NF),
                 "conv3x3_narrow_dgrad: output stride / PixelUnshuffle geometry");
  KAIR_CHECK_ARG(ldo % 4 == 0 && ((uintptr_t)out & 15) == 0 && (long)B * H * W < (1L << 31), "conv3x3_narrow_dgrad: alignment");
  hipStream_t s = (hipStream_t)stream;
  KAIR_LAUNCH(narrow_dgrad_pack_kernel, dim3(16), dim3(256), 0, s, w, NR, (bf16*)ws);
  NarrowDgradArgs a;
  a.dE = (const bf16*)dE; a.lde = lde; a.w = (const bf16*)ws; a.out = out; a.odt = out_dtype; a.ldo = ldo; a.ps_r = ps_r;
  a.B = B; a.H = H; a.W = W;
  KAIR_LAUNCH(conv3x3_narrow_dgrad_kernel, dim3(grid_rows((long)B * (W / SEG) * H, 4)), dim3(256), 0, s, a);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" long kair_conv3x3_narrow_wgrad_ws(int NR) {
  return 4L * num_cus() * (NR * NF * 9 + NR);
}

extern "C" int kair_conv3x3_narrow_wgrad(const void* dE, long lde, const void* x, long ldx, int NR, float* ws, float* grad_w,
                                         float* grad_b, int accumulate, int B, int H, int W, void* stream) {
  KAIR_CHECK_ARG(dE && x && ws && grad_w && NR >= 1 && NR <= 4 && lde >= 4 && lde % 4 == 0 && ldx >= NF && ldx % 8 == 0 &&
                     ((uintptr_t)dE & 7) == 0 && ((uintptr_t)x & 15) == 0,
                 "conv3x3_narrow_wgrad: bad operands");
  KAIR_CHECK_ARG(W % SEG == 0, "conv3x3_narrow_wgrad: W must be a multiple of 64 (row segments)");
  KAIR_CHECK_ARG((long)B * H * W < (1L << 31), "conv3x3_narrow_wgrad: too many pixels");
  NarrowWgradArgs a;
  a.dE = (const bf16*)dE; a.lde = lde; a.x = (const bf16*)x; a.ldx = ldx; a.NR = NR;
  a.B = B; a.H = H; a.W = W;
  a.part = ws;
  const int grid = grid_rows((long)B * (W / SEG) * H, 4);
  hipStream_t s = (hipStream_t)stream;
  KAIR_LAUNCH(conv3x3_narrow_wgrad_kernel, dim3(grid), dim3(256), 0, s, a);
  KAIR_CHECK_LAUNCH();
  const int stride = NR * NF * 9 + NR;
  KAIR_LAUNCH(narrow_wgrad_finalize_kernel, dim3((stride + FIN_E - 1) / FIN_E), dim3(256), 0, s, ws, grid, NR, grad_w,
                     grad_b, accumulate);
  KAIR_CHECK_LAUNCH();
  return 0;
}

// ---- fp32x3 forms ---------------------------------------------------------------------------------
extern "C" long kair_conv3x3_narrow_x3_ws(void) { return 18 * 2 * 64 * 8 / 2; }   // floats (fp16 fragments)

extern "C" int kair_conv3x3_narrow_fwd_x3(const float* x, long ldx, int ex, const float* w, const float* bias, int NR,
                                          void* ws, const float* mean, float img_range, const float* resid, float* out,
                                          int B, int H, int W, void* stream) {
  KAIR_CHECK_ARG(x && w && ws && bias && out && NR >= 1 && NR <= 4 && B > 0 && H > 0 && W > 0, "conv3x3_narrow_fwd_x3: bad args");
  KAIR_CHECK_ARG(W % SEG == 0, "conv3x3_narrow_fwd_x3: W must be a multiple of 64 (row segments)");
  KAIR_CHECK_ARG(ldx % 4 == 0 && ldx >= NF && ((uintptr_t)x & 15) == 0 && ((uintptr_t)ws & 15) == 0,
                 "conv3x3_narrow_fwd_x3: x rows of >= 64 fp32 channels, 16-byte aligned; 16-byte aligned ws");
  KAIR_CHECK_ARG((long)B * H * W < (1L << 31), "conv3x3_narrow_fwd_x3: too many pixels");
  hipStream_t s = (hipStream_t)stream;
  KAIR_LAUNCH(narrow_fwd_x3_pack_kernel, dim3(18 * 2 * 64 * 8 / 256), dim3(256), 0, s, w, NR, (f16*)ws);
  NarrowFwdX3Args a;
  a.x = x; a.ldx = ldx; a.w = (const f16*)ws; a.bias = bias; a.mean = mean; a.range = img_range; a.NR = NR;
  a.resid = resid; a.out = out; a.B = B; a.H = H; a.W = W;
  a.sx = ldexpf(1.f, ex); a.oscale = ldexpf(1.f, -(ex + KAIR_X3_WEXP));
  KAIR_LAUNCH(conv3x3_narrow_fwd_x3_kernel, dim3(grid_rows((long)B * (W / SEG) * H, 2)), dim3(256), 0, s, a);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_conv3x3_narrow_dgrad_x3(const float* dE, long lde, int eg, const float* w, int NR, void* ws, float* out,
                                            long ldo, int ps_r, int B, int H, int W, void* stream) {
  KAIR_CHECK_ARG(dE && w && ws && out && NR >= 1 && NR <= 4 && lde >= 4 && lde % 4 == 0 && ((uintptr_t)dE & 15) == 0 &&
                     ((uintptr_t)ws & 15) == 0,
                 "conv3x3_narrow_dgrad_x3: dE rows of >= 4 fp32 channels, 16-byte aligned; 16-byte aligned ws");
  KAIR_CHECK_ARG(W % SEG == 0, "conv3x3_narrow_dgrad_x3: W must be a multiple of 64 (row segments)");
  KAIR_CHECK_ARG(ps_r <= 1 ? ldo >= NF : (H % ps_r == 0 && W % ps_r == 0 && ldo >= (long)ps_r * ps_r * NF),
                 "conv3x3_narrow_dgrad_x3: output stride / PixelUnshuffle geometry");
  KAIR_CHECK_ARG(ldo % 4 == 0 && ((uintptr_t)out & 15) == 0 && (long)B * H * W < (1L << 31), "conv3x3_narrow_dgrad_x3: alignment");
  hipStream_t s = (hipStream_t)stream;
  KAIR_LAUNCH(narrow_dgrad_x3_pack_kernel, dim3(4 * 2 * 2 * 64 * 8 / 256), dim3(256), 0, s, w, NR, (f16*)ws);
  NarrowDgradX3Args a;
  a.dE = dE; a.lde = lde; a.w = (const f16*)ws; a.out = out; a.ldo = ldo; a.ps_r = ps_r; a.B = B; a.H = H; a.W = W;
  a.se = ldexpf(1.f, eg); a.oscale = ldexpf(1.f, -(eg + KAIR_X3_WEXP));
  KAIR_LAUNCH(conv3x3_narrow_dgrad_x3_kernel, dim3(grid_rows((long)B * (W / SEG) * H, 4)), dim3(256), 0, s, a);
  KAIR_CHECK_LAUNCH();
  return 0;
}

extern "C" int kair_conv3x3_narrow_wgrad_x3(const float* dE, long lde, int eg, const float* x, long ldx, int ex, int NR,
                                            float* ws, float* grad_w, float* grad_b, int accumulate, int B, int H, int W,
                                            void* stream) {
  KAIR_CHECK_ARG(dE && x && ws && grad_w && NR >= 1 && NR <= 4 && lde >= 4 && lde % 4 == 0 && ldx >= NF && ldx % 4 == 0 &&
                     ((uintptr_t)dE & 15) == 0 && ((uintptr_t)x & 15) == 0,
                 "conv3x3_narrow_wgrad_x3: bad operands");
  KAIR_CHECK_ARG(W % SEG == 0, "conv3x3_narrow_wgrad_x3: W must be a multiple of 64 (row segments)");
  KAIR_CHECK_ARG((long)B * H * W < (1L << 31), "conv3x3_narrow_wgrad_x3: too many pixels");
  NarrowWgradX3Args a;
  a.dE = dE; a.lde = lde; a.x = x; a.ldx = ldx; a.NR = NR; a.B = B; a.H = H; a.W = W; a.part = ws;
  a.se = ldexpf(1.f, eg); a.sx = ldexpf(1.f, ex); a.oscale = ldexpf(1.f, -(eg + ex)); a.bscale = ldexpf(1.f, -eg);
  const int grid = grid_rows((long)B * (W / SEG) * H, 4);
  hipStream_t s = (hipStream_t)stream;
  KAIR_LAUNCH(conv3x3_narrow_wgrad_x3_kernel, dim3(grid), dim3(256), 0, s, a);
  KAIR_CHECK_LAUNCH();
  const int stride = NR * NF * 9 + NR;
  KAIR_LAUNCH(narrow_wgrad_finalize_kernel, dim3((stride + FIN_E - 1) / FIN_E), dim3(256), 0, s, ws, grid, NR, grad_w,
                     grad_b, accumulate);
  KAIR_CHECK_LAUNCH();
  return 0;
}
