/*
 * kair_hip.h — C ABI of libkair_hip.so, the MI355X (gfx950) kernels behind the KAIR hot path.
 *
 * The reference (Owen1B/KAIR) has NO native code on this path: models/network_{swinir,dncnn,
 * rrdb,rrdbnet,usrnet}.py run on ATen (cuDNN / cuBLAS in the reference).  These entry points
 * replace the ATen calls that those files make; each declaration names the reference site.
 *
 * Conventions:
 *   - plain device pointers + sizes, caller (PyTorch caching allocator) owns every buffer,
 *     including outputs and workspaces; no allocation, no host sync, no global mutable state;
 *   - every call takes the hipStream_t to launch on (passed as void* to keep this header
 *     HIP-free) and is graph-capturable;
 *   - return 0 on success or a negative KAIR_ERR_* code; kair_last_error() returns a
 *     thread-local message for the last failure.
 *
 * Activation layouts: NHWC token matrices with the channel dimension padded
 * to a multiple of 32 (e.g. SwinIR C=180 -> 192), head-padded q/k/v (head_dim 30 -> 32),
 * fp32 residual stream, bf16 (or fp32 in parity mode) GEMM operands, fp32 accumulation.
 */
#ifndef KAIR_HIP_H
#define KAIR_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define KAIR_OK 0
#define KAIR_ERR_ARG (-1)
#define KAIR_ERR_HIP (-2)

typedef enum { KAIR_F32 = 0, KAIR_BF16 = 1, KAIR_F16 = 3 } kair_dtype;
/* `compute` of kair_gemm_nt / kair_gemm_tn besides the dtypes: the split-fp16 ("x3") arithmetic of the
 * fp32 engine on the 16-bit matrix cores.  Every operand x enters as a pair of fp16 values of x * 2^e
 * (hi = f16(x 2^e), lo = f16(x 2^e - hi); e = kair_operand.x3_exp, a power-of-2 scale that centres the
 * operand in fp16's range) and every product as hi.hi + hi.lo + lo.hi with fp32 accumulation, rescaled by
 * 2^-(eA + eB): ~2^-21 relative per product, the precision class of fp32 arithmetic (one bf16 product:
 * 2^-8; bf16 pairs: 2^-16).  Operands: fp32 (split in the kernel) or fp16 hi planes with
 * kair_operand.lo_ptr (their stored values carry x3_exp).  Packed weights (kinds 9 / 17 / 18 / 19 with an
 * fp16 destination) hold w * 2^KAIR_X3_WEXP. */
#define KAIR_COMPUTE_X3 2
#define KAIR_X3_WEXP 12

/* How a GEMM operand element (row m, column k) is addressed. */
typedef enum {
  KAIR_LD_ROWS = 0,    /* ptr[rowmap(m) * ld + k]                                           */
  KAIR_LD_IM2COL3 = 1, /* 3x3/pad1/stride1 patch of an NHWC image [B, im_H, im_W, im_C]:
                          k = tap * im_C + c                                                 */
  KAIR_LD_QKVBLK = 2,  /* head-blocked q/k/v: [part][window][head][tok][hdp], k = part*nh*hdp
                          + head*hdp + d                                                    */
  KAIR_LD_S2D = 3      /* 2x2 / stride-2 patch (space-to-depth) of an NHWC image
                          [B, 2*im_H, 2*im_W, im_C]: row m = (b, y, x) of the im_H x im_W OUTPUT grid,
                          k = (i*2 + j) * im_C + c -> pixel (2y+i, 2x+j); ld = pixel stride (0: im_C).
                          basicblock.downsample_strideconv forward / upsample_convtranspose dgrad */
} kair_load_mode;

typedef struct {
  const void* ptr;
  int dtype;           /* kair_dtype                                                         */
  int mode;            /* kair_load_mode                                                     */
  long ld;             /* ROWS: row stride in elements                                       */
  int win_H, win_W, win_ws, win_shift; /* ROWS: Swin window->token row map (ws==0: identity)  */
  int im_H, im_W, im_C, im_flip;       /* IM2COL3 (im_flip: tap (dy,dx) -> (-dy,-dx), dgrad)
                                          im_H x im_W is the CONV grid; ld = pixel stride (0: im_C) */
  int qkv_nh, qkv_hdp, qkv_tok;        /* QKVBLK                                              */
  const float* rowscale; int rows_per_scale; /* optional per-sample scale (DropPath)          */
  int ones_col;        /* >=0: this column reads as 1.0 (fused bias gradient), else -1       */
  int ones_in_data;    /* 1: the producer already stored 1.0 in column ones_col of every row
                          (lets DMA loaders skip the injection); 0: loaders inject it         */
  int im_up;           /* IM2COL3: 2 = the source image is im_H/2 x im_W/2 and is read through a
                          nearest x2 upsample (F.interpolate(scale 2, 'nearest')); 0/1 = none  */
  int w_split;         /* kair_gemm_nt B only (bf16 compute): 1 = the packed weight rows hold a
                          hi/lo bf16 pair per value (w = hi + lo, pack kind 9), interleaved per 64
                          columns [hi k0..k0+63 | lo k0..k0+63 | hi k0+64.. ...]; row length
                          2*ceil(K/64)*64.  The A operand is read once per pair, so the product
                          carries ~16 mantissa bits of the fp32 master weights (bf16 weight
                          rounding biases the output, see DESIGN.md "parity at bf16")        */
  int a_split;         /* kair_gemm_nt A only (bf16 compute).  1 (ROWS / IM2COL3, no rowscale): the
                          activation enters the product as a hi/lo bf16 pair, x = hi + lo with
                          lo = bf16(x - hi), adding the product a_lo . w_hi (with w_split also
                          a_hi . w_lo): ~16 mantissa bits of the activation instead of 8.
                          fp32 A: lo is formed in the kernel from the fp32 value; bf16 A: ptr
                          holds the hi plane and lo_ptr the lo plane (same layout).
                          2 (bf16 IM2COL3 with w_split): the image's im_C channels are the [hi | lo]
                          halves of one activation and B is packed tied over both halves (kair_wmap
                          kG = 2), so the plain product is already the split one; the flag lets
                          the 3x3 halo kernel skip the negligible lo . w_lo chunk products   */
  const void* lo_ptr;  /* bf16 A with a_split: the lo plane (kair_epilogue.out_lo of its producer);
                          x3 compute: the lo plane of an fp16 operand                           */
  int x3_exp;          /* x3 compute: the operand's power-of-2 exponent (fp32: applied before the fp16
                          split; fp16 planes: carried by the stored values); packed weights KAIR_X3_WEXP */
} kair_operand;

typedef enum {
  KAIR_OUT_ROWS = 0,      /* out[rowmap(m) * ldo + n]                                         */
  KAIR_OUT_QKVBLK = 1,    /* head-blocked q/k/v layout (as KAIR_LD_QKVBLK)                    */
  KAIR_OUT_PSHUF = 2,     /* PixelShuffle(r): m=(b,y,x) of [ps_H,ps_W], n=c*r*r+i*r+j
                             -> out NHWC [b, y*r+i, x*r+j, c] with channel stride ldo          */
  KAIR_OUT_PUNSHUF = 3,   /* inverse: m = pixel of the [ps_H*r, ps_W*r] image, n = c
                             -> out[(b,y,x) of ps_H x ps_W][c*r*r+i*r+j], stride ldo          */
  KAIR_OUT_NCHW = 4,      /* image out[b][n][y][x] (n < img_C) of [img_H, img_W],
                             value = v / img_range + img_mean[n] (+ resid[b][n][y][x] when resid
                             is set: SwinIR's denoising head x + conv_last(res), v:831-835)   */
  KAIR_OUT_PSHUF_NCHW = 5, /* PixelShuffle(r) straight into an NCHW image [b][c][y*r+i][x*r+j]
                             (c < img_C), value = v / img_range + img_mean[c]  (UpsampleOneStep) */
  KAIR_OUT_PSHUF_SPM = 6, /* as PSHUF with the GEMM columns sub-pixel-major, n = (i*r+j)*(N/r^2) + c
                             (weights packed with kair_wmap.n_perm = r^2): 8 consecutive columns
                             are 8 consecutive channels of one output pixel -> 16-byte stores      */
  KAIR_OUT_PUNSHUF_SPM = 7 /* inverse of PSHUF_SPM: out[(b,y,x)][(i*r+j)*ldc + c], ldc = ps_C       */
} kair_out_mode;

typedef enum { KAIR_ACT_NONE = 0, KAIR_ACT_GELU = 1, KAIR_ACT_LEAKY = 2, KAIR_ACT_RELU = 3 } kair_act;

typedef struct {
  void* out; int out_dtype; int out_mode; long ldo;
  int win_H, win_W, win_ws, win_shift;  /* row map for KAIR_OUT_ROWS / residual / gate         */
  const float* bias;                    /* [N] or NULL                                        */
  int act; float slope;                 /* kair_act; slope for LEAKY                          */
  void* out_pre; int pre_dtype; long ldp; /* optional: pre-activation copy (same row map)     */
  const float* resid; long ldr;          /* optional: out = resid + rowscale * value (fp32)    */
  const float* rowscale; int rows_per_scale;
  const void* gate; int gate_dtype; long ldg; int gate_kind; /* value *= act'(gate):
                                           1 gelu'(gate)  2 leaky'(sign of gate)  3 relu'
                                           4 gate itself (a stored activation derivative)     */
  int ps_r, ps_H, ps_W;                 /* pixel (un)shuffle geometry                         */
  int qkv_nh, qkv_hdp, qkv_tok;         /* KAIR_OUT_QKVBLK                                    */
  const float* img_mean; float img_range; int img_C, img_H, img_W; /* KAIR_OUT_NCHW          */
  int out_ones_col_p1;                  /* ROWS: 1 + column whose `out` value is forced to 1.0
                                           (the next weight-gradient GEMM's ones column); 0 none */
  const float* resid2; long ldr2;        /* optional second fp32 residual (ROWS): out += resid2
                                           (U-Net skip additions, network_usrnet_v1.py:159-162)  */
  int pre_kind;                         /* out_pre holds: 0 the pre-activation x; 1 act'(x) (GELU
                                           only: the backward gate, gate_kind 4, with no erf
                                           left in the backward epilogue)                        */
  void* a_copy; long ld_acopy;          /* optional bf16 copy of the A operand's image (IM2COL3 A,
                                           3x3 halo-conv path only, else KAIR_ERR_ARG): pixel m,
                                           channels [0, im_C) -> a_copy[m * ld_acopy + c] -- the
                                           weight gradient's operand, written from the halo the conv
                                           loads anyway (no extra read of the fp32 image)           */
  int acopy_ones_col_p1;                /* 1 + channel of a_copy forced to 1.0 (bias gradient); 0 none */
  void* out_lo;                         /* optional, bf16 `out` in ROWS / PSHUF_SPM mode: the lo plane
                                           lo = bf16(v - bf16(v)) at the same offsets, so the next
                                           conv can read the activation as a hi/lo pair
                                           (kair_operand.a_split); x3 compute with an fp16 `out` (ROWS /
                                           QKVBLK): the fp16 lo plane of v * 2^x3_out_exp          */
  int x3_out_exp;                       /* x3 compute, fp16 out: the stored pair holds v * 2^x3_out_exp */
} kair_epilogue;

/* C[m,n] = sum_k A[m,k] * B[n,k]  (+ epilogue).  compute: KAIR_BF16 -> v_mfma_f32_16x16x32_bf16,
 * KAIR_F32 -> v_mfma_f32_16x16x4_f32 (exact fp32).  K must be a multiple of 8.
 * Replaces: nn.Linear (network_swinir.py:19-20,105,107 forward/dgrad), nn.Conv2d 3x3
 * (network_swinir.py:465,669,729,742,745,584; network_dncnn.py:62-66; network_rrdbnet.py:82-90)
 * forward and input-gradient. */
int kair_gemm_nt(const kair_operand* A, const kair_operand* B, const kair_epilogue* E,
                 long M, int N, int K, int compute, void* stream);

/* 1 if kair_gemm_nt runs a bf16 3x3 conv of this geometry (image H x W x C, M = B*H*W rows, N outputs;
 * 16-byte aligned rows, pixel stride C, plain ROWS epilogue) on the halo-conv path, the one that can
 * write kair_epilogue.a_copy; else 0. */
int kair_conv3x3_halo_geometry(int H, int W, int C, long M, int N);

/* Weight gradient: partial[s][n][k] = sum_{m in split s} A[m,n] * B[m,k]; then
 * kair_wgrad_finalize sums the splits.  ws needs splits*N*K floats (kair_wgrad_splits()).
 * Replaces the weight-gradient half of the same nn.Linear / nn.Conv2d backward. */
int kair_wgrad_splits(long M, int N, int K);
int kair_gemm_tn(const kair_operand* A, const kair_operand* B, float* ws, int splits,
                 long M, int N, int K, int compute, void* stream);

/* Weight layout maps between reference (fp32 master, torch layout) and packed (padded) forms. */
typedef struct {
  int kind;          /* 0 linear [N][K]; 1 conv3x3 [Co][Ci][3][3] -> [Cop][9*Cip];
                        2 conv3x3 dgrad form -> [Cip][9*Cop] (flipped taps, swapped channels);
                        3 linear transposed -> [Kp][Np]; 4 bias vector;
                        7 conv2x2 [N][K][2][2] -> [Np][4*Kp], k = tap*Kp + kp (stride-2 conv
                          forward / transposed-conv dgrad over (N, K) = (Ci, Co));
                        8 conv2x2 -> [4*Kp][Np], row = kp*4 + tap (pixel-shuffle forms: stride-2
                          conv dgrad, transposed-conv forward over (N, K) = (Ci, Co));
                        9 conv3x3 forward, hi/lo split (bf16 only): [Cop][2*ceil(9*Cip/64)*64],
                          64-column chunks alternate hi = bf16(w), lo = bf16(w - hi);
                        10 linear in MFMA-fragment order [Np/32][Kp/16][64][8]: the
                          v_mfma_f32_32x32x16 operand of rows 32nb.. and k-step kb is one
                          contiguous 1 KiB block (lane l: row 32nb + l%32, k 16kb + 8(l/32) + j);
                        12 kind 10 with hi/lo halves (bf16 only): [Np/32][Kp/16][2][64][8], the hi
                          block of (nb, kb) followed by its lo block;
                        13 kind 10 of the TRANSPOSED weight: [Kp/32][Np/16][64][8], lane l: W[n][k]
                          with k = 32kb' + l%32 (output), n = 16kb + 8(l/32) + j (contraction);
                        14 linear in v_mfma_f32_16x16x32 fragment order [Np/16][Kp/32][64][8]: the
                          operand of rows 16nb.. and k-step kb is one contiguous 1 KiB block (lane l:
                          row 16nb + l%16, k 32kb + 8(l/16) + j);
                        15 conv3x3 forward in the kind-14 fragment order with hi/lo halves (bf16 only):
                          [Np/16][9*Kp/32][2][64][8], contraction index k = tap*Kp + cip (the
                          narrow-N conv's register-resident weights, kair_conv3x3_narrow_fwd;
                          kair_conv3x3_wr's split form);
                        16 conv3x3 dgrad form (kind 2) in the kind-14 fragment order (bf16):
                          [Kp/16][9*Np/32][64][8], rows = input channels, k = tap*Np + cop
                          (kair_conv3x3_wr's plain form over the output gradient, flip = 1) */
  int N, K;          /* reference dims: linear (out,in); conv (Cout,Cin)                     */
  int nG, nGr, nGp;  /* out dim = nG groups of nGr real rows padded to nGp                   */
  int kG, kGr, kGp;  /* in  dim = kG groups of kGr real cols padded to kGp (kinds 1 / 9 only: kG*kGr
                        may be a multiple of K -- tied copies, packed col -> reference col % K)   */
  int n_perm;        /* > 1: the out dim is stored sub-pixel-major for a PixelShuffle(r), n_perm =
                        r*r: packed (unpadded) row s*(N/r^2) + c holds reference row c*r^2 + s
                        (KAIR_OUT_PSHUF_SPM / KAIR_OUT_PUNSHUF_SPM layouts); 0 or 1: identity     */
} kair_wmap;

/* dst (packed, dtype) <- src (reference fp32).  Pad entries written as 0. */
int kair_pack_weight(const float* src, void* dst, int dst_dtype, const kair_wmap* map, void* stream);
/* Batched packing: every weight re-pack of a step in one launch (one job per kair_pack_weight call). */
typedef struct kair_pack_job {
  const float* src;
  void* dst;
  int dst_dtype;
  int reserved;
  kair_wmap map;
  long total; /* filled by kair_pack_table_build */
} kair_pack_job;
/* bytes of device memory the job table needs */
long kair_pack_table_bytes(int njobs);
/* validate jobs, copy the table to device memory (synchronous); returns the launch's block count
 * (> 0) or a negative error code.  Call outside stream capture. */
long kair_pack_table_build(kair_pack_job* jobs, int njobs, void* table_dev);
int kair_pack_weights(const void* table_dev, int njobs, long nblocks, void* stream);
/* grad_ref (fp32 reference layout) = sum_s partial[s] (packed layout [Np][Kp]);
 * bias_grad (if non-NULL) = column ones_col of the sum.  accumulate: += instead of =. */
int kair_wgrad_finalize(const float* partial, int splits, const kair_wmap* map, float* grad_ref,
                        float* bias_grad, int ones_col, int accumulate, void* stream);
/* Grouped weight gradients (bf16): the linear layers of a group of Swin blocks in ONE TN launch +
 * ONE finalize launch.  Job i: grad_i (reference layout [N_ref][K_ref], via map_i, kind 0) =
 * sum_m A_i[m][n] * B_i[m][k] over n < N_i, k < K_i (the packed dims), bias_grad_i = column
 * ones_col_i of that sum (B_i holds 1.0 there: ones_in_data).  A: ROWS or QKVBLK (one q/k/v
 * geometry per group); B: ROWS.  Up to 24 jobs sharing M rows; ws: kair_wgrad_grouped_ws() floats.
 * Replaces the weight-gradient half of nn.Linear backward (network_swinir.py:19-20, 105, 107) for
 * every block of an RSTB at once; the sums are in fixed order (deterministic).
 * fp32x3 (round 6): jobs whose A and B are fp16 pairs (dtype KAIR_F16 + lo_ptr, x3_exp each; ROWS, no window map,
 * 16-byte aligned, N and K % 8) run on the split-fp16 TN ring (192 x 192 tiles, three fp16-pair products per
 * multiply, accumulator x 2^-(eA + eB)) -- one launch for all jobs, then the same grouped finalize. */
typedef struct {
  kair_operand A, B;
  int N, K;
  kair_wmap map;
  float* grad;
  float* bias_grad;
  int ones_col;
} kair_wgrad_job;
long kair_wgrad_grouped_ws(const kair_wgrad_job* jobs, int njobs, long M);
int kair_wgrad_grouped(const kair_wgrad_job* jobs, int njobs, long M, float* ws, void* stream);
/* As kair_wgrad_grouped with at most max_ctas workgroups (max_ctas == 0: no cap; fewer row splits,
 * never fewer tiles): the per-RSTB deferred weight gradients run on a side stream beside the next
 * RSTB's data-gradient chain, and a launch spread over every CU would hold the chain's kernels off the
 * chip until it ends.  The workspace of the uncapped form is always large enough.  max_ctas < 0:
 * -max_ctas times the default row splits instead (shorter workgroups; workspace -max_ctas times
 * kair_wgrad_grouped_ws()). */
int kair_wgrad_grouped_ex(const kair_wgrad_job* jobs, int njobs, long M, float* ws, int max_ctas, void* stream);
/* bias_grad[n_ref] (+)= sum_m G[m][n]  for an operand G of width Np (conv biases without a pad
 * column).  ws: 1024 * Np floats. */
int kair_colsum(const kair_operand* G, long M, int Np, const kair_wmap* map, float* bias_grad,
                float* ws, int accumulate, void* stream);

/* LayerNorm over the last dim (nn.LayerNorm eps 1e-5; network_swinir.py:199,205,520,725).
 * x fp32 [M, ldx] token order -> y (dtype) at rows rowmap^-1 (window order when win_ws > 0),
 * y pad columns [C, ldy) written 0.  mean/rstd fp32 [M] indexed by token row. */
int kair_layernorm_fwd(const float* x, long ldx, void* y, int y_dtype, long ldy, const float* gamma,
                       const float* beta, float* mean, float* rstd, long M, int C, float eps,
                       int win_H, int win_W, int win_ws, int win_shift, int one_col, void* stream);
/* kair_layernorm_fwd with an x3 fp16-pair output (the fp32x3 engine's GEMM operand, split once here instead of
 * in every consuming GEMM): y_hi = f16(y 2^x3_exp), y_lo = f16(y 2^x3_exp - y_hi); the ones column reads 2^x3_exp. */
int kair_layernorm_fwd_x3(const float* x, long ldx, void* y_hi, void* y_lo, long ldy, const float* gamma,
                          const float* beta, float* mean, float* rstd, long M, int C, float eps,
                          int win_H, int win_W, int win_ws, int win_shift, int one_col, int x3_exp, void* stream);
/* A row-scaled, cast copy of an fp32 token-row matrix (the next GEMM's A operand):
 * out[token_to_win(t)][c] = rowscale[t / rows_per_scale] * src[t][c]  (window order when win_ws > 0).
 * dtype KAIR_F16: an x3 fp16 pair -- out holds hi = f16(v 2^x3_exp), out_lo lo = f16(v 2^x3_exp - hi). */
typedef struct {
  void* out;
  int dtype;
  long ld;
  const float* rowscale; /* NULL => 1 */
  int rows_per_scale;
  int win_H, win_W, win_ws, win_shift;
  void* out_lo;          /* dtype KAIR_F16: the lo plane (same layout as out)                          */
  int x3_exp;            /* dtype KAIR_F16: the pair's power-of-2 exponent                              */
} kair_copy_desc;
int kair_row_copy(const float* src, long ld_src, long M, int C, const kair_copy_desc* copy, void* stream);

/* dx_acc[t] (+)= LN-backward(dy) for token rows t; dgamma/dbeta (+)= column sums.
 * dy (dtype) is addressed like y in the forward.  ws: 2 * 2048 * C floats.
 * copy (optional): also write the finished dx rows as a kair_copy_desc. */
int kair_layernorm_bwd(const float* x, long ldx, const void* dy, int dy_dtype, long ldy,
                       const float* gamma, const float* mean, const float* rstd, float* dx_acc,
                       long ld_dx, int dx_accumulate, float* dgamma, float* dbeta, int dparam_accumulate,
                       float* ws, long M, int C, int win_H, int win_W, int win_ws, int win_shift,
                       const kair_copy_desc* copy, void* stream);

/* Deferred LayerNorm parameter gradients: kair_layernorm_bwd with dgamma = dbeta = NULL leaves its
 * [kair_layernorm_bwd_blocks(M)][2C] partial sums in ws; one grouped launch then reduces several
 * LayerNorms' partials (fixed order, the same sums as the immediate form): up to 32 jobs. */
long kair_layernorm_bwd_blocks(long M);
typedef struct {
  const float* part; long nb; int C;
  float* dgamma; float* dbeta; int accumulate;
} kair_ln_param_job;
int kair_ln_param_reduce_grouped(const kair_ln_param_job* jobs, int njobs, void* stream);

/* Fused Swin window attention (network_swinir.py:114-145) for ws=8 (64 tokens), head_dim <= 32:
 *   O = softmax(q*scale @ k^T + table[relidx] + shift_mask) @ v   per (window, head).
 * qkv: head-blocked [3][nWin][nh][64][32] (dtype); table: fp32 [(2ws-1)^2][nh] (reference
 * layout); O written to rows [nWin*64, ldo] window order, head h at columns h*32..h*32+31;
 * lse fp32 [nWin][nh][64] (for backward).  Region mask is computed analytically for a
 * shift>0 block on an H x W token grid (calculate_mask, network_swinir.py:216-237).
 * mask (optional, shift must be 0): an explicit additive fp32 mask [mask_nw][64][64] indexed by
 * window % mask_nw -- WindowAttention.forward(x, mask) with a caller-built mask (:132-136). */
int kair_window_attn_fwd(const void* qkv, int dtype, const float* table, void* O, long ldo, float* lse,
                         long nWin, int nh, int hd, float scale, int H, int W, int shift, int ones_col,
                         const float* mask, int mask_nw, void* stream);
/* Backward: dO rows [nWin*64, lddo] (dtype, same layout as O); writes dqkv head-blocked (dtype);
 * dtable (+)= bias-table gradient (ws: partials*nh*225 floats, kair_window_attn_bwd_ws(): each wave bins
 * its (group, head) 64 x 64 bias gradient into the 225 relative positions before it leaves LDS). */
long kair_window_attn_bwd_ws(long nWin, int nh);
int kair_window_attn_bwd(const void* qkv, const void* O, long ldo, const void* dO, long lddo, int dtype,
                         const float* table, const float* lse, void* dqkv, float* dtable, int dtable_accumulate,
                         float* ws, long nWin, int nh, int hd, float scale, int H, int W, int shift,
                         const float* mask, int mask_nw, void* stream);
/* Same, dqkv_rows != 0 (bf16 only): dqkv written as token rows [nWin*64][3*nh*hp] in window order,
 * column (part*nh + h)*hp + d -- the plain A operand of the q/k/v input-gradient GEMM and of the q/k/v
 * weight gradient.  head_pad hp: 32 (the layouts above), or 16 (bf16, head_dim <= 16: every "32" of the
 * q/k/v, O, dO and dqkv layouts reads 16 -- SwinIR-lightweight's head dim 10, network_swinir.py:85). */
int kair_window_attn_bwd_ex(const void* qkv, const void* O, long ldo, const void* dO, long lddo, int dtype,
                            const float* table, const float* lse, void* dqkv, int dqkv_rows, float* dtable,
                            int dtable_accumulate, float* ws, long nWin, int nh, int hd, float scale, int H, int W,
                            int shift, const float* mask, int mask_nw, int head_pad, void* stream);
/* kair_window_attn_fwd with the head pad explicit (32, or 16 in bf16 as kair_window_attn_bwd_ex). */
int kair_window_attn_fwd_ex(const void* qkv, int dtype, const float* table, void* O, long ldo, float* lse,
                            long nWin, int nh, int hd, float scale, int H, int W, int shift, int ones_col,
                            const float* mask, int mask_nw, int head_pad, void* stream);

/* Split-fp16 ("x3", KAIR_COMPUTE_X3) window attention: the fp32 reference's arithmetic on the 16-bit
 * matrix cores.  Every tensor is an fp16 pair of planes holding x 2^e (hi = f16(x 2^e), lo = f16(x 2^e -
 * hi)) in the bf16 layouts above and every product hi.hi + hi.lo + lo.hi.  fwd: qkv / qkv_lo head-blocked
 * (exponent e_in), O / O_lo rows (written with e_out), lse fp32.  bwd: q/k/v and O carry e_act, dO carries
 * e_grad and dqkv / dqkv_lo are written with e_grad as token rows [nWin*64][3*nh*32] (window order,
 * column (part*nh + h)*32 + d); dtable (natural units) as kair_window_attn_bwd (NULL: partials left in ws
 * for kair_attn_dtable_grouped with dtype KAIR_COMPUTE_X3).  O_lo = NULL: O is fp32 rows in natural units
 * (16-byte aligned, ldo % 4 == 0; the ones column reads 1.0); dqkv_lo = NULL: dqkv is fp32 in natural units. */
int kair_window_attn_fwd_x3(const void* qkv, const void* qkv_lo, const float* table, void* O, void* O_lo, long ldo,
                            float* lse, long nWin, int nh, int hd, float scale, int H, int W, int shift, int ones_col,
                            int e_in, int e_out, void* stream);
int kair_window_attn_bwd_x3(const void* qkv, const void* qkv_lo, const void* O, const void* O_lo, long ldo,
                            const void* dO, const void* dO_lo, long lddo, const float* table, const float* lse,
                            void* dqkv, void* dqkv_lo, float* dtable, int dtable_accumulate, float* ws, long nWin,
                            int nh, int hd, float scale, int H, int W, int shift, int e_act, int e_grad, void* stream);

/* Deferred bias-table gradient: kair_window_attn_bwd with dtable = NULL leaves its per-group
 * partials (kair_window_attn_bwd_groups() planes of [nh][225]) in ws; one grouped launch then
 * reduces several blocks' partials into their dtable (+)= (network_swinir.py:94-98 gather, backward):
 * up to 32 jobs, deterministic. */
long kair_window_attn_bwd_groups(long nWin, int nh, int dtype);
typedef struct {
  const float* ws; long nWin; int nh; int dtype;
  float* dtable; int accumulate;
} kair_attn_dtable_job;
int kair_attn_dtable_grouped(const kair_attn_dtable_job* jobs, int njobs, void* stream);

/* Fused attention half of a Swin block (bf16; nh = 6 heads, C < 32*nh, window 8):
 *   out = x + rowscale * proj(W-MSA(LN1(x)))        network_swinir.py:239-272 + 114-145
 * in one launch (one workgroup per window, one wave per head).  x / out fp32 token rows; the LN1
 * output (window order, 1.0 at column C), mean / rstd, the head-blocked q/k/v, O (1.0 at
 * o_ones_col) and lse are stored exactly as kair_layernorm_fwd / kair_gemm_nt / kair_window_attn_fwd
 * would, for the unchanged backward.  wqkv: [3*nh*32][32*nh] (head-padded rows), wproj:
 * [32*nh][nh*32], both in MFMA-fragment order (pack kind 10, or kind 12 hi/lo pairs when
 * w_split); rowscale per sample (rows_per_scale = H*W) or NULL. */
int kair_swin_attn_fwd(const float* x, long ldx, const float* gamma, const float* beta, float eps, int C,
                       void* ln, long ldln, float* mean, float* rstd, const void* wqkv, const float* bqkv,
                       void* qkv, const float* table, float scale, void* O, long ldo, int o_ones_col,
                       float* lse, const void* wproj, const float* bproj, const float* rowscale,
                       int rows_per_scale, float* out, long ldout, long nWin, int nh, int H, int W, int shift,
                       int w_split, void* stream);
/* Fused MLP half of a Swin block (bf16; Cp = 192, hidden padded to Hp = 384):
 *   out = x + rowscale * fc2(GELU(fc1(LN2(x))))     network_swinir.py:274-276, Mlp.forward :24-30
 * in one launch over row tiles of token rows (M a multiple of 32).  Saved for the unchanged backward
 * as kair_layernorm_fwd / kair_gemm_nt (pre_kind 1) store them: ln (1.0 at column C), mean / rstd,
 * u = GELU'(x) of the fc1 pre-activation x and h = GELU(x) (1.0 at column hd), both [M][ldh].
 * w1 [Hp][Cp] in MFMA-fragment order (kind 10) and w2 [Cp][Hp] in 16x16x32 fragment order (kind 14);
 * w_split: both in kind 12 (hi/lo pairs, M a multiple of 64).  b1 [Hp], b2 [Cp] padded. */
int kair_swin_mlp_fwd(const float* x, long ldx, const float* gamma, const float* beta, float eps, int C,
                      void* ln, long ldln, float* mean, float* rstd, const void* w1, const float* b1, void* u,
                      void* h, long ldh, int hd, const void* w2, const float* b2, const float* rowscale,
                      int rows_per_scale, float* out, long ldout, long M, int Cp, int Hp, int w_split,
                      void* stream);

/* Fused MLP half backward (bf16; Cp = 192, hidden 384): with D = dL/dout (fp32 token rows) and
 * dc = rowscale_mlp * D (bf16 token rows),
 *   du  = (dc . W2) * gd            gd = GELU'(fc1 pre-activation) as the forward stored it
 *   D  += LN2-backward(du . W1)     (network_swinir.py:274-276 backward)  -> dL/dmid
 *   dco = rowscale * dL/dmid         bf16, rows in window order (H, W, shift): the proj operand
 *   dgamma / dbeta (+)= LN2 parameter gradients (dparam_acc)
 * in one launch + a small reduction.  w2t / w1t: fc2 / fc1 weights in transposed fragment order
 * (pack kind 13).  dco must not alias dc.  ws: kair_swin_mlp_bwd_ws() floats. */
long kair_swin_mlp_bwd_ws(void);
int kair_swin_mlp_bwd(const void* dc, long lddc, const void* gd, long ldg, const void* w2t, const void* w1t,
                      void* du, long lddu, const float* x, long ldx, const float* gamma, const float* mean,
                      const float* rstd, int C, float* D, long ldD, void* dco, long lddo, const float* rowscale,
                      int rows_per_scale, int H, int W, int shift, float* dgamma, float* dbeta, int dparam_acc,
                      float* ws, long M, int Cp, int Hp, void* stream);

/* 3x3 conv, stride 1, pad 1, with the weights streamed from global memory into registers (one wave
 * per SIMD, the input tile's halo in LDS; csrc/conv_wr.hip) -- replaces the RSTB conv and its input
 * gradient of the implicit GEMM (kair_gemm_nt over KAIR_LD_IM2COL3, network_swinir.py:263-279 RSTB.conv).
 * x: NHWC rows [B*H*W][ldx], fp32 or bf16.  split = 1 (fp32 x): split activations -- the kernel forms
 * lo = bf16(x - bf16(x)) and multiplies hi.W_hi + hi.W_lo + lo.W_hi (w = pack kind 15, Np = 192);
 * split = 0: one bf16 product (w = pack kind 16, the dgrad form, with flip = 1 for an input gradient).  n_blocks = Np/16
 * (12).  out[m][n] = conv + bias[n] (+ resid[m][n]), fp32 or bf16 rows, n < N.  acopy (optional): the
 * bf16 copy of the image rows (hi half) with 1.0 at column acones (bias gradient), as kair_epilogue
 * a_copy.  C a multiple of 64, <= 192; N <= 192, N % 4 == 0; tiles of 96 (split) or 144 pixels: whole
 * rows of W <= tile or tile-sized pieces of wider rows (kair_conv3x3_wr_tile: 0 = unsupported). */
int kair_conv3x3_wr_tile(int split, int B, int H, int W, int C, int N);
int kair_conv3x3_wr(const void* x, int x_dtype, long ldx, int split, int flip, const void* w, int n_blocks,
                    const float* bias, const float* resid, long ldr, void* out, int out_dtype, long ldo, void* acopy,
                    long ldac, int acones, int B, int H, int W, int C, int N, void* stream);
/* kair_conv3x3_wr with two more forms: a bf16 [hi | lo] pair image (split = 1, x_dtype KAIR_BF16: rows of
 * 2 C channels, C per half; the SwinIR x4 upsampling convs, N in (192, 256], pack kind 15 with Np = 256,
 * n_blocks 16) and a PixelShuffle(ps_r) sub-pixel-major store (packed column n = (i r + j) N/r^2 + c ->
 * pixel (y r + i, x r + j), channel c; ldo = the shuffled rows' stride) with, for a bf16 output, the lo
 * plane bf16(v - bf16(v)) at the same offsets from out_lo (a pair output for the next split conv).  N <= 64
 * (n_blocks 4, split, row output: conv_before_upsample) with act KAIR_ACT_LEAKY(slope) and out_lo.  The
 * upsampling convs' input gradients: plain bf16 image of C <= 256 channels, N <= 64, with ps_r < 0 a
 * PixelUnshuffle(-ps_r) store into the previous conv's pre-shuffle rows (KAIR_OUT_PUNSHUF_SPM layout) or a
 * LeakyReLU' gate (gate bf16 rows, ldg; v *= gate > 0 ? 1 : slope). */
int kair_conv3x3_wr_ex(const void* x, int x_dtype, long ldx, int split, int flip, const void* w, int n_blocks,
                       const float* bias, const float* resid, long ldr, void* out, int out_dtype, long ldo, void* out_lo,
                       int ps_r, int act, float slope, const void* gate, long ldg, void* acopy, long ldac, int acones,
                       int B, int H, int W, int C, int N, void* stream);

/* Narrow-output 3x3 convs (csrc/tail.hip): a 64-channel NHWC bf16 image <-> NR <= 4 output channels,
 * the last conv of the reconstruction head (network_swinir.py:745, :817 conv_last).
 * fwd:   out NCHW [B][NR][H][W] = conv(x) + bias, / img_range + mean (mean may be NULL; resid, optional,
 *        an NCHW image added last).  x rows [B*H*W][ldx]: channels [0, 64) = hi, and with lo_off > 0 the
 *        lo halves at [lo_off, lo_off + 64) (split activations); w = pack kind 15 of the conv weight
 *        (hi/lo split, Np = 16).  W % 64 == 0 for all three (64-pixel row segments).
 * dgrad: dX = conv^T(dE): dE rows [B*H*W][lde] bf16 (channels [0, NR)), w the fp32 reference weight
 *        [NR][64][3][3] (re-laid into ws, kair_conv3x3_narrow_dgrad_ws() floats, by the same call); out rows [B*H*W][ldo] (ps_r <= 1) or, with ps_r = r, the PixelUnshuffle(r)
 *        sub-pixel-major layout of the previous conv's pre-shuffle rows (KAIR_OUT_PUNSHUF_SPM).
 * wgrad: grad_w [NR][64][3][3] (and grad_b [NR] if non-NULL) = / += (accumulate) sum over pixels, from
 *        per-workgroup partials in ws (kair_conv3x3_narrow_wgrad_ws(NR) floats) summed in fixed order. */
int kair_conv3x3_narrow_fwd(const void* x, long ldx, int lo_off, const void* w, const float* bias, int NR,
                            const float* mean, float img_range, const float* resid, float* out, int B, int H, int W,
                            void* stream);
long kair_conv3x3_narrow_dgrad_ws(void);
int kair_conv3x3_narrow_dgrad(const void* dE, long lde, const float* w, int NR, void* ws, void* out, int out_dtype,
                              long ldo, int ps_r, int B, int H, int W, void* stream);
long kair_conv3x3_narrow_wgrad_ws(int NR);
int kair_conv3x3_narrow_wgrad(const void* dE, long lde, const void* x, long ldx, int NR, float* ws, float* grad_w,
                              float* grad_b, int accumulate, int B, int H, int W, void* stream);

/* fp32x3 forms of the three narrow convs (the fp32 engine's arithmetic, KAIR_COMPUTE_X3): fp32 operands, each
 * staged into LDS as the fp16 pair of v 2^e and multiplied hi.hi + lo.hi + hi.lo (fp32 accumulation).  x: fp32
 * rows [B*H*W][ldx], channels [0, 64), exponent ex; dE: fp32 rows [B*H*W][lde] (channels [0, 4) read, the
 * weights zero for n >= NR), exponent eg; w: the fp32 conv weight [NR][64][3][3] (split as w 2^KAIR_X3_WEXP
 * into ws, kair_conv3x3_narrow_x3_ws() floats, by the fwd / dgrad call itself; one ws per concurrent call).
 * Outputs as the bf16 forms: fwd the NCHW image, dgrad fp32 rows or the PixelUnshuffle(ps_r) sub-pixel-major
 * layout, wgrad grad_w / grad_b from per-workgroup partials in ws (kair_conv3x3_narrow_wgrad_ws(NR) floats). */
long kair_conv3x3_narrow_x3_ws(void);
int kair_conv3x3_narrow_fwd_x3(const float* x, long ldx, int ex, const float* w, const float* bias, int NR, void* ws,
                               const float* mean, float img_range, const float* resid, float* out, int B, int H, int W,
                               void* stream);
int kair_conv3x3_narrow_dgrad_x3(const float* dE, long lde, int eg, const float* w, int NR, void* ws, float* out, long ldo,
                                 int ps_r, int B, int H, int W, void* stream);
int kair_conv3x3_narrow_wgrad_x3(const float* dE, long lde, int eg, const float* x, long ldx, int ex, int NR, float* ws,
                                 float* grad_w, float* grad_b, int accumulate, int B, int H, int W, void* stream);

/* Elementwise / small kernels ------------------------------------------------------------- */
/* NCHW fp32 image -> NHWC (dtype) with channel stride ldc, x' = (x - mean[c]) * img_range
 * (network_swinir.py:809-810); mean may be NULL.  Pad channels written 0. */
int kair_image_to_nhwc(const float* img, void* out, int dtype, int ldc, const float* mean, float img_range,
                       int B, int C, int H, int W, void* stream);
/* The same as a hi/lo bf16 pair (conv_first of the split-operand engine): channel c < C holds
 * hi = bf16(x'), channel ldc/2 + c holds bf16(x' - hi); pad channels 0.  Needs 2*C <= ldc, ldc even.
 * The conv reading it packs its weights tied over both halves (kair_wmap kG*kGr = 2K, kinds 1 / 9). */
int kair_image_to_nhwc_hilo(const float* img, void* out, int ldc, const float* mean, float img_range,
                            int B, int C, int H, int W, void* stream);
/* L1 loss (nn.L1Loss, mean): loss_out[0] = weight*mean|E-H|; grad dE = weight*sign(E-H)/numel written
 * for the last conv's dgrad: NHWC (dtype, channel stride ldc) when ps_r == 1, or in the
 * pre-PixelShuffle(ps_r) layout [b][y/r][x/r][c*r*r + (y%r)*r + x%r] otherwise.  ws: 1024 floats. */
int kair_l1_loss(const float* E, const float* H, float* loss_out, void* dE, int dtype, int ldc, int ps_r, float weight,
                 int B, int C, int Hh, int Ww, float* ws, void* stream);
/* Charbonnier loss (models/loss.py:208-218, model_plain.py:191-192; SwinIR denoising / JPEG options):
 * loss_out[0] = weight*mean(sqrt((E-H)^2 + eps)); dE = weight*(E-H)/sqrt((E-H)^2 + eps)/numel, laid out as
 * kair_l1_loss. */
int kair_charbonnier_loss(const float* E, const float* H, float* loss_out, void* dE, int dtype, int ldc, int ps_r,
                          float weight, float eps, int B, int C, int Hh, int Ww, float* ws, void* stream);
/* y[i] += a * x[i] over n fp32 elements (residual-gradient merges). */
int kair_axpy(float* y, const float* x, float a, long n, void* stream);
/* BatchNorm2d over NHWC rows z [M, C] fp32 (basicblock.py:69: momentum 0.9, eps 1e-4), fused act
 * (0 none, 1 ReLU, 2 LeakyReLU(slope)).  training: batch statistics (two-pass, deterministic) ->
 * mean/rstd [C] and the running-stat update (unbiased running_var); else running statistics.
 * ws: kair_bn_ws(C) floats.  (network_dncnn.py:40-71 BN layers) */
long kair_bn_ws(int C);
int kair_bn_fwd(const float* z, long ldz, void* out, int out_dtype, long ldo, long M, int C, const float* gamma,
                const float* beta, float* running_mean, float* running_var, float momentum, float eps, int training,
                float* mean, float* rstd, int act, float slope, float* ws, void* stream);
/* dz = BN'(act'(a) * da) with the saved mean/rstd; dgamma/dbeta (+)= column sums. */
int kair_bn_bwd(const float* z, long ldz, const void* a, int a_dtype, long lda, const float* da, long ldda, void* dz,
                int dz_dtype, long lddz, long M, int C, const float* gamma, const float* mean, const float* rstd,
                int act, float slope, float* dgamma, float* dbeta, int accumulate, float* ws, void* stream);

/* y = a * x + b * y (fp32, n elements) */
int kair_axpby(float* y, const float* x, float a, float b, long n, void* stream);
/* y[m][c] = a * x[m][c] + b * y[m][c] for c < C over strided fp32 rows */
int kair_axpby_rows(float* y, long ldy, const float* x, long ldx, long M, int C, float a, float b, void* stream);
/* out[m][c] (dtype) = G[m][c] * act'(X[m][c]) for c < C  (act' from the POST-activation value X:
 * kind 1 ReLU, 2 LeakyReLU(slope); 0 identity; kind 3: exact-erf GELU' of the PRE-activation X),
 * optionally * scale.  Row strides ldg / ldx / ldo. */
int kair_act_grad_cast(const float* G, long ldg, const void* X, int x_dtype, long ldx, void* out, int out_dtype,
                       long ldo, long M, int C, int kind, float slope, float scale, void* stream);
/* 2x2 sum-pool (adjoint of nearest x2 upsample): dst[b][y][x][c] (+)= sum_{i,j<2} src[b][2y+i][2x+j][c].
 * src fp32 [B, 2H, 2W] rows of stride lds; dst fp32 [B, H, W] rows of stride ldd. */
int kair_sumpool2x(const float* src, long lds, float* dst, long ldd, int B, int H, int W, int C, int accumulate,
                   void* stream);
/* Fused Adam (torch.optim.Adam maths, model_plain.py:210-222,302) + EMA (model_base.py:247-252)
 * over flat fp32 buffers.  lr_t is a DEVICE array {lr / (1 - beta1^t), sqrt(1 - beta2^t)} written by
 * the host before each (graph-replayed) step; ema may be NULL (E_decay = 0). */
int kair_adam_ema(float* p, const float* g, float* m, float* v, float* ema, long n, const float* lr_t,
                  float beta1, float beta2, float eps, float weight_decay, float ema_decay, void* stream);
/* kair_adam_ema with a device skip flag (NULL: never): *skip != 0 drops the step -- parameters, moments and
 * EMA untouched -- the way torch.cuda.amp.GradScaler.step skips an inf/NaN step.  The fp32x3 range guard. */
int kair_adam_ema_ex(float* p, const float* g, float* m, float* v, float* ema, long n, const float* lr_t,
                     float beta1, float beta2, float eps, float weight_decay, float ema_decay, const unsigned* skip,
                     void* stream);
/* fp32x3 range guard: *flag = (any non-finite g: 1) | (non-finite *loss: 2) | (any |p| >= p_limit or
 * non-finite p: 4), over the flat gradient / parameter buffers of n floats (loss may be NULL).  A split-fp16
 * operand that leaves fp16's range turns into inf/NaN in every product it enters, so the step's gradients
 * show it; p_limit = 2^(16 - KAIR_X3_WEXP) bounds the weights' fp16 window.  (No reference counterpart: the
 * fp32 reference has no operand window.) */
int kair_range_check(const float* g, const float* p, long n, const float* loss, float p_limit, unsigned* flag,
                     void* stream);
/* fp32x3: the input-gradient GEMM of a Swin linear fused with the LayerNorm backward in front of it (network_swinir.py
 * :199 / :205 norm1 / norm2 -> qkv / fc1; replaces kair_gemm_nt into a dxn buffer + kair_layernorm_bwd, same math):
 *   dxn = A B^T (A: fp16-pair gradient rows, B: the split-packed weight, N = 192 >= C: one tile holds whole rows),
 *   row r of the GEMM (window order when win_ws > 0) is token t;
 *   D[t] += rstd (g - mean_c(g) - xh mean_c(g xh)),  g = dxn gamma,  xh = (x[t] - mean[t]) rstd[t]   (c < C);
 *   copy (optional, fp16 pair): the finished D row as in kair_layernorm_bwd;
 *   part: [kair_gemm_nt_x3_lnbwd_parts(M, N)][2 C] dgamma / dbeta partial rows (one per 16 GEMM rows) for
 *   kair_ln_param_reduce_grouped. */
long kair_gemm_nt_x3_lnbwd_parts(long M, int N);
int kair_gemm_nt_x3_lnbwd(const kair_operand* A, const kair_operand* B, long M, int N, int K, int win_H, int win_W,
                          int win_ws, int win_shift, const float* x, long ldx, const float* gamma, const float* mean,
                          const float* rstd, int C, float* D, long ldd, float* part, const kair_copy_desc* copy,
                          void* stream);

/* Measurement (bench.py's in-step kernel table; no reference counterpart): open a kernel timing window of n slots.
 * Until kair_ktime_end, each libkair launch into a non-capturing stream takes the next slot and is dispatched with
 * hipExtLaunchKernel and the slot's event pair, which the runtime stamps with the dispatch packet's start / end (the
 * kernel duration rocprofv3 --kernel-trace reports).  kair_ktime_count: slots taken (by the last window once closed);
 * kair_ktime_read(i): slot i's duration in ms (waits for it) and the kernel's symbol name.  Host state of the
 * calling thread. */
int kair_ktime_begin(int n);
int kair_ktime_count(void);
int kair_ktime_end(void);
int kair_ktime_read(int i, float* ms, const char** name);

/* Measurement: kair_gate_hold queues one wave on the stream that waits until kair_gate_release (or timeout_ms), so
 * an eager pass queued behind it runs back to back; kair_gate_status: 0 pending, 1 released, 2 timed out. */
int kair_gate_hold(int timeout_ms, void* stream);
int kair_gate_release(void);
int kair_gate_status(void);

/* USRNet (network_usrnet_v1.py) -------------------------------------------------------------
 * Complex plane sets are float2 [planes][W][H] (TRANSPOSED: column-major per plane).            */
#define KAIR_USR_SRC_NCHW 0  /* fp32 NCHW planes [planes][H][W]                                    */
#define KAIR_USR_SRC_PSF 1   /* p2o of a PSF [B][1][kh][kw]: zero-pad + circular shift (v1:48-69)  */
#define KAIR_USR_SRC_ZUP 2   /* s-fold zero-upsample of LQ planes [planes][H/sf][W/sf] (v1:72-82)   */
#define KAIR_USR_SRC_NHWC 3  /* channel plane%C of fp32 NHWC rows [B][H][W][ld]                     */
#define KAIR_USR_COL_FB 0        /* T <- FB (in place), invW[b][g][u'] = alias-mean |FB|^2           */
#define KAIR_USR_COL_FBFY 1      /* T <- conj(FB) * F(T)                                             */
#define KAIR_USR_COL_DATA_FWD 2  /* DataNet.forward (v1:183-194); FR saved when non-null            */
#define KAIR_USR_COL_DATA_BWD 3  /* DataNet backward: T <- dL/dx spectrum, part <- partial dL/dalpha */
#define KAIR_USR_CHAN_CHUNKS 64
/* forward DFT along W of every row, written transposed (replaces torch.fft.fftn's first axis,
 * v1:66/185/251 and the p2o / upsample inputs) */
int kair_usr_fft_rows(const float* src, int src_mode, int C, long ld, int kh, int kw, int sf, void* T,
                      int planes, int H, int W, void* stream);
/* DFT along H of sf alias column lines per CTA + the closed form of `mode`, then (data modes) the
 * inverse DFT along H.  alpha[b * alpha_stride]; part: [planes][W/sf] (bwd). */
int kair_usr_fft_cols(int mode, const void* T, void* T_out, const void* FB, const void* FBFy, void* FR,
                      float* invW, const float* alpha, int alpha_stride, float* part, int planes, int C,
                      int H, int W, int sf, void* stream);
/* inverse DFT along W, real part * scale: NCHW fp32 planes (nhwc 0) or channel plane%C of NHWC
 * rows [B][H][W][ld] of dst_dtype (nhwc 1)  (torch.real(torch.fft.ifftn(..)), v1:192) */
int kair_usr_ifft_rows(const void* T, void* dst, int nhwc, int dst_dtype, int C, long ld, float scale,
                       int planes, int H, int W, void* stream);
/* out[s*ostride] (+)= scale * sum_j ws[s*seglen + j]  (fixed order) */
int kair_usr_seg_sum(const float* ws, int seglen, int nseg, float scale, float* out, int ostride,
                     int accumulate, void* stream);
/* out[b*ostride] (+)= sum_p x[(b*HW + p)*ld + c]  (ws: B * KAIR_USR_CHAN_CHUNKS floats) */
int kair_usr_chan_sum(const float* x, long ld, int c, long HW, int B, float* ws, float* out, int ostride,
                      int accumulate, void* stream);
/* ResUNet's ReplicationPad2d((0, Wp-W, 0, Hp-H)) and crop x[..., :H, :W] (network_usrnet_v1.py:148-151,
 * 164) with their adjoints.  nb: images (NHWC modes, channel stride ldc) or planes (CROP_NCHW).
 * REPLICATE / ZERO: H x W -> Hp x Wp (fp32 or bf16); FOLD (replicate adjoint, pad pixels summed onto
 * the edge they copy): Hp x Wp -> H x W; CROP_NCHW: Hp x Wp planes -> H x W (fp32). */
enum { KAIR_USR_PAD_REPLICATE = 0, KAIR_USR_PAD_ZERO = 1, KAIR_USR_PAD_FOLD = 2, KAIR_USR_CROP_NCHW = 3 };
int kair_usr_pad(const void* src, void* dst, int dtype, int mode, int ldc, int nb, int H, int W, int Hp, int Wp,
                 void* stream);
/* F.interpolate(x, scale_factor=sf, mode='nearest') of fp32 NCHW planes (v1:252) */
int kair_usr_upsample_nearest(const float* L, float* out, int planes, int h, int w, int sf, void* stream);
/* ResUNet input torch.cat((x, beta), 1) (v1:261) as NHWC rows of width ld: x channels, beta[b*bstride], 0 */
int kair_usr_pack_input(const float* x, const float* beta, int beta_stride, void* out, int dtype, int ld,
                        int B, int C, long HW, void* stream);
/* HyPaNet (v1:204-216) on [sigma, sf]: ab [B][no] = softplus(MLP) + 1e-6; one block (B*(4hc+2no)*4 <= 64 KiB) */
int kair_hypanet_fwd(const float* sigma, float sf, const float* W1, const float* b1, const float* W2,
                     const float* b2, const float* W3, const float* b3, int hc, int no, int B, float* ab,
                     void* stream);
int kair_hypanet_bwd(const float* sigma, float sf, const float* W1, const float* b1, const float* W2,
                     const float* b2, const float* W3, const float* b3, int hc, int no, int B, const float* gab,
                     float* gW1, float* gb1, float* gW2, float* gb2, float* gW3, float* gb3, int accumulate,
                     void* stream);

/* ---- Swin-block input gradients as row GEMMs with fused consumers (bf16, rowgemm.hip) --------
 * Y[m, :] = A[m, :K] . W^T for the input gradient of one block linear (nn.Linear backward,
 * network_swinir.py:19-20 fc1 / fc2, :105 qkv, :107 proj).  A: bf16 rows [M][lda] (K = 192, 384 or
 * 576 columns, 16-byte aligned); W: the linear's weight in transposed MFMA-fragment order (pack
 * kind 13: [N/32][K/16][64][8], the dgrad output dimension N = 192 or 384 first).
 *   kair_rowgemm_store: out[m][n] = bf16(Y)                       (proj input gradient -> dO)
 *   kair_rowgemm_gate:  out[m][n] = bf16(Y * gate[m][n])           (fc2 input gradient through the
 *                                                                   stored GELU'(fc1 pre-activation))
 *   kair_rowgemm_lnbwd: N = 192; Y = dL/d(LayerNorm output) of rows in the window order `win`
 *     (nn.LayerNorm backward, network_swinir.py:199 norm1 / :205 norm2): D[t] += LN-backward(Y)
 *     for token t = win_to_token(m) (x, mean, rstd, D token rows; x and D share the row stride),
 *     the finished row also written as `copy` (bf16, optional), and the dgamma / dbeta partials
 *     [kair_rowgemm_ln_blocks(M, K)][2][C] left in `part` for kair_ln_param_reduce_grouped.
 *   Replaces kair_gemm_nt / hipBLASLt + kair_layernorm_bwd for these products: Y stays fp32 in
 *   registers (the unfused path rounded it to bf16 and round-tripped it through HBM). */
int kair_rowgemm_store(const void* A, long lda, long M, int K, const void* W, int N, void* out, long ldo,
                       void* stream);
int kair_rowgemm_gate(const void* A, long lda, long M, int K, const void* W, int N, const void* gate, long ldg,
                      void* out, long ldo, void* stream);
long kair_rowgemm_ln_blocks(long M, int K);
int kair_rowgemm_lnbwd(const void* A, long lda, long M, int K, const void* W, const float* x, long ldx,
                       const float* gamma, const float* mean, const float* rstd, int C, float* D, long ldD,
                       int win_H, int win_W, int win_ws, int win_shift, const kair_copy_desc* copy, float* part,
                       void* stream);

/* ---- training-patch synthesis ------------------------------------------
 * pool: fp32 NCHW image pool [N][C][Hs][Ws] in [0, 1] (HBM-resident); params: int4 per sample
 * {image, rnd_h, rnd_w, mode} (rnd_* in L coordinates for SR, H coordinates for denoising; mode the
 * utils_image.augment_img mode 0..7).  Outputs fp32 NCHW [B][C][PS][PS] (H) and L.
 * kair_synth_sr replaces DatasetSR.__getitem__ (data/dataset_sr.py:35-92): L = MATLAB bicubic x1/sf
 * of the whole image (utils_image.imresize, utils_image.py:938-1005; separable taps wh/ih [Hs/sf][P],
 * ww/iw [Ws/sf][P] from calculate_weights_indices :880-932, source indices already reflected),
 * cropped at (rnd_h, rnd_w) and augmented; H the aligned sf x larger crop.
 * kair_synth_dn replaces DatasetDnCNN.__getitem__ train branch (data/dataset_dncnn.py:50-75):
 * L = H + sigma * N(0,1) (sigma = sigma_255 / 255), Philox-4x32-10 normals keyed by (seed, step). */
int kair_synth_sr(const float* pool, int C, int Hs, int Ws, const int* params, int B, int PS, int sf,
                  const float* wh, const int* ih, const float* ww, const int* iw, int P, float* outH,
                  float* outL, void* stream);
int kair_synth_dn(const float* pool, int C, int Hs, int Ws, const int* params, int B, int PS, float sigma,
                  unsigned long long seed, unsigned long long step, float* outH, float* outL, void* stream);

const char* kair_last_error(void);
int kair_device_arch(char* buf, int len);

/* Perf investigation only: per-wave phase stamps of the last bf16 attention backward launched with
 * KAIR_ATTN_STAMP=1 in the environment (s_memtime cycles, 8 per wave: 7 phase boundaries of the
 * wave's third window + its window count).  n = number of u64 values to copy. */
int kair_debug_attn_stamps(unsigned long long* host, int n);
/* Perf investigation only: per-wave phase stamps (8 s_memtime values) of the fused attention half's last
 * window per workgroup (cleared by the read), from a library built with --debug-ablations and KAIR_ATTN_DBG bit 8 set. */
int kair_debug_fused_stamps(unsigned long long* host, int n);
/* Perf investigation only: phase stamps of the last x3 NT ring launch (CTAs 0-3, 8 waves, iterations 0-63, 5
 * s_memtime values each; cleared by the read), from a --debug-ablations library with KAIR_RING_DBG bit 8 set. */
int kair_debug_x3_stamps(unsigned long long* host, int n);

#ifdef __cplusplus
}
#endif
#endif
