/*
 * avsr_hip.h — C-ABI of libavsr_hip.so, the MI355X (gfx950) kernel library behind the
 * AV-HuBERT AVSR forward/backward hot path.
 *
 * Boundary contract:
 *   - every entry point is `extern "C"`, takes plain device pointers + sizes (in a POD
 *     params struct) and a hipStream_t passed as `void*`; returns 0 on success or a
 *     hipError_t / AVSR_E_* code.
 *   - the caller owns every buffer (the PyTorch caching allocator in the Python host);
 *     kernels never allocate, free or synchronise the host, so every launch is
 *     graph-capturable.
 *   - dtype tag: AVSR_F32 = fp32 storage ("parity mode": operands are split into
 *     bf16 hi+lo and fed to the same bf16 MFMA tiles, 3 products per step),
 *     AVSR_BF16 = bf16 storage (throughput mode). Accumulation is always fp32.
 *
 * Each entry point names the reference operation it replaces (file:line in
 * quanpn90/avsr @ 2025-08-29 unless prefixed HF: = transformers 4.52.4
 * models/wav2vec2/modeling_wav2vec2.py, or ATen: = torch 2.7.1 operator).
 */
#ifndef AVSR_HIP_H
#define AVSR_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { AVSR_F32 = 0, AVSR_BF16 = 1 };
enum { AVSR_ACT_NONE = 0, AVSR_ACT_GELU = 1, AVSR_ACT_RELU = 2 };
enum { AVSR_E_SHAPE = 1001, AVSR_E_ALIGN = 1002, AVSR_E_DTYPE = 1003, AVSR_E_ARG = 1004 };

/* library identity: returns a static string ("avsr_hip <version> gfx950") */
const char* avsr_version(void);

/* ------------------------------------------------------------------------------------
 * Process-wide kernel-selection options. These are the only switches that change which
 * kernel an entry point launches; the library reads no environment variables. Every option
 * defaults to the measured production choice (value in brackets); the others exist for A/B
 * measurements (tools/) and the tests that pin each variant. Set them between launches, not
 * while another host thread is enqueueing work. Results of the variants are identical
 * unless an option says otherwise.
 *   AVSR_OPT_GEMM_TILE      [0]  0: automatic tile choice (gemm.hip tile_cfg); k + 1 forces
 *                                 tile configuration k (AVSR_TILE_* below) on the bf16 core
 *   AVSR_OPT_ATTN_SQ_FWD    [1]  1: query-tiled streamed self-attention forward for bf16,
 *                                 L >= 128; 0: the resident-K/V kernel (same rows to 1e-2)
 *   AVSR_OPT_ATTN_SQ_BWD    [0]  retired: accepts 0 only (the small-footprint dQ kernel it
 *                                 selected measured 0.4 % slower in the step and was removed)
 *   AVSR_OPT_WGRAD_DUAL     [1]  1: two-wave-group weight-gradient kernel (fp32 C, both
 *                                 operands r-contiguous); 0: the 4-wave core
 *   AVSR_OPT_CONV_192       [1]  1: 192x128 tiles for conv fwd / data-grad where they still
 *                                 run >= 2 blocks per CU; 0: 128x128 (bit-identical)
 *   AVSR_OPT_CONV_S2PHASE   [1]  1: stride-2 data-grads as four parity-class GEMMs; 0: one
 *                                 col2im GEMM over all taps (bit-identical)
 *   AVSR_OPT_CONV_PATCH     [1]  1: patch-resident 3x3 kernel for 64-channel stride-1 fwd /
 *                                 data-grad; 0: the general implicit GEMM (bit-identical)
 *   AVSR_OPT_CONV_WPATCH    [1]  1: patch-resident weight-grad (stage 1 / 2 geometries); 0:
 *                                 the general split-K weight-grad (fp32 re-association)
 *   AVSR_OPT_STEM_POOL_2X2  [1]  1: stem max-pool forward / backward apply over 2x2 output
 *                                 blocks; 0: one output pixel per thread (bit-identical)
 *   AVSR_OPT_STEM_WPATCH    [1]  1: patch-resident stem weight-grad (packed 8-channel input,
 *                                 7x7 / stride 2); 0: the general split-K weight-grad (fp32
 *                                 re-association)
 * avsr_set_option returns 0, or AVSR_E_ARG for an unknown option or a value out of range;
 * avsr_get_option returns the value, or -1 for an unknown option.
 * ------------------------------------------------------------------------------------ */
enum {
  AVSR_OPT_GEMM_TILE = 0,
  AVSR_OPT_ATTN_SQ_FWD = 1,
  AVSR_OPT_ATTN_SQ_BWD = 2,
  AVSR_OPT_WGRAD_DUAL = 3,
  AVSR_OPT_CONV_192 = 4,
  AVSR_OPT_CONV_S2PHASE = 5,
  AVSR_OPT_CONV_PATCH = 6,
  AVSR_OPT_CONV_WPATCH = 7,
  AVSR_OPT_STEM_POOL_2X2 = 8,
  AVSR_OPT_STEM_WPATCH = 9,
  AVSR_OPT_COUNT = 10
};
/* tile configurations of the bf16 GEMM core (AVSR_OPT_GEMM_TILE = k + 1) */
enum {
  AVSR_TILE_128 = 0, AVSR_TILE_256 = 1, AVSR_TILE_256x128 = 2, AVSR_TILE_128x256 = 3, AVSR_TILE_128s3 = 4,
  AVSR_TILE_128s4 = 5, AVSR_TILE_128w8s3 = 6, AVSR_TILE_128w8s4 = 7, AVSR_TILE_PP = 8, AVSR_TILE_96 = 9,
  AVSR_TILE_128x64 = 10, AVSR_TILE_192 = 11, AVSR_TILE_192x256 = 12, AVSR_TILE_192s3 = 13, AVSR_TILE_192w8 = 14,
  AVSR_TILE_192w8s3 = 15, AVSR_TILE_64 = 16, AVSR_TILE_192w8s4 = 17, AVSR_TILE_64s4 = 18, AVSR_TILE_COUNT = 19
};
int avsr_set_option(int option, int64_t value);
int64_t avsr_get_option(int option);

/* ------------------------------------------------------------------------------------
 * GEMM with fused epilogue, fp32 accumulate: v_mfma_f32_16x16x32_bf16 on the LDS-DMA core
 * (128x128 / 192x128 tiles, bf16), v_mfma_f32_32x32x16_bf16 on the register-staged core
 * (fp32 parity mode: bf16 hi/lo split; shapes under 128 rows / columns).
 *   C[b][m][n] = epi( alpha * sum_k A(b,m,k) * B(b,n,k) )
 *   A(m,k) = A[m*lda + k] if a_kmajor else A[k*lda + m]
 *   B(n,k) = B[n*ldb + k] if b_kmajor else B[k*ldb + n]
 * Forward epilogue (epi_bwd = 0):  h = alpha*acc + bias[n];  if (preact) preact[m][n] = h;
 *   y = act(h); y = dropout(y; drop_p, seed); y += res[m][n]; C = y (+ beta*C_old)
 * Backward epilogue (epi_bwd = 1): g = alpha*acc; g = dropout_mask(g; drop_p, seed);
 *   g *= act'(gate[m][n]); C = g (+ beta*C_old)
 * Replaces: torch.nn.Linear (ATen addmm) everywhere on the path — encoder q/k/v/out
 *   (HF:Wav2Vec2Attention), FFN (HF:Wav2Vec2FeedForward :551-572), post_extract_proj
 *   (src/nets/backend/backbones/avhubert.py:259-263), SubModel.proj (:187-198),
 *   ctc_lo (src/nets/backend/ctc.py:25), decoder linears
 *   (src/nets/backend/transformer/attention.py:31-34, positionwise_feed_forward.py:25-30,
 *   decoder.py:117) — forward, input-grad and weight-grad.
 * Requirements: lda/ldb/ldc and the contiguous extent multiples of 8 elements, pointers
 *   16-byte aligned (AVSR_E_ALIGN otherwise).
 * ------------------------------------------------------------------------------------ */
typedef struct {
  int M, N, K, batch;
  int dtype;                 /* AVSR_F32 / AVSR_BF16: storage of A, B, res, preact, gate */
  int a_kmajor, b_kmajor;
  int c_f32;                 /* 1: C is fp32 regardless of dtype (weight grads) */
  const void* A; int64_t lda, strideA;
  const void* B; int64_t ldb, strideB;
  void* C;       int64_t ldc, strideC;
  float alpha, beta;
  const float* bias;         /* [N] fp32 or NULL (forward only) */
  int act;                   /* AVSR_ACT_* */
  int epi_bwd;               /* 0 forward epilogue, 1 backward (gate) epilogue */
  void* preact;              /* forward: store pre-activation h (dtype, ld = ldc) or NULL */
  const void* res;  int64_t ldr, strideR;   /* residual (dtype) or NULL */
  const void* gate;          /* backward: pre-activation h (dtype, ld = ldc) or NULL */
  float drop_p;              /* dropout probability (0 = off) */
  uint64_t seed;             /* counter-based dropout stream id */
  int splitk;                /* >1: K split over blocks (C must be fp32) */
  float* ws;                 /* split-K slab workspace, AVSR_GEMM_SLAB_WS(batch, splitk, M, N) fp32:
                                each split stores its partial tile, a reduce pass writes
                                C = alpha*sum + beta*C (plain epilogue only). NULL: C += alpha*acc
                                by fp32 atomics. Ignored when splitk <= 1. */
  float* db;                 /* optional: db[n] += sum_m C[m][n] of the stored tile values (the
                                bias gradient of the layer whose output gradient C is, e.g.
                                FFN1's bias from the FFN2 data-grad); bf16, N % 8 == 0, no split */
  float* db_ws;              /* its row-tile partials, AVSR_GEMM_COLSUM_WS(M, N) fp32 */
  unsigned long long* stamp; /* optional diagnostic (bench.py roofline probe; bf16 LDS-DMA path):
                                {min start, max end} in s_memrealtime ticks (100 MHz) — every
                                workgroup folds its first / last instant in by vector atomics.
                                Caller initialises {~0ull, 0}. No output depends on it. */
  float* skinny_ws;          /* optional, AVSR_SKINNY_WS_BYTES: with splitk <= 1 and M <= 64 (the
                                vector-ALU path of decoder steps) the launch splits K over
                                avsr_gemm_skinny_splits(N, K) workgroup rows: AVSR_SKINNY_WS fp32
                                partials, then AVSR_SKINNY_CNT uint32 arrival counters that the
                                caller zeroes once (every launch leaves them zero); the last
                                workgroup of a column block adds the partials in a fixed order
                                and runs the epilogue. NULL: one workgroup row. */
  const float* ln_c1;        /* optional LayerNorm prologue (fp32, M <= 64, K <= 1024, K % 16 == 0,
                                unsplit): A holds the LayerNorm inputs x and B = gamma o W (W's
                                columns scaled by the LayerNorm weight); per row the kernel takes
                                mean and 1/sqrt(var + ln_eps) of x and computes
                                C = epilogue(rstd * (x B^T - mean * ln_c1[n])) with ln_c1[n] =
                                sum_k B[n][k] and bias = W beta + b — LayerNorm followed by the
                                linear (decoder.py:98-134 norm1/2/3 + linear) in one launch */
  float ln_eps;
  void* kv_k;                /* optional KV-cache append (fp32 few-row path, N % 3 == 0, D = N / 3):
                                output columns [D, 2D) of row m go to kv_k row (*kv_pos * kv_rows +
                                m) instead of C, columns [2D, 3D) to kv_v (the self-attention K / V
                                cache of the device-side beam search; avsr_beam_kv_put fused into
                                the QKV projection); columns [0, D) to C as usual */
  void* kv_v;
  const int* kv_pos;
  int kv_rows;
  unsigned* slab_cnt;        /* optional, AVSR_SLAB_CNT uint32 arrival counters for the slab split-K
                                weight-gradient path (splitk > 1 with ws, both operands r-contiguous,
                                fp32 C, plain epilogue): the last-arriving split of each output
                                tile reduces the slabs inside the GEMM (no separate reduction pass).
                                The caller zeroes them once; every launch leaves them zero. Launches
                                that share a counter buffer must be ordered (one stream). NULL: a
                                separate reduction pass. */
} avsr_gemm_params;
#define AVSR_GEMM_COLSUM_WS(M, N) ((int64_t)(((M) + 63) / 64) * (N))
/* slabs are AVSR_GEMM_SLAB_PAD floats apart beyond M*N: power-of-two slab strides put the
 * reduce pass's split-many reads of one vector on the same HBM channels (measured 0.55 TB/s for
 * 8 slabs of 4 MiB) */
#define AVSR_GEMM_SLAB_PAD 1088
#define AVSR_SKINNY_WS (1 << 19)
#define AVSR_SKINNY_CNT 4096
#define AVSR_SLAB_CNT 4096
#define AVSR_SKINNY_WS_BYTES ((int64_t)AVSR_SKINNY_WS * 4 + AVSR_SKINNY_CNT * 4)
#define AVSR_GEMM_SLAB_WS(batch, splitk, M, N) ((int64_t)(batch) * (splitk) * ((int64_t)(M) * (N) + AVSR_GEMM_SLAB_PAD))

int avsr_gemm(const avsr_gemm_params* p, void* stream);
/* n <= 4 weight-gradient GEMMs (C fp32 += alpha * A^T B with both operands r-contiguous bf16, no
 * epilogue, no split: the avsr_gemm weight-gradient shape) in ONE launch whose grid holds every
 * problem's output tiles — problems that each fill part of the chip fill it together (encoder
 * out-proj 64 + QKV 192 tiles = 256 = one block per CU). Results equal avsr_gemm's per problem
 * bit for bit; problems of another shape run one by one through avsr_gemm. Replaces the
 * nn.Linear weight-gradients of Wav2Vec2Attention (avhubert.py:747-768). */
int avsr_gemm_wgrad_group(const avsr_gemm_params* p, int n, void* stream);
/* K-split count the few-row path uses for an N x K weight of this dtype when skinny_ws is given
 * (depends on dtype, N and K only, never on M: a row's result does not depend on how many rows
 * share the launch; fp32 with K % 16 == 0 and 16-byte aligned rows runs the matrix-core kernel) */
int avsr_gemm_skinny_splits(int dtype, int N, int K);

/* ------------------------------------------------------------------------------------
 * Implicit-GEMM convolution over NHWC activations (no im2col buffer), grouped.
 *   x [nimg][hin][win][ldx] (group g uses channels g*cin .. g*cin+cin-1)
 *   y [nimg][hout][wout][ldy] (group g: channels g*cout ..)
 *   w [groups*cout][kh][kw][cin]  (= torch channels_last physical order)
 * fwd:         y  = conv(x, w)                          (+ BN partial statistics if stats)
 * bwd_data:    dx = alpha * conv_transpose(dy, w) (+ beta * dx)
 * bwd_weight:  dw (fp32) += conv_wgrad(x, dy)   (split-K over pixels: fp32 slabs in ws, reduced
 *              by a second kernel; without ws, fp32 atomics)
 * Replaces: nn.Conv2d in src/nets/backend/backbones/resnet.py:10-22 (3x3 and 1x1
 *   downsample, ResNet-18 trunk), nn.Conv3d stem resnet.py:132 (as a 2-D conv over 5
 *   time-stacked channels, see avsr_stem_pack), and the grouped pos-conv Conv1d
 *   (k=128, groups 16) of HF:Wav2Vec2PositionalConvEmbedding (:326-369) as a 1-D conv
 *   (win = wout = kw = 1).
 * Requirements: cin, cout powers of two >= 8; ldx, ldy multiples of 8; 16-B aligned.
 * ------------------------------------------------------------------------------------ */
typedef struct {
  int dtype;
  int nimg, hin, win, cin;
  int hout, wout, cout;
  int kh, kw, sh, sw, ph, pw;
  int groups;
  int64_t ldx, ldy;
  const void* x; const void* w; void* y;   /* forward operands / output */
  void* dx; const void* dy; float* dw;     /* backward */
  float* stats;   /* fwd only: [cout][avsr_conv_stat_tiles()][3] (count, mean, M2) or NULL */
  float alpha, beta;                       /* bwd_data scaling */
  int splitk;     /* bwd_weight: 0 = auto */
  /* fwd epilogue (optional): h = conv + bias[c]; preact = h; y = act(h) + res  (res/preact
   * laid out like y; used by the pos-conv: x + GELU(conv(x) + b)) */
  const float* bias; int act; void* preact; const void* res;
  float* ws;      /* bwd_weight split-K workspace of avsr_conv_wgrad_ws() floats, or NULL */
  /* bwd_data, optional (bf16, groups 1): BatchNorm+PReLU backward reduction in the epilogue.
   * The value v = alpha*conv_transpose(dy, w) + beta*dx is the gradient of prelu(z),
   * z = h*scale + shift (+ res | + res*scale2 + shift2); dx receives dz = prelu'(z)*v and
   * bnr_ws[avsr_conv_bnr_tiles()][4][cin] the per-tile column sums (sum dz, sum dz*xhat,
   * sum dz*xhat2, sum v*z*[z<=0]) that avsr_bn_bwd_finalize folds. h / res laid out like dx.
   * Replaces the separate avsr_bn_act_bwd_reduce pass over dx (resnet.py:45-62 backward). */
  const void* bnr_h; const void* bnr_res;
  const float* bnr_scale; const float* bnr_shift; const float* bnr_prelu;
  const float* bnr_mean; const float* bnr_invstd;
  const float* bnr_scale2; const float* bnr_shift2; const float* bnr_mean2; const float* bnr_invstd2;
  float* bnr_ws;
} avsr_conv_params;

int avsr_conv_fwd(const avsr_conv_params* p, void* stream);
int avsr_conv_bwd_data(const avsr_conv_params* p, void* stream);
int avsr_conv_bwd_weight(const avsr_conv_params* p, void* stream);
/* number of row tiles the forward partial statistics are split into */
int avsr_conv_stat_tiles(const avsr_conv_params* p);
/* number of row tiles of a bwd_data with the BN-backward epilogue (rows of bnr_ws) */
int avsr_conv_bnr_tiles(const avsr_conv_params* p);
/* fp32 workspace (floats) bwd_weight uses when p->ws is given (0: it needs none) */
int64_t avsr_conv_wgrad_ws(const avsr_conv_params* p);

/* ------------------------------------------------------------------------------------
 * LayerNorm over the last dim (rows of N), fp32 statistics.
 * fwd: y = (x - mean) * rstd * gamma + beta; stores mean/rstd per row (fp32).
 * bwd: dx = (dres ? dres : 0) + rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * gamma;
 *      dgamma += sum dy * xhat, dbeta += sum dy   (fp32, atomics)
 * Replaces: torch.nn.LayerNorm at avhubert.py:184-185/:484 (2048, eps 1e-5),
 *   HF:Wav2Vec2EncoderLayer layer_norm / final_layer_norm and encoder layer_norm (1e-5),
 *   src/nets/backend/transformer/layer_norm.py:12-33 (decoder, eps 1e-12).
 * ------------------------------------------------------------------------------------ */
typedef struct {
  int dtype, rows, N;
  float eps;
  const void* x; int64_t ldx;
  void* y; int64_t ldy;
  const float* gamma; const float* beta;
  float* mean; float* rstd;                 /* [rows] */
  const void* dy; int64_t lddy;             /* bwd */
  void* dx; int64_t lddx;                   /* bwd output */
  const void* dres; int64_t lddres;         /* bwd: residual gradient added to dx (may alias dx) */
  float* dgamma; float* dbeta;              /* bwd: fp32 accumulators [N] or NULL */
  float* ws;                                /* bwd with dgamma: workspace >= AVSR_LN_WS(N) floats */
  /* bwd, optional: the next elementwise backward of the chain fused in (avsr_ew_bwd with out,
   * drop_p, seed, db): g = dropout-backward(dx as stored) and db += column sums of g. The
   * reference applies dropout to the sublayer output that is added to this LayerNorm's input
   * (HF Wav2Vec2EncoderLayer), so its gradient is the residual gradient dx masked. With db the
   * workspace needs AVSR_LN_WS3(N) floats. */
  void* g; int64_t ldg; float drop_p; uint64_t seed; float* db;
} avsr_layernorm_params;
#define AVSR_LN_BLOCKS 256
#define AVSR_LN_WS(N) (AVSR_LN_BLOCKS * 2 * (N))
#define AVSR_LN_WS3(N) (AVSR_LN_BLOCKS * 3 * (N))
int avsr_layernorm_fwd(const avsr_layernorm_params* p, void* stream);
int avsr_layernorm_bwd(const avsr_layernorm_params* p, void* stream);

/* ------------------------------------------------------------------------------------
 * BatchNorm (NHWC, per-channel) for the ResNet-18 lip frontend, resnet.py:30-164.
 * finalize: combine conv-epilogue partials (count, mean, M2) -> mean / invstd; scale =
 *   gamma*invstd, shift = beta - mean*scale; training also updates running stats
 *   (momentum 0.1, unbiased running_var, as torch.nn.BatchNorm2d/3d). Eval mode builds
 *   scale/shift from the running statistics.
 * act_fwd: y = prelu(h*scale + shift + r), r = res (identity) or res*scale2 + shift2
 *   (downsample BN) or 0;  prelu weight per channel (nn.PReLU(num_parameters=C)).
 * act_bwd_reduce: z recomputed; dz = dy * prelu'(z) (stored); accumulates per channel
 *   sum dz, sum dz*xhat (and for the downsample BN), prelu-weight grad sum dy*z*[z<=0];
 *   also dgamma/dbeta of both BNs.
 * bwd_apply: dh = scale*(dz - sum dz/M - xhat*sum(dz xhat)/M) (+beta*dh), same for the
 *   downsample BN into dhd.
 * ------------------------------------------------------------------------------------ */
typedef struct {
  int tiles, C;               /* partial tiles, channels */
  const float* partials;      /* [C][tiles][3] or NULL (eval) */
  const float* gamma; const float* beta;
  float* running_mean; float* running_var;
  float momentum, eps;
  int training;
  float* mean; float* invstd; float* scale; float* shift;   /* [C] outputs */
} avsr_bn_finalize_params;
int avsr_bn_finalize(const avsr_bn_finalize_params* p, void* stream);

typedef struct {
  int dtype, M, C;
  const void* h;                                   /* conv output (pre-BN) [M][C] */
  const float* scale; const float* shift;          /* BN of h */
  const void* res;                                 /* residual [M][C] or NULL */
  const float* scale2; const float* shift2;        /* BN of res (downsample) or NULL (identity) */
  const float* prelu;                              /* [C] */
  void* y;                                         /* fwd output */
  /* backward */
  const void* dy; void* dz;
  const float* mean; const float* invstd;          /* BN of h (for xhat) */
  const float* mean2; const float* invstd2;        /* BN of res when scale2 */
  float* sums;    /* [C][3] out: sum dz, sum dz*xhat, sum dz*xhat2 (fp32; written, not accumulated) */
  float* dprelu;  /* [C] fp32 grad accumulator */
  float* dgamma; float* dbeta; float* dgamma2; float* dbeta2;   /* fp32 grad accumulators or NULL */
  void* dh; void* dh2; float beta_acc;             /* bwd_apply outputs (dh2 for the downsample BN) */
  float* ws;                                       /* bwd_reduce workspace >= AVSR_BN_WS(C) floats */
} avsr_bn_act_params;
/* partial sums of `tiles` row blocks [tiles][4][C] plus the fold area finalize uses */
#define AVSR_BN_FIN_WS(tiles, C) (((int64_t)(tiles) + ((tiles) > 256 ? ((tiles) + 15) / 16 : 0)) * 4 * (C))
#define AVSR_BN_WS(C) AVSR_BN_FIN_WS(2048, C)
int avsr_bn_act_fwd(const avsr_bn_act_params* p, void* stream);
/* reduce + finalize (sums, dgamma/dbeta, dprelu) */
int avsr_bn_act_bwd_reduce(const avsr_bn_act_params* p, void* stream);
/* finalize only, from partials ws[tiles][4][C] written by a data-grad BN epilogue
 * (avsr_conv_params.bnr_ws, tiles = avsr_conv_bnr_tiles) */
int avsr_bn_bwd_finalize(const avsr_bn_act_params* p, int tiles, void* stream);
int avsr_bn_bwd_apply(const avsr_bn_act_params* p, void* stream);

/* stem: y[n][oh][ow][c] = max_{3x3, s2, p1} prelu(bn(h)) (+argmax index, + hmax = h at the
 * argmax), resnet.py:132-136 (BatchNorm3d + PReLU + MaxPool3d((1,3,3),(1,2,2),(0,1,1))).
 * Backward in the pooled domain: the BN/PReLU reduction is avsr_bn_act_bwd_reduce (or a
 * data-grad BN epilogue) over the POOLED grid with h = hmax, dy = pooled gradient, giving the
 * pooled dz and the sums over input pixels (dz vanishes off the argmax positions);
 * bwd_apply: dh[n][h][w][c] = scale*(dz - S0/M - xhat*S1/M), dz routed back through the
 * argmax (M = m_total, or nimg*H*W). */
typedef struct {
  int dtype, nimg, H, W, C, Ho, Wo;
  const void* h; const float* scale; const float* shift; const float* prelu;
  void* y; uint8_t* argmax;
  const void* dy; void* dz;                        /* bwd_apply: dz = pooled dz [n][Ho][Wo][C] */
  const float* mean; const float* invstd;
  float* sums; float* dprelu; float* dgamma; float* dbeta;
  float* ws;
  void* hmax;                                      /* fwd output [n][Ho][Wo][C] (optional) */
  void* dh;                                        /* bwd_apply output [n][H][W][C] */
  int64_t m_total;                                 /* bwd_apply: pixels M the BN statistics
                                                      cover (0: nimg*H*W); a launch over a range
                                                      of images passes the whole batch's M */
} avsr_stem_pool_params;
int avsr_stem_pool_fwd(const avsr_stem_pool_params* p, void* stream);
int avsr_stem_pool_bwd_apply(const avsr_stem_pool_params* p, void* stream);

/* global average pool over P pixels: y[n][c] = mean_p x[n][p][c] (nn.AdaptiveAvgPool2d(1),
 * resnet.py:83,121); bwd: dx[n][p][c] = dy[n][c] / P */
int avsr_avgpool_fwd(int dtype, int nimg, int P, int C, const void* x, void* y, void* stream);
int avsr_avgpool_bwd(int dtype, int nimg, int P, int C, const void* dy, void* dx, void* stream);

/* ------------------------------------------------------------------------------------
 * Fused multi-head attention, head dim 64, fp32 online softmax (flash-style; the Lq x Lk
 * score matrix is never stored).  o = softmax(scale * q k^T + mask) v  per (batch, head).
 *   q row (b, i), head h: q[(b*Lq + i)*ldq + h*64 .. +63]; likewise k, v (Lk rows), o.
 *   mask: key j of batch b valid iff j < klen[b] (klen NULL: all Lk valid) and, if causal,
 *   j <= i.  Optional dropout on the probabilities (counter-based; bwd recomputes it).
 * fwd stores lse[b][h][i] (natural log) for the backward.
 * bwd: dq (fp32 accumulator [B*Lq][ldq_f32], atomics, caller zeroes) or dq_out (dtype),
 *   dk, dv (dtype); needs delta[b][h][i] = sum_d dO*O from avsr_attn_bwd_prep. bf16 runs
 *   two streaming kernels (dK/dV per key block, dQ per query block), fp32 one atomic kernel.
 * Replaces: HF:eager_attention_forward + Wav2Vec2Attention core (:438-548; encoder, key
 *   padding mask from avhubert.py:688-696) and MultiHeadedAttention.forward_attention
 *   (src/nets/backend/transformer/attention.py:56-106; decoder causal self-attention and
 *   memory-masked source attention).
 * ------------------------------------------------------------------------------------ */
typedef struct {
  int dtype, B, H, Lq, Lk;
  float scale;
  const void* q; int64_t ldq;
  const void* k; int64_t ldk;
  const void* v; int64_t ldv;
  void* o; int64_t ldo;
  float* lse;                 /* [B][H][Lq] */
  const int* klen;            /* [B] or NULL */
  int causal;
  float drop_p; uint64_t seed;
  /* backward */
  const void* dout; int64_t lddo;
  float* delta;               /* [B][H][Lq] */
  float* dq; int64_t lddq;    /* fp32 */
  void* dk; int64_t lddk;
  void* dv; int64_t lddv;
  /* bf16 only: if non-NULL, dQ is written here in the activation dtype (dq unused);
   * otherwise bf16 writes dq (fp32) with plain stores (= accumulate onto a zeroed buffer) */
  void* dq_out; int64_t lddq_out;
  /* optional (backward): db[s*H*64 + h*64 + d] += column sums over all B*L rows of the dQ
   * (s = 0), dK (s = 1), dV (s = 2) values as stored (bf16-rounded in bf16) — the fused q/k/v
   * projection bias gradients. db_ws: AVSR_ATTN_DB_WS(B, H) floats of per-utterance partials,
   * finalised through the column-sum path (deferred like avsr_gemm db: keep it alive until the
   * flush). The resident bf16 kernels sum them in their store epilogues; other paths run one
   * extra pass over dq/dk/dv. NULL: off. */
  float* db; float* db_ws;
  /* optional probability-dropout keep mask (bf16, non-causal): written once per (seed, shape)
   * by avsr_attn_dropmask, then read by avsr_attn_fwd / avsr_attn_bwd in place of re-hashing
   * the counter dropout per element (same bits: the mask IS the hash's keep decision). 64-bit
   * lane masks, AVSR_ATTN_MASK_WORDS(B, H, Lq, Lk) words, per (b, h) and 32 x 32 tile (query
   * block qb of 32, key block kb of 32, kb padded to an even count NKB = 2 * ceil(Lk / 64)), 16
   * words per tile, query on the lane: word ((bh * NQB + qb) * NKB + kb) * 16 + r, bit l keeps
   * (q = 32 qb + (l & 31), k = 32 kb + (r & 3) + 8 (r >> 2) + 4 (l >> 5)); 0 past Lq / Lk.
   * NULL: the kernels hash (decoder attention, fp32). */
  uint64_t* drop_mask;
} avsr_attn_params;
#define AVSR_ATTN_DB_WS(B, H) ((int64_t)(B) * 3 * (H) * 64)
#define AVSR_ATTN_MASK_WORDS(B, H, Lq, Lk) \
  ((int64_t)(B) * (H) * (((Lq) + 31) / 32) * (2 * (((Lk) + 63) / 64)) * 16)
/* diagnostic (not product path): per-workgroup s_memrealtime stamps (start, first round
 * landed, compute done, end, HW_ID, XCC_ID) of the resident attention forward into
 * buf[6 * workgroups], and of the encoder backward's dQ / dK-dV kernels into buf[6 * B * H]
 * / buf[6 * B * H ..]; buf = NULL turns them off */
int avsr_debug_attn_stamps(unsigned long long* buf);
int avsr_attn_fwd(const avsr_attn_params* p, void* stream);
int avsr_attn_bwd_prep(const avsr_attn_params* p, void* stream);   /* delta = rowsum(dO * O) */
int avsr_attn_bwd(const avsr_attn_params* p, void* stream);
/* fills p->drop_mask (AVSR_ATTN_MASK_WORDS words) with the keep decisions of drop_p / seed for
 * (B, H, Lq, Lk): the data-independent half of the attention dropout, runnable ahead of the
 * forward on another stream. Same replacement as avsr_attn_fwd (the dropout of
 * Wav2Vec2Attention / eager_attention_forward, avhubert.py:747-768). */
int avsr_attn_dropmask(const avsr_attn_params* p, void* stream);

/* ------------------------------------------------------------------------------------
 * Losses on logits [rows][ldx] (V valid columns; columns V..ldx-1 of every gradient row are
 * written as 0 so padded GEMM operands stay finite).
 * avsr_row_lse:   lse[row] = log sum_k exp(x[row][k])
 * avsr_lsm_fwd:   LabelSmoothingLoss rows (src/nets/backend/transformer/label_smoothing_loss.py
 *   :41-63, KL(q || softmax) with q = smoothing/(V-1) off-target, 1-smoothing on target,
 *   target -1 ignored) -> row_loss, and th_accuracy's argmax match (nets_utils.py:303-323)
 * avsr_lsm_bwd:   dx = (*dloss * coef) * (softmax - q), 0 on ignored rows
 * avsr_ctc_fwd:   torch.nn.CTCLoss(blank=0, reduction none, zero_infinity=True) per utterance
 *   (ctc.py:64-81): log-space alpha and beta over the extended label sequence; nll[b] and the
 *   state occupancies gamma[b][t][s] = P(path at state s at t | x) (0 if infeasible)
 * avsr_ctc_bwd:   dx[b,t,k] = (*dloss * coef) * (softmax_t(k) - sum_{s: ext_s = k} gamma_t(s))
 *   for t < in_len[b] (0 otherwise and for infeasible utterances)
 * avsr_loss_finalize: loss_ctc = sum nll / B, loss_att = sum row_loss / B (att_per_token = 0) or
 *   / the number of target tokens, i.e. rows with row_correct >= 0 (att_per_token = 1:
 *   transformer_length_normalized_loss, label_smoothing_loss.py:61; needs row_correct),
 *   loss = mtl*ctc + (1-mtl)*att, acc = correct / valid  (e2e_asr_avhubert.py:150-159)
 *   out[4] = {loss, loss_ctc, loss_att, acc}, all on device (no host sync)
 * ------------------------------------------------------------------------------------ */
typedef struct {
  int dtype, rows, V;
  const void* x; int64_t ldx;
  const int* target;        /* [rows], -1 = ignore */
  float smoothing;
  float* lse; float* row_loss; int* row_correct;   /* [rows]; row_correct: 1/0, -1 ignored */
  const float* dloss; float coef;
  void* dx; int64_t lddx;
} avsr_xent_params;
int avsr_row_lse(const avsr_xent_params* p, void* stream);
int avsr_lsm_fwd(const avsr_xent_params* p, void* stream);
int avsr_lsm_bwd(const avsr_xent_params* p, void* stream);

typedef struct {
  int dtype, B, T, V, Lmax;
  const void* x; int64_t ldx;          /* rows b*T + t */
  const float* lse;                    /* [B*T] */
  const int* labels;                   /* [B][Lmax] */
  const int* label_len; const int* in_len;   /* [B] */
  float* alpha; float* gamma;          /* workspaces [B][T][2*Lmax+1] */
  float* nll;                          /* [B] */
  const float* dloss; float coef;
  void* dx; int64_t lddx;
} avsr_ctc_params;
int avsr_ctc_fwd(const avsr_ctc_params* p, void* stream);
int avsr_ctc_bwd(const avsr_ctc_params* p, void* stream);

int avsr_loss_finalize(int B, const float* nll, int rows, const float* row_loss, const int* row_correct,
                       float mtlalpha, int att_per_token, float* out, void* stream);

/* ------------------------------------------------------------------------------------
 * Elementwise / data-movement kernels around the GEMMs.
 * avsr_ew_bwd:     out = alpha * dy * dropmask(drop_p, seed; idx = row*N + col) * act'(gate),
 *                  db[n] += sum_rows out  (bias gradients of the Linear layers; out optional)
 * avsr_dropout_fwd: out = dy * dropmask (nn.Dropout on a [rows][N] view: CTC input dropout
 *                  ctc.py:27,98, encoder dropout after pos-conv avhubert.py:704)
 * avsr_mask_rows:  x[b*T + t][:] = 0 for t >= len[b]   (avhubert.py:683-686)
 * avsr_embed_fwd:  y[r] = dropout(table[tok[r]] * scale + pe[r % L])  (decoder embed +
 *                  PositionalEncoding, decoder.py:89-93, embedding.py:80-87); bwd: dtable
 *                  += per-token sums of the row gradients in row order (no atomics)
 * avsr_cast:       dst = alpha * src + beta * dst over a [rows][cols] strided view
 * avsr_cast_flat:  dst = src over n contiguous elements (fp32 <-> bf16 vectorised: the arena's
 *                  master -> compute-shadow refresh after load_state_dict / optimizer steps; the
 *                  bf16-compressed gradient all-reduce's compress / decompress)
 * avsr_stem_pack:  videos (B,1,T,88,88) fp32 -> (B*T, 88, 88, 8): channel c = frame t+c-2
 *                  (c < 5, zero outside [0,T)), the Conv3d(k=5x7x7, pad 2x3x3) stem as a 2-D conv
 * avsr_stem_wpack / avsr_stem_wgrad_unpack: Conv3d weight (64,1,5,7,7) <-> [64][7][7][8]
 * avsr_audio_pack: audios (B, F, T) fp32 -> (B*T, F)  (SubModel.proj input, avhubert.py:194-196)
 * avsr_weightnorm_fwd/bwd: w = g * v / ||v|| per tap k, v stored [o][k][c] (HF weight_norm
 *                  dim=2 of the pos-conv, modeling_wav2vec2.py:336-356)
 * avsr_sumsq / avsr_adamw: fused clip_grad_norm_(max_norm) + torch.optim.AdamW step over a
 *                  flat fp32 parameter range; optionally refreshes the bf16 shadow copy
 * ------------------------------------------------------------------------------------ */
typedef struct {
  int dtype, rows, N;
  const void* dy; int64_t lddy;
  void* out; int64_t ldout;
  const void* gate; int64_t ldgate; int act;
  float drop_p; uint64_t seed;
  float alpha;
  float* db;
  float* ws;                                       /* with db: workspace >= AVSR_EW_WS(N) floats */
} avsr_ew_params;
#define AVSR_EW_ROWBLOCKS 256
#define AVSR_EW_WS(N) (AVSR_EW_ROWBLOCKS * (N))
int avsr_ew_bwd(const avsr_ew_params* p, void* stream);
/* Deferred finalisation of the column-sum partials (bias gradients of avsr_ew_bwd /
 * avsr_gemm db, LayerNorm dgamma/dbeta): between avsr_colsum_defer(1) and avsr_colsum_flush the
 * finalise passes are queued on the host and a flush reduces all of them in one batched launch
 * on `stream` (stream-ordered after the producers). The caller keeps the partial workspaces
 * alive until the flush. avsr_colsum_defer returns the previous setting. (A training step's
 * ~200 separate 5 us finalise launches become one per encoder layer.) */
int avsr_colsum_defer(int on);
int avsr_colsum_flush(void* stream);
/* avsr_colsum_inline(1): finalise passes launch at once on their producer's stream even while
 * deferral is on (the queue is left untouched) -- for a column sum issued on another stream
 * than the flush (the weight-grad side stream); returns the previous setting */
int avsr_colsum_inline(int on);
int avsr_dropout_fwd(const avsr_ew_params* p, void* stream);
int avsr_mask_rows(int dtype, int B, int T, int N, void* x, int64_t ldx, const int* len, void* stream);

typedef struct {
  int dtype, rows, L, D;
  const int* tok; const void* table; const float* pe; float scale;
  void* y; float drop_p; uint64_t seed;
  const void* dy; float* dtable;
  const int* pe_row;         /* forward, optional: device int, every row adds pe[pe_row[0]] (L ignored):
                                the position of a beam-search step kept on the device */
} avsr_embed_params;
int avsr_embed_fwd(const avsr_embed_params* p, void* stream);
int avsr_embed_bwd(const avsr_embed_params* p, void* stream);

int avsr_cast(int src_dtype, int dst_dtype, int rows, int cols, const void* src, int64_t lds,
              void* dst, int64_t ldd, float alpha, float beta, void* stream);
int avsr_cast_flat(int src_dtype, int dst_dtype, int64_t n, const void* src, void* dst, void* stream);
int avsr_stem_pack(int dtype, int B, int T, const float* video, void* out, void* stream);
int avsr_stem_wpack(int dtype, const float* w, void* wp, void* stream);
/* avsr_stem_conv_fwd (bf16): the stem Conv3d (resnet.py:132) read straight from videos
 *                  (B,1,T,88,88) fp32 (zero frames outside the clip) -> h [B*T][44][44][64] bf16,
 *                  and (stats != NULL) BN partials stats[64][avsr_stem_conv_tiles(B, T)][3]
 *                  (count, mean, M2) as avsr_conv_fwd writes them; wk from avsr_stem_wpack2:
 *                  [64][288] bf16, k = (dt*7 + kh)*8 + kw (kw = 7 and k >= 280 zero) */
int avsr_stem_conv_tiles(int B, int T);
int avsr_stem_wpack2(const float* w, void* wk, void* stream);
int avsr_stem_conv_fwd(int B, int T, const float* video, const void* wk, void* h, float* stats, void* stream);
int avsr_stem_wgrad_unpack(const float* gp, float* gw, void* stream);
int avsr_audio_pack(int dtype, int B, int F, int T, const float* audio, void* out, void* stream);

int avsr_weightnorm_fwd(int dtype, int O, int K, int C, const float* v, const float* g, float* norm,
                        void* w, void* stream);
int avsr_weightnorm_bwd(int O, int K, int C, const float* v, const float* g, const float* norm,
                        const float* dw, float* dv, float* dg, float* scratch, void* stream);

/* *out += sum x^2 in a fixed summation order (deterministic); ws: AVSR_SUMSQ_WS floats */
#define AVSR_SUMSQ_WS 1024
int avsr_sumsq(const float* x, int64_t n, float* out, float* ws, void* stream);
typedef struct {
  int64_t n;
  float* param; const float* grad; float* exp_avg; float* exp_avg_sq;
  void* shadow; int shadow_dtype;        /* bf16 copy of the updated params, or NULL */
  float lr, beta1, beta2, eps, weight_decay;
  float bias_corr1, bias_corr2;          /* 1 - beta^t */
  const float* sumsq; float max_norm;    /* clip: coef = min(1, max_norm / (sqrt(*sumsq) + 1e-6)); sumsq NULL = no clip */
  float grad_scale;                      /* extra multiplier on the gradient (1/accumulation etc.) */
  int max_blocks;                        /* grid cap (0: 4096 = the whole chip). An update running
                                            beside other work on another stream takes fewer, so its
                                            grid-stride blocks leave CU slots to that work; the
                                            result does not depend on it */
  float* grad_clear;                     /* NULL, or = grad: each gradient element is set to 0 after the
                                            update has read it (the next step's gradient clear done
                                            by the update, e.g. while it overlaps the next forward) */
} avsr_adamw_params;
int avsr_adamw(const avsr_adamw_params* p, void* stream);

/* ------------------------------------------------------------------------------------
 * Joint CTC / attention beam search. Replaces, for the decoder
 * that get_beam_search_decoder builds (src/avhubert_avsr/avhubert_avsr_model.py:12-36):
 *   Decoder.batch_score / forward_one_step    src/nets/backend/transformer/decoder.py:153-227
 *     (one query per hypothesis; the reference recomputes the cross-attention K/V of the
 *      memory every step, here they are computed once per utterance)
 *   CTCPrefixScoreTH.__call__                 src/nets/ctc_prefix_score.py:65-187
 *   BatchBeamSearch.search / batch_beam       src/nets/batch_beam_search.py:102-260
 *   index_select of the hypothesis states     src/nets/batch_beam_search.py:53-66
 * avsr_log_softmax_rows: out[r][c] = x[r][c] - max - log(sum exp(x - max)), c < V (fp32 out)
 * avsr_dec_attn: o[i][h*64..] = softmax(scale * q_i k_j^T, j < klen[i]) v  per hypothesis i
 *   and head h; key j of hypothesis i at k[i*k_bstride + j*ldk + h*64] (bstride 0: the keys
 *   are shared, e.g. the encoder memory). dynamic LDS: (klen_max + 256) * 4 bytes.
 * avsr_row_topk: ids[r][0..K) = indices of the K largest x[r][c], c < V, descending
 *   (ties: smaller index first); K <= 16.
 * avsr_ctc_prefix: for hypothesis h (prefix length out_len + 1 incl. sos, last token
 *   last[h], CTC forward variables r_prev[h][T][2] or NULL at the first step) and its P
 *   scored tokens ids[h][:]: r_new[h][j][T][2] and psi[h][j] = log prefix probability
 *   (LOGZERO for blank, r_sum[T-1] for eos), psi[h][P] = r_sum[T-1] (the eos score).
 * avsr_beam_select: weighted[h][v] = w_dec*dec[h][v] + w_ctc*(psi(h,v) - s_prev[h]) +
 *   score[h]; the beam best (h, v) in descending order -> out_prev/out_tok/out_score,
 *   out_dec = dec[h][v], out_ctc = psi - s_prev, out_s = psi, out_col = column of v in
 *   ids[h] (P-1 when v was not scored, the reference's scoring_idmap -1 index).
 * Batched decoding (several utterances per step, avsr_amd.decode.BatchBeamSearch.decode_batch):
 *   the optional kidx / uidx+tlen / nseg+seg fields route each hypothesis to its utterance's
 *   memory, CTC log-probs and beam selection; the reference decodes one utterance at a time
 *   (script/evaluation.py:280-296), results are identical per utterance.
 * avsr_gather_rows: dst[g][i] = src[g][idx[i]] for i < n, rows of row_bytes; sizes, strides and
 *   pointers multiples of 4 bytes (16-byte words when everything is 16-byte aligned).
 * ------------------------------------------------------------------------------------ */
int avsr_log_softmax_rows(int dtype, int rows, int V, const void* x, int64_t ldx, float* out, int64_t ldo,
                          void* stream);

typedef struct {
  int dtype, n, H, klen_max;
  float scale;
  const void* q; int64_t ldq;
  const void* k; int64_t ldk, k_bstride;
  const void* v; int64_t ldv, v_bstride;
  const int* klen;            /* [n] or NULL (= klen_max) */
  void* o; int64_t ldo;
  const int* kidx;            /* [n] or NULL: hypothesis i reads key block kidx[i] (base kidx[i]*k_bstride,
                                 v likewise) instead of block i — batched decoding of several
                                 utterances whose memories sit in one [U][T][..] buffer */
  const int* kmap; int64_t ldmap;   /* optional [n][ldmap]: key j of hypothesis i is row kmap[i*ldmap + j]
                                 of k (v likewise; bstride / kidx ignored) — the self-attention
                                 cache of a device-side beam search, [step][row] rows addressed
                                 through each hypothesis's ancestry instead of being reordered */
  int group;                  /* >= 1 (0 = 1): hypotheses i0 .. i0+group-1 (i0 % group == 0) share one
                                 key block and klen (kidx / klen equal within a group, no kmap; the
                                 beams of one utterance over its memory): one workgroup reads each
                                 key / value row once for all of them */
  int ksplit;                 /* >= 2: a workgroup row's keys split over up to ksplit workgroups
                                 (min(ksplit, ceil(klen / 192)) of them: a function of the row's
                                 klen only), each writing (max, sum, unnormalised o) partials to
                                 ws; the last-arriving one (counter cnt[group][head], zeroed by
                                 the caller once, left zero) merges them in split order. 0 / 1: none */
  float* ws;                  /* ksplit >= 2: ceil(n / group) * H * ksplit * group * 66 floats */
  unsigned* cnt;              /* ksplit >= 2: ceil(n / group) * H counters */
} avsr_dec_attn_params;
int avsr_dec_attn(const avsr_dec_attn_params* p, void* stream);

typedef struct {
  int rows, V, K;
  const float* x; int64_t ldx;
  int* ids;                   /* [rows][K] */
} avsr_topk_params;
int avsr_row_topk(const avsr_topk_params* p, void* stream);
/* avsr_log_softmax_topk: avsr_log_softmax_rows followed by avsr_row_topk on its output, in one
 * pass over each row (decode steps: the decoder output layer's log-probs and the pre-beam,
 * batch_beam_search.py:228-236 + scorers/ctc.py pre-beam); results identical to the two calls */
int avsr_log_softmax_topk(int dtype, int rows, int V, const void* x, int64_t ldx, float* out, int64_t ldo,
                          int K, int* ids, void* stream);

typedef struct {
  int n, T, V, P;
  int blank, eos, out_len;
  const float* logp;          /* [T][V] CTC log-probs */
  const float* r_prev;        /* [n][T][2] or NULL (first step) */
  const int* last;            /* [n] */
  const int* ids;             /* [n][P] */
  float* r_new;               /* [n][P][T][2] */
  float* psi;                 /* [n][P+1] */
  /* batched utterances (uidx NULL: one utterance): hypothesis h scores utterance uidx[h],
   * whose log-probs start at logp + uidx[h]*logp_ustride and whose length is tlen[uidx[h]]
   * (<= T, the row stride of r_prev / r_new) */
  const int* uidx; int64_t logp_ustride; const int* tlen;
  const int* out_len_dev;     /* optional device int overriding out_len (graph-captured steps) */
} avsr_ctc_prefix_params;
int avsr_ctc_prefix(const avsr_ctc_prefix_params* p, void* stream);

typedef struct {
  int n, V, P, beam;
  int blank, eos;
  float w_dec, w_ctc;
  const float* dec; int64_t ld;        /* decoder log-probs [n][ld] */
  const int* ids;                      /* [n][P] */
  const float* psi;                    /* [n][P+1] */
  const float* s_prev;                 /* [n] */
  const float* score;                  /* [n] */
  int* out_prev; int* out_tok; int* out_col;
  float* out_score; float* out_dec; float* out_ctc; float* out_s;
  /* batched utterances (nseg 0: one selection over all n rows): selection u runs over rows
   * [seg[u], seg[u+1]) and writes out_*[u*beam + r]; out_prev is the global row index */
  int nseg; const int* seg;
} avsr_beam_select_params;
int avsr_beam_select(const avsr_beam_select_params* p, void* stream);

int avsr_gather_rows(int groups, int n, int64_t row_bytes, const void* src, int64_t src_gstride,
                     int64_t src_rstride, void* dst, int64_t dst_gstride, int64_t dst_rstride,
                     const int* idx, void* stream);

/* Device-side beam bookkeeping (avsr_amd.decode: the whole step lives on the device and is
 * replayed as a HIP graph; the host reads only a done count every few steps and the history at
 * the end). Fixed geometry: U utterances x beam rows = R rows; a finished hypothesis / utterance
 * becomes a dead row (score -inf, never selected: identical to the reference removing it,
 * batch_beam_search.py:262-349, beam_search.py:330-372).
 * avsr_beam_step_prep: at the start of step pos (= *pos): anc[r][pos] = pos*R + r (the
 *   self-attention cache row this step writes for row r) and klen[r] = pos + 1.
 * avsr_beam_kv_put: cache_k[(pos*R + r)*D ..] = qkv[r][D..2D), cache_v from qkv[r][2D..3D).
 * avsr_beam_post: after avsr_beam_select of step pos: new running state per row (token,
 *   score, decoder / CTC score sums in double like the reference's Python floats, CTC prefix
 *   score), the back-pointers and ended-hypothesis records of the step, per-utterance end
 *   detection (e2e_asr_common.py:18-48 over the per-length best ended scores) and stop rules;
 *   src[0..R) = rows to gather the ancestry from, src[R..2R) = r_new rows for r_prev; *pos += 1. */
typedef struct {
  int U, beam, P, R, Lmax, steps_cap, eos, end_detect;
  double d_end;
  int* pos;
  const int* maxlen;
  const int* sel_prev; const int* sel_tok; const int* sel_col;
  const float* sel_score; const float* sel_dec; const float* sel_ctc; const float* sel_s;
  int* tok; float* score; double* sdec; double* sctc; float* s_prev;
  int* src;
  int* bp_prev; int* bp_tok; int* end_flag; float* end_score; double* end_dec; double* end_ctc;
  float* best_len;           /* [U][Lmax + 3] */
  float* best_end;           /* [U] */
  int* done;                 /* [U + 1]: per utterance, then the count */
} avsr_beam_post_params;
int avsr_beam_step_prep(int R, int Lmax, const int* pos, int* anc, int* klen, void* stream);
int avsr_beam_kv_put(int dtype, int R, int D, const void* qkv, int64_t ldqkv, void* cache_k, void* cache_v,
                     const int* pos, void* stream);
int avsr_beam_post(const avsr_beam_post_params* p, void* stream);

/* ------------------------------------------------------------------------------------
 * Input front end (the collator's per-clip CPU transforms moved on device).
 * avsr_fbank_stack: log mel filterbank features of 16 kHz waveforms, stacked 4 frames per
 *   video frame and layer-normalised per row, written in the model's audios layout.
 *   Replaces FBanksAndStack.forward src/dataset/avhubert_dataset.py:108-116 (logfbank of
 *   python_speech_features 0.6 at :111: preemphasis 0.97, 400-sample frames every 160,
 *   rectangular window, |rfft_512|^2 / 512, 26 triangular mel filters, eps floor, log;
 *   stacker :91-106; F.layer_norm over 104, eps 1e-5) + collate_pad's 0.0 row padding
 *   (:280-311) + the permute to (B, 104, T) (:351).
 *   wav [B][ldw] f32 (clip b uses n_samples[b] >= 1 samples, e.g. 640 * video frames after
 *   cut_or_pad :22-33); out [B][104][T] f32, rows >= ceil(frames_b / 4) are zero.
 *   bins: the 28 filter edges floor(513 * mel2hz(linspace(0, hz2mel(8000), 28)) / 16000).
 * avsr_video_normalize: uint8 frames [B][T][H][W] -> f32 [B][1][T][crop][crop] =
 *   ((x / 255) cropped at (oy, ox) - mean) / std.  Replaces VideoTransform
 *   (avhubert_dataset.py:225-246: /255, CenterCrop(88) or RandomCrop(88) offsets,
 *   Normalize(0.421, 0.165)) + the collator permute (:350).
 * ------------------------------------------------------------------------------------ */
typedef struct {
  int B, T;                  /* clips, output rows (>= the longest clip's rows) */
  const float* wav; int64_t ldw;
  const int64_t* n_samples;  /* device [B] */
  int bins[28];
  float preemph, ln_eps;
  float* out;
} avsr_fbank_params;
int avsr_fbank_stack(const avsr_fbank_params* p, void* stream);

typedef struct {
  int B, T, H, W, crop, oy, ox;
  const uint8_t* frames;
  float mean, std;
  float* out;
} avsr_video_norm_params;
int avsr_video_normalize(const avsr_video_norm_params* p, void* stream);

/* ------------------------------------------------------------------------------------
 * Train-time augmentation on device (the collator's CPU transforms).
 * avsr_time_mask: zero spans of rows of x [B][L][row_bytes] (any dtype: row_bytes bytes per
 *   time step): rows [spans[b][s][0], spans[b][s][1]) of clip b for s < nspan (empty / negative
 *   spans ignored). Replaces AdaptiveTimeMask.forward's `cloned[t_start:t_end] = 0`
 *   (src/dataset/avhubert_dataset.py:131-151; the span draws stay on the host, :141-149).
 * avsr_add_noise: y[b] = x[b] + s_b * n[b] over the first len_b samples of each clip, with
 *   s_b = 10^((snr0_b - snr_b) / 20), snr0_b = 10 (log10 |x_b|^2 - log10 |n_b|^2) (energies in
 *   fp64 over the clip) — torchaudio.functional.add_noise as AddNoise / AddMultiSpk call it
 *   (avhubert_dataset.py:154-222: :178, :214, :220). y may alias x. ws: 2 * B * 64 doubles.
 * avsr_rgb_to_gray: uint8 RGB [n][3] -> uint8 gray [n], cv2.COLOR_RGB2GRAY fixed point
 *   (R*4899 + G*9617 + B*1868 + 8192) >> 14 (load_video, avhubert_dataset.py:45).
 * ------------------------------------------------------------------------------------ */
typedef struct {
  int B, L, nspan;
  int64_t row_bytes, clip_stride_bytes;     /* bytes per time step, bytes between clips */
  void* x;
  const int* spans;                         /* device [B][nspan][2] */
} avsr_time_mask_params;
int avsr_time_mask(const avsr_time_mask_params* p, void* stream);

typedef struct {
  int B, L;
  const float* x; int64_t ldx;
  const float* noise; int64_t ldn;
  const int* lengths;                       /* device [B] or NULL (all L) */
  const float* snr_db;                      /* device [B] */
  float* y; int64_t ldy;
  double* ws;                               /* >= AVSR_NOISE_WS(B) doubles */
} avsr_add_noise_params;
#define AVSR_NOISE_WS(B) (2 * 64 * (int64_t)(B))
int avsr_add_noise(const avsr_add_noise_params* p, void* stream);

int avsr_rgb_to_gray(const uint8_t* rgb, uint8_t* gray, int64_t n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* AVSR_HIP_H */
