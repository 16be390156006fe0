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
 * GEMM with fused epilogue (bf16 MFMA 32x32x16 tiles, fp32 accumulate).
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
  int splitk;                /* >1: K split over blocks, C (fp32) += alpha*acc by atomics */
} avsr_gemm_params;

int avsr_gemm(const avsr_gemm_params* p, void* stream);

/* ------------------------------------------------------------------------------------
 * Implicit-GEMM convolution over NHWC activations (no im2col buffer), grouped.
 *   x [nimg][hin][win][ldx] (group g uses channels g*cin .. g*cin+cin-1)
 *   y [nimg][hout][wout][ldy] (group g: channels g*cout ..)
 *   w [groups*cout][kh][kw][cin]  (= torch channels_last physical order)
 * fwd:         y  = conv(x, w)                          (+ BN partial statistics if stats)
 * bwd_data:    dx = alpha * conv_transpose(dy, w) (+ beta * dx)
 * bwd_weight:  dw (fp32) += conv_wgrad(x, dy)   (split-K, fp32 atomics)
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
  float* stats;   /* fwd only: [avsr_conv_stat_tiles()][groups*cout][3] (count, mean, M2) or NULL */
  float alpha, beta;                       /* bwd_data scaling */
  int splitk;     /* bwd_weight: 0 = auto */
} avsr_conv_params;

int avsr_conv_fwd(const avsr_conv_params* p, void* stream);
int avsr_conv_bwd_data(const avsr_conv_params* p, void* stream);
int avsr_conv_bwd_weight(const avsr_conv_params* p, void* stream);
/* number of row tiles the forward partial statistics are split into */
int avsr_conv_stat_tiles(const avsr_conv_params* p);

#ifdef __cplusplus
}
#endif
#endif /* AVSR_HIP_H */
