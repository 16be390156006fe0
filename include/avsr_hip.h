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
} avsr_gemm_params;

int avsr_gemm(const avsr_gemm_params* p, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* AVSR_HIP_H */
