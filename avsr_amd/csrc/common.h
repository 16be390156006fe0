// Shared device helpers for the gfx950 kernels of libavsr_hip.so.
// Wave = 64 lanes everywhere; bf16 is clang's __bf16 (same bits as torch.bfloat16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "avsr_hip.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int v4i32 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define AVSR_DEV __device__ __forceinline__

AVSR_DEV float to_f(float x) { return x; }
AVSR_DEV float to_f(bf16 x) { return (float)x; }
template <typename T> AVSR_DEV T from_f(float x);
template <> AVSR_DEV float from_f<float>(float x) { return x; }
template <> AVSR_DEV bf16 from_f<bf16>(float x) { return (bf16)x; }

// 16-byte vector of T (8 bf16 or 4 f32)
struct alignas(16) v16 { uint32_t w[4]; };

// hardware 2^x (v_exp_f32, ~1 ulp; no denormal-result fix-up): softmax / log-sum-exp inner loops
AVSR_DEV float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Wave reductions on DPP row rotations (v_mov_b32_dpp row_ror: cross-lane moves inside each
// 16-lane row, no LDS), then the four row results read as scalars (lanes 0 / 16 / 32 / 48) and
// combined in a fixed order: the result is wave-uniform and deterministic. (A __shfl_xor
// butterfly is six ds_bpermute round trips through the LDS unit on the reduction's dependent
// chain.) Call in converged control flow, like the butterfly they replace.
template <int R> AVSR_DEV float rorf(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x120 + R, 0xf, 0xf, false));
}
template <int R> AVSR_DEV int rori(int x) { return __builtin_amdgcn_update_dpp(0, x, 0x120 + R, 0xf, 0xf, false); }
AVSR_DEV float lanef(float x, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l)); }
// sum over each 16-lane row (every lane of the row holds it; lanes may differ in the last bit)
AVSR_DEV float row_sum16(float x) {
  x += rorf<8>(x); x += rorf<4>(x); x += rorf<2>(x); x += rorf<1>(x);
  return x;
}
AVSR_DEV float wave_sum(float x) {
  x = row_sum16(x);
  return (lanef(x, 0) + lanef(x, 16)) + (lanef(x, 32) + lanef(x, 48));
}
// max / sum with the lane 32 apart (the two halves of a wave): v_permlane32_swap (gfx950) hands
// every lane both x[l mod 32] and x[32 + l mod 32] without an LDS round trip (ds_bpermute);
// the sum is lo + hi in every lane (the __shfl_xor form gave hi + lo in the upper half: equal)
AVSR_DEV float xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
AVSR_DEV float xor32_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
AVSR_DEV float wave_max(float x) {
  x = fmaxf(x, rorf<8>(x)); x = fmaxf(x, rorf<4>(x)); x = fmaxf(x, rorf<2>(x)); x = fmaxf(x, rorf<1>(x));
  return fmaxf(fmaxf(lanef(x, 0), lanef(x, 16)), fmaxf(lanef(x, 32), lanef(x, 48)));
}

// ---- counter-based dropout stream: keep(seed, idx) with P(keep) = 1 - p ------------
// Two murmur3 finalisers over (seed, idx) -> 32-bit uniform (~16 VALU per element; the
// outer mix of (hi, seed_hi) is loop-invariant in every caller's inner loop). Identical
// in forward and backward so no mask is ever stored (the backward recomputes it).
AVSR_DEV uint32_t fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85EBCA6Bu;
  h ^= h >> 13; h *= 0xC2B2AE35u;
  return h ^ (h >> 16);
}
// mix32 = mix32_lo(mix32_hi(seed, hi), lo): callers whose index range shares one high word
// hoist mix32_hi and pay one finaliser per element (bit-identical mask)
AVSR_DEV uint32_t mix32_hi(uint64_t seed, uint32_t hi) {
  return (uint32_t)seed ^ fmix32(hi ^ (uint32_t)(seed >> 32) ^ 0x68E31DA4u);
}
AVSR_DEV uint32_t mix32_lo(uint32_t pre, uint32_t lo) { return fmix32((lo * 0x9E3779B1u) ^ pre); }
AVSR_DEV uint32_t mix32(uint64_t seed, uint64_t idx) {
  return mix32_lo(mix32_hi(seed, (uint32_t)(idx >> 32)), (uint32_t)idx);
}
// Elementwise dropout (GEMM epilogues, ew_bwd / dropout_fwd, the LayerNorm backward's fused
// ew_bwd): element idx reads the 16-bit half (idx & 1) of the hash of PAIR idx >> 1 — one
// finaliser per two elements, the scheme of the attention kernels' AttnDrop — and is dropped iff
// that half < thr = round(p * 65536) (p_eff within 8e-6 of p); kept values are scaled by
// 65536 / (65536 - thr), so E[mask] = 1 exactly. Every site evaluates this same function of
// (seed, idx): masks are recomputed, never stored.
AVSR_DEV uint32_t drop_thr16(float p) { return (uint32_t)(p * 65536.f + 0.5f); }
AVSR_DEV float drop_keep_scale(uint32_t thr) { return thr < 65536u ? 65536.f / (float)(65536u - thr) : 0.f; }
AVSR_DEV uint32_t drop_half(uint32_t h, bool odd) { return odd ? (h >> 16) : (h & 0xFFFFu); }

AVSR_DEV float drop_scale(float p, uint64_t seed, uint64_t idx) {
  // returns 0 for dropped, 65536 / (65536 - thr) for kept
  const uint32_t thr = drop_thr16(p);
  return drop_half(mix32(seed, idx >> 1), idx & 1) >= thr ? drop_keep_scale(thr) : 0.0f;
}

// drop_scale over indices d0 .. d0+7, multiplied into v: for even d0 the 4 pairs are hashed once
// each, with the high-word finaliser shared when they have one high word (same mask as
// drop_scale element by element)
AVSR_DEV void drop8(float p, uint64_t seed, uint64_t d0, float* v) {
  const uint32_t thr = drop_thr16(p);
  const float ks = drop_keep_scale(thr);
  const uint64_t p0 = d0 >> 1;
  const uint32_t lo = (uint32_t)p0;
  if (!(d0 & 1) && lo <= 0xFFFFFFFCu) {
    const uint32_t pre = mix32_hi(seed, (uint32_t)(p0 >> 32));
    const uint32_t g0 = lo * 0x9E3779B1u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t h = fmix32((g0 + (uint32_t)q * 0x9E3779B1u) ^ pre);
      v[2 * q] *= (h & 0xFFFFu) >= thr ? ks : 0.0f;
      v[2 * q + 1] *= (h >> 16) >= thr ? ks : 0.0f;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] *= drop_scale(p, seed, d0 + q);
  }
}

AVSR_DEV float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
AVSR_DEV float gelu_erf_grad(float x) {
  float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}
// bf16 paths: erf by Abramowitz-Stegun 7.1.26 (|err| < 1.5e-7, far below bf16 rounding),
// sharing one exp(-x^2/2) between erf and the GELU derivative's pdf (~14 VALU vs ocml erff)
AVSR_DEV float erf_as(float z, float ez2) {   // ez2 = exp(-z*z)
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, fabsf(z), 1.0f));
  const float p = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f), 0.254829592f);
  return copysignf(fmaf(-p, ez2, 1.0f), z);
}
AVSR_DEV float gelu_fast(float x) {
  const float z = x * 0.70710678118654752f;
  return 0.5f * x * (1.0f + erf_as(z, __expf(-z * z)));
}
AVSR_DEV float gelu_fast_grad(float x) {
  const float z = x * 0.70710678118654752f, e = __expf(-z * z);
  return 0.5f * (1.0f + erf_as(z, e)) + x * 0.39894228040143268f * e;
}
// two elements at a time: the polynomial, the scalings and the final blend in packed fp32
// (v_pk_fma_f32 / v_pk_mul_f32), only rcp and exp per element
typedef float f32x2 __attribute__((ext_vector_type(2)));
AVSR_DEV f32x2 erf_as2(f32x2 z, f32x2 ez2) {
  const f32x2 az = {fabsf(z.x), fabsf(z.y)};
  const f32x2 d = az * 0.3275911f + 1.0f;
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 p = t * 1.061405429f + -1.453152027f;
  p = p * t + 1.421413741f;
  p = p * t + -0.284496736f;
  p = p * t + 0.254829592f;
  const f32x2 r = 1.0f - (p * t) * ez2;
  return f32x2{copysignf(r.x, z.x), copysignf(r.y, z.y)};
}
AVSR_DEV f32x2 exp_negsq2(f32x2 z) {
  const f32x2 q = z * z;
  return f32x2{__expf(-q.x), __expf(-q.y)};
}
AVSR_DEV f32x2 gelu_fast2(f32x2 x) {
  const f32x2 z = x * 0.70710678118654752f;
  const f32x2 hx = x * 0.5f;
  return hx + hx * erf_as2(z, exp_negsq2(z));
}
AVSR_DEV f32x2 gelu_fast_grad2(f32x2 x) {
  const f32x2 z = x * 0.70710678118654752f, e = exp_negsq2(z);
  return 0.5f + 0.5f * erf_as2(z, e) + (x * 0.39894228040143268f) * e;
}
template <typename T> AVSR_DEV float act_fwd_t(int act, float h) {
  if constexpr (sizeof(T) == 2) return act == AVSR_ACT_GELU ? gelu_fast(h) : (act == AVSR_ACT_RELU ? fmaxf(h, 0.f) : h);
  else return act == AVSR_ACT_GELU ? gelu_erf(h) : (act == AVSR_ACT_RELU ? fmaxf(h, 0.f) : h);
}
template <typename T> AVSR_DEV float act_bwd_t(int act, float h) {
  if constexpr (sizeof(T) == 2) return act == AVSR_ACT_GELU ? gelu_fast_grad(h) : (act == AVSR_ACT_RELU ? (h > 0.f ? 1.f : 0.f) : 1.f);
  else return act == AVSR_ACT_GELU ? gelu_erf_grad(h) : (act == AVSR_ACT_RELU ? (h > 0.f ? 1.f : 0.f) : 1.f);
}
AVSR_DEV float act_fwd(int act, float h) {
  return act == AVSR_ACT_GELU ? gelu_erf(h) : (act == AVSR_ACT_RELU ? fmaxf(h, 0.f) : h);
}
AVSR_DEV float act_bwd(int act, float h) {
  return act == AVSR_ACT_GELU ? gelu_erf_grad(h) : (act == AVSR_ACT_RELU ? (h > 0.f ? 1.f : 0.f) : 1.f);
}

// split an fp32 fragment into bf16 hi + lo parts (parity mode: 3 MFMA products)
AVSR_DEV void split8(const float* x, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    bf16 h = (bf16)x[j];
    hi[j] = h;
    lo[j] = (bf16)(x[j] - (float)h);
  }
}

// v_mfma_f32_16x16x32_bf16: lane l holds A[row l&15][k 8(l>>4)..+7], B[k 8(l>>4)..+7][col l&15];
// C/D: 4 registers, C[row 4(l>>4) + r][col l&15]
AVSR_DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
AVSR_DEV f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// kernel-selection options (avsr_set_option, version.hip); the library reads no environment
int64_t avsr_opt(int option);

#define AVSR_CHECK_LAUNCH() do { hipError_t e_ = hipGetLastError(); if (e_ != hipSuccess) return (int)e_; } while (0)

static inline int avsr_aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// ---- 16-byte vector load/store of VE = 16/sizeof(T) elements as floats ----------------
template <typename T> struct VecW { static constexpr int VE = 16 / (int)sizeof(T); };
template <typename T> AVSR_DEV void ldv(const T* p, float* o) {
  if constexpr (sizeof(T) == 2) {
    bf16x8 v = *(const bf16x8*)p;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (float)v[j];
  } else {
    f32x4 v = *(const f32x4*)p;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = v[j];
  }
}
template <typename T> AVSR_DEV void stv(T* p, const float* o) {
  if constexpr (sizeof(T) == 2) {
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (bf16)o[j];
    *(bf16x8*)p = v;
  } else {
    f32x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = o[j];
    *(f32x4*)p = v;
  }
}
// q = n / d for 0 <= n < 2^31 (Granlund-Montgomery round-up multiplier)
struct FastDiv {
  uint32_t d, m, s;
};
static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f; f.d = d; uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}
AVSR_DEV uint32_t fdiv(uint32_t n, const FastDiv& f) { return (__umulhi(n, f.m) + n) >> f.s; }

// grid-stride launch size for memory-bound kernels (<= 8 blocks of 256 per CU)
static inline int avsr_grid(long work, int per_block = 256, int cap = 2048) {
  long g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (int)(g < cap ? g : cap);
}

// Column sums of a row-block partial workspace: out[c] += sum_b ws[b*ld + c] for c < N, or,
// when out1 != nullptr, columns [N1, N) go to out1[c - N1] (LayerNorm dgamma/dbeta in one
// launch). Block = 32 columns (one 128-byte line per row) x 32 row lanes (1024 threads): each
// thread adds nb/32 partial rows with four independent accumulators, then the row lanes are
// summed in a fixed order (deterministic). (8 row lanes: ~6.7 us per 256 x 1024 workspace,
// a latency-bound chain of 32 loads per thread.)
constexpr int COLSUM_THREADS = 1024;
AVSR_DEV void colsum_block(const float* ws, int nb, int64_t ld, int N, float* out, int N1, float* out1, int cb) {
  __shared__ float red[32][33];
  const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c = cb * 32 + cl;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (c < N) {
    int b = rl;
    for (; b + 96 < nb; b += 128) {
      s0 += ws[(int64_t)b * ld + c];
      s1 += ws[(int64_t)(b + 32) * ld + c];
      s2 += ws[(int64_t)(b + 64) * ld + c];
      s3 += ws[(int64_t)(b + 96) * ld + c];
    }
    for (; b < nb; b += 32) s0 += ws[(int64_t)b * ld + c];
  }
  red[rl][cl] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (rl == 0 && c < N) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) s += red[i][cl];
    if (out1 && c >= N1) out1[c - N1] += s;
    else out[c] += s;
  }
}
static __global__ __launch_bounds__(COLSUM_THREADS) void colsum_finalize_kernel(const float* ws, int nb, int64_t ld, int N,
                                                                                 float* out, int N1, float* out1) {
  colsum_block(ws, nb, ld, N, out, N1, out1, blockIdx.x);
}
static inline dim3 colsum_grid(int N) { return dim3((N + 31) / 32); }

// The row-block partial workspaces of bias / LayerNorm parameter gradients are finalised by
// colsum_launch: at once, or — between avsr_colsum_defer(1) and avsr_colsum_flush() — queued
// host-side and reduced by ONE batched launch per flush (misc.hip). Callers keep the
// workspaces alive until the flush.
int colsum_launch(const float* ws, int nb, int64_t ld, int N, float* out, int N1, float* out1, hipStream_t st);
