// Elementwise / data-movement kernels around the GEMMs (declarations, reference call sites:
// include/avsr_hip.h): bias-gradient column sums with dropout/activation masks, dropout,
// padded-frame masking, decoder embedding + positional encoding, casts, stem/audio input
// packing, pos-conv weight norm, and the fused clip-grad-norm + AdamW step.
// All HBM-bound: 16-byte vectors where the layout allows, grid-stride loops.
#include "common.h"
#include <hip/hip_ext.h>
#include <vector>

namespace {

struct EwArgs {
  int rows, N;
  const void* dy; int64_t lddy; void* out; int64_t ldout;
  const void* gate; int64_t ldgate; int act;
  float drop_p; uint64_t seed; float alpha; float* db; float* ws;
};

// block = 64 column vectors x 4 row lanes over a chunk of rows; column partial sums are
// reduced in LDS and written (plain stores) to ws[row_block][N], then colsum_finalize adds
// the row-block partials into db: no atomic contention, deterministic order.
template <typename T>
__global__ __launch_bounds__(256) void ew_bwd_kernel(EwArgs a) {
  constexpr int VE = VecW<T>::VE;
  __shared__ float red[4 * 64 * 8];
  const int nv = a.N / VE;
  const int cvl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int cv = blockIdx.x * 64 + cvl;
  const int chunk = (a.rows + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * chunk, r1 = min(a.rows, r0 + chunk);
  float acc[VE];
#pragma unroll
  for (int j = 0; j < VE; ++j) acc[j] = 0.f;
  if (cv < nv) {
    for (int r = r0 + rl; r < r1; r += 4) {
      float d[VE], g[VE];
      ldv((const T*)a.dy + (int64_t)r * a.lddy + cv * VE, d);
      if (a.gate) ldv((const T*)a.gate + (int64_t)r * a.ldgate + cv * VE, g);
#pragma unroll
      for (int j = 0; j < VE; ++j) d[j] *= a.alpha;
      if (a.drop_p > 0.f) {
        const uint64_t i0 = (uint64_t)r * a.N + cv * VE;
        if constexpr (VE == 8) drop8(a.drop_p, a.seed, i0, d);
        else {
#pragma unroll
          for (int j = 0; j < VE; ++j) d[j] *= drop_scale(a.drop_p, a.seed, i0 + j);
        }
      }
#pragma unroll
      for (int j = 0; j < VE; ++j) {
        float v = d[j];
        if (a.gate) v *= act_bwd_t<T>(a.act, g[j]);
        acc[j] += v;
        d[j] = v;
      }
      if (a.out) stv((T*)a.out + (int64_t)r * a.ldout + cv * VE, d);
    }
  }
  if (!a.db) return;
#pragma unroll
  for (int j = 0; j < VE; ++j) red[(rl * 64 + cvl) * VE + j] = acc[j];
  __syncthreads();
  if (rl == 0 && cv < nv) {
#pragma unroll
    for (int j = 0; j < VE; ++j) {
      const float t = red[(0 * 64 + cvl) * VE + j] + red[(1 * 64 + cvl) * VE + j] + red[(2 * 64 + cvl) * VE + j] +
                      red[(3 * 64 + cvl) * VE + j];
      a.ws[(int64_t)blockIdx.y * a.N + cv * VE + j] = t;
    }
  }
}


template <typename T>
__global__ __launch_bounds__(256) void mask_rows_kernel(int B, int T_, int N, T* x, int64_t ldx, const int* len) {
  constexpr int VE = VecW<T>::VE;
  const int nv = N / VE;
  const int64_t total = (int64_t)B * T_ * nv;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t row = i / nv;
    const int b = (int)(row / T_), t = (int)(row % T_);
    if (t >= len[b]) {
      float z[VE];
#pragma unroll
      for (int j = 0; j < VE; ++j) z[j] = 0.f;
      stv(x + row * ldx + (i % nv) * VE, z);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void embed_kernel(avsr_embed_params p, int bwd) {
  constexpr int VE = VecW<T>::VE;
  const int nv = p.D / VE;
  const int64_t total = (int64_t)p.rows * nv;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int r = (int)(i / nv), d0 = (int)(i % nv) * VE;
    const int tok = p.tok[r];
    const int pos = p.pe_row ? p.pe_row[0] : r % p.L;
    if (!bwd) {
      float e[VE], o[VE];
      ldv((const T*)p.table + (int64_t)tok * p.D + d0, e);
#pragma unroll
      for (int j = 0; j < VE; ++j) {
        float v = e[j] * p.scale + p.pe[(int64_t)pos * p.D + d0 + j];
        if (p.drop_p > 0.f) v *= drop_scale(p.drop_p, p.seed, (uint64_t)r * p.D + d0 + j);
        o[j] = v;
      }
      stv((T*)p.y + (int64_t)r * p.D + d0, o);
    }
  }
}

// embedding backward without atomics (deterministic): block r owns the table row of token
// tok[r] iff r is that token's first occurrence; it adds the row gradients of every occurrence
// in row order. Other blocks exit.
template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_kernel(avsr_embed_params p) {
  constexpr int VE = VecW<T>::VE;
  const int r = blockIdx.x;
  const int tok = p.tok[r];
  __shared__ int seen;
  if (threadIdx.x == 0) seen = 0;
  __syncthreads();
  for (int q = threadIdx.x; q < r; q += 256)
    if (p.tok[q] == tok) seen = 1;
  __syncthreads();
  if (seen) return;
  const int nv = p.D / VE;
  for (int c = threadIdx.x; c < nv; c += 256) {
    const int d0 = c * VE;
    float acc[VE];
#pragma unroll
    for (int j = 0; j < VE; ++j) acc[j] = 0.f;
    for (int q = r; q < p.rows; ++q) {
      if (p.tok[q] != tok) continue;
      float g[VE];
      ldv((const T*)p.dy + (int64_t)q * p.D + d0, g);
#pragma unroll
      for (int j = 0; j < VE; ++j) {
        float v = g[j] * p.scale;
        if (p.drop_p > 0.f) v *= drop_scale(p.drop_p, p.seed, (uint64_t)q * p.D + d0 + j);
        acc[j] += v;
      }
    }
    float* dt = p.dtable + (int64_t)tok * p.D + d0;
#pragma unroll
    for (int j = 0; j < VE; ++j) dt[j] += acc[j];
  }
}

template <typename S, typename D>
__global__ __launch_bounds__(256) void cast_kernel(int rows, int cols, const S* src, int64_t lds, D* dst,
                                                   int64_t ldd, float alpha, float beta) {
  const int64_t c0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (c0 >= cols) return;
  for (int r = blockIdx.y; r < rows; r += gridDim.y) {
    const S* s = src + (int64_t)r * lds + c0;
    D* d = dst + (int64_t)r * ldd + c0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (c0 + q < cols) {
        float v = alpha * to_f(s[q]);
        if (beta != 0.f) v += beta * to_f(d[q]);
        d[q] = from_f<D>(v);
      }
    }
  }
}

// contiguous n-element cast, 8 elements per thread per iteration (two 16-byte fp32 loads,
// one 16-byte bf16 store), grid-stride: the arena's fp32 master -> bf16 shadow refresh
// (428 M parameters: 1.7 GB read + 0.86 GB written, HBM-bound).
__global__ __launch_bounds__(256) void cast_flat_f32_bf16_kernel(int64_t n8, const float4* __restrict__ src,
                                                                 bf16x8* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const float4 a = src[2 * i], b = src[2 * i + 1];
    bf16x8 o;
    o[0] = (bf16)a.x; o[1] = (bf16)a.y; o[2] = (bf16)a.z; o[3] = (bf16)a.w;
    o[4] = (bf16)b.x; o[5] = (bf16)b.y; o[6] = (bf16)b.z; o[7] = (bf16)b.w;
    dst[i] = o;
  }
}

// bf16 -> fp32 over 8-element vectors (the compressed gradient all-reduce's decompress,
// parallel.GradReducer(compress="bf16"))
__global__ __launch_bounds__(256) void cast_flat_bf16_f32_kernel(int64_t n8, const bf16x8* __restrict__ src,
                                                                 float4* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const bf16x8 v = src[i];
    dst[2 * i] = float4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
    dst[2 * i + 1] = float4{(float)v[4], (float)v[5], (float)v[6], (float)v[7]};
  }
}

// grid (clip x chunk of PACK_TC frames, pixel blocks): a thread walks one pixel through a
// chunk of output frames, loading each of the chunk's PACK_TC + 4 source frames once (all
// loads issued first) instead of 5 loads per output (the source video is read ~1.25x, not 5x)
constexpr int PACK_TC = 16;
template <typename T>
__global__ __launch_bounds__(256) void stem_pack_kernel(int B, int T_, const float* video, T* out) {
  constexpr int HW = 88 * 88;
  const int pix = blockIdx.y * 256 + threadIdx.x;
  if (pix >= HW) return;
  const int nch = (T_ + PACK_TC - 1) / PACK_TC;
  const int b = blockIdx.x / nch, t0 = (blockIdx.x - b * nch) * PACK_TC;
  const float* src = video + (int64_t)b * T_ * HW + pix;
  float f[PACK_TC + 4];
#pragma unroll
  for (int k = 0; k < PACK_TC + 4; ++k) {
    const int tt = t0 + k - 2;
    f[k] = (tt >= 0 && tt < T_) ? src[(int64_t)tt * HW] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < PACK_TC; ++u) {
    const int t = t0 + u;
    if (t >= T_) break;
    float o[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) o[c] = c < 5 ? f[u + c] : 0.f;
    T* dst = out + (((int64_t)b * T_ + t) * HW + pix) * 8;
    if constexpr (sizeof(T) == 2) {
      stv(dst, o);
    } else {
      stv(dst, o);
      stv(dst + 4, o + 4);
    }
  }
}

template <typename T>
__global__ void stem_wpack_kernel(const float* w, T* wp) {
  const int i = blockIdx.x * 256 + threadIdx.x;   // [64][7][7][8]
  if (i >= 64 * 49 * 8) return;
  const int c = i % 8, khw = (i / 8) % 49, o = i / (49 * 8);
  wp[i] = from_f<T>(c < 5 ? w[(o * 5 + c) * 49 + khw] : 0.f);
}

__global__ void stem_wgrad_unpack_kernel(const float* gp, float* gw) {
  const int i = blockIdx.x * 256 + threadIdx.x;   // [64][5][7][7]
  if (i >= 64 * 5 * 49) return;
  const int khw = i % 49, c = (i / 49) % 5, o = i / (5 * 49);
  gw[i] += gp[(o * 49 + khw) * 8 + c];
}

template <typename T>
__global__ __launch_bounds__(256) void audio_pack_kernel(int B, int F, int T_, const float* a, T* out) {
  const int64_t total = (int64_t)B * T_ * F;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int f = (int)(i % F);
    const int64_t bt = i / F;
    const int b = (int)(bt / T_), t = (int)(bt % T_);
    out[i] = from_f<T>(a[((int64_t)b * F + f) * T_ + t]);
  }
}

// norm[k] = ||v[:, k, :]||  (v stored [O][K][C]); one block per k
__global__ __launch_bounds__(256) void wn_norm_kernel(int O, int K, int C, const float* v, const float* dw,
                                                      float* out) {
  const int k = blockIdx.x;
  float s = 0.f;
  for (int i = threadIdx.x; i < O * C; i += 256) {
    const int o = i / C, c = i % C;
    const int64_t idx = ((int64_t)o * K + k) * C + c;
    s += dw ? dw[idx] * v[idx] : v[idx] * v[idx];
  }
  s = wave_sum(s);
  __shared__ float sh[4];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t = sh[0] + sh[1] + sh[2] + sh[3];
    out[k] = dw ? t : sqrtf(t);
  }
}

// same reduction with 16-byte loads and 16 waves per k (C % 4 == 0, v / dw 16-byte aligned):
// the 128 blocks of the pos-conv weight stream 256 KB each instead of one 4-byte load per thread
// and iteration behind a runtime division (125 -> ~15 us per call)
__global__ __launch_bounds__(1024) void wn_norm4_kernel(int O, int K, int C, const float* v, const float* dw,
                                                        float* out) {
  const int k = blockIdx.x, c4n = C >> 2, per = O * c4n;
  float s = 0.f;
#pragma unroll 4
  for (int i = threadIdx.x; i < per; i += 1024) {
    const int o = i / c4n, c4 = i - o * c4n;
    const int64_t idx = ((int64_t)o * K + k) * C + 4 * c4;
    const f32x4 a = *(const f32x4*)(v + idx);
    const f32x4 b = dw ? *(const f32x4*)(dw + idx) : a;
    s += a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
  }
  s = wave_sum(s);
  __shared__ float sh[16];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += sh[w];
    out[k] = dw ? t : sqrtf(t);
  }
}

static void wn_norm_launch(int O, int K, int C, const float* v, const float* dw, float* out, hipStream_t st) {
  if (C % 4 == 0 && avsr_aligned16(v) && (!dw || avsr_aligned16(dw)))
    hipLaunchKernelGGL(wn_norm4_kernel, dim3(K), dim3(1024), 0, st, O, K, C, v, dw, out);
  else
    hipLaunchKernelGGL(wn_norm_kernel, dim3(K), dim3(256), 0, st, O, K, C, v, dw, out);
}

template <typename T>
__global__ __launch_bounds__(256) void wn_apply_kernel(int O, int K, int C, const float* v, const float* g,
                                                       const float* norm, T* w) {
  const int64_t total = (int64_t)O * K * C;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int k = (int)((i / C) % K);
    w[i] = from_f<T>(g[k] * v[i] / norm[k]);
  }
}

__global__ __launch_bounds__(256) void wn_bwd_kernel(int O, int K, int C, const float* v, const float* g,
                                                     const float* norm, const float* dw, const float* s,
                                                     float* dv) {
  const int64_t total = (int64_t)O * K * C;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int k = (int)((i / C) % K);
    const float n = norm[k];
    dv[i] += g[k] / n * dw[i] - g[k] * s[k] / (n * n * n) * v[i];
  }
}

__global__ void wn_dg_kernel(int K, const float* s, const float* norm, float* dg) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k < K) dg[k] += s[k] / norm[k];
}

// sum of squares in two deterministic passes: per-block partials -> ws, then one block sums
// them in a fixed order and adds the total to *out
__global__ __launch_bounds__(256) void sumsq_kernel(const float* x, int64_t n, float* ws) {
  float s = 0.f;
  const int64_t n4 = n / 4;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const f32x4 v = ((const f32x4*)x)[i];
    s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
  }
  if (blockIdx.x == 0)
    for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += 256) s += x[i] * x[i];
  s = wave_sum(s);
  __shared__ float sh[4];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) ws[blockIdx.x] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

__global__ __launch_bounds__(256) void sumsq_final_kernel(const float* ws, int nb, float* out) {
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += 256) s += ws[i];
  s = wave_sum(s);
  __shared__ float sh[4];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *out += (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

struct AdamCoef { float coef, step, rbc2, decay; };

AVSR_DEV AdamCoef adam_coef(const avsr_adamw_params& p) {
  AdamCoef c;
  c.coef = p.grad_scale;
  if (p.sumsq) {
    const float tn = sqrtf(*p.sumsq) * p.grad_scale;
    c.coef *= fminf(1.f, p.max_norm / (tn + 1e-6f));
  }
  c.step = p.lr / p.bias_corr1;
  c.rbc2 = 1.f / sqrtf(p.bias_corr2);
  c.decay = p.lr * p.weight_decay;
  return c;
}

// one element (torch.optim.AdamW arithmetic: decoupled decay, then the moment update)
AVSR_DEV float adam_elem(const avsr_adamw_params& p, const AdamCoef& c, float g, float w, float& m, float& v) {
  g *= c.coef;
  w -= c.decay * w;
  m = p.beta1 * m + (1.f - p.beta1) * g;
  v = p.beta2 * v + (1.f - p.beta2) * g * g;
  return w - c.step * m / (sqrtf(v) * c.rbc2 + p.eps);
}

// Four elements per thread and iteration with 16-byte loads / stores: elements [0, head) and
// [head + 4*nv, n) (fewer than 4 each, to reach / past the 16-byte boundary) by block 0.
template <typename S>
__global__ __launch_bounds__(256) void adamw_kernel(avsr_adamw_params p, int head, int64_t nv) {
  const AdamCoef c = adam_coef(p);
  if (blockIdx.x == 0 && threadIdx.x < 8) {
    const int t = threadIdx.x;
    const int64_t i = t < 4 ? t : head + 4 * nv + (t - 4);
    if ((t < 4 && t < head) || (t >= 4 && i < p.n)) {
      float m = p.exp_avg[i], v = p.exp_avg_sq[i];
      const float w = adam_elem(p, c, p.grad[i], p.param[i], m, v);
      p.exp_avg[i] = m; p.exp_avg_sq[i] = v; p.param[i] = w;
      if (p.shadow) ((S*)p.shadow)[i] = from_f<S>(w);
      if (p.grad_clear) p.grad_clear[i] = 0.f;
    }
  }
  float* P = p.param + head; const float* G = p.grad + head;
  float* M = p.exp_avg + head; float* V = p.exp_avg_sq + head;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < nv; q += (int64_t)gridDim.x * 256) {
    const f32x4 g = *(const f32x4*)(G + 4 * q);
    f32x4 w = *(const f32x4*)(P + 4 * q), m = *(const f32x4*)(M + 4 * q), v = *(const f32x4*)(V + 4 * q);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float mj = m[j], vj = v[j];
      w[j] = adam_elem(p, c, g[j], w[j], mj, vj);
      m[j] = mj; v[j] = vj;
    }
    *(f32x4*)(P + 4 * q) = w; *(f32x4*)(M + 4 * q) = m; *(f32x4*)(V + 4 * q) = v;
    if (p.grad_clear) *(f32x4*)(p.grad_clear + head + 4 * q) = f32x4{0.f, 0.f, 0.f, 0.f};
    if (p.shadow) {
      S* sh = (S*)p.shadow + head + 4 * q;
      if constexpr (sizeof(S) == 2) {
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (bf16)w[j];
        *(bf16x4*)sh = o;
      } else {
        *(f32x4*)sh = w;
      }
    }
  }
}

EwArgs ew_args(const avsr_ew_params* p) {
  EwArgs a;
  a.rows = p->rows; a.N = p->N; a.dy = p->dy; a.lddy = p->lddy; a.out = p->out; a.ldout = p->ldout;
  a.gate = p->gate; a.ldgate = p->ldgate; a.act = p->act; a.drop_p = p->drop_p; a.seed = p->seed;
  a.alpha = p->alpha; a.db = p->db; a.ws = p->ws;
  return a;
}

int ew_launch(const avsr_ew_params* p, hipStream_t st) {
  const int ve = p->dtype == AVSR_BF16 ? 8 : 4;
  if (p->N % ve) return AVSR_E_SHAPE;
  if (p->rows == 0) return 0;
  if (p->db && !p->ws) return AVSR_E_ARG;
  const int nv = p->N / ve;
  dim3 grid((nv + 63) / 64, 1);
  // ~4096 blocks (16 waves per CU) for latency hiding; at most AVSR_EW_ROWBLOCKS row blocks
  // of column partials for colsum_finalize
  int gy = 4096 / (int)grid.x;
  gy = gy < 16 ? 16 : (gy > AVSR_EW_ROWBLOCKS ? AVSR_EW_ROWBLOCKS : gy);
  gy = gy > p->rows ? p->rows : gy;
  grid.y = gy;
  EwArgs a = ew_args(p);
  if (p->dtype == AVSR_BF16) hipLaunchKernelGGL(ew_bwd_kernel<bf16>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(ew_bwd_kernel<float>, grid, dim3(256), 0, st, a);
  AVSR_CHECK_LAUNCH();
  if (p->db) return colsum_launch((const float*)p->ws, (int)grid.y, (int64_t)p->N, p->N, p->db, 0, nullptr, st);
  return 0;
}

// ---- deferred column-sum finalisation (one launch per flush) ----------------------------
constexpr int COLSUM_BATCH = 32;
struct ColsumBatch {
  const float* ws[COLSUM_BATCH]; float* out[COLSUM_BATCH]; float* out1[COLSUM_BATCH];
  int64_t ld[COLSUM_BATCH]; int nb[COLSUM_BATCH], N[COLSUM_BATCH], N1[COLSUM_BATCH];
};
__global__ __launch_bounds__(COLSUM_THREADS) void colsum_batch_kernel(ColsumBatch b) {
  const int d = blockIdx.y;
  if ((int)blockIdx.x * 32 >= b.N[d]) return;          // block-uniform
  colsum_block(b.ws[d], b.nb[d], b.ld[d], b.N[d], b.out[d], b.N1[d], b.out1[d], blockIdx.x);
}
struct ColsumQueue { bool on = false, inl = false; std::vector<ColsumBatch> full; ColsumBatch cur; int n = 0; int maxn = 0; };
ColsumQueue g_colsum;

}  // namespace

int colsum_launch(const float* ws, int nb, int64_t ld, int N, float* out, int N1, float* out1, hipStream_t st) {
  if (!g_colsum.on || g_colsum.inl) {
    hipLaunchKernelGGL(colsum_finalize_kernel, colsum_grid(N), dim3(COLSUM_THREADS), 0, st, ws, nb, ld, N, out, N1, out1);
    AVSR_CHECK_LAUNCH();
    return 0;
  }
  ColsumQueue& q = g_colsum;
  const int i = q.n % COLSUM_BATCH;
  q.cur.ws[i] = ws; q.cur.nb[i] = nb; q.cur.ld[i] = ld; q.cur.N[i] = N; q.cur.out[i] = out; q.cur.N1[i] = N1;
  q.cur.out1[i] = out1;
  q.n++;
  q.maxn = q.maxn > N ? q.maxn : N;
  if (q.n % COLSUM_BATCH == 0) q.full.push_back(q.cur);
  return 0;
}

extern "C" int avsr_colsum_defer(int on) {
  const int was = g_colsum.on ? 1 : 0;
  g_colsum.on = on != 0;
  if (!g_colsum.on && g_colsum.n) {   // switched off with passes still queued (an aborted step):
    g_colsum.full.clear();            // drop them rather than reduce workspaces that may be gone
    g_colsum.n = 0; g_colsum.maxn = 0;
  }
  return was;
}

extern "C" int avsr_colsum_inline(int on) {
  const int was = g_colsum.inl ? 1 : 0;
  g_colsum.inl = on != 0;
  return was;
}

extern "C" int avsr_colsum_flush(void* stream) {
  ColsumQueue& q = g_colsum;
  hipStream_t st = (hipStream_t)stream;
  const dim3 gx = colsum_grid(q.maxn > 0 ? q.maxn : 1);
  for (const ColsumBatch& b : q.full) hipLaunchKernelGGL(colsum_batch_kernel, dim3(gx.x, COLSUM_BATCH), dim3(COLSUM_THREADS), 0, st, b);
  const int rest = q.n % COLSUM_BATCH;
  if (rest) hipLaunchKernelGGL(colsum_batch_kernel, dim3(gx.x, rest), dim3(COLSUM_THREADS), 0, st, q.cur);
  q.full.clear(); q.n = 0; q.maxn = 0;
  AVSR_CHECK_LAUNCH();
  return 0;
}


extern "C" int avsr_ew_bwd(const avsr_ew_params* p, void* stream) {
  if (!p) return AVSR_E_ARG;
  return ew_launch(p, (hipStream_t)stream);
}

extern "C" int avsr_dropout_fwd(const avsr_ew_params* p, void* stream) {
  if (!p || !p->out) return AVSR_E_ARG;
  avsr_ew_params q = *p;
  q.gate = nullptr; q.db = nullptr;
  return ew_launch(&q, (hipStream_t)stream);
}

extern "C" int avsr_mask_rows(int dtype, int B, int T, int N, void* x, int64_t ldx, const int* len, void* stream) {
  const int ve = dtype == AVSR_BF16 ? 8 : 4;
  if (N % ve || ldx % ve) return AVSR_E_ALIGN;
  const int g = avsr_grid((int64_t)B * T * N / ve);
  if (dtype == AVSR_BF16) hipLaunchKernelGGL(mask_rows_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, B, T, N, (bf16*)x, ldx, len);
  else hipLaunchKernelGGL(mask_rows_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, B, T, N, (float*)x, ldx, len);
  AVSR_CHECK_LAUNCH();
  return 0;
}

static int embed_launch(const avsr_embed_params* p, int bwd, hipStream_t st) {
  const int ve = p->dtype == AVSR_BF16 ? 8 : 4;
  if (p->D % ve) return AVSR_E_SHAPE;
  if (p->rows <= 0) return 0;
  if (bwd) {
    if (p->dtype == AVSR_BF16) hipLaunchKernelGGL(embed_bwd_kernel<bf16>, dim3(p->rows), dim3(256), 0, st, *p);
    else hipLaunchKernelGGL(embed_bwd_kernel<float>, dim3(p->rows), dim3(256), 0, st, *p);
    AVSR_CHECK_LAUNCH();
    return 0;
  }
  const int g = avsr_grid((int64_t)p->rows * p->D / ve);
  if (p->dtype == AVSR_BF16) hipLaunchKernelGGL(embed_kernel<bf16>, dim3(g), dim3(256), 0, st, *p, bwd);
  else hipLaunchKernelGGL(embed_kernel<float>, dim3(g), dim3(256), 0, st, *p, bwd);
  AVSR_CHECK_LAUNCH();
  return 0;
}
extern "C" int avsr_embed_fwd(const avsr_embed_params* p, void* stream) { return p ? embed_launch(p, 0, (hipStream_t)stream) : AVSR_E_ARG; }
extern "C" int avsr_embed_bwd(const avsr_embed_params* p, void* stream) { return p ? embed_launch(p, 1, (hipStream_t)stream) : AVSR_E_ARG; }

extern "C" int avsr_cast(int sd, int dd, int rows, int cols, const void* src, int64_t lds, void* dst, int64_t ldd,
                         float alpha, float beta, void* stream);

extern "C" int avsr_cast_flat(int sd, int dd, int64_t n, const void* src, void* dst, void* stream) {
  if (n <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (sd == AVSR_F32 && dd == AVSR_BF16 && n % 8 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0) {
    const int64_t n8 = n / 8;
    int64_t g = (n8 + 255) / 256;
    g = g > 256 * 32 ? 256 * 32 : g;           // 32 waves-worth of blocks per CU, grid-stride
    hipLaunchKernelGGL(cast_flat_f32_bf16_kernel, dim3((unsigned)g), dim3(256), 0, st, n8, (const float4*)src, (bf16x8*)dst);
    AVSR_CHECK_LAUNCH();
    return 0;
  }
  if (sd == AVSR_BF16 && dd == AVSR_F32 && n % 8 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0) {
    const int64_t n8 = n / 8;
    int64_t g = (n8 + 255) / 256;
    g = g > 256 * 32 ? 256 * 32 : g;
    hipLaunchKernelGGL(cast_flat_bf16_f32_kernel, dim3((unsigned)g), dim3(256), 0, st, n8, (const bf16x8*)src, (float4*)dst);
    AVSR_CHECK_LAUNCH();
    return 0;
  }
  // general case: a [rows][4096] view of the flat buffer plus a tail row
  const int64_t cols = 4096, rows = n / cols, tail = n - rows * cols;
  const size_t es = sd == AVSR_F32 ? 4 : 2, ed = dd == AVSR_F32 ? 4 : 2;
  if (rows > 0) {
    const int rc = avsr_cast(sd, dd, (int)rows, (int)cols, src, cols, dst, cols, 1.f, 0.f, stream);
    if (rc) return rc;
  }
  if (tail > 0) return avsr_cast(sd, dd, 1, (int)tail, (const char*)src + rows * cols * es, tail,
                                 (char*)dst + rows * cols * ed, tail, 1.f, 0.f, stream);
  return 0;
}

extern "C" int avsr_cast(int sd, int dd, int rows, int cols, const void* src, int64_t lds, void* dst, int64_t ldd,
                         float alpha, float beta, void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  const int64_t gx = ((int64_t)cols + 1023) / 1024;
  int64_t gy = 4096 / gx;
  gy = gy < 1 ? 1 : (gy > rows ? rows : gy);
  gy = gy > 65535 ? 65535 : gy;
  const dim3 g((unsigned)gx, (unsigned)gy);
  hipStream_t st = (hipStream_t)stream;
  if (sd == AVSR_F32 && dd == AVSR_BF16) hipLaunchKernelGGL((cast_kernel<float, bf16>), dim3(g), dim3(256), 0, st, rows, cols, (const float*)src, lds, (bf16*)dst, ldd, alpha, beta);
  else if (sd == AVSR_F32 && dd == AVSR_F32) hipLaunchKernelGGL((cast_kernel<float, float>), dim3(g), dim3(256), 0, st, rows, cols, (const float*)src, lds, (float*)dst, ldd, alpha, beta);
  else if (sd == AVSR_BF16 && dd == AVSR_F32) hipLaunchKernelGGL((cast_kernel<bf16, float>), dim3(g), dim3(256), 0, st, rows, cols, (const bf16*)src, lds, (float*)dst, ldd, alpha, beta);
  else if (sd == AVSR_BF16 && dd == AVSR_BF16) hipLaunchKernelGGL((cast_kernel<bf16, bf16>), dim3(g), dim3(256), 0, st, rows, cols, (const bf16*)src, lds, (bf16*)dst, ldd, alpha, beta);
  else return AVSR_E_DTYPE;
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_stem_pack(int dtype, int B, int T, const float* video, void* out, void* stream) {
  if ((int64_t)B * T == 0) return 0;
  const int64_t nx = (int64_t)B * ((T + PACK_TC - 1) / PACK_TC);
  if (nx > 0x7fffffffLL) return AVSR_E_SHAPE;
  const dim3 g((unsigned)nx, (88 * 88 + 255) / 256);
  if (dtype == AVSR_BF16) hipLaunchKernelGGL(stem_pack_kernel<bf16>, g, dim3(256), 0, (hipStream_t)stream, B, T, video, (bf16*)out);
  else hipLaunchKernelGGL(stem_pack_kernel<float>, g, dim3(256), 0, (hipStream_t)stream, B, T, video, (float*)out);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_stem_wpack(int dtype, const float* w, void* wp, void* stream) {
  const int g = (64 * 49 * 8 + 255) / 256;
  if (dtype == AVSR_BF16) hipLaunchKernelGGL(stem_wpack_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, w, (bf16*)wp);
  else hipLaunchKernelGGL(stem_wpack_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, w, (float*)wp);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_stem_wgrad_unpack(const float* gp, float* gw, void* stream) {
  hipLaunchKernelGGL(stem_wgrad_unpack_kernel, dim3((64 * 5 * 49 + 255) / 256), dim3(256), 0, (hipStream_t)stream, gp, gw);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_audio_pack(int dtype, int B, int F, int T, const float* audio, void* out, void* stream) {
  const int g = avsr_grid((int64_t)B * T * F);
  if (dtype == AVSR_BF16) hipLaunchKernelGGL(audio_pack_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, B, F, T, audio, (bf16*)out);
  else hipLaunchKernelGGL(audio_pack_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, B, F, T, audio, (float*)out);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_weightnorm_fwd(int dtype, int O, int K, int C, const float* v, const float* g, float* norm,
                                   void* w, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  wn_norm_launch(O, K, C, v, nullptr, norm, st);
  const int gr = avsr_grid((int64_t)O * K * C);
  if (dtype == AVSR_BF16) hipLaunchKernelGGL(wn_apply_kernel<bf16>, dim3(gr), dim3(256), 0, st, O, K, C, v, g, norm, (bf16*)w);
  else hipLaunchKernelGGL(wn_apply_kernel<float>, dim3(gr), dim3(256), 0, st, O, K, C, v, g, norm, (float*)w);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_weightnorm_bwd(int O, int K, int C, const float* v, const float* g, const float* norm,
                                   const float* dw, float* dv, float* dg, float* scratch, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  wn_norm_launch(O, K, C, v, dw, scratch, st);
  hipLaunchKernelGGL(wn_dg_kernel, dim3((K + 255) / 256), dim3(256), 0, st, K, (const float*)scratch, norm, dg);
  hipLaunchKernelGGL(wn_bwd_kernel, dim3(avsr_grid((int64_t)O * K * C)), dim3(256), 0, st, O, K, C, v, g, norm, dw,
                     (const float*)scratch, dv);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_sumsq(const float* x, int64_t n, float* out, float* ws, void* stream) {
  if (!avsr_aligned16(x)) return AVSR_E_ALIGN;
  if (!out || !ws) return AVSR_E_ARG;
  const int nb = avsr_grid(n / 4 + 1, 256, AVSR_SUMSQ_WS);
  hipLaunchKernelGGL(sumsq_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, x, n, ws);
  AVSR_CHECK_LAUNCH();
  hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, (const float*)ws, nb, out);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_adamw(const avsr_adamw_params* p, void* stream) {
  if (!p) return AVSR_E_ARG;
  if (p->n == 0) return 0;
  // the four fp32 arrays share their offset modulo 16 bytes (one arena index); the shadow must
  // then be 8-byte (bf16) / 16-byte (fp32) aligned at the same element
  const uintptr_t a0 = (uintptr_t)p->param & 15;
  if ((((uintptr_t)p->grad & 15) != a0) || (((uintptr_t)p->exp_avg & 15) != a0) || (((uintptr_t)p->exp_avg_sq & 15) != a0) || (a0 & 3))
    return AVSR_E_ALIGN;
  int head = (int)(((16 - a0) & 15) / 4);
  if (head > p->n) head = (int)p->n;
  const int64_t nv = (p->n - head) / 4;
  const size_t ssz = p->shadow_dtype == AVSR_F32 ? 4 : 2;
  if (p->shadow && (((uintptr_t)p->shadow + head * ssz) & (4 * ssz - 1))) return AVSR_E_ALIGN;
  if (p->max_blocks < 0) return AVSR_E_ARG;
  if (p->grad_clear && p->grad_clear != p->grad) return AVSR_E_ARG;
  const int g = avsr_grid(nv > 0 ? nv : 1, 256, p->max_blocks > 0 && p->max_blocks < 4096 ? p->max_blocks : 4096);
  if (p->shadow_dtype == AVSR_F32) hipLaunchKernelGGL(adamw_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, *p, head, nv);
  else hipLaunchKernelGGL(adamw_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, *p, head, nv);
  AVSR_CHECK_LAUNCH();
  return 0;
}

