// LayerNorm, BatchNorm (+PReLU, +residual), stem max-pool and global average pool —
// forward and backward, for the AVSR hot path (declarations and reference call sites in
// include/avsr_hip.h). All are HBM-bound: 16-byte vector loads/stores, fp32 statistics,
// one pass per tensor where the math allows.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "common.h"

namespace {

// =============================================================== LayerNorm
struct LnArgs {
  int rows, N; float eps;
  const void* x; int64_t ldx; void* y; int64_t ldy;
  const float* gamma; const float* beta; float* mean; float* rstd;
  const void* dy; int64_t lddy; void* dx; int64_t lddx; const void* dres; int64_t lddres;
  float* dgamma; float* dbeta; float* ws;
  void* g; int64_t ldg; float drop_p; uint64_t seed; bool db;   // fused ew_bwd (see avsr_layernorm_params)
};

// one wave per row; lane owns vectors lane, lane+64, ... (VPL of them)
template <typename T, int VPL>
__global__ __launch_bounds__(256) void ln_fwd_kernel(LnArgs a) {
  constexpr int VE = VecW<T>::VE;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= a.rows) return;
  const T* x = (const T*)a.x + (int64_t)row * a.ldx;
  float v[VPL][VE];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = (lane + i * 64) * VE;
    if (c < a.N) ldv(x + c, v[i]);
    else
#pragma unroll
      for (int j = 0; j < VE; ++j) v[i][j] = 0.f;
#pragma unroll
    for (int j = 0; j < VE; ++j) s += v[i][j];
  }
  const float mean = wave_sum(s) / a.N;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = (lane + i * 64) * VE;
    if (c < a.N)
#pragma unroll
      for (int j = 0; j < VE; ++j) { const float d = v[i][j] - mean; q += d * d; }
  }
  const float rstd = rsqrtf(wave_sum(q) / a.N + a.eps);
  T* y = (T*)a.y + (int64_t)row * a.ldy;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = (lane + i * 64) * VE;
    if (c < a.N) {
      float o[VE];
#pragma unroll
      for (int j = 0; j < VE; ++j) o[j] = (v[i][j] - mean) * rstd * a.gamma[c + j] + a.beta[c + j];
      stv(y + c, o);
    }
  }
  if (lane == 0) { a.mean[row] = mean; a.rstd[row] = rstd; }
}

// grid-stride over rows, W waves per block, each wave R rows at a time with all their loads
// (x, dy, dres) issued together; dgamma/dbeta accumulated per lane in registers, summed over
// the block's waves in LDS (dynamic, W*N floats) and written as one partial row per block
// (colsum_finalize adds the blocks)
template <typename T, int VPL, int W, int R>
__global__ __launch_bounds__(64 * W) void ln_bwd_kernel(LnArgs a) {
  constexpr int VE = VecW<T>::VE;
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * W;
  float dg[VPL][VE], db[VPL][VE], gm[VPL][VE], gb[VPL][VE];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = (lane + i * 64) * VE;
#pragma unroll
    for (int j = 0; j < VE; ++j) {
      dg[i][j] = 0.f; db[i][j] = 0.f; gb[i][j] = 0.f; gm[i][j] = c < a.N ? a.gamma[c + j] : 0.f;
    }
  }
  for (int row0 = blockIdx.x * W + (threadIdx.x >> 6); row0 < a.rows; row0 += R * nw) {
    float xv[R][VPL][VE], dv[R][VPL][VE], rv[R][VPL][VE];
    float mean[R], rstd[R];
    bool live[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int row = min(row0 + u * nw, a.rows - 1);
      live[u] = row0 + u * nw < a.rows;
      const T* x = (const T*)a.x + (int64_t)row * a.ldx;
      const T* dy = (const T*)a.dy + (int64_t)row * a.lddy;
      const T* dr = a.dres ? (const T*)a.dres + (int64_t)row * a.lddres : nullptr;
      mean[u] = a.mean[row]; rstd[u] = a.rstd[row];
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        const int c = min((lane + i * 64) * VE, a.N - VE);
        ldv(x + c, xv[u][i]);
        ldv(dy + c, dv[u][i]);
        if (dr) ldv(dr + c, rv[u][i]);
        else
#pragma unroll
          for (int j = 0; j < VE; ++j) rv[u][i][j] = 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < R; ++u) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        const bool cok = (lane + i * 64) * VE < a.N && live[u];
#pragma unroll
        for (int j = 0; j < VE; ++j) {
          const float xh = (xv[u][i][j] - mean[u]) * rstd[u];
          const float g = cok ? dv[u][i][j] * gm[i][j] : 0.f;
          s1 += g;
          s2 += g * xh;
          dg[i][j] += cok ? dv[u][i][j] * xh : 0.f;
          db[i][j] += cok ? dv[u][i][j] : 0.f;
          xv[u][i][j] = xh;             // keep xhat and g for the output pass
          dv[u][i][j] = g;
        }
      }
      s1 = wave_sum(s1) / a.N;
      s2 = wave_sum(s2) / a.N;
      if (live[u]) {
        T* dx = (T*)a.dx + (int64_t)(row0 + u * nw) * a.lddx;
#pragma unroll
        for (int i = 0; i < VPL; ++i) {
          const int c = (lane + i * 64) * VE;
          if (c < a.N) {
            float o[VE];
#pragma unroll
            for (int j = 0; j < VE; ++j) o[j] = rv[u][i][j] + rstd[u] * (dv[u][i][j] - s1 - xv[u][i][j] * s2);
            stv(dx + c, o);
            if (a.g) {
              // the fused ew_bwd: dropout backward of dx AS STORED (rounded to T), same mask
              // stream and column sums as ew_bwd_kernel
              float d[VE];
#pragma unroll
              for (int j = 0; j < VE; ++j) d[j] = to_f(from_f<T>(o[j]));
              if (a.drop_p > 0.f) {
                const uint64_t i0 = (uint64_t)(row0 + u * nw) * a.N + c;
                if constexpr (VE == 8) drop8(a.drop_p, a.seed, i0, d);
                else {
#pragma unroll
                  for (int j = 0; j < VE; ++j) d[j] *= drop_scale(a.drop_p, a.seed, i0 + j);
                }
              }
#pragma unroll
              for (int j = 0; j < VE; ++j) gb[i][j] += d[j];
              stv((T*)a.g + (int64_t)(row0 + u * nw) * a.ldg + c, d);
            }
          }
        }
      }
    }
  }
  if (!a.dgamma) return;
  // per-block column partials (the block's waves summed in LDS) -> ws[block][2 or 3][N]
  extern __shared__ __attribute__((aligned(16))) float red[];   // [W][N]
  const int w = threadIdx.x >> 6;
  const int nq = a.db ? 3 : 2;
  for (int q = 0; q < nq; ++q) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = (lane + i * 64) * VE;
      if (c < a.N) {
        // 16-byte stores of the lane's VE consecutive columns (scalar stores at a VE-float lane
        // stride were 4-8-way bank conflicts: 78 % of the kernel's LDS cycles, profiles/r05_sq_counters.txt)
        float* dst = red + w * a.N + c;
#pragma unroll
        for (int j = 0; j < VE; j += 4)
          *(f32x4*)(dst + j) = q == 0 ? f32x4{dg[i][j], dg[i][j + 1], dg[i][j + 2], dg[i][j + 3]}
                             : q == 1 ? f32x4{db[i][j], db[i][j + 1], db[i][j + 2], db[i][j + 3]}
                                      : f32x4{gb[i][j], gb[i][j + 1], gb[i][j + 2], gb[i][j + 3]};
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < a.N; c += 64 * W) {
      float t = 0.f;
#pragma unroll
      for (int v = 0; v < W; ++v) t += red[v * a.N + c];
      a.ws[((int64_t)blockIdx.x * nq + q) * a.N + c] = t;
    }
  }
}

// LayerNorm backward launch shape: 4 waves per block, one row in flight per wave. In isolation
// 6000 x 1024 takes 18.3-20.1 us with 4-8 waves (2 waves: 26 us; 16 waves: 38 us), 8-16 waves
// lose 2x at N = 2048, and in the step 4,1 beats 2,x and 8,x by 0.5-1 %
// (profiles/r02_ln_bwd_shape_ab.txt)
static void ln_bwd_shape(int& W, int& R) { W = 4; R = 1; }

static int ln_bwd_blocks() { return AVSR_LN_BLOCKS; }

template <typename T>
int ln_launch(const avsr_layernorm_params* p, bool bwd, hipStream_t st) {
  constexpr int VE = VecW<T>::VE;
  LnArgs a;
  a.rows = p->rows; a.N = p->N; a.eps = p->eps;
  a.x = p->x; a.ldx = p->ldx; a.y = p->y; a.ldy = p->ldy; a.gamma = p->gamma; a.beta = p->beta;
  a.mean = p->mean; a.rstd = p->rstd; a.dy = p->dy; a.lddy = p->lddy; a.dx = p->dx; a.lddx = p->lddx;
  a.dres = p->dres; a.lddres = p->lddres; a.dgamma = p->dgamma; a.dbeta = p->dbeta; a.ws = p->ws;
  a.g = bwd ? p->g : nullptr; a.ldg = p->ldg; a.drop_p = p->drop_p; a.seed = p->seed; a.db = bwd && p->db != nullptr;
  if (a.db && (!a.g || !p->dgamma)) return AVSR_E_ARG;     // the bias partials ride on the dgamma workspace
  const int vpl = (p->N / VE + 63) / 64;
  int blocks = (p->rows + 3) / 4;
  int W = 4, R = 1;
  if (bwd) {
    ln_bwd_shape(W, R);
    blocks = (p->rows + W - 1) / W;
    blocks = blocks < AVSR_LN_BLOCKS ? blocks : AVSR_LN_BLOCKS;
  }
  if (bwd && p->dgamma && (!p->ws || p->N > 2048)) return AVSR_E_ARG;
  while (W > 4 && (size_t)W * p->N * sizeof(float) > 64 * 1024) W >>= 1;   // default dynamic-LDS limit
  if (bwd) blocks = std::min((p->rows + W - 1) / W, ln_bwd_blocks());
  const size_t red = (size_t)W * p->N * sizeof(float);
#define LNB(V, W_, R_) hipLaunchKernelGGL((ln_bwd_kernel<T, V, W_, R_>), dim3(blocks), dim3(64 * W_), red, st, a)
#define LNL(V)                                                                                   \
  if (vpl <= V) {                                                                                \
    if (bwd) {                                                                                   \
      if (W == 16) { if (R == 2) LNB(V, 16, 2); else LNB(V, 16, 1); }                            \
      else if (W == 8) { if (R == 2) LNB(V, 8, 2); else LNB(V, 8, 1); }                          \
      else if (W == 4) { if (R == 2) LNB(V, 4, 2); else LNB(V, 4, 1); }                          \
      else { if (R == 2) LNB(V, 2, 2); else LNB(V, 2, 1); }                                      \
      if (p->dgamma) {                                                                           \
        AVSR_CHECK_LAUNCH();                                                                     \
        const int nq = a.db ? 3 : 2;                                                             \
        const int rc = colsum_launch((const float*)p->ws, blocks, (int64_t)nq * p->N, 2 * p->N,   \
                                     p->dgamma, p->N, p->dbeta, st);                             \
        if (rc || !a.db) return rc;                                                              \
        return colsum_launch((const float*)p->ws + 2 * p->N, blocks, (int64_t)3 * p->N, p->N,    \
                             p->db, 0, nullptr, st);                                             \
      }                                                                                          \
    } else {                                                                                     \
      hipLaunchKernelGGL((ln_fwd_kernel<T, V>), dim3(blocks), dim3(256), 0, st, a);              \
    }                                                                                            \
    AVSR_CHECK_LAUNCH();                                                                         \
    return 0;                                                                                    \
  }
  LNL(1) LNL(2) LNL(4) LNL(8)
#undef LNL
#undef LNB
  return AVSR_E_SHAPE;
}

int ln_check(const avsr_layernorm_params* p) {
  if (!p) return AVSR_E_ARG;
  const int ve = p->dtype == AVSR_BF16 ? 8 : 4;
  if (p->N % ve || p->ldx % ve || p->ldy % ve) return AVSR_E_ALIGN;
  return 0;
}

// =============================================================== BatchNorm
// one block of BNF_THREADS per channel: Chan-merge of the conv epilogue's (count, mean, M2)
// tile partials (the stem has ~45 k tiles per channel: 1024 threads keep that under ~40 us)
constexpr int BNF_THREADS = 1024;
__global__ __launch_bounds__(BNF_THREADS) void bn_finalize_kernel(avsr_bn_finalize_params a) {
  const int c = blockIdx.x;
  __shared__ double sn[BNF_THREADS], sm[BNF_THREADS], sq[BNF_THREADS];
  double n = 0, mean = 0, m2 = 0;
  if (a.training) {
    const float* pp = a.partials + (int64_t)c * a.tiles * 3;
    for (int t = threadIdx.x; t < a.tiles; t += blockDim.x) {
      const double nb = pp[t * 3 + 0], mb = pp[t * 3 + 1], qb = pp[t * 3 + 2];
      if (nb > 0) {
        const double nn = n + nb, d = mb - mean;
        mean += d * nb / nn;
        m2 += qb + d * d * n * nb / nn;
        n = nn;
      }
    }
    sn[threadIdx.x] = n; sm[threadIdx.x] = mean; sq[threadIdx.x] = m2;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {     // blockDim.x: 256 or 1024
      if (threadIdx.x < o) {
        const double na = sn[threadIdx.x], nb = sn[threadIdx.x + o];
        if (nb > 0) {
          const double nn = na + nb, d = sm[threadIdx.x + o] - sm[threadIdx.x];
          sm[threadIdx.x] += d * nb / nn;
          sq[threadIdx.x] += sq[threadIdx.x + o] + d * d * na * nb / nn;
          sn[threadIdx.x] = nn;
        }
      }
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) {
    double mu, var;
    if (a.training) {
      n = sn[0]; mu = sm[0]; var = n > 0 ? sq[0] / n : 0.0;
      if (a.running_mean) {
        const double unb = n > 1 ? sq[0] / (n - 1) : var;
        a.running_mean[c] = (float)((1.0 - a.momentum) * a.running_mean[c] + a.momentum * mu);
        a.running_var[c] = (float)((1.0 - a.momentum) * a.running_var[c] + a.momentum * unb);
      }
    } else {
      mu = a.running_mean[c]; var = a.running_var[c];
    }
    const float inv = (float)(1.0 / sqrt(var + (double)a.eps));
    const float g = a.gamma ? a.gamma[c] : 1.f, b = a.beta ? a.beta[c] : 0.f;
    a.mean[c] = (float)mu; a.invstd[c] = inv;
    a.scale[c] = g * inv; a.shift[c] = b - (float)mu * g * inv;
  }
}

struct BnArgs {
  int M, C;
  const void* h; const float* scale; const float* shift;
  const void* res; const float* scale2; const float* shift2;
  const float* prelu; void* y;
  const void* dy; void* dz;
  const float* mean; const float* invstd; const float* mean2; const float* invstd2;
  float* sums; float* dprelu; float* dgamma; float* dbeta; float* dgamma2; float* dbeta2;
  void* dh; void* dh2; float beta_acc; float* ws;
};

// Per-channel parameters of the thread's fixed channel group (the grid stride is a multiple
// of C/VE, so every vector a thread visits has the same channels): loaded once.
template <int VE>
AVSR_DEV void chan_load(const float* p, int c0, float (&o)[VE]) {
#pragma unroll
  for (int j = 0; j < VE; ++j) o[j] = p ? p[c0 + j] : 0.f;
}

// y = PReLU(h*scale + shift [+ res*scale2 + shift2 | + res]); two vectors per iteration so
// each wave keeps two independent 16-byte loads (x2 with the residual) in flight.
template <typename T>
__global__ __launch_bounds__(256) void bn_act_fwd_kernel(BnArgs a) {
  constexpr int VE = VecW<T>::VE;
  const int cpv = a.C / VE;
  const int64_t nv = (int64_t)a.M * cpv, stride = (int64_t)gridDim.x * 256;
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int c0 = (int)(t0 % cpv) * VE;
  float sc[VE], sh[VE], pw[VE], sc2[VE], sh2[VE];
  chan_load(a.scale, c0, sc); chan_load(a.shift, c0, sh); chan_load(a.prelu, c0, pw);
  chan_load(a.scale2, c0, sc2); chan_load(a.shift2, c0, sh2);
  const bool res = a.res != nullptr, res_bn = a.scale2 != nullptr;
  for (int64_t v = t0; v < nv; v += 2 * stride) {
    const bool two = v + stride < nv;
    float h[2][VE], r[2][VE];
    ldv((const T*)a.h + v * VE, h[0]);
    if (two) ldv((const T*)a.h + (v + stride) * VE, h[1]);
    if (res) {
      ldv((const T*)a.res + v * VE, r[0]);
      if (two) ldv((const T*)a.res + (v + stride) * VE, r[1]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !two) break;
      float o[VE];
#pragma unroll
      for (int j = 0; j < VE; ++j) {
        float z = h[u][j] * sc[j] + sh[j];
        if (res) z += res_bn ? r[u][j] * sc2[j] + sh2[j] : r[u][j];
        o[j] = z > 0.f ? z : z * pw[j];
      }
      stv((T*)a.y + (v + u * stride) * VE, o);
    }
  }
}

// block-level reduction of per-thread channel partials (a thread's channel group is fixed:
// the grid stride is a multiple of C/VE) -> ws[block][q][C] (plain stores)
template <int VE>
__device__ void block_chan_partial(const float (&q)[VE], float* lds, int cpv, float* ws_row) {
#pragma unroll
  for (int j = 0; j < VE; ++j) lds[threadIdx.x * VE + j] = q[j];
  __syncthreads();
  if ((int)threadIdx.x < cpv) {
    float acc[VE];
#pragma unroll
    for (int j = 0; j < VE; ++j) acc[j] = 0.f;
    for (int t = threadIdx.x; t < 256; t += cpv)
#pragma unroll
      for (int j = 0; j < VE; ++j) acc[j] += lds[t * VE + j];
#pragma unroll
    for (int j = 0; j < VE; ++j) ws_row[threadIdx.x * VE + j] = acc[j];
  }
  __syncthreads();
}

// per channel: S_q = sum over blocks; sums[c][0..2] = S0..S2 (set); grads accumulate
__global__ __launch_bounds__(256) void bn_grad_finalize_kernel(const float* ws, int nb, int C, float* sums,
                                                               float* dbeta, float* dgamma, float* dbeta2,
                                                               float* dgamma2, float* dprelu) {
  const int c = blockIdx.x;
  __shared__ float sh[4][4];
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  for (int b = threadIdx.x; b < nb; b += 256)
#pragma unroll
    for (int q = 0; q < 4; ++q) s[q] += ws[((int64_t)b * 4 + q) * C + c];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float v = wave_sum(s[q]);
    if ((threadIdx.x & 63) == 0) sh[q][threadIdx.x >> 6] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float t[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] = sh[q][0] + sh[q][1] + sh[q][2] + sh[q][3];
    if (sums) { sums[c * 3 + 0] = t[0]; sums[c * 3 + 1] = t[1]; sums[c * 3 + 2] = t[2]; }
    if (dbeta) dbeta[c] += t[0];
    if (dgamma) dgamma[c] += t[1];
    if (dbeta2) dbeta2[c] += t[0];
    if (dgamma2) dgamma2[c] += t[2];
    if (dprelu) dprelu[c] += t[3];
  }
}

// dz = prelu'(z)*dy with z recomputed; per-block channel partials of sum dz, sum dz*xhat,
// sum dz*xhat2 and the PReLU-weight sum dy*z*[z<=0] -> ws[block][4][C]. Two vectors per
// iteration (independent 16-byte loads in flight).
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(BnArgs a) {
  constexpr int VE = VecW<T>::VE;
  __shared__ float lds[256 * VE];
  const int cpv = a.C / VE;
  const int64_t nv = (int64_t)a.M * cpv, stride = (int64_t)gridDim.x * 256;
  float s0[VE], s1[VE], s2[VE], s3[VE];
#pragma unroll
  for (int j = 0; j < VE; ++j) { s0[j] = s1[j] = s2[j] = s3[j] = 0.f; }
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int c0 = (int)(t0 % cpv) * VE;
  float sc[VE], sh[VE], pw[VE], mu[VE], is[VE], sc2[VE], sh2[VE], mu2[VE], is2[VE];
  chan_load(a.scale, c0, sc); chan_load(a.shift, c0, sh); chan_load(a.prelu, c0, pw);
  chan_load(a.mean, c0, mu); chan_load(a.invstd, c0, is);
  chan_load(a.scale2, c0, sc2); chan_load(a.shift2, c0, sh2); chan_load(a.mean2, c0, mu2); chan_load(a.invstd2, c0, is2);
  const bool res = a.res != nullptr, res_bn = a.scale2 != nullptr;
  for (int64_t v = t0; v < nv; v += 2 * stride) {
    const bool two = v + stride < nv;
    float h[2][VE], r[2][VE], d[2][VE];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !two) break;
      const int64_t w = v + u * stride;
      ldv((const T*)a.h + w * VE, h[u]);
      ldv((const T*)a.dy + w * VE, d[u]);
      if (res) ldv((const T*)a.res + w * VE, r[u]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !two) break;
      float dzo[VE];
#pragma unroll
      for (int j = 0; j < VE; ++j) {
        float z = h[u][j] * sc[j] + sh[j];
        if (res) z += res_bn ? r[u][j] * sc2[j] + sh2[j] : r[u][j];
        const bool pos = z > 0.f;
        const float dz = pos ? d[u][j] : d[u][j] * pw[j];
        s3[j] += pos ? 0.f : d[u][j] * z;
        dzo[j] = dz;
        s0[j] += dz;
        s1[j] += dz * (h[u][j] - mu[j]) * is[j];
        if (res_bn) s2[j] += dz * (r[u][j] - mu2[j]) * is2[j];
      }
      stv((T*)a.dz + (v + u * stride) * VE, dzo);
    }
  }
  // channel partials of this block -> ws[block][q][C]; bn_grad_finalize sums the blocks
  float* wsb = a.ws + (int64_t)blockIdx.x * 4 * a.C;
  block_chan_partial<VE>(s0, lds, cpv, wsb + 0 * a.C);
  block_chan_partial<VE>(s1, lds, cpv, wsb + 1 * a.C);
  block_chan_partial<VE>(s2, lds, cpv, wsb + 2 * a.C);
  block_chan_partial<VE>(s3, lds, cpv, wsb + 3 * a.C);
}

// ws[nb][4][C] -> ws2[slices][4][C]: one wave per (channel group of 64, slice of BN_FOLD_PER
// block rows), four rows per iteration (16 independent 256-byte coalesced loads in flight per
// lane), no LDS. Single-wave blocks: the fold runs on the main stream while the side stream's
// persistent weight-gradient blocks (conv_wgrad_patch, one 4-wave block per CU with up to 152 KB
// of LDS) hold every CU, and the former 8-wave / 8 KB-LDS blocks found no room beside them
// (6 us alone, 180 us in the step: they waited for the weight-gradient tail).
constexpr int BN_FOLD_PER = 16;
__global__ __launch_bounds__(64) void bn_ws_fold_kernel(const float* ws, int nb, int C, float* ws2) {
  const int c = blockIdx.x * 64 + threadIdx.x, sl = blockIdx.y;
  const int b0 = sl * BN_FOLD_PER, b1 = min(nb, b0 + BN_FOLD_PER);
  if (c >= C) return;
  float s[4][4] = {};
  int b = b0;
  for (; b + 3 < b1; b += 4)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) s[u][q] += ws[((int64_t)(b + u) * 4 + q) * C + c];
  for (; b < b1; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) s[0][q] += ws[((int64_t)b * 4 + q) * C + c];
#pragma unroll
  for (int q = 0; q < 4; ++q) ws2[((int64_t)sl * 4 + q) * C + c] = (s[0][q] + s[1][q]) + (s[2][q] + s[3][q]);
}

template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(BnArgs a) {
  constexpr int VE = VecW<T>::VE;
  const int cpv = a.C / VE;
  const int64_t nv = (int64_t)a.M * cpv, stride = (int64_t)gridDim.x * 256;
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int c0 = (int)(t0 % cpv) * VE;
  const float invM = 1.f / (float)a.M;
  // dh = scale*(dz - S0/M - xh*S1/M) with xh = (h-mean)*invstd  ==  A*dz + B*(h-mean) + Cc
  float ka[VE], kb[VE], kc[VE], km[VE], ka2[VE], kb2[VE], kc2[VE], km2[VE];
#pragma unroll
  for (int j = 0; j < VE; ++j) {
    const int c = c0 + j;
    const float s0 = a.sums[c * 3 + 0] * invM, s1 = a.sums[c * 3 + 1] * invM;
    ka[j] = a.scale[c];
    kb[j] = -a.scale[c] * s1 * a.invstd[c];
    kc[j] = -a.scale[c] * s0;
    km[j] = a.mean[c];
    if (a.dh2) {
      const float s2 = a.sums[c * 3 + 2] * invM;
      ka2[j] = a.scale2[c];
      kb2[j] = -a.scale2[c] * s2 * a.invstd2[c];
      kc2[j] = -a.scale2[c] * s0;
      km2[j] = a.mean2[c];
    }
  }
  const bool acc = a.beta_acc != 0.f;
  // U grid-stride vectors per iteration with every load issued first (memory-level
  // parallelism: one vector in flight per thread left this pass at ~65 % of HBM bandwidth)
  constexpr int U = 4;
  for (int64_t v0 = t0; v0 < nv; v0 += U * stride) {
    float dz[U][VE], h[U][VE], o[U][VE], r[U][VE];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v = v0 + u * stride;
      ok[u] = v < nv;
      const int64_t vv = ok[u] ? v : v0;
      ldv((const T*)a.dz + vv * VE, dz[u]);
      ldv((const T*)a.h + vv * VE, h[u]);
      if (acc) ldv((const T*)a.dh + vv * VE, o[u]);
      if (a.dh2) ldv((const T*)a.res + vv * VE, r[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) break;
      const int64_t v = v0 + u * stride;
      float g[VE];
#pragma unroll
      for (int j = 0; j < VE; ++j) {
        const float gg = ka[j] * dz[u][j] + kb[j] * (h[u][j] - km[j]) + kc[j];
        g[j] = acc ? a.beta_acc * o[u][j] + gg : gg;
      }
      stv((T*)a.dh + v * VE, g);
      if (a.dh2) {
        float o2[VE];
#pragma unroll
        for (int j = 0; j < VE; ++j) o2[j] = ka2[j] * dz[u][j] + kb2[j] * (r[u][j] - km2[j]) + kc2[j];
        stv((T*)a.dh2 + v * VE, o2);
      }
    }
  }
}

BnArgs bn_args(const avsr_bn_act_params* p) {
  BnArgs a;
  a.M = p->M; a.C = p->C; a.h = p->h; a.scale = p->scale; a.shift = p->shift; a.res = p->res;
  a.scale2 = p->scale2; a.shift2 = p->shift2; a.prelu = p->prelu; a.y = p->y; a.dy = p->dy; a.dz = p->dz;
  a.mean = p->mean; a.invstd = p->invstd; a.mean2 = p->mean2; a.invstd2 = p->invstd2; a.sums = p->sums;
  a.dprelu = p->dprelu; a.dgamma = p->dgamma; a.dbeta = p->dbeta; a.dgamma2 = p->dgamma2; a.dbeta2 = p->dbeta2;
  a.dh = p->dh; a.dh2 = p->dh2; a.beta_acc = p->beta_acc; a.ws = p->ws;
  return a;
}

// =============================================================== stem max-pool
// grid (vector blocks of one image, image): 32-bit in-image indexing, the nine window
// loads issued together (clamped addresses, masked values)
template <typename T>
__global__ __launch_bounds__(256) void stem_pool_fwd_kernel(avsr_stem_pool_params p, FastDiv fwo) {
  constexpr int VE = VecW<T>::VE;
  const int cpv = p.C / VE;
  const int per_img = p.Ho * p.Wo * cpv;
  const int v = blockIdx.x * 256 + threadIdx.x;
  if (v >= per_img) return;
  const int n = blockIdx.y;
  const int cv = v % cpv, c0 = cv * VE;
  const uint32_t opix = (uint32_t)(v / cpv);
  const int oh = (int)fdiv(opix, fwo), ow = (int)(opix - oh * fwo.d);
  float sc[VE], sh[VE], pw[VE];
  chan_load(p.scale, c0, sc); chan_load(p.shift, c0, sh); chan_load(p.prelu, c0, pw);
  const T* base = (const T*)p.h + (int64_t)n * p.H * p.W * p.C + c0;
  float hv[9][VE];
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    const int ih = min(max(2 * oh - 1 + q / 3, 0), p.H - 1), iw = min(max(2 * ow - 1 + q % 3, 0), p.W - 1);
    ldv(base + (ih * p.W + iw) * p.C, hv[q]);
  }
  float best[VE], bh[VE];
  uint8_t idx[VE];
#pragma unroll
  for (int j = 0; j < VE; ++j) { best[j] = -INFINITY; bh[j] = 0.f; idx[j] = 0; }
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    const int ih = 2 * oh - 1 + q / 3, iw = 2 * ow - 1 + q % 3;
    if (ih < 0 || ih >= p.H || iw < 0 || iw >= p.W) continue;
#pragma unroll
    for (int j = 0; j < VE; ++j) {
      const float z = hv[q][j] * sc[j] + sh[j];
      const float y = z > 0.f ? z : z * pw[j];
      if (y > best[j]) { best[j] = y; bh[j] = hv[q][j]; idx[j] = (uint8_t)q; }
    }
  }
  const int64_t ov = (int64_t)n * per_img + v;
  stv((T*)p.y + ov * VE, best);
  if (p.hmax) stv((T*)p.hmax + ov * VE, bh);
  if constexpr (VE == 8) *(uint2*)(p.argmax + ov * VE) = *(const uint2*)idx;
  else *(uint32_t*)(p.argmax + ov * VE) = *(const uint32_t*)idx;
}

// Same outputs for H = 2*Ho, W = 2*Wo: one thread per 2x2 block of pooled outputs and channel
// group. The block's four 3x3 windows cover a 5x5 input patch: each input is loaded and put
// through BN+PReLU once (25 per 4 outputs instead of 36), row by row; every window still
// visits its taps in row-major order with the strict '>' (same maximum, same argmax on ties).
// Grid-stride with the channel group fixed (per-channel coefficients loaded once).
template <typename T>
__global__ __launch_bounds__(256) void stem_pool_fwd2_kernel(avsr_stem_pool_params p, FastDiv fbwo, FastDiv fbho) {
  constexpr int VE = VecW<T>::VE;
  const int cpv = p.C / VE, cshift = 31 - __builtin_clz(cpv);
  const int bho = p.Ho >> 1, bwo = p.Wo >> 1;
  // 32-bit indices with multiply-shift divisions (the launcher checks nv < 2^31)
  const uint32_t nv = (uint32_t)p.nimg * bho * bwo * cpv, stride = gridDim.x * 256u;
  const uint32_t t0 = blockIdx.x * 256u + threadIdx.x;
  const int cv = (int)(t0 & (cpv - 1)), c0 = cv * VE;
  float sc[VE], sh[VE], pw[VE];
  chan_load(p.scale, c0, sc); chan_load(p.shift, c0, sh); chan_load(p.prelu, c0, pw);
  for (uint32_t v = t0; v < nv; v += stride) {
    const uint32_t blk = v >> cshift, q = fdiv(blk, fbwo);
    const int bw = (int)(blk - q * fbwo.d);
    const uint32_t nq = fdiv(q, fbho);
    const int bh = (int)(q - nq * fbho.d);
    const int64_t n = nq;
    const int ih0 = 4 * bh - 1, iw0 = 4 * bw - 1;        // patch origin (may be -1)
    const T* base = (const T*)p.h + n * p.H * p.W * p.C + c0;
    float best[4][VE], bhv[4][VE];
    uint8_t idx[4][VE];
#pragma unroll
    for (int o = 0; o < 4; ++o)
#pragma unroll
      for (int j = 0; j < VE; ++j) { best[o][j] = -INFINITY; bhv[o][j] = 0.f; idx[o][j] = 0; }
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const int ih = ih0 + r;
      const bool rok = ih >= 0 && ih < p.H;
      float hv[5][VE];
#pragma unroll
      for (int c = 0; c < 5; ++c) {
        const int iw = min(max(iw0 + c, 0), p.W - 1);
        ldv(base + ((int64_t)min(max(ih, 0), p.H - 1) * p.W + iw) * p.C, hv[c]);
      }
      if (!rok) continue;
#pragma unroll
      for (int c = 0; c < 5; ++c) {
        const int iw = iw0 + c;
        if (iw < 0 || iw >= p.W) continue;
#pragma unroll
        for (int o = 0; o < 4; ++o) {
          const int a = o >> 1, b = o & 1;
          const int wr = r - 2 * a, wc = c - 2 * b;       // tap position in window o
          if (wr < 0 || wr > 2 || wc < 0 || wc > 2) continue;
#pragma unroll
          for (int j = 0; j < VE; ++j) {
            const float z = hv[c][j] * sc[j] + sh[j];
            const float y = z > 0.f ? z : z * pw[j];
            if (y > best[o][j]) { best[o][j] = y; bhv[o][j] = hv[c][j]; idx[o][j] = (uint8_t)(wr * 3 + wc); }
          }
        }
      }
    }
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const int oh = 2 * bh + (o >> 1), ow = 2 * bw + (o & 1);
      const int64_t ov = ((n * p.Ho + oh) * p.Wo + ow) * cpv + cv;
      stv((T*)p.y + ov * VE, best[o]);
      if (p.hmax) stv((T*)p.hmax + ov * VE, bhv[o]);
      if constexpr (VE == 8) *(uint2*)(p.argmax + ov * VE) = *(const uint2*)idx[o];
      else *(uint32_t*)(p.argmax + ov * VE) = *(const uint32_t*)idx[o];
    }
  }
}

// Stem backward, dense part. The BN reductions run over the pooled grid (h at the argmax,
// saved by the forward as hmax; dz is nonzero only where an input pixel is some window's
// argmax, so sum_p dz*xhat = sum_o dzp[o]*xhat(hmax[o])); here dz[p] = sum of dzp[o] over the
// (at most 4) windows o whose argmax is p, and dh = scale*(dz - S0/M - xhat*S1/M).
// Grid-stride over 16-byte vectors with the thread's channel group fixed (the stride is a
// multiple of C/VE), so the per-channel coefficients are formed once per thread.
template <typename T>
__global__ __launch_bounds__(256) void stem_bwd_apply_kernel(avsr_stem_pool_params p, FastDiv fw, FastDiv fhw) {
  constexpr int VE = VecW<T>::VE;
  const int cpv = p.C / VE, cshift = 31 - __builtin_clz(cpv);
  const int64_t nv = (int64_t)p.nimg * p.H * p.W * cpv, stride = (int64_t)gridDim.x * 256;
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int cv = (int)(t0 % cpv), c0 = cv * VE;
  const float invM = 1.f / (p.m_total > 0 ? (float)p.m_total : (float)p.nimg * p.H * p.W);
  float ka[VE], kb[VE], kc[VE], km[VE];
#pragma unroll
  for (int j = 0; j < VE; ++j) {
    const int c = c0 + j;
    const float s0 = p.sums[c * 3 + 0] * invM, s1 = p.sums[c * 3 + 1] * invM;
    ka[j] = p.scale[c]; kb[j] = -p.scale[c] * s1 * p.invstd[c]; kc[j] = -p.scale[c] * s0; km[j] = p.mean[c];
  }
  // two vectors per iteration: both h loads and all window gathers in flight together
  for (int64_t v = t0; v < nv; v += 2 * stride) {
    const bool two = v + stride < nv;
    float h[2][VE], d[2][VE];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int j = 0; j < VE; ++j) d[u][j] = 0.f;
      if (u == 1 && !two) break;
      const int64_t w = v + u * stride;
      const uint32_t pix = (uint32_t)(w >> cshift);
      const uint32_t n = fdiv(pix, fhw), rem = pix - n * fhw.d;
      const int ih = (int)fdiv(rem, fw), iw = (int)(rem - ih * fw.d);
      ldv((const T*)p.h + w * VE, h[u]);
      // windows (oh, ow) with 2*o-1 <= i <= 2*o+1
      const int oh0 = (ih + 1) / 2 - 1, ow0 = (iw + 1) / 2 - 1;
#pragma unroll
      for (int dh = 0; dh < 2; ++dh) {
        const int oh = oh0 + dh;
        if (oh < 0 || oh >= p.Ho || ih < 2 * oh - 1 || ih > 2 * oh + 1) continue;
#pragma unroll
        for (int dw = 0; dw < 2; ++dw) {
          const int ow = ow0 + dw;
          if (ow < 0 || ow >= p.Wo || iw < 2 * ow - 1 || iw > 2 * ow + 1) continue;
          const int64_t ov = (((int64_t)n * p.Ho + oh) * p.Wo + ow) * cpv + cv;
          const uint8_t want = (uint8_t)((ih - 2 * oh + 1) * 3 + (iw - 2 * ow + 1));
          float g[VE];
          ldv((const T*)p.dz + ov * VE, g);
          uint8_t am[VE];
          if constexpr (VE == 8) *(uint2*)am = *(const uint2*)(p.argmax + ov * VE);
          else *(uint32_t*)am = *(const uint32_t*)(p.argmax + ov * VE);
#pragma unroll
          for (int j = 0; j < VE; ++j) d[u][j] += am[j] == want ? g[j] : 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !two) break;
      float o[VE];
#pragma unroll
      for (int j = 0; j < VE; ++j) o[j] = ka[j] * d[u][j] + kb[j] * (h[u][j] - km[j]) + kc[j];
      stv((T*)p.dh + (v + u * stride) * VE, o);
    }
  }
}

// Same result for even H, W (Ho = H/2, Wo = W/2), one thread per 2x2 pixel block (2oh+dy, 2ow+dx)
// and channel group: the block's pixels lie in windows (oh, ow), (oh, ow+1) [dx = 1],
// (oh+1, ow) [dy = 1], (oh+1, ow+1) [both], so the four windows' dz / argmax are loaded once
// for four outputs (2.25 window gathers per pixel otherwise), with no per-pixel divisions and
// every load of the block issued together. Windows are added in the per-pixel kernel's order
// (bit-identical).
template <typename T, int U>
__global__ __launch_bounds__(256) void stem_bwd_apply2_kernel(avsr_stem_pool_params p, FastDiv fwo, FastDiv fho) {
  constexpr int VE = VecW<T>::VE;
  const int cpv = p.C / VE, cshift = 31 - __builtin_clz(cpv);
  // 32-bit indices with multiply-shift divisions (the launcher checks nv < 2^31; the int64
  // divisions they replace were ~1/3 of this HBM-bound pass, 900 -> 737 us at C2). U blocks per
  // iteration with every load issued first (U = 2 needs 198 VGPRs: 2 waves per SIMD instead of 3)
  const uint32_t nv = (uint32_t)p.nimg * p.Ho * p.Wo * cpv, stride = gridDim.x * 256u;
  const uint32_t t0 = blockIdx.x * 256u + threadIdx.x;
  const int cv = (int)(t0 & (cpv - 1)), c0 = cv * VE;
  const float invM = 1.f / (p.m_total > 0 ? (float)p.m_total : (float)p.nimg * p.H * p.W);
  float ka[VE], kb[VE], kc[VE], km[VE];
#pragma unroll
  for (int j = 0; j < VE; ++j) {
    const int c = c0 + j;
    const float s0 = p.sums[c * 3 + 0] * invM, s1 = p.sums[c * 3 + 1] * invM;
    ka[j] = p.scale[c]; kb[j] = -p.scale[c] * s1 * p.invstd[c]; kc[j] = -p.scale[c] * s0; km[j] = p.mean[c];
  }
  for (uint32_t v0 = t0; v0 < nv; v0 += U * stride) {
    float g[U][4][VE], h[U][4][VE];
    uint8_t am[U][4][VE];
    bool wok[U][4], ok[U];
    uint32_t hb[U];                                    // vector index of pixel (2oh, 2ow)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t v = v0 + u * stride;
      ok[u] = v < nv;
      const uint32_t blk = (ok[u] ? v : v0) >> cshift;   // (n, oh, ow)
      const uint32_t q = fdiv(blk, fwo), n = fdiv(q, fho);
      const int ow = (int)(blk - q * fwo.d), oh = (int)(q - n * fho.d);
      // windows w = (oh + a, ow + b), a, b in {0, 1}; out-of-range windows contribute nothing
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const int wa = w >> 1, wb = w & 1;
        wok[u][w] = oh + wa < p.Ho && ow + wb < p.Wo;
        const uint32_t ov = ((n * p.Ho + min(oh + wa, p.Ho - 1)) * p.Wo + min(ow + wb, p.Wo - 1)) * cpv + cv;
        ldv((const T*)p.dz + (int64_t)ov * VE, g[u][w]);
        if constexpr (VE == 8) *(uint2*)am[u][w] = *(const uint2*)(p.argmax + (int64_t)ov * VE);
        else *(uint32_t*)am[u][w] = *(const uint32_t*)(p.argmax + (int64_t)ov * VE);
      }
      hb[u] = ((n * p.H + 2 * oh) * p.W + 2 * ow) * cpv + cv;
#pragma unroll
      for (int qd = 0; qd < 4; ++qd)
        ldv((const T*)p.h + (int64_t)(hb[u] + ((qd >> 1) * p.W + (qd & 1)) * cpv) * VE, h[u][qd]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) break;
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        const int dy = qd >> 1, dx = qd & 1;
        float d[VE];
#pragma unroll
        for (int j = 0; j < VE; ++j) d[j] = 0.f;
        // pixel (2oh+dy, 2ow+dx) sits at window-local position (dy+1, dx+1) of window (oh, ow)
        // and at (dy-1, dx+1), (dy+1, dx-1), (dy-1, dx-1) of the others (rows: 3 per window)
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const int wa = w >> 1, wb = w & 1;
          if ((wa && !dy) || (wb && !dx)) continue;      // the pixel is not in that window
          const uint8_t want = (uint8_t)((dy - 2 * wa + 1) * 3 + (dx - 2 * wb + 1));
#pragma unroll
          for (int j = 0; j < VE; ++j) d[j] += (wok[u][w] && am[u][w][j] == want) ? g[u][w][j] : 0.f;
        }
        float o[VE];
#pragma unroll
        for (int j = 0; j < VE; ++j) o[j] = ka[j] * d[j] + kb[j] * (h[u][qd][j] - km[j]) + kc[j];
        stv((T*)p.dh + (int64_t)(hb[u] + (dy * p.W + dx) * cpv) * VE, o);
      }
    }
  }
}

// =============================================================== avg pool
template <typename T>
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(int nimg, int P, int C, const T* x, T* y) {
  constexpr int VE = VecW<T>::VE;
  const int cpv = C / VE;
  const int64_t nv = (int64_t)nimg * cpv;
  for (int64_t v = blockIdx.x * 256 + threadIdx.x; v < nv; v += (int64_t)gridDim.x * 256) {
    const int64_t n = v / cpv;
    const int c0 = (int)(v % cpv) * VE;
    float s[VE], t[VE];
#pragma unroll
    for (int j = 0; j < VE; ++j) s[j] = 0.f;
    for (int q = 0; q < P; ++q) {
      ldv(x + ((n * P + q) * C + c0), t);
#pragma unroll
      for (int j = 0; j < VE; ++j) s[j] += t[j];
    }
#pragma unroll
    for (int j = 0; j < VE; ++j) s[j] /= (float)P;
    stv(y + v * VE, s);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void avgpool_bwd_kernel(int nimg, int P, int C, const T* dy, T* dx) {
  constexpr int VE = VecW<T>::VE;
  const int cpv = C / VE;
  const int64_t nv = (int64_t)nimg * P * cpv;
  for (int64_t v = blockIdx.x * 256 + threadIdx.x; v < nv; v += (int64_t)gridDim.x * 256) {
    const int64_t n = v / ((int64_t)P * cpv);
    const int c0 = (int)(v % cpv) * VE;
    float t[VE];
    ldv(dy + (n * C + c0), t);
#pragma unroll
    for (int j = 0; j < VE; ++j) t[j] /= (float)P;
    stv(dx + v * VE, t);
  }
}

int bn_grid(int64_t nv, int cpv) {
  // grid stride (blocks*256) must be a multiple of cpv: 256 % cpv == 0 for cpv <= 256 power of 2
  (void)cpv;
  return avsr_grid(nv, 256, 2048);
}

}  // namespace

extern "C" int avsr_layernorm_fwd(const avsr_layernorm_params* p, void* stream) {
  int rc = ln_check(p);
  if (rc) return rc;
  if (p->rows == 0) return 0;
  if (p->dtype == AVSR_BF16) return ln_launch<bf16>(p, false, (hipStream_t)stream);
  if (p->dtype == AVSR_F32) return ln_launch<float>(p, false, (hipStream_t)stream);
  return AVSR_E_DTYPE;
}

extern "C" int avsr_layernorm_bwd(const avsr_layernorm_params* p, void* stream) {
  int rc = ln_check(p);
  if (rc) return rc;
  if (p->rows == 0) return 0;
  if (p->dtype == AVSR_BF16) return ln_launch<bf16>(p, true, (hipStream_t)stream);
  if (p->dtype == AVSR_F32) return ln_launch<float>(p, true, (hipStream_t)stream);
  return AVSR_E_DTYPE;
}

extern "C" int avsr_bn_finalize(const avsr_bn_finalize_params* p, void* stream) {
  if (!p || p->C <= 0) return AVSR_E_ARG;
  if (p->training && !p->partials) return AVSR_E_ARG;
  if (!p->training && (!p->running_mean || !p->running_var)) return AVSR_E_ARG;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(p->C), dim3(p->training && p->tiles > 2048 ? BNF_THREADS : 256), 0,
                     (hipStream_t)stream, *p);
  AVSR_CHECK_LAUNCH();
  return 0;
}

static int bn_check(const avsr_bn_act_params* p) {
  if (!p) return AVSR_E_ARG;
  const int ve = p->dtype == AVSR_BF16 ? 8 : 4;
  if (p->C % ve || (p->C / ve) > 256 || (256 % (p->C / ve))) return AVSR_E_SHAPE;
  return 0;
}

extern "C" int avsr_bn_act_fwd(const avsr_bn_act_params* p, void* stream) {
  int rc = bn_check(p);
  if (rc) return rc;
  BnArgs a = bn_args(p);
  const int ve = p->dtype == AVSR_BF16 ? 8 : 4;
  const int g = bn_grid((int64_t)p->M * p->C / ve, p->C / ve);
  if (p->dtype == AVSR_BF16) hipLaunchKernelGGL(bn_act_fwd_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(bn_act_fwd_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, a);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_bn_act_bwd_reduce(const avsr_bn_act_params* p, void* stream) {
  int rc = bn_check(p);
  if (rc) return rc;
  if (!p->ws) return AVSR_E_ARG;
  BnArgs a = bn_args(p);
  const int ve = p->dtype == AVSR_BF16 ? 8 : 4;
  const int g = bn_grid((int64_t)p->M * p->C / ve, p->C / ve);
  if (p->dtype == AVSR_BF16) hipLaunchKernelGGL(bn_bwd_reduce_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(bn_bwd_reduce_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, a);
  AVSR_CHECK_LAUNCH();
  return avsr_bn_bwd_finalize(p, g, stream);
}

// ws[tiles][4][C] (from the reduce kernel or a data-grad BN epilogue) -> sums + parameter
// grads. More than 256 partial rows are first folded into ceil(tiles / 16) slices, stored after
// the partials (ws holds AVSR_BN_FIN_WS(tiles, C) floats).
extern "C" int avsr_bn_bwd_finalize(const avsr_bn_act_params* p, int tiles, void* stream) {
  if (!p || !p->ws || p->C <= 0 || tiles <= 0) return AVSR_E_ARG;
  const float* ws = p->ws;
  int nb = tiles;
  hipStream_t st = (hipStream_t)stream;
  if (tiles > 256) {
    const int SL = (tiles + BN_FOLD_PER - 1) / BN_FOLD_PER;
    if (SL > 65535) return AVSR_E_SHAPE;
    float* ws2 = p->ws + (int64_t)tiles * 4 * p->C;
    hipLaunchKernelGGL(bn_ws_fold_kernel, dim3((p->C + 63) / 64, SL), dim3(64), 0, st, (const float*)p->ws, tiles,
                       p->C, ws2);
    ws = ws2; nb = SL;
  }
  hipLaunchKernelGGL(bn_grad_finalize_kernel, dim3(p->C), dim3(256), 0, st, ws, nb, p->C, p->sums, p->dbeta,
                     p->dgamma, p->dbeta2, p->dgamma2, p->dprelu);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_bn_bwd_apply(const avsr_bn_act_params* p, void* stream) {
  int rc = bn_check(p);
  if (rc) return rc;
  if (!p->sums || !p->dz || !p->dh) return AVSR_E_ARG;
  BnArgs a = bn_args(p);
  const int ve = p->dtype == AVSR_BF16 ? 8 : 4;
  const int g = bn_grid((int64_t)p->M * p->C / ve, p->C / ve);
  if (p->dtype == AVSR_BF16) hipLaunchKernelGGL(bn_bwd_apply_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(bn_bwd_apply_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, a);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_stem_pool_fwd(const avsr_stem_pool_params* p, void* stream) {
  if (!p) return AVSR_E_ARG;
  const int ve = p->dtype == AVSR_BF16 ? 8 : 4;
  if (p->C % ve) return AVSR_E_SHAPE;
  if (p->nimg > 65535) return AVSR_E_SHAPE;
  if (p->H == 2 * p->Ho && p->W == 2 * p->Wo && !(p->Ho & 1) && !(p->Wo & 1) && avsr_opt(AVSR_OPT_STEM_POOL_2X2) &&
      256 % (p->C / ve) == 0) {
    const int64_t nv2 = (int64_t)p->nimg * (p->Ho / 2) * (p->Wo / 2) * p->C / ve;
    if (nv2 >= (1ll << 31)) return AVSR_E_SHAPE;
    const int g2 = bn_grid(nv2, p->C / ve);
    const FastDiv fbwo = make_fastdiv(p->Wo / 2), fbho = make_fastdiv(p->Ho / 2);
    if (p->dtype == AVSR_BF16) hipLaunchKernelGGL(stem_pool_fwd2_kernel<bf16>, dim3(g2), dim3(256), 0, (hipStream_t)stream, *p, fbwo, fbho);
    else hipLaunchKernelGGL(stem_pool_fwd2_kernel<float>, dim3(g2), dim3(256), 0, (hipStream_t)stream, *p, fbwo, fbho);
    AVSR_CHECK_LAUNCH();
    return 0;
  }
  const dim3 g((p->Ho * p->Wo * p->C / ve + 255) / 256, p->nimg);
  const FastDiv fwo = make_fastdiv(p->Wo);
  if (p->dtype == AVSR_BF16) hipLaunchKernelGGL(stem_pool_fwd_kernel<bf16>, g, dim3(256), 0, (hipStream_t)stream, *p, fwo);
  else hipLaunchKernelGGL(stem_pool_fwd_kernel<float>, g, dim3(256), 0, (hipStream_t)stream, *p, fwo);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_stem_pool_bwd_apply(const avsr_stem_pool_params* p, void* stream) {
  if (!p || !p->dz || !p->dh || !p->sums || !p->argmax) return AVSR_E_ARG;
  const int ve = p->dtype == AVSR_BF16 ? 8 : 4;
  if (p->C % ve) return AVSR_E_SHAPE;
  if (256 % (p->C / ve)) return AVSR_E_SHAPE;
  if ((int64_t)p->nimg * p->H * p->W >= (1ll << 31)) return AVSR_E_SHAPE;
  if (p->Ho != (p->H + 1) / 2 || p->Wo != (p->W + 1) / 2) return AVSR_E_SHAPE;
  if (!(p->H & 1) && !(p->W & 1) && avsr_opt(AVSR_OPT_STEM_POOL_2X2)) {     // 2x2-block kernel (same result)
    const int64_t nv2 = (int64_t)p->nimg * p->Ho * p->Wo * p->C / ve;
    if (nv2 >= (1ll << 31) || (int64_t)p->nimg * p->H * p->W * p->C / ve >= (1ll << 31)) return AVSR_E_SHAPE;
    const int g2 = bn_grid(nv2, p->C / ve);
    const FastDiv fwo = make_fastdiv(p->Wo), fho = make_fastdiv(p->Ho);
    if (p->dtype == AVSR_BF16) hipLaunchKernelGGL((stem_bwd_apply2_kernel<bf16, 1>), dim3(g2), dim3(256), 0, (hipStream_t)stream, *p, fwo, fho);
    else hipLaunchKernelGGL((stem_bwd_apply2_kernel<float, 1>), dim3(g2), dim3(256), 0, (hipStream_t)stream, *p, fwo, fho);
    AVSR_CHECK_LAUNCH();
    return 0;
  }
  const int g = bn_grid((int64_t)p->nimg * p->H * p->W * p->C / ve, p->C / ve);
  const FastDiv fw = make_fastdiv(p->W), fhw = make_fastdiv(p->H * p->W);
  if (p->dtype == AVSR_BF16) hipLaunchKernelGGL(stem_bwd_apply_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, *p, fw, fhw);
  else hipLaunchKernelGGL(stem_bwd_apply_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, *p, fw, fhw);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_avgpool_fwd(int dtype, int nimg, int P, int C, const void* x, void* y, void* stream) {
  const int ve = dtype == AVSR_BF16 ? 8 : 4;
  if (C % ve) return AVSR_E_SHAPE;
  const int g = avsr_grid((int64_t)nimg * C / ve);
  if (dtype == AVSR_BF16) hipLaunchKernelGGL(avgpool_fwd_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, nimg, P, C, (const bf16*)x, (bf16*)y);
  else hipLaunchKernelGGL(avgpool_fwd_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, nimg, P, C, (const float*)x, (float*)y);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_avgpool_bwd(int dtype, int nimg, int P, int C, const void* dy, void* dx, void* stream) {
  const int ve = dtype == AVSR_BF16 ? 8 : 4;
  if (C % ve) return AVSR_E_SHAPE;
  const int g = avsr_grid((int64_t)nimg * P * C / ve);
  if (dtype == AVSR_BF16) hipLaunchKernelGGL(avgpool_bwd_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, nimg, P, C, (const bf16*)dy, (bf16*)dx);
  else hipLaunchKernelGGL(avgpool_bwd_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, nimg, P, C, (const float*)dy, (float*)dx);
  AVSR_CHECK_LAUNCH();
  return 0;
}
