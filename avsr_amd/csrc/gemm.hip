// GEMM with fused epilogue for gfx950: 128x128x32 block tile, 4 waves (2x2), each wave a
// 64x64 sub-tile = 2x2 v_mfma_f32_32x32x16_bf16 accumulators (fp32). Operands are staged
// global -> registers -> LDS (double-buffered, one barrier per K-tile; the next tile's
// global loads are in flight while the current tile's MFMAs run). LDS rows are padded by
// one 16-byte vector, which makes the ds_read_b128 fragment reads conflict-free.
//
// Replaces every torch.nn.Linear on the AVSR hot path (see include/avsr_hip.h).
// fp32 storage ("parity mode") runs the same tiles with each operand split into
// bf16 hi + lo and three MFMA products (hi*hi + hi*lo + lo*hi) per step.
#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BKE = 32, NT = 256;

template <typename T> struct Cfg {
  static constexpr int VE = 16 / (int)sizeof(T);   // elements per 16-byte vector
  static constexpr int ROW = BKE + VE;             // padded LDS row (elements)
  static constexpr int TILE = BM * ROW;            // elements per operand tile
  static constexpr int NVEC = BM * BKE / VE;       // 16-byte vectors per operand tile
  static constexpr int VPT = NVEC / NT;            // vectors per thread
};

struct GemmArgs {
  int M, N, K;
  const void* A; int64_t lda, sA;
  const void* B; int64_t ldb, sB;
  void* C; int64_t ldc, sC;
  float alpha, beta;
  const float* bias;
  int act, bwd;
  void* preact;
  const void* res; int64_t ldr, sR;
  const void* gate;
  float drop_p;
  uint64_t seed;
};

// Load one operand tile (rows r0..r0+127 of the operand, k0..k0+31) into registers.
template <typename T, bool KMAJ>
AVSR_DEV void gload(const T* __restrict__ base, int64_t ld, int r0, int rext, int k0, int K,
                    v16 (&reg)[Cfg<T>::VPT], int tid) {
  constexpr int VE = Cfg<T>::VE;
#pragma unroll
  for (int i = 0; i < Cfg<T>::VPT; ++i) {
    int v = tid + i * NT;
    const T* p;
    bool ok;
    if constexpr (KMAJ) {
      int r = v / (BKE / VE), kv = v % (BKE / VE);
      int k = k0 + kv * VE;
      ok = (r0 + r < rext) && (k < K);
      p = base + (int64_t)(r0 + r) * ld + k;
    } else {
      int kk = v / (BM / VE), rv = v % (BM / VE);
      int k = k0 + kk, rr = r0 + rv * VE;
      ok = (k < K) && (rr < rext);
      p = base + (int64_t)k * ld + rr;
    }
    if (ok) reg[i] = *(const v16*)p;
    else { reg[i].w[0] = reg[i].w[1] = reg[i].w[2] = reg[i].w[3] = 0u; }
  }
}

template <typename T, bool KMAJ>
AVSR_DEV void lstore(T* lds, const v16 (&reg)[Cfg<T>::VPT], int tid) {
  constexpr int VE = Cfg<T>::VE, ROW = Cfg<T>::ROW;
#pragma unroll
  for (int i = 0; i < Cfg<T>::VPT; ++i) {
    int v = tid + i * NT;
    if constexpr (KMAJ) {
      int r = v / (BKE / VE), kv = v % (BKE / VE);
      *(v16*)(lds + r * ROW + kv * VE) = reg[i];
    } else {
      int kk = v / (BM / VE), rv = v % (BM / VE);
      const T* vals = (const T*)&reg[i];
#pragma unroll
      for (int e = 0; e < VE; ++e) lds[(rv * VE + e) * ROW + kk] = vals[e];
    }
  }
}

// Read the MFMA operand fragment: rows rb..rb+31 (row = lane&31), k = s*16 + 8*(lane>>5) + 0..7
template <typename T>
AVSR_DEV void frag(const T* lds, int rb, int s, int lane, bf16x8& hi, bf16x8& lo) {
  constexpr int ROW = Cfg<T>::ROW;
  const T* p = lds + (rb + (lane & 31)) * ROW + s * 16 + 8 * (lane >> 5);
  if constexpr (sizeof(T) == 2) {
    hi = *(const bf16x8*)p;
  } else {
    f32x4 x0 = *(const f32x4*)p, x1 = *(const f32x4*)(p + 4);
    float x[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    split8(x, hi, lo);
  }
}

template <typename T, typename OutT, bool AK, bool BK>
__global__ __launch_bounds__(NT) void gemm_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* lA = (T*)smem;                 // [2][TILE]
  T* lB = lA + 2 * Cfg<T>::TILE;    // [2][TILE]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int bz = blockIdx.z;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const T* A = (const T*)g.A + (int64_t)bz * g.sA;
  const T* B = (const T*)g.B + (int64_t)bz * g.sB;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  v16 ra[Cfg<T>::VPT], rb[Cfg<T>::VPT];
  const int nk = (g.K + BKE - 1) / BKE;
  gload<T, AK>(A, g.lda, m0, g.M, 0, g.K, ra, tid);
  gload<T, BK>(B, g.ldb, n0, g.N, 0, g.K, rb, tid);
  lstore<T, AK>(lA, ra, tid);
  lstore<T, BK>(lB, rb, tid);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      gload<T, AK>(A, g.lda, m0, g.M, (kt + 1) * BKE, g.K, ra, tid);
      gload<T, BK>(B, g.ldb, n0, g.N, (kt + 1) * BKE, g.K, rb, tid);
    }
    const T* cA = lA + cur * Cfg<T>::TILE;
    const T* cB = lB + cur * Cfg<T>::TILE;
#pragma unroll
    for (int s = 0; s < BKE / 16; ++s) {
      bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) frag<T>(cA, wm * 64 + i * 32, s, lane, ah[i], al[i]);
#pragma unroll
      for (int j = 0; j < 2; ++j) frag<T>(cB, wn * 64 + j * 32, s, lane, bh[j], bl[j]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = mfma32(ah[i], bh[j], acc[i][j]);
          if constexpr (sizeof(T) == 4) {
            acc[i][j] = mfma32(ah[i], bl[j], acc[i][j]);
            acc[i][j] = mfma32(al[i], bh[j], acc[i][j]);
          }
        }
    }
    if (more) {
      lstore<T, AK>(lA + (cur ^ 1) * Cfg<T>::TILE, ra, tid);
      lstore<T, BK>(lB + (cur ^ 1) * Cfg<T>::TILE, rb, tid);
    }
    __syncthreads();
  }

  // ---- epilogue ----
  OutT* C = (OutT*)g.C + (int64_t)bz * g.sC;
  const T* R = g.res ? (const T*)g.res + (int64_t)bz * g.sR : nullptr;
  T* P = g.preact ? (T*)g.preact + (int64_t)bz * g.sC : nullptr;
  const T* G = g.gate ? (const T*)g.gate + (int64_t)bz * g.sC : nullptr;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 64 + j * 32 + (lane & 31);
      if (col >= g.N) continue;
      const float bcol = (g.bias && !g.bwd) ? g.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row >= g.M) continue;
        float v = g.alpha * acc[i][j][r];
        const int64_t off = (int64_t)row * g.ldc + col;
        const uint64_t didx = ((uint64_t)bz * g.M + row) * (uint64_t)g.N + col;
        if (!g.bwd) {
          v += bcol;
          if (P) P[off] = from_f<T>(v);
          v = act_fwd(g.act, v);
          if (g.drop_p > 0.f) v *= drop_scale(g.drop_p, g.seed, didx);
          if (R) v += to_f(R[(int64_t)row * g.ldr + col]);
        } else {
          if (g.drop_p > 0.f) v *= drop_scale(g.drop_p, g.seed, didx);
          if (G) v *= act_bwd(g.act, to_f(G[off]));
        }
        if (g.beta != 0.f) v += g.beta * to_f(C[off]);
        C[off] = from_f<OutT>(v);
      }
    }
}

template <typename T, typename OutT, bool AK, bool BK>
int launch(const GemmArgs& g, int batch, hipStream_t st) {
  dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, batch);
  size_t lds = 4 * (size_t)Cfg<T>::TILE * sizeof(T);
  hipLaunchKernelGGL((gemm_kernel<T, OutT, AK, BK>), grid, dim3(NT), lds, st, g);
  AVSR_CHECK_LAUNCH();
  return 0;
}

template <typename T, typename OutT>
int dispatch_layout(const avsr_gemm_params* p, const GemmArgs& g, hipStream_t st) {
  if (p->a_kmajor && p->b_kmajor) return launch<T, OutT, true, true>(g, p->batch, st);
  if (p->a_kmajor && !p->b_kmajor) return launch<T, OutT, true, false>(g, p->batch, st);
  if (!p->a_kmajor && p->b_kmajor) return launch<T, OutT, false, true>(g, p->batch, st);
  return launch<T, OutT, false, false>(g, p->batch, st);
}

}  // namespace

extern "C" int avsr_gemm(const avsr_gemm_params* p, void* stream) {
  if (!p) return AVSR_E_ARG;
  if (p->M <= 0 || p->N <= 0 || p->K <= 0 || p->batch <= 0) return p->M == 0 || p->N == 0 ? 0 : AVSR_E_SHAPE;
  if (p->dtype != AVSR_F32 && p->dtype != AVSR_BF16) return AVSR_E_DTYPE;
  const int ve = p->dtype == AVSR_BF16 ? 8 : 4;
  if (!avsr_aligned16(p->A) || !avsr_aligned16(p->B)) return AVSR_E_ALIGN;
  if (p->lda % ve || p->ldb % ve || p->strideA % ve || p->strideB % ve) return AVSR_E_ALIGN;
  if ((p->a_kmajor || p->b_kmajor) && (p->K % ve)) return AVSR_E_ALIGN;
  GemmArgs g;
  g.M = p->M; g.N = p->N; g.K = p->K;
  g.A = p->A; g.lda = p->lda; g.sA = p->strideA;
  g.B = p->B; g.ldb = p->ldb; g.sB = p->strideB;
  g.C = p->C; g.ldc = p->ldc; g.sC = p->strideC;
  g.alpha = p->alpha; g.beta = p->beta; g.bias = p->bias;
  g.act = p->act; g.bwd = p->epi_bwd; g.preact = p->preact;
  g.res = p->res; g.ldr = p->ldr; g.sR = p->strideR; g.gate = p->gate;
  g.drop_p = p->drop_p; g.seed = p->seed;
  hipStream_t st = (hipStream_t)stream;
  if (p->dtype == AVSR_F32) return dispatch_layout<float, float>(p, g, st);
  if (p->c_f32) return dispatch_layout<bf16, float>(p, g, st);
  return dispatch_layout<bf16, bf16>(p, g, st);
}
