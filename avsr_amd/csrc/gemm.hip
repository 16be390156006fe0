// Dense GEMM with fused epilogue (C-ABI avsr_gemm). Mainloop/epilogue: gemm_core.h.
// Replaces every torch.nn.Linear on the AVSR hot path (forward, data-grad, weight-grad);
// see include/avsr_hip.h for the reference call sites.
#include "gemm_core.h"

using namespace gemmcore;

namespace {

struct DenseArgs {
  int M, N, K, splits, kchunk;
  const void* A; int64_t lda, sA;
  const void* B; int64_t ldb, sB;
  int64_t sC, sR;
  Epi e;
};

template <typename T, typename OutT, int WM, int WN, bool AK, bool BK>
__global__ __launch_bounds__(NT) void dense_kernel(DenseArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using TL = Tile<T, WM, WN, AK, BK>;
  const int z = blockIdx.z, bz = z / a.splits, sp = z % a.splits;
  const int m0 = blockIdx.y * TL::BM, n0 = blockIdx.x * TL::BN;
  using LA = typename std::conditional<AK, LdDenseK<T, TL::BM>, LdDenseR<T, TL::BM>>::type;
  using LB = typename std::conditional<BK, LdDenseK<T, TL::BN>, LdDenseR<T, TL::BN>>::type;
  LA la; la.p = (const T*)a.A + (int64_t)bz * a.sA; la.ld = a.lda; la.rext = a.M; la.K = a.K;
  LB lb; lb.p = (const T*)a.B + (int64_t)bz * a.sB; lb.ld = a.ldb; lb.rext = a.N; lb.K = a.K;
  const int kbeg = sp * a.kchunk, kend = min(a.K, kbeg + a.kchunk);
  f32x16 acc[2][2];
  mainloop<T, WM, WN>(la, lb, m0, n0, kbeg, kend, acc, smem);
  Epi e = a.e;
  e.C = (OutT*)e.C + (int64_t)bz * a.sC;
  if (e.res) e.res = (const T*)e.res + (int64_t)bz * a.sR;
  if (e.preact) e.preact = (T*)e.preact + (int64_t)bz * a.sC;
  if (e.gate) e.gate = (const T*)e.gate + (int64_t)bz * a.sC;
  e.drop_base = (uint64_t)bz * (uint64_t)a.M * (uint64_t)a.N;
  epilogue<T, OutT, WM, WN>(e, m0, n0, acc, smem);
}

template <typename T, typename OutT, int WM, int WN, bool AK, bool BK>
int launch(const DenseArgs& a, int batch, hipStream_t st) {
  using TL = Tile<T, WM, WN, AK, BK>;
  dim3 grid((a.N + TL::BN - 1) / TL::BN, (a.M + TL::BM - 1) / TL::BM, batch * a.splits);
  hipLaunchKernelGGL((dense_kernel<T, OutT, WM, WN, AK, BK>), grid, dim3(NT), TL::LDS_BYTES, st, a);
  AVSR_CHECK_LAUNCH();
  return 0;
}

template <typename T, typename OutT, int WM, int WN>
int by_layout(const avsr_gemm_params* p, const DenseArgs& a, hipStream_t st) {
  if (p->a_kmajor && p->b_kmajor) return launch<T, OutT, WM, WN, true, true>(a, p->batch, st);
  if (p->a_kmajor) return launch<T, OutT, WM, WN, true, false>(a, p->batch, st);
  if (p->b_kmajor) return launch<T, OutT, WM, WN, false, true>(a, p->batch, st);
  return launch<T, OutT, WM, WN, false, false>(a, p->batch, st);
}

template <typename T, typename OutT>
int by_tile(const avsr_gemm_params* p, const DenseArgs& a, hipStream_t st) {
  if (p->N <= 64) return by_layout<T, OutT, 4, 1>(p, a, st);
  if (p->M <= 64) return by_layout<T, OutT, 1, 4>(p, a, st);
  return by_layout<T, OutT, 2, 2>(p, a, st);
}

}  // namespace

extern "C" int avsr_gemm(const avsr_gemm_params* p, void* stream) {
  if (!p) return AVSR_E_ARG;
  if (p->M == 0 || p->N == 0) return 0;
  if (p->M < 0 || p->N < 0 || p->K < 0 || p->batch <= 0) return AVSR_E_SHAPE;
  if (p->dtype != AVSR_F32 && p->dtype != AVSR_BF16) return AVSR_E_DTYPE;
  const int ve = p->dtype == AVSR_BF16 ? 8 : 4;
  if (!avsr_aligned16(p->A) || !avsr_aligned16(p->B)) return AVSR_E_ALIGN;
  if (p->lda % ve || p->ldb % ve || p->strideA % ve || p->strideB % ve) return AVSR_E_ALIGN;
  if ((p->a_kmajor || p->b_kmajor) && (p->K % ve)) return AVSR_E_ALIGN;
  const int splits = p->splitk > 1 ? p->splitk : 1;
  if (splits > 1 && !(p->c_f32 || p->dtype == AVSR_F32)) return AVSR_E_ARG;
  DenseArgs a;
  a.M = p->M; a.N = p->N; a.K = p->K;
  a.splits = splits;
  a.kchunk = ((p->K + splits - 1) / splits + BKE - 1) / BKE * BKE;
  a.A = p->A; a.lda = p->lda; a.sA = p->strideA;
  a.B = p->B; a.ldb = p->ldb; a.sB = p->strideB;
  a.sC = p->strideC; a.sR = p->strideR;
  Epi& e = a.e;
  e.M = p->M; e.N = p->N; e.C = p->C; e.ldc = p->ldc;
  e.alpha = p->alpha; e.beta = p->beta; e.bias = p->bias;
  e.act = p->act; e.bwd = p->epi_bwd; e.atomic = splits > 1;
  e.preact = p->preact; e.res = p->res; e.ldr = p->ldr; e.gate = p->gate;
  e.drop_p = p->drop_p; e.seed = p->seed; e.drop_base = 0; e.stats = nullptr; e.stats_tiles = 0;
  hipStream_t st = (hipStream_t)stream;
  if (p->K == 0) return AVSR_E_SHAPE;
  if (p->dtype == AVSR_F32) return by_tile<float, float>(p, a, st);
  if (p->c_f32) return by_tile<bf16, float>(p, a, st);
  return by_tile<bf16, bf16>(p, a, st);
}
