// Implicit-GEMM convolution (NHWC, grouped) forward / data-grad / weight-grad.
// C-ABI: avsr_conv_fwd / avsr_conv_bwd_data / avsr_conv_bwd_weight (include/avsr_hip.h).
//
//  fwd         C[m = y pixel][co]        = sum_{k=(kh,kw,ci)} x[im2col(m, k)] * w[co][k]
//              (+ fused BatchNorm partial statistics of the stored tile)
//  bwd_data    C[m = x pixel][ci]        = sum_{k=(kh,kw,co)} dy[col2im(m, k)] * w[co][kh][kw][ci]
//  bwd_weight  dw[co][(kh,kw,ci)]       += sum_{m = y pixel} dy[m][co] * x[im2col(m, (kh,kw,ci))]
//              (K = pixels is split over blocks; fp32 atomics into the gradient)
#include "gemm_core.h"

using namespace gemmcore;

namespace {

static int ilog2(int v) { int s = 0; while ((1 << s) < v) ++s; return (1 << s) == v ? s : -1; }

static int make_geom(const avsr_conv_params* p, ConvGeom& g) {
  g.nimg = p->nimg; g.hin = p->hin; g.win = p->win; g.hout = p->hout; g.wout = p->wout;
  g.kh = p->kh; g.kw = p->kw; g.sh = p->sh; g.sw = p->sw; g.ph = p->ph; g.pw = p->pw;
  g.cin = p->cin; g.cout = p->cout; g.ldx = p->ldx; g.ldy = p->ldy;
  g.f_hw_out = make_fastdiv((uint32_t)(p->hout * p->wout));
  g.f_w_out = make_fastdiv((uint32_t)p->wout);
  g.f_hw_in = make_fastdiv((uint32_t)(p->hin * p->win));
  g.f_w_in = make_fastdiv((uint32_t)p->win);
  g.f_kw = make_fastdiv((uint32_t)p->kw);
  g.cin_shift = ilog2(p->cin); g.cout_shift = ilog2(p->cout);
  const int ve = p->dtype == AVSR_BF16 ? 8 : 4;
  if (g.cin_shift < 0 || g.cout_shift < 0 || p->cin < ve || p->cout < ve) return AVSR_E_SHAPE;
  if (p->ldx % ve || p->ldy % ve) return AVSR_E_ALIGN;
  if (p->groups < 1 || p->ldx < (int64_t)p->groups * p->cin || p->ldy < (int64_t)p->groups * p->cout) return AVSR_E_SHAPE;
  return 0;
}

struct ConvArgs {
  ConvGeom g;
  const void* a; const void* b;   // operand bases (group 0)
  int64_t a_gstride, b_gstride, c_gstride;
  int M, N, K, splits, kchunk;
  Epi e;
};

enum { K_FWD = 0, K_DGRAD = 1, K_WGRAD = 2 };

template <typename T, typename OutT, int WM, int WN, int KIND>
__global__ __launch_bounds__(NT) void conv_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using TL = Tile<T, WM, WN>;   // BM/BN only (LDS sizing: conv_lds below)
  const int z = blockIdx.z, grp = z / a.splits, sp = z % a.splits;
  const int m0 = blockIdx.y * TL::BM, n0 = blockIdx.x * TL::BN;
  const T* pa = (const T*)a.a + (int64_t)grp * a.a_gstride;
  const T* pb = (const T*)a.b + (int64_t)grp * a.b_gstride;
  f32x16 acc[2][2];
  const int kbeg = sp * a.kchunk, kend = min(a.K, kbeg + a.kchunk);
  if constexpr (KIND == K_FWD) {
    LdConvK<T, TL::BM, false> la; la.p = pa; la.g = a.g; la.rext = a.M; la.K = a.K;
    LdDenseK<T, TL::BN> lb; lb.p = pb; lb.ld = a.K; lb.rext = a.N; lb.K = a.K;
    mainloop<T, WM, WN>(la, lb, m0, n0, kbeg, kend, acc, smem);
  } else if constexpr (KIND == K_DGRAD) {
    LdConvK<T, TL::BM, true> la; la.p = pa; la.g = a.g; la.rext = a.M; la.K = a.K;
    LdWgtR<T, TL::BN> lb; lb.p = pb; lb.g = a.g; lb.rext = a.N; lb.K = a.K;
    mainloop<T, WM, WN>(la, lb, m0, n0, kbeg, kend, acc, smem);
  } else {
    LdDenseR<T, TL::BM> la; la.p = pa; la.ld = a.g.ldy; la.rext = a.M; la.K = a.K;
    LdConvR<T, TL::BN> lb; lb.p = pb; lb.g = a.g; lb.rext = a.N; lb.K = a.K;
    mainloop<T, WM, WN>(la, lb, m0, n0, kbeg, kend, acc, smem);
  }
  Epi e = a.e;
  e.C = (OutT*)e.C + (int64_t)grp * a.c_gstride;
  if (e.res) e.res = (const T*)e.res + (int64_t)grp * a.c_gstride;
  if (e.preact) e.preact = (T*)e.preact + (int64_t)grp * a.c_gstride;
  if (e.bias) e.bias += (int64_t)grp * a.c_gstride;
  epilogue<T, OutT, WM, WN>(e, m0, n0, acc, smem);
}

template <typename T, typename OutT, int WM, int WN, int KIND>
int launch(const ConvArgs& a, int groups, hipStream_t st) {
  // operand kinds per convolution direction (fwd: K/K, dgrad: K/R, wgrad: R/R)
  using TL = Tile<T, WM, WN, KIND != K_WGRAD, KIND == K_FWD>;
  dim3 grid((a.N + TL::BN - 1) / TL::BN, (a.M + TL::BM - 1) / TL::BM, groups * a.splits);
  if (grid.y > 65535) return AVSR_E_SHAPE;
  hipLaunchKernelGGL((conv_kernel<T, OutT, WM, WN, KIND>), grid, dim3(NT), TL::LDS_BYTES, st, a);
  AVSR_CHECK_LAUNCH();
  return 0;
}

// tile shapes: N <= 64 -> 256x64; M <= 64 -> 64x256; else 128x128
template <typename T, typename OutT, int KIND>
int by_tile(const ConvArgs& a, int groups, hipStream_t st) {
  if (a.N <= 64) return launch<T, OutT, 4, 1, KIND>(a, groups, st);
  if (a.M <= 64) return launch<T, OutT, 1, 4, KIND>(a, groups, st);
  return launch<T, OutT, 2, 2, KIND>(a, groups, st);
}

static int tile_bm(int M, int N) { return N <= 64 ? 256 : (M <= 64 ? 64 : 128); }

static void base_epi(Epi& e) {
  e.alpha = 1.f; e.beta = 0.f; e.bias = nullptr; e.act = 0; e.bwd = 0; e.atomic = 0;
  e.preact = nullptr; e.res = nullptr; e.ldr = 0; e.gate = nullptr; e.drop_p = 0.f; e.seed = 0;
  e.drop_base = 0; e.stats = nullptr; e.stats_tiles = 0;
}

}  // namespace

extern "C" int avsr_conv_stat_tiles(const avsr_conv_params* p) {
  const int M = p->nimg * p->hout * p->wout;
  const int bm = tile_bm(M, p->cout);
  return (M + bm - 1) / bm;
}

extern "C" int avsr_conv_fwd(const avsr_conv_params* p, void* stream) {
  if (!p) return AVSR_E_ARG;
  ConvArgs a;
  int rc = make_geom(p, a.g);
  if (rc) return rc;
  if (!avsr_aligned16(p->x) || !avsr_aligned16(p->w) || !avsr_aligned16(p->y)) return AVSR_E_ALIGN;
  if (p->stats && p->groups != 1) return AVSR_E_ARG;
  a.a = p->x; a.b = p->w;
  a.a_gstride = p->cin; a.b_gstride = (int64_t)p->cout * p->kh * p->kw * p->cin; a.c_gstride = p->cout;
  a.M = p->nimg * p->hout * p->wout; a.N = p->cout; a.K = p->kh * p->kw * p->cin;
  a.splits = 1; a.kchunk = a.K;
  base_epi(a.e);
  a.e.M = a.M; a.e.N = a.N; a.e.C = p->y; a.e.ldc = p->ldy; a.e.stats = p->stats;
  a.e.stats_tiles = avsr_conv_stat_tiles(p);
  a.e.bias = p->bias; a.e.act = p->act; a.e.preact = p->preact; a.e.res = p->res; a.e.ldr = p->ldy;
  if (p->stats && (p->bias || p->act || p->res)) return AVSR_E_ARG;
  if (a.M == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (p->dtype == AVSR_F32) return by_tile<float, float, K_FWD>(a, p->groups, st);
  if (p->dtype == AVSR_BF16) return by_tile<bf16, bf16, K_FWD>(a, p->groups, st);
  return AVSR_E_DTYPE;
}

extern "C" int avsr_conv_bwd_data(const avsr_conv_params* p, void* stream) {
  if (!p) return AVSR_E_ARG;
  ConvArgs a;
  int rc = make_geom(p, a.g);
  if (rc) return rc;
  if (!avsr_aligned16(p->dx) || !avsr_aligned16(p->w) || !avsr_aligned16(p->dy)) return AVSR_E_ALIGN;
  a.a = p->dy; a.b = p->w;
  a.a_gstride = p->cout; a.b_gstride = (int64_t)p->cout * p->kh * p->kw * p->cin; a.c_gstride = p->cin;
  a.M = p->nimg * p->hin * p->win; a.N = p->cin; a.K = p->kh * p->kw * p->cout;
  a.splits = 1; a.kchunk = a.K;
  base_epi(a.e);
  a.e.M = a.M; a.e.N = a.N; a.e.C = p->dx; a.e.ldc = p->ldx; a.e.alpha = p->alpha; a.e.beta = p->beta;
  if (a.M == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (p->dtype == AVSR_F32) return by_tile<float, float, K_DGRAD>(a, p->groups, st);
  if (p->dtype == AVSR_BF16) return by_tile<bf16, bf16, K_DGRAD>(a, p->groups, st);
  return AVSR_E_DTYPE;
}

extern "C" int avsr_conv_bwd_weight(const avsr_conv_params* p, void* stream) {
  if (!p) return AVSR_E_ARG;
  ConvArgs a;
  int rc = make_geom(p, a.g);
  if (rc) return rc;
  if (!avsr_aligned16(p->x) || !avsr_aligned16(p->dy) || !p->dw) return AVSR_E_ALIGN;
  a.a = p->dy; a.b = p->x;
  const int64_t ktot = (int64_t)p->kh * p->kw * p->cin;
  a.a_gstride = p->cout; a.b_gstride = p->cin; a.c_gstride = p->cout * ktot;
  a.M = p->cout; a.N = (int)ktot; a.K = p->nimg * p->hout * p->wout;
  if (a.K == 0) return 0;
  int splits = p->splitk;
  if (splits <= 0) {
    const int bm = tile_bm(a.M, a.N), bn = a.N <= 64 ? 64 : (a.M <= 64 ? 256 : 128);
    const long tiles = (long)((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn) * p->groups;
    long want = (2048 + tiles - 1) / tiles;                 // ~8 blocks per CU
    long maxs = (a.K + 2047) / 2048;                          // keep >= 64 K-tiles per block
    splits = (int)(want < maxs ? want : maxs);
    if (splits < 1) splits = 1;
  }
  a.splits = splits;
  a.kchunk = ((a.K + splits - 1) / splits + BKE - 1) / BKE * BKE;
  a.splits = (a.K + a.kchunk - 1) / a.kchunk;
  base_epi(a.e);
  a.e.M = a.M; a.e.N = a.N; a.e.C = p->dw; a.e.ldc = ktot; a.e.atomic = 1; a.e.alpha = 1.f;
  hipStream_t st = (hipStream_t)stream;
  if (p->dtype == AVSR_F32) return by_tile<float, float, K_WGRAD>(a, p->groups, st);
  if (p->dtype == AVSR_BF16) return by_tile<bf16, float, K_WGRAD>(a, p->groups, st);
  return AVSR_E_DTYPE;
}
