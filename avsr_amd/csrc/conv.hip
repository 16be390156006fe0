// Implicit-GEMM convolution (NHWC, grouped) forward / data-grad / weight-grad.
// C-ABI: avsr_conv_fwd / avsr_conv_bwd_data / avsr_conv_bwd_weight (include/avsr_hip.h).
//
//  fwd         C[m = y pixel][co]        = sum_{k=(kh,kw,ci)} x[im2col(m, k)] * w[co][k]
//              (+ fused BatchNorm partial statistics of the stored tile)
//  bwd_data    C[m = x pixel][ci]        = sum_{k=(kh,kw,co)} dy[col2im(m, k)] * w[co][kh][kw][ci]
//  bwd_weight  dw[co][(kh,kw,ci)]       += sum_{m = y pixel} dy[m][co] * x[im2col(m, (kh,kw,ci))]
//              (K = pixels is split over blocks; fp32 atomics into the gradient)
#include "gemm_core.h"
#include "gemm_glds.h"

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
  g.ktot_w = p->kh * p->kw * p->cin; g.tap_kfw = p->kw; g.tap_kh0 = 0; g.tap_kw0 = 0; g.tap_step = 1;
  const int ve = p->dtype == AVSR_BF16 ? 8 : 4;
  if (g.cin_shift < 0 || g.cout_shift < 0 || p->cin < ve || p->cout < ve) return AVSR_E_SHAPE;
  if (p->ldx % ve || p->ldy % ve) return AVSR_E_ALIGN;
  if (p->groups < 1 || p->ldx < (int64_t)p->groups * p->cin || p->ldy < (int64_t)p->groups * p->cout) return AVSR_E_SHAPE;
  return 0;
}

struct ConvArgs {
  ConvGeom g;
  uint32_t a_bytes, b_bytes;      // per-group operand extents for the buffer-DMA loaders (0: pointer loaders)
  const void* a; const void* b;   // operand bases (group 0)
  int64_t a_gstride, b_gstride, c_gstride;
  int M, N, K, splits, kchunk;
  float* ws;                      // bwd_weight split-K slabs [groups][splits][M][N] (nullptr: direct / atomics)
  Epi e;
  gemmg::BnrArgs bnr;             // K_DGRAD_BNR: BatchNorm-backward reduction of the stored tile
};

// K_DGRAD_BNR + r: data-grad whose epilogue is gemmg::epilogue_bnr with residual mode r
// (0 none, 1 identity, 2 under its own BN); bf16 LDS-DMA path only
enum { K_FWD = 0, K_DGRAD = 1, K_WGRAD = 2, K_DGRAD_BNR = 3 };

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
  if (KIND == K_WGRAD && a.ws) e.C = a.ws + ((int64_t)grp * a.splits + sp) * a.M * a.N;
  else e.C = (OutT*)e.C + (int64_t)grp * a.c_gstride;
  if (e.res) e.res = (const T*)e.res + (int64_t)grp * a.c_gstride;
  if (e.preact) e.preact = (T*)e.preact + (int64_t)grp * a.c_gstride;
  if (e.bias) e.bias += (int64_t)grp * a.c_gstride;
  epilogue<T, OutT, WM, WN>(e, m0, n0, acc, smem);
}

// ---------------------------------------------------------------- LDS-DMA (bf16) loaders
// Same operand views as the register-staged loaders above, but every 16-byte vector is
// DMA'd straight into the swizzled LDS image (gemm_glds.h); invalid taps -> zero line.
using gemmg::GBK;
using gemmg::glds16;
using gemmg::g_zero_line;

// A of forward (TRANSP=false: r = output pixel, gather x) / data-grad (TRANSP=true: r = input
// pixel, gather dy): k-major image, k = (kh, kw, c) with c fastest.
template <int R, int NW, bool TRANSP> struct GConvK {
  static constexpr bool KMAJ = true;
  static constexpr int SLOTS = R / 8 / NW;
  const bf16* p; ConvGeom g; int kend;
  int pn[SLOTS], ph_[SLOTS], pw_[SLOTS], kc[SLOTS];
  AVSR_DEV void init(const bf16* base, const ConvGeom& g_, int r0, int rext, int kend_, int wave, int lane) {
    p = base; g = g_; kend = kend_;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int pc = i * NW + wave, pr = pc * 8 + (lane >> 3);
      kc[i] = ((lane & 7) ^ ((pr >> 1) & 7)) * 8;
      const int r = r0 + pr;
      if (r >= rext) { pn[i] = 0; ph_[i] = -1000000; pw_[i] = 0; continue; }
      if (!TRANSP) {
        uint32_t n = fdiv(r, g.f_hw_out); uint32_t rem = r - n * g.f_hw_out.d;
        uint32_t oh = fdiv(rem, g.f_w_out); uint32_t ow = rem - oh * g.f_w_out.d;
        pn[i] = n * g.hin * g.win; ph_[i] = oh * g.sh - g.ph; pw_[i] = ow * g.sw - g.pw;
      } else {
        uint32_t n = fdiv(r, g.f_hw_in); uint32_t rem = r - n * g.f_hw_in.d;
        uint32_t h = fdiv(rem, g.f_w_in); uint32_t w = rem - h * g.f_w_in.d;
        pn[i] = n * g.hout * g.wout; ph_[i] = h + g.ph; pw_[i] = w + g.pw;
      }
    }
  }
  AVSR_DEV void issue(char* img, int k0, int wave) const {
    const int cs = TRANSP ? g.cout_shift : g.cin_shift;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int k = k0 + kc[i];
      const int c = k & ((1 << cs) - 1), khw = k >> cs;
      const int kh = fdiv(khw, g.f_kw), kw = khw - kh * g.f_kw.d;
      bool ok = k < kend;
      int64_t off;
      if (!TRANSP) {
        const int ih = ph_[i] + kh, iw = pw_[i] + kw;
        ok = ok && ih >= 0 && ih < g.hin && iw >= 0 && iw < g.win;
        off = (int64_t)(pn[i] + ih * g.win + iw) * g.ldx + c;
      } else {
        const int th = ph_[i] - kh, tw = pw_[i] - kw;
        const int oh = th / g.sh, ow = tw / g.sw;
        ok = ok && th >= 0 && tw >= 0 && oh * g.sh == th && ow * g.sw == tw && oh < g.hout && ow < g.wout;
        off = (int64_t)(pn[i] + oh * g.wout + ow) * g.ldy + c;
      }
      glds16(ok ? (const void*)(p + off) : (const void*)g_zero_line, img + (i * NW + wave) * 1024);
    }
  }
};

// B of data-grad: weight [cout][kh][kw][cin] viewed as (r = cin, k = (kh, kw, cout)); r-contiguous.
template <int R, int NW> struct GWgtR {
  static constexpr bool KMAJ = false;
  static constexpr int CPR = R / 8, RPP = 64 / CPR, SLOTS = GBK / RPP / NW;
  const bf16* p; ConvGeom g; int kend;
  int kr[SLOTS], rr[SLOTS];
  AVSR_DEV void init(const bf16* base, const ConvGeom& g_, int r0, int rext, int kend_, int wave, int lane) {
    p = base; g = g_; kend = kend_;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int pc = i * NW + wave, pk = pc * RPP + lane / CPR;
      const int c = (lane % CPR) ^ gemmg::rswz<CPR>(pk);
      kr[i] = pk;
      rr[i] = r0 + c * 8 < rext ? r0 + c * 8 : -1;
    }
  }
  AVSR_DEV void issue(char* img, int k0, int wave) const {
    const int ktot = g.kh * g.kw * g.cin;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int k = k0 + kr[i];
      const int co = k & ((1 << g.cout_shift) - 1), khw = k >> g.cout_shift;
      const bool ok = k < kend && rr[i] >= 0;
      glds16(ok ? (const void*)(p + (int64_t)co * ktot + khw * g.cin + rr[i]) : (const void*)g_zero_line,
             img + (i * NW + wave) * 1024);
    }
  }
};

// B of weight-grad: r = (kh, kw, cin) (vectors along cin), k = output pixel; r-contiguous.
template <int R, int NW> struct GConvR {
  static constexpr bool KMAJ = false;
  static constexpr int CPR = R / 8, RPP = 64 / CPR, SLOTS = GBK / RPP / NW;
  const bf16* p; ConvGeom g; int kend;
  int kr[SLOTS], rk[SLOTS], rw[SLOTS], rc[SLOTS];
  AVSR_DEV void init(const bf16* base, const ConvGeom& g_, int r0, int rext, int kend_, int wave, int lane) {
    p = base; g = g_; kend = kend_;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int pc = i * NW + wave, pk = pc * RPP + lane / CPR;
      const int r = r0 + ((lane % CPR) ^ gemmg::rswz<CPR>(pk)) * 8;
      kr[i] = pk;
      if (r >= rext) { rk[i] = -1000000; rw[i] = 0; rc[i] = 0; continue; }
      const int c = r & ((1 << g.cin_shift) - 1), khw = r >> g.cin_shift;
      const int kh = fdiv(khw, g.f_kw);
      rk[i] = kh; rw[i] = khw - kh * g.f_kw.d; rc[i] = c;
    }
  }
  AVSR_DEV void issue(char* img, int k0, int wave) const {
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int k = k0 + kr[i];
      bool ok = k < kend;
      const uint32_t kk = ok ? k : 0;
      const uint32_t n = fdiv(kk, g.f_hw_out), rem = kk - n * g.f_hw_out.d;
      const uint32_t oh = fdiv(rem, g.f_w_out), ow = rem - oh * g.f_w_out.d;
      const int ih = (int)oh * g.sh - g.ph + rk[i], iw = (int)ow * g.sw - g.pw + rw[i];
      ok = ok && ih >= 0 && ih < g.hin && iw >= 0 && iw < g.win;
      glds16(ok ? (const void*)(p + (int64_t)(n * g.hin * g.win + ih * g.win + iw) * g.ldx + rc[i])
                : (const void*)g_zero_line,
             img + (i * NW + wave) * 1024);
    }
  }
};

// ---------------------------------------------------------------- buffer-DMA conv loaders
// Tap-uniform K-tiles: with cin (forward) / cout (data-grad) a multiple of 64, one K-tile of
// 64 lies inside one (kh, kw) tap, so the tap decomposition is wave-uniform (scalar) and a
// lane's work per DMA piece is its bounds check and one add (see gemm_glds.h BDenseK).
using gemmg::OOB;
using gemmg::bglds16;
using gemmg::make_rsrc;

// forward A: r = output pixel, gather x
template <int R, int NW> struct BConvK {
  static constexpr bool KMAJ = true;
  static constexpr int SLOTS = R / 8 / NW;
  __amdgpu_buffer_rsrc_t rs; ConvGeom g;
  int ih0[SLOTS], iw0[SLOTS], ro[SLOTS];
  AVSR_DEV void init(const bf16* base, uint32_t bytes, const ConvGeom& g_, int r0, int rext, int wave, int lane) {
    rs = make_rsrc(base, bytes); g = g_;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int pc = i * NW + wave, pr = pc * 8 + (lane >> 3);
      const int kc = ((lane & 7) ^ ((pr >> 1) & 7)) * 8;
      const int r = r0 + pr;
      if (r >= rext) { ih0[i] = -1000000; iw0[i] = 0; ro[i] = 0; continue; }
      const uint32_t n = fdiv(r, g.f_hw_out), rem = r - n * g.f_hw_out.d;
      const uint32_t oh = fdiv(rem, g.f_w_out), ow = rem - oh * g.f_w_out.d;
      ih0[i] = oh * g.sh - g.ph; iw0[i] = ow * g.sw - g.pw;
      ro[i] = (int)((((int64_t)n * g.hin * g.win + (int64_t)ih0[i] * g.win + iw0[i]) * g.ldx + kc) * 2);
    }
  }
  AVSR_DEV void issue(char* img, int k0, int wave) const {
    const int khw = k0 >> g.cin_shift, cb = k0 & ((1 << g.cin_shift) - 1);
    const int kh = (int)fdiv(khw, g.f_kw), kw = khw - kh * (int)g.f_kw.d;
    const int tap = (int)(((int64_t)(kh * g.win + kw) * g.ldx + cb) * 2);
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const bool ok = (unsigned)(ih0[i] + kh) < (unsigned)g.hin && (unsigned)(iw0[i] + kw) < (unsigned)g.win;
      bglds16(rs, ok ? (uint32_t)(ro[i] + tap) : OOB, 0u, img + (i * NW + wave) * 1024);
    }
  }
};

// data-grad A: r = input pixel, gather dy at ((h+ph-kh)/sh, (w+pw-kw)/sw); strides 1 or 2
template <int R, int NW> struct BConvKT {
  static constexpr bool KMAJ = true;
  static constexpr int SLOTS = R / 8 / NW;
  __amdgpu_buffer_rsrc_t rs; ConvGeom g;
  int th0[SLOTS], tw0[SLOTS], ro[SLOTS];
  AVSR_DEV void init(const bf16* base, uint32_t bytes, const ConvGeom& g_, int r0, int rext, int wave, int lane) {
    rs = make_rsrc(base, bytes); g = g_;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int pc = i * NW + wave, pr = pc * 8 + (lane >> 3);
      const int kc = ((lane & 7) ^ ((pr >> 1) & 7)) * 8;
      const int r = r0 + pr;
      if (r >= rext) { th0[i] = -1000000; tw0[i] = 0; ro[i] = 0; continue; }
      const uint32_t n = fdiv(r, g.f_hw_in), rem = r - n * g.f_hw_in.d;
      const uint32_t h = fdiv(rem, g.f_w_in), w = rem - h * g.f_w_in.d;
      th0[i] = h + g.ph; tw0[i] = w + g.pw;
      ro[i] = (int)(((int64_t)n * g.hout * g.wout * g.ldy + kc) * 2);
    }
  }
  AVSR_DEV void issue(char* img, int k0, int wave) const {
    const int khw = k0 >> g.cout_shift, cb = k0 & ((1 << g.cout_shift) - 1);
    const int kh = (int)fdiv(khw, g.f_kw), kw = khw - kh * (int)g.f_kw.d;
    const int ldy2 = (int)g.ldy * 2, cb2 = cb * 2;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int th = th0[i] - kh, tw = tw0[i] - kw;
      bool ok;
      int pix;
      if (g.sh == 1) {
        ok = (unsigned)th < (unsigned)g.hout && (unsigned)tw < (unsigned)g.wout;
        pix = th * g.wout + tw;
      } else {
        ok = ((th | tw) & 1) == 0 && (unsigned)(th >> 1) < (unsigned)g.hout && (unsigned)(tw >> 1) < (unsigned)g.wout;
        pix = (th >> 1) * g.wout + (tw >> 1);
      }
      bglds16(rs, ok ? (uint32_t)(ro[i] + pix * ldy2 + cb2) : OOB, 0u, img + (i * NW + wave) * 1024);
    }
  }
};

// data-grad B: weight [cout][kh][kw][cin] as (r = cin, k = (kh, kw, cout)), r-contiguous
template <int R, int NW> struct BWgtR {
  static constexpr bool KMAJ = false;
  static constexpr int CPR = R / 8, RPP = 64 / CPR, SLOTS = GBK / RPP / NW;
  __amdgpu_buffer_rsrc_t rs; ConvGeom g;
  uint32_t vo[SLOTS];
  AVSR_DEV void init(const bf16* base, uint32_t bytes, const ConvGeom& g_, int r0, int rext, int wave, int lane) {
    rs = make_rsrc(base, bytes); g = g_;
    const int ktot = g.ktot_w;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int pc = i * NW + wave, pk = pc * RPP + lane / CPR;
      const int r = r0 + ((lane % CPR) ^ gemmg::rswz<CPR>(pk)) * 8;
      vo[i] = r < rext ? (uint32_t)(((int64_t)pk * ktot + r) * 2) : OOB;
    }
  }
  AVSR_DEV void issue(char* img, int k0, int wave) const {
    const int ktot = g.ktot_w;
    int tap = k0 >> g.cout_shift;
    if (g.tap_step != 1) {      // parity class of a stride-2 data-grad: class tap (u, v) -> kernel tap
      const int u = (int)fdiv(tap, g.f_kw), v = tap - u * (int)g.f_kw.d;
      tap = (g.tap_kh0 + g.tap_step * u) * g.tap_kfw + g.tap_kw0 + g.tap_step * v;
    }
    const uint32_t so = (uint32_t)((((int64_t)(k0 & ((1 << g.cout_shift) - 1))) * ktot + (int64_t)tap * g.cin) * 2);
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) bglds16(rs, vo[i], so, img + (i * NW + wave) * 1024);
  }
};

// weight-grad B: r = (kh, kw, cin) (vectors along cin), k = output pixel; r-contiguous
template <int R, int NW> struct BConvR {
  static constexpr bool KMAJ = false;
  static constexpr int CPR = R / 8, RPP = 64 / CPR, SLOTS = GBK / RPP / NW;
  __amdgpu_buffer_rsrc_t rs; ConvGeom g; int kend;
  int kr[SLOTS], rk[SLOTS], rw[SLOTS], rc[SLOTS];
  AVSR_DEV void init(const bf16* base, uint32_t bytes, const ConvGeom& g_, int r0, int rext, int kend_, int wave, int lane) {
    rs = make_rsrc(base, bytes); g = g_; kend = kend_;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int pc = i * NW + wave, pk = pc * RPP + lane / CPR;
      const int r = r0 + ((lane % CPR) ^ gemmg::rswz<CPR>(pk)) * 8;
      kr[i] = pk;
      if (r >= rext) { rk[i] = -1000000; rw[i] = 0; rc[i] = 0; continue; }
      const int c = r & ((1 << g.cin_shift) - 1), khw = r >> g.cin_shift;
      const int kh = fdiv(khw, g.f_kw);
      rk[i] = kh - g.ph; rw[i] = khw - kh * g.f_kw.d - g.pw; rc[i] = c * 2;
    }
  }
  AVSR_DEV void issue(char* img, int k0, int wave) const {
    const int ldx2 = (int)g.ldx * 2;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int k = k0 + kr[i];
      const uint32_t kk = k < kend ? k : 0;
      const uint32_t n = fdiv(kk, g.f_hw_out), rem = kk - n * g.f_hw_out.d;
      const uint32_t oh = fdiv(rem, g.f_w_out), ow = rem - oh * g.f_w_out.d;
      const int ih = (int)oh * g.sh + rk[i], iw = (int)ow * g.sw + rw[i];
      const bool ok = k < kend && (unsigned)ih < (unsigned)g.hin && (unsigned)iw < (unsigned)g.win;
      const uint32_t v = (uint32_t)(((int)n * g.hin * g.win + ih * g.win + iw) * ldx2 + rc[i]);
      bglds16(rs, ok ? v : OOB, 0u, img + (i * NW + wave) * 1024);
    }
  }
};

// dense wrappers with the conv loaders' init signature
template <int R, int NW> struct GDenseKc : gemmg::GDenseK<R, NW> {
  AVSR_DEV void init(const bf16* base, int64_t ld, const ConvGeom&, int r0, int rext, int kend, int wave, int lane) {
    gemmg::GDenseK<R, NW>::init(base, ld, r0, rext, kend, wave, lane);
  }
};

template <typename OutT, int KIND, class CF>
__global__ __launch_bounds__(CF::NTH, CF::MINB) void conv_glds_kernel(ConvArgs a, int tiles_m, int tiles_n) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int id = gemmg::xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn, z;
  gemmg::tile_of(id, tiles_m, tiles_n, tm, tn, z);
  const int grp = z / a.splits, sp = z % a.splits;
  const int m0 = tm * CF::BM, n0 = tn * CF::BN;
  const bf16* pa = (const bf16*)a.a + (int64_t)grp * a.a_gstride;
  const bf16* pb = (const bf16*)a.b + (int64_t)grp * a.b_gstride;
  const int kbeg = sp * a.kchunk, kend = min(a.K, kbeg + a.kchunk);
  const int nk = (kend - kbeg + GBK - 1) / GBK;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  f32x4 acc[CF::TM][CF::TN];
  if (a.a_bytes) {                // buffer-DMA loaders (tap-uniform K-tiles, extents < 2 GiB)
    if constexpr (KIND == K_FWD) {
      BConvK<CF::BM, CF::NW> la; la.init(pa, a.a_bytes, a.g, m0, a.M, wave, lane);
      gemmg::BDenseK<CF::BN, CF::NW> lb; lb.init(pb, a.b_bytes, a.K, n0, a.N, kend, wave, lane);
      gemmg::mainloop_glds<CF>(la, lb, kbeg, nk, acc, smem);
    } else if constexpr (KIND == K_DGRAD || KIND >= K_DGRAD_BNR) {
      BConvKT<CF::BM, CF::NW> la; la.init(pa, a.a_bytes, a.g, m0, a.M, wave, lane);
      BWgtR<CF::BN, CF::NW> lb; lb.init(pb, a.b_bytes, a.g, n0, a.N, wave, lane);
      gemmg::mainloop_glds<CF>(la, lb, kbeg, nk, acc, smem);
    } else {
      gemmg::BDenseR<CF::BM, CF::NW> la; la.init(pa, a.a_bytes, a.g.ldy, m0, a.M, kend, wave, lane);
      BConvR<CF::BN, CF::NW> lb; lb.init(pb, a.b_bytes, a.g, n0, a.N, kend, wave, lane);
      gemmg::mainloop_glds<CF>(la, lb, kbeg, nk, acc, smem);
    }
  } else if constexpr (KIND == K_FWD) {
    GConvK<CF::BM, CF::NW, false> la; la.init(pa, a.g, m0, a.M, kend, wave, lane);
    gemmg::GDenseK<CF::BN, CF::NW> lb; lb.init(pb, a.K, n0, a.N, kend, wave, lane);
    gemmg::mainloop_glds<CF>(la, lb, kbeg, nk, acc, smem);
  } else if constexpr (KIND == K_DGRAD || KIND >= K_DGRAD_BNR) {
    GConvK<CF::BM, CF::NW, true> la; la.init(pa, a.g, m0, a.M, kend, wave, lane);
    GWgtR<CF::BN, CF::NW> lb; lb.init(pb, a.g, n0, a.N, kend, wave, lane);
    gemmg::mainloop_glds<CF>(la, lb, kbeg, nk, acc, smem);
  } else {
    gemmg::GDenseR<CF::BM, CF::NW> la; la.init(pa, a.g.ldy, m0, a.M, kend, wave, lane);
    GConvR<CF::BN, CF::NW> lb; lb.init(pb, a.g, n0, a.N, kend, wave, lane);
    gemmg::mainloop_glds<CF>(la, lb, kbeg, nk, acc, smem);
  }
  if constexpr (KIND >= K_DGRAD_BNR) {
    gemmg::epilogue_bnr<CF, KIND - K_DGRAD_BNR>(a.e, a.bnr, m0, n0, acc, smem);
    return;
  }
  Epi e = a.e;
  if (KIND == K_WGRAD && a.ws) e.C = a.ws + ((int64_t)grp * a.splits + sp) * a.M * a.N;
  else e.C = (OutT*)e.C + (int64_t)grp * a.c_gstride;
  if (e.res) e.res = (const bf16*)e.res + (int64_t)grp * a.c_gstride;
  if (e.preact) e.preact = (bf16*)e.preact + (int64_t)grp * a.c_gstride;
  if (e.bias) e.bias += (int64_t)grp * a.c_gstride;
  gemmg::epilogue_g<bf16, OutT, CF>(e, m0, n0, acc, smem);
}

using CCfg128 = gemmg::GCfg<2, 2, 2, 2, 2>;    // 128x128
using CCfg256x64 = gemmg::GCfg<4, 1, 2, 2, 2>; // 256x64  (N <= 64: cout / cin = 64)
using CCfg64x256 = gemmg::GCfg<1, 4, 2, 2, 2>; // 64x256  (M <= 64: weight-grad with cout = 64)
using CCfg192 = gemmg::GCfg<2, 2, 3, 2, 2>;    // 192x128 (96x64 per wave), k-major A (fwd / data-grad)

template <typename OutT, int KIND, class CF>
int launch_glds(const ConvArgs& a, int groups, hipStream_t st) {
  const int tm = (a.M + CF::BM - 1) / CF::BM, tn = (a.N + CF::BN - 1) / CF::BN;
  if (a.e.stats && a.e.stats_tiles != tm) return AVSR_E_SHAPE;   // partials sized for another tile height
  const long nwg = (long)tm * tn * groups * a.splits;
  if (nwg > 0x7fffffffL) return AVSR_E_SHAPE;
  hipLaunchKernelGGL((conv_glds_kernel<OutT, KIND, CF>), dim3((unsigned)nwg), dim3(CF::NTH), CF::LDS_BYTES, st, a,
                     tm, tn);
  AVSR_CHECK_LAUNCH();
  return 0;
}

static bool conv_glds_enabled() { return true; }

// 192x128 for the k-major-A directions (forward, data-grad) where it still runs >= 2 blocks per
// CU and its rounds carry no more work than 128x128's (the dense rule, gemm.hip tile_cfg):
// ResNet stages 2-3 at C2 (video fwd 9.09 -> 8.83 ms, bwd 17.13 -> 16.84, profiles/r02_resnet_c192_ab.txt)
static bool conv192(int M, int N, int groups) {
  if (N <= 64 || M <= 64 || !conv_glds_enabled() || !avsr_opt(AVSR_OPT_CONV_192)) return false;
  const long tn = (long)((N + 127) / 128) * groups;
  const long n128 = ((long)((M + 127) / 128) * tn + 255) / 256, n192 = ((long)((M + 191) / 192) * tn + 255) / 256;
  return n192 >= 2 && 3 * n192 * 50 <= 2 * n128 * 51;
}

template <typename OutT, int KIND>
int glds_by_tile(const ConvArgs& a, int groups, hipStream_t st) {
  if constexpr (KIND != K_WGRAD) {
    if (conv192(a.M, a.N, groups)) return launch_glds<OutT, KIND, CCfg192>(a, groups, st);
  }
  if (a.N <= 64) return launch_glds<OutT, KIND, CCfg256x64>(a, groups, st);
  if (a.M <= 64) return launch_glds<OutT, KIND, CCfg64x256>(a, groups, st);
  return launch_glds<OutT, KIND, CCfg128>(a, groups, st);
}

template <typename T, typename OutT, int WM, int WN, int KIND>
int launch(const ConvArgs& a, int groups, hipStream_t st) {
  // operand kinds per convolution direction (fwd: K/K, dgrad: K/R, wgrad: R/R)
  using TL = Tile<T, WM, WN, KIND != K_WGRAD, KIND == K_FWD>;
  dim3 grid((a.N + TL::BN - 1) / TL::BN, (a.M + TL::BM - 1) / TL::BM, groups * a.splits);
  if (a.e.stats && a.e.stats_tiles != (int)grid.y) return AVSR_E_SHAPE;   // partials sized for another tile height
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
// row-tile height of a forward / data-grad launch: per-tile BN partials. 192 rows only on the
// bf16 LDS-DMA path (glds_by_tile); the fp32 / register-staged path keeps tile_bm
static int tile_bm_k(int M, int N, int dtype) {
  return dtype == AVSR_BF16 && conv192(M, N, 1) ? 192 : tile_bm(M, N);
}

// extents (elements, one group) of the A / B operands -> buffer-DMA loaders when allowed
static void set_extents(ConvArgs& a, const avsr_conv_params* p, bool tap_uniform, int64_t ea, int64_t eb) {
  const int64_t lim = ((int64_t)gemmg::OOB - (1 << 20)) / 2;
  const bool ok = p->dtype == AVSR_BF16 && tap_uniform && ea > 0 && eb > 0 && ea < lim && eb < lim;
  a.a_bytes = ok ? (uint32_t)(ea * 2) : 0u;
  a.b_bytes = ok ? (uint32_t)(eb * 2) : 0u;
}

static void base_epi(Epi& e) {
  e.alpha = 1.f; e.beta = 0.f; e.bias = nullptr; e.act = 0; e.bwd = 0; e.atomic = 0;
  e.preact = nullptr; e.res = nullptr; e.ldr = 0; e.gate = nullptr; e.drop_p = 0.f; e.seed = 0;
  e.drop_base = 0; e.stats = nullptr; e.stats_tiles = 0;
  e.rm_wc = 0; e.rm_hc = 0; e.rm_hin = 0; e.rm_win = 0; e.rm_a = 0; e.rm_b = 0; e.colsum = nullptr;
}

// weight-gradient split-K plan. The LDS-DMA path writes per-split fp32 slabs (plain stores)
// and reduces them afterwards: device-scope fp32 atomics on the 8-XCD part are resolved beyond
// the per-XCD L2 and sustain only ~50 G adds/s (measured: splits x M x N atomics dominated the
// ResNet wgrad at 683 splits), while a slab costs 8 bytes/float of HBM traffic.
struct WgradPlan { int splits, kchunk; bool slab; };

static WgradPlan wgrad_plan(const avsr_conv_params* p, bool glds, bool with_ws) {
  const int M = p->cout, N = p->kh * p->kw * p->cin, K = p->nimg * p->hout * p->wout;
  const int bm = tile_bm(M, N), bn = N <= 64 ? 64 : (M <= 64 ? 256 : 128);
  const long tiles = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn) * p->groups;
  WgradPlan w;
  const int kq = glds ? GBK : BKE;
  long splits = p->splitk;
  w.slab = with_ws;   // deterministic: per-split slabs + an ordered reduce (no fp32 atomics)
  if (splits <= 0) {
    // slab: ~2 full rounds of 512 block slots (2 per CU), rounded DOWN so the last round is
    // not a 1-block tail (513 blocks cost 2 rounds: measured 812 -> ~550 us on stage 1)
    const long target = w.slab ? 1024 : 2048;   // 512-2048 measured within noise (r02_conv_wgrad_target_ab)
    const long want = w.slab ? (target / tiles > 0 ? target / tiles : 1) : (target + tiles - 1) / tiles;
    const long maxs = w.slab ? (K + 1023) / 1024 : (K + 2047) / 2048;
    splits = want < maxs ? want : maxs;
    if (splits < 1) splits = 1;
  }
  w.kchunk = (int)(((K + splits - 1) / splits + kq - 1) / kq * kq);
  w.splits = (K + w.kchunk - 1) / w.kchunk;
  if (w.splits <= 1) { w.splits = 1; w.slab = false; }
  return w;
}

// dw[g] += sum over the splits of ws[g][s], in split order (deterministic). With chunks > 1
// (few output elements, many splits) a first pass folds each chunk of splits into its first
// slab (in place), and a second pass (chunks == -nchunks) sums those chunk heads in order.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(float* ws, int splits, int chunks, int64_t mn,
                                                           float* dw, int64_t dw_gstride) {
  const int g = blockIdx.y, c = blockIdx.z;
  float* w = ws + (int64_t)g * splits * mn;
  float* d = dw + (int64_t)g * dw_gstride;
  const int nch = chunks < 0 ? -chunks : chunks;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < mn; i += (int64_t)gridDim.x * 1024) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    if (chunks < 0) {            // pass 2: the chunk heads
      for (int q = 0; q < nch; ++q) s += *(const f32x4*)(w + (int64_t)((int64_t)splits * q / nch) * mn + i);
    } else {
      const int s0 = (int)((int64_t)splits * c / chunks), s1 = (int)((int64_t)splits * (c + 1) / chunks);
      for (int q = s0; q < s1; ++q) s += *(const f32x4*)(w + (int64_t)q * mn + i);
      if (chunks > 1) {          // pass 1: fold into the chunk's first slab
        *(f32x4*)(w + (int64_t)s0 * mn + i) = s;
        continue;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) d[i + r] += s[r];   // dw is a view into the parameter arena: 4-byte aligned only
  }
}

// Stride-2 data-grad by parity class of the input pixel. Class (a, b) = pixels (2i+a, 2j+b)
// receives contributions only from the taps kh = kh0 + 2u, kh0 = (a + ph) mod 2 (kw likewise),
// through dy at (i + ci - u, j + cj - v), ci = (a + ph - kh0) / 2: a stride-1 data-grad over
// the class grid. The four class GEMMs do 1/4 of the multiply-adds of the full one, whose
// other taps land on the zeros between the strided output pixels. A class with no taps (1x1
// kernels) still runs its epilogue (zeros, or the fused BatchNorm reduction of beta * dx).
struct S2Class { int a, b, hc, wc, nkh, nkw, kh0, kw0, ci, cj; };

static void s2_classes(const avsr_conv_params* p, S2Class (&c)[4]) {
  for (int q = 0; q < 4; ++q) {
    S2Class& k = c[q];
    k.a = q >> 1; k.b = q & 1;
    k.hc = (p->hin - k.a + 1) / 2; k.wc = (p->win - k.b + 1) / 2;
    k.kh0 = (k.a + p->ph) & 1; k.kw0 = (k.b + p->pw) & 1;
    k.nkh = k.kh0 < p->kh ? (p->kh - k.kh0 + 1) / 2 : 0;
    k.nkw = k.kw0 < p->kw ? (p->kw - k.kw0 + 1) / 2 : 0;
    k.ci = (k.a + p->ph - k.kh0) / 2; k.cj = (k.b + p->pw - k.kw0) / 2;
  }
}

// the parity-class path: bf16 buffer-DMA loaders (tap-uniform K-tiles), one group, stride 2
static bool s2_phase(const avsr_conv_params* p) {
  if (!avsr_opt(AVSR_OPT_CONV_S2PHASE)) return false;
  if (p->sh != 2 || p->sw != 2 || p->groups != 1 || p->dtype != AVSR_BF16 || !conv_glds_enabled()) return false;
  if (p->cout % 64) return false;
  ConvArgs t;
  set_extents(t, p, true, ((int64_t)p->nimg * p->hout * p->wout - 1) * p->ldy + p->cout,
              (int64_t)p->cout * p->kh * p->kw * p->cin);
  return t.a_bytes != 0;
}

// ---------------------------------------------------------------- patch-resident 3x3 / stride 1
// 3x3 / stride 1 / pad 1 convolutions with 64 channels on both sides (ResNet stage 1 at 22 x 22:
// layer1 conv1 / conv2 forward and data-grad). The general kernel builds each of the 9 tap
// K-tiles by re-gathering the block's pixels, so a block streams its input 9x through L2 — at
// N = 64 that made stage 1 L2-bandwidth bound (21 % of MFMA peak). Here a block of 256 output
// pixels DMAs the input patch around them into LDS ONCE, in padded coordinates ((H+2) x (W+2)
// per image; border and out-of-range positions come from the buffer's out-of-range zeros), and
// every tap of every pixel is a row offset into that image: no per-fragment masking, 9x fewer
// input bytes per block. The weight K-tiles (one tap x 64 channels, 8 KiB) stream through a
// 3-stage LDS ring as in gemm_glds.h; epilogues (BN statistics, fused BN-backward reduction)
// are gemm_glds.h's, unchanged. Forward reads x at p + (kh-1, kw-1); the data-grad reads dy at
// p - (kh-1, kw-1) against the weight viewed (ci, (kh, kw, co)).
struct PatchGeom {
  int nimg, H, W, Wp, PP;        // Wp = W + 2, PP = (H + 2) * Wp
  FastDiv f_pp, f_wp, f_hw, f_w;
  int sign;                      // +1 forward, -1 data-grad
};
constexpr int PATCH_ROWS = 384;                        // padded pixels of 64 channels (128 B) per block
constexpr int PATCH_BYTES = PATCH_ROWS * 128;
using PCfg = gemmg::GCfg<4, 1, 2, 2, 3>;               // 256 x 64, 4 waves of 64 x 64, 3-stage weight ring
constexpr int PATCH_SB = PCfg::BN * GBK * 2;           // one weight K-tile
constexpr int PATCH_LDS = PATCH_BYTES + PCfg::S * PATCH_SB;   // 72 KiB: two blocks per CU
static_assert(PCfg::EP_BYTES <= PATCH_LDS && PCfg::NTH * 33 * 4 <= PATCH_LDS, "epilogue staging exceeds LDS");

AVSR_DEV int patch_pos(int p, const PatchGeom& pg) {   // output pixel -> padded position
  const uint32_t n = fdiv((uint32_t)p, pg.f_hw), rem = (uint32_t)p - n * pg.f_hw.d;
  const uint32_t y = fdiv(rem, pg.f_w), x = rem - y * pg.f_w.d;
  return (int)(n * pg.PP + (y + 1) * pg.Wp + x + 1);
}

// the patch image [PATCH_ROWS][64] (k-major row swizzle of gemm_glds.h on the patch row)
template <int NW> struct PatchLoad {
  static constexpr int PIECES = PATCH_ROWS * 8 / 64 / NW;
  __amdgpu_buffer_rsrc_t rs;
  uint32_t vo[PIECES];
  AVSR_DEV void init(const bf16* base, uint32_t bytes, const PatchGeom& pg, int qmin, int wave, int lane) {
    rs = make_rsrc(base, bytes);
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const int pr = (i * NW + wave) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((pr >> 1) & 7);
      const uint32_t q = (uint32_t)(qmin + pr);
      const uint32_t n = fdiv(q, pg.f_pp), rem = q - n * (uint32_t)pg.PP;
      const uint32_t yy = fdiv(rem, pg.f_wp), xx = rem - yy * (uint32_t)pg.Wp;
      const bool ok = n < (uint32_t)pg.nimg && yy - 1u < (uint32_t)pg.H && xx - 1u < (uint32_t)pg.W;
      vo[i] = ok ? (((n * pg.H + yy - 1) * pg.W + xx - 1) * 64u + c * 8u) * 2u : OOB;
    }
  }
  AVSR_DEV void issue(char* img, int wave) const {
#pragma unroll
    for (int i = 0; i < PIECES; ++i) bglds16(rs, vo[i], 0u, img + (i * NW + wave) * 1024);
  }
};

template <class LB>
struct PatchFrags {
  bf16x8 a[PCfg::TM], b[PCfg::TN];
  AVSR_DEV void load(const char* patch, const int (&row)[PCfg::TM], int toff, const char* wstage, int s, int lane) {
#pragma unroll
    for (int i = 0; i < PCfg::TM; ++i) {
      const int r = row[i] + toff;
      const int c = (4 * s + (lane >> 4)) ^ ((r >> 1) & 7);
      a[i] = *(const bf16x8*)(patch + r * 128 + c * 16);
    }
#pragma unroll
    for (int j = 0; j < PCfg::TN; ++j) b[j] = gemmg::gfrag<PCfg::BN, LB::KMAJ>(wstage, j * 16, s, lane);
  }
  AVSR_DEV void mma(f32x4 (&acc)[PCfg::TM][PCfg::TN]) const {
#pragma unroll
    for (int i = 0; i < PCfg::TM; ++i)
#pragma unroll
      for (int j = 0; j < PCfg::TN; ++j) acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
  }
};

template <int KIND>
__global__ __launch_bounds__(PCfg::NTH, 2) void conv_patch_kernel(ConvArgs a, PatchGeom pg) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int S = PCfg::S, NK = 9, KS = GBK / 32, GLB = PATCH_SB / 1024 / PCfg::NW;
  const int m0 = gemmg::xcd_remap(blockIdx.x, gridDim.x) * PCfg::BM;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int qmin = patch_pos(m0, pg) - pg.Wp - 1;
  char* patch = smem;
  char* ring = smem + PATCH_BYTES;
  PatchLoad<PCfg::NW> lp;
  lp.init((const bf16*)a.a, a.a_bytes, pg, qmin, wave, lane);
  using LB = typename std::conditional<KIND == K_FWD, gemmg::BDenseK<PCfg::BN, PCfg::NW>,
                                       BWgtR<PCfg::BN, PCfg::NW>>::type;
  LB lb;
  if constexpr (KIND == K_FWD) lb.init((const bf16*)a.b, a.b_bytes, a.K, 0, a.N, a.K, wave, lane);
  else lb.init((const bf16*)a.b, a.b_bytes, a.g, 0, a.N, wave, lane);
  int row[PCfg::TM];                 // patch row of this lane's output pixel in each 16-row block
#pragma unroll
  for (int i = 0; i < PCfg::TM; ++i) {
    const int p = min(m0 + wave * 64 + i * 16 + (lane & 15), a.M - 1);
    row[i] = patch_pos(p, pg) - qmin;
  }
  f32x4 acc[PCfg::TM][PCfg::TN];
#pragma unroll
  for (int i = 0; i < PCfg::TM; ++i)
#pragma unroll
    for (int j = 0; j < PCfg::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  lp.issue(patch, wave);
#pragma unroll
  for (int p = 0; p < S; ++p) lb.issue(ring + p * PATCH_SB, p * GBK, wave);
  gemmg::wait_vmcnt<GLB * (S - 1)>();      // the patch and weight tile 0 have landed
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  auto toff = [&](int kt) {                 // row offset of tap kt = (kh, kw) in the padded patch
    const int kh = kt / 3, kw = kt - 3 * kh;
    return pg.sign * ((kh - 1) * pg.Wp + (kw - 1));
  };
  // two fragment sets in fixed roles (k-step 0 / 1 of a tap): no register copies (gemm_glds.h)
  static_assert(KS == 2, "the fragment sets alternate over two k-steps per K-tile");
  PatchFrags<LB> f0, f1;
  f0.load(patch, row, toff(0), ring, 0, lane);
  int cs = 0;
  for (int kt = 0; kt < NK; ++kt) {
    const int ns = cs + 1 == S ? 0 : cs + 1;
    f1.load(patch, row, toff(kt), ring + cs * PATCH_SB, 1, lane);
    f0.mma(acc);
    if (kt + 1 < NK) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (kt + S - 1 < NK) gemmg::wait_vmcnt<GLB * (S - 2)>();
      else gemmg::wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + S < NK) lb.issue(ring + cs * PATCH_SB, (kt + S) * GBK, wave);
      f0.load(patch, row, toff(kt + 1), ring + ns * PATCH_SB, 0, lane);
    }
    f1.mma(acc);
    cs = ns;
  }
  __syncthreads();
  if constexpr (KIND >= K_DGRAD_BNR) {
    gemmg::epilogue_bnr<PCfg, KIND - K_DGRAD_BNR>(a.e, a.bnr, m0, 0, acc, smem);
  } else {
    gemmg::epilogue_g<bf16, bf16, PCfg>(a.e, m0, 0, acc, smem);
  }
}

// ---------------------------------------------------------------- patch-resident weight-grad
// dW[co][(kh, kw, ci)] = sum_p dy[p][co] * x[p + (kh-1, kw-1)][ci] for the 3x3 / stride 1 /
// pad 1 convolutions of ResNet stages 1 (22 x 22 x 64) and 2 (11 x 11 x 128). The general
// weight-grad re-gathers x for every tap (9 passes of the input through L2; at stage 1 its
// 64 x 256 tiles are 1/4 padding). Here persistent blocks (WP_BLOCKS, below) walk tiles of TR whole
// image rows; a block owns a 64 x 64 (co, ci) block of every tap. Per tile the block's dy
// channels and the zero-padded (TR+2) x (W+2) patch of its x channels are DMA'd into LDS once,
// double buffered, and all 9 taps read the patch at row offsets. Every tile has the same
// geometry, so each LDS address of the main loop is a per-lane base fixed for the kernel plus a
// compile-time offset. The 64 x 576 gradient block stays in registers: wave w owns input
// channels [16w, 16w + 16) of all 9 taps (36 accumulators of 16 x 16). Both operands are
// pixel-major, so both fragments are transposed LDS reads (ds_read_b64_tr_b16); the MFMA k
// order within a fragment is permuted (k bits 2 and 3 swapped) so that each half-wave read
// covers 8 consecutive pixels: the dy image (128-byte rows) is conflict-free with a chunk XOR
// on pixel bits 1-2, the patch (padded rows, no XOR) is (nearly) conflict-free. The
// DMAs of the next tile are spread over the k-steps. With several (co, ci) blocks (stage 2:
// 2 x 2), the blocks that share an XCD (ids b, b+8, ...) take the blocks of the same tile range,
// so x and dy come from that XCD's L2 after the first read. Each block writes its fp32 partial
// once to a slab [block][64][576]; wpatch_reduce_kernel sums them in block order (deterministic).
// Persistent blocks of the stage-1 / stage-2 weight-grads: 128, one on every other CU. These run
// on the side stream beside the ResNet backward's data-gradient chain, and a block holds up to
// 152 KB of LDS, so at one block per CU (256) every chain kernel needing LDS waited for free CUs;
// 128 blocks take longer on the side but the step is shorter (6 of 6 interleaved pairs, +0.3-0.5 %
// value_expected; 64: slower; profiles/r05_wpatch_blocks_ab.txt). A/B builds may override.
#ifndef AVSR_WP_BLOCKS
#define AVSR_WP_BLOCKS 128
#endif
#ifndef AVSR_WP34          // A/B builds only: stages 3-4 on the general weight-grad
#define AVSR_WP34 1
#endif
#ifndef AVSR_WP34_BLOCKS
#define AVSR_WP34_BLOCKS 128
#endif
constexpr int WP_BLOCKS = AVSR_WP_BLOCKS, WP34_BLOCKS = AVSR_WP34_BLOCKS, WP_COLS = 576;

// Stages 3 (6 x 6, 256 channels) and 4 (3 x 3, 512 channels): a tile is IPT whole images stacked
// vertically in the patch with ONE shared zero row between neighbours (a tap above an image's
// first row or below its last reads that row), so the 9 taps stay row offsets; IPT is chosen so
// that IPT x H x W pixels nearly fill whole 32-pixel k-steps (180 of 192, 126 of 128). NBLK
// persistent blocks; the next tile's DMAs are issued over the first SPREAD k-steps of the current
// one (with few k-steps per tile, DMAs issued at the last one would have no time to land).
template <int W_, int TR_, int TPI_, int NBUF_, int PST_, int IPT_ = 1, int NBLK_ = WP_BLOCKS, int SPREAD_ = 0>
struct WPGeo {
  static constexpr int W = W_, TR = TR_, TPI = TPI_, H = TR * TPI, NBUF = NBUF_, PST = PST_, IPT = IPT_, NBLK = NBLK_;
  static constexpr int IMGT = TR * W;                // pixels of one image in a tile
  static constexpr int PX = IPT * IMGT;              // pixels per tile
  static constexpr int KS = (PX + 31) / 32;          // k-steps of 32 pixels
  static constexpr int DYR = KS * 32;                // dy image rows (>= PX: zero)
  static constexpr int WP = W + 2, PROWS = (IPT * (TR + 1) + 1) * WP;
  static constexpr int SLOTS = PST / 16;             // 16-byte slots per patch row (8 data + pad)
  static constexpr int PPIECE = (PROWS * SLOTS + 255) / 256;   // patch DMA pieces per wave
  static constexpr int PBYTES = PPIECE * 4 * 1024;
  static constexpr int DYPIECE = DYR * 128 / 4096;   // dy DMA pieces per wave
  static constexpr int DYB = DYR * 128;
  static constexpr int BUF = DYB + PBYTES;
  static constexpr int LDS = NBUF * BUF;
  static constexpr int NP = DYPIECE + PPIECE;        // DMAs per wave per tile
  static constexpr int SPREAD = SPREAD_ > 0 ? SPREAD_ : KS;
  static_assert(LDS <= 160 * 1024, "the tile buffers must fit the CU's LDS");
  static_assert(IPT == 1 || TPI == 1, "a tile is part of one image or whole images");
  static_assert(NBUF >= 2 && (NBUF - 2) * NP <= 63 && SPREAD <= KS, "vmcnt range / DMA spread");
  static_assert(NBLK % 8 == 0, "blocks come in XCD groups of 8");
};
// patch row stride 144 B: one 2-way overlap among 8 consecutive rows' 32-byte windows; 160 B:
// none (what the LDS allows)
using WPStage1 = WPGeo<22, 11, 2, 2, 144>;   // half images: 242 pixels, 13 x 24 patch, double buffered
using WPStage2 = WPGeo<11, 11, 1, 3, 160>;   // whole images: 121 pixels, 13 x 13 patch, 3 buffers (short tiles)
using WPStage3 = WPGeo<6, 6, 1, 2, 144, 5, WP34_BLOCKS, 3>;    // 5 images: 180 pixels, 36 x 8 patch
using WPStage4 = WPGeo<3, 3, 1, 2, 160, 14, WP34_BLOCKS, 2>;   // 14 images: 126 pixels, 57 x 5 patch

AVSR_DEV int whswz(int row) { return ((row >> 1) & 3) << 1; }
AVSR_DEV bf16x8 trpair(const char* pa, const char* pb) {
  const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)pa);
  const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)pb);
  union { v4i16 s4[2]; bf16x8 h; } u;
  u.s4[0] = a; u.s4[1] = b;
  return u.h;
}

// (co, ci) block q and tile range r of block b among nblk: blocks b, b+8, ... share an XCD under
// round-robin placement (S = nblk / 8 per XCD). nq <= S (S % nq == 0): the nq blocks with the same
// range sit on one XCD; nq > S (nq % S == 0): a range's blocks fill nq / S XCDs. Ranges per
// block kind: bpq = nblk / nq either way.
AVSR_DEV void wp_block(int b, int nq, int nblk, int& q, int& r) {
  const int x = b & 7, s = b >> 3, S = nblk >> 3;
  if (nq <= S) {
    q = s % nq;
    r = (s / nq) * 8 + x;
  } else {
    const int k = nq / S;
    r = x / k;
    q = (x - r * k) * S + s;
  }
}

// wait until at most min(ahead, K) tiles of NP DMAs each are still in flight (vmcnt is an immediate)
template <int NP, int K>
AVSR_DEV void wp_wait_ahead(int ahead) {
  if constexpr (K == 0) {
    gemmg::wait_vmcnt<0>();
  } else {
    if (ahead >= K) gemmg::wait_vmcnt<NP * K>();
    else wp_wait_ahead<NP, K - 1>(ahead);
  }
}

template <class G>
__global__ __launch_bounds__(256, 1) void conv_wgrad_patch_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                                  uint32_t x_bytes, uint32_t dy_bytes, int nimg,
                                                                  int cin, int cout, float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int IMG = G::H * G::W;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ncih = cin / 64, nq = (cout / 64) * ncih, bpq = gridDim.x / nq;
  int q, rng;
  wp_block(blockIdx.x, nq, gridDim.x, q, rng);
  const int coh = q / ncih, cih = q - coh * ncih;
  const int ntiles = (nimg * G::TPI + G::IPT - 1) / G::IPT;   // a last part tile reads zeros past the end
  const int ta = (int)((int64_t)ntiles * rng / bpq), tb = (int)((int64_t)ntiles * (rng + 1) / bpq);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(x, x_bytes), rdy = make_rsrc(dy, dy_bytes);
  // DMA pieces of a tile (offsets recomputed per issue: compile-time divisors, no registers held)
  auto tile_px = [&](int t) { return (t / G::TPI) * IMG * G::IPT + (t % G::TPI) * G::PX; };
  auto issue_dy = [&](int i, int t, char* buf) {
    const int s = (wave + 4 * i) * 64 + lane, row = s >> 3;
    const int c = (s & 7) ^ whswz(row);
    const uint32_t vo = row < G::PX ? (uint32_t)(tile_px(t) + row) * (uint32_t)(cout * 2) + coh * 128 + c * 16 : gemmg::OOB;
    gemmg::bglds16(rdy, vo, 0u, buf + (wave + 4 * i) * 1024);
  };
  auto issue_patch = [&](int i, int t, char* buf) {
    const int s = (wave + 4 * i) * 64 + lane, row = s / G::SLOTS, ch = s - row * G::SLOTS;
    const int py = row / G::WP, pxp = row - py * G::WP;
    bool ok;
    int src;                                           // input pixel of this slot (relative to the tile's first)
    if constexpr (G::IPT == 1) {
      const int y = (t % G::TPI) * G::TR + py - 1;     // image row of this slot's patch row
      ok = y >= 0 && y < G::H;
      src = (py - 1) * G::W + pxp - 1;
    } else {                                           // image i's rows 1 + i (H + 1) ..., shared zero rows between
      const int i = (py - 1) / (G::TR + 1), yl = py - 1 - i * (G::TR + 1);
      ok = py >= 1 && yl < G::TR;
      src = i * G::IMGT + yl * G::W + pxp - 1;
    }
    ok = ok && ch < 8 && row < G::PROWS && pxp >= 1 && pxp <= G::W;
    const uint32_t vo = ok ? (uint32_t)(tile_px(t) + src) * (uint32_t)(cin * 2) + cih * 128 + ch * 16 : gemmg::OOB;
    gemmg::bglds16(rx, vo, 0u, buf + G::DYB + (wave + 4 * i) * 1024);
  };
  // fragment bases: lane group g holds k = 8g + j <-> pixel 32kb + 16(g >> 1) + 4(g & 1) + (j & 3) + 8(j >> 2)
  const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  const int pxa = 16 * (g >> 1) + 4 * (g & 1) + qq;
  const int sw = whswz(pxa);
  int dA[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dA[i] = pxa * 128 + (((2 * i + (pp >> 1)) ^ sw) << 4) + 8 * (pp & 1);
  auto prow = [&](int px) {                        // tile pixel -> patch row
    px = min(px, G::PX - 1);
    const int i = px / G::IMGT, r = px - i * G::IMGT, yy = r / G::W, xx = r - yy * G::W;
    return (i * (G::TR + 1) + yy + 1) * G::WP + xx + 1;
  };
  int pA[G::KS], pB[G::KS];               // patch byte bases (tap (0, 0) = offset 0) per k-step
#pragma unroll
  for (int kb = 0; kb < G::KS; ++kb) {
    pA[kb] = (prow(32 * kb + pxa) - G::WP - 1) * G::PST + 32 * wave + 8 * pp;
    pB[kb] = (prow(32 * kb + pxa + 8) - G::WP - 1) * G::PST + 32 * wave + 8 * pp;
  }
  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int PD = G::NBUF - 1;          // tiles in flight ahead of the one computed
#pragma unroll
  for (int d = 0; d < PD; ++d)
    if (ta + d < tb) {
#pragma unroll
      for (int i = 0; i < G::DYPIECE; ++i) issue_dy(i, ta + d, smem + d * G::BUF);
#pragma unroll
      for (int i = 0; i < G::PPIECE; ++i) issue_patch(i, ta + d, smem + d * G::BUF);
    }
  constexpr int PER = (G::NP + G::SPREAD - 1) / G::SPREAD;   // DMAs per k-step
  for (int t = ta; t < tb; ++t) {
    const char* buf = smem + ((t - ta) % G::NBUF) * G::BUF;
    char* nbuf = smem + ((t + PD - ta) % G::NBUF) * G::BUF;
    const bool more = t + PD < tb;
    // tile t has landed: the DMAs of the (up to PD - 1) later tiles already issued may still fly
    wp_wait_ahead<G::NP, PD - 1>(tb - 1 - t);
    __builtin_amdgcn_s_barrier();         // ... for every wave; every wave is done with tile t-1
    asm volatile("" ::: "memory");
    const char* patch = buf + G::DYB;
    // fragments of k-step kb: 4 dy (A) and 9 tap (B) transposed reads; the reads of step kb+1
    // are issued before the MFMAs of step kb (one wave per SIMD: nothing else hides their
    // latency), the next tile's DMAs after them (the asm DMA is a compiler memory barrier)
    struct Fr { bf16x8 a[4], b[9]; };
    auto load = [&](Fr& f, int kb) {
#pragma unroll
      for (int i = 0; i < 4; ++i) f.a[i] = trpair(buf + dA[i] + kb * 4096, buf + dA[i] + kb * 4096 + 1024);
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) {
        const int off = ((tp / 3) * G::WP + tp % 3) * G::PST;
        f.b[tp] = trpair(patch + pA[kb] + off, patch + pB[kb] + off);
      }
    };
    Fr cur, nxt;
    load(cur, 0);
#pragma unroll
    for (int kb = 0; kb < G::KS; ++kb) {
      if (kb + 1 < G::KS) load(nxt, kb + 1);
      if (more && kb < G::SPREAD) {
#pragma unroll
        for (int d = 0; d < PER; ++d) {
          const int pc = kb * PER + d;
          if (pc < G::DYPIECE) issue_dy(pc, t + PD, nbuf);
          else if (pc < G::DYPIECE + G::PPIECE) issue_patch(pc - G::DYPIECE, t + PD, nbuf);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) acc[i][tp] = mfma16(cur.a[i], cur.b[tp], acc[i][tp]);
      if (kb + 1 < G::KS) cur = nxt;
    }
  }
  // partial -> ws[block][co 64][576]: accumulator (i, tap) register r = co 16i + 4g + r, column
  // tap * 64 + 16 * wave + (lane & 15)
  float* o = ws + (int64_t)blockIdx.x * 64 * WP_COLS;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int tp = 0; tp < 9; ++tp)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[(16 * i + 4 * g + r) * WP_COLS + tp * 64 + 16 * wave + (lane & 15)] = acc[i][tp][r];
}

AVSR_DEV int wp_bid(int q, int r, int nq, int nblk) {   // inverse of wp_block
  const int S = nblk >> 3;
  if (nq <= S) return ((((r >> 3) * nq) + q) << 3) + (r & 7);
  const int k = nq / S;
  return ((q % S) << 3) + r * k + q / S;
}

// dw[co][tap][ci] += sum over the tile ranges r of block kind q of ws[wp_bid(q, r)][co % 64][tap * 64 + ci % 64],
// in range order (deterministic), in two passes: chunk c of WPR_CHUNKS folds its ranges into the
// slab of its first range (in place); pass 2 (chunk < 0) adds the chunk heads in order to dw.
// 4 consecutive ci per thread.
constexpr int WPR_CHUNKS = 8;
__global__ __launch_bounds__(256) void wpatch_reduce_kernel(float* __restrict__ ws, int nblk, int cin, int cout,
                                                            float* dw, int pass2) {
  const int ncih = cin / 64, nq = (cout / 64) * ncih, bpq = nblk / nq;
  const int e = (blockIdx.x * 256 + threadIdx.x) * 4;      // element of the 64 x 576 block
  const int q = blockIdx.y, c = blockIdx.z;
  if (e >= 64 * WP_COLS) return;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (!pass2) {
    const int r0 = bpq * c / WPR_CHUNKS, r1 = bpq * (c + 1) / WPR_CHUNKS;
    for (int r = r0; r < r1; ++r) s += *(const f32x4*)(ws + (int64_t)wp_bid(q, r, nq, nblk) * 64 * WP_COLS + e);
    if (r1 > r0) *(f32x4*)(ws + (int64_t)wp_bid(q, r0, nq, nblk) * 64 * WP_COLS + e) = s;
    return;
  }
  for (int k = 0; k < WPR_CHUNKS; ++k) {
    const int r0 = bpq * k / WPR_CHUNKS, r1 = bpq * (k + 1) / WPR_CHUNKS;
    if (r1 > r0) s += *(const f32x4*)(ws + (int64_t)wp_bid(q, r0, nq, nblk) * 64 * WP_COLS + e);
  }
  const int r = e / WP_COLS, col = e - r * WP_COLS, tap = col >> 6, ci = col & 63;
  const int coh = q / ncih, cih = q - coh * ncih;
  float* d = dw + ((int64_t)(coh * 64 + r) * 9 + tap) * cin + cih * 64 + ci;
#pragma unroll
  for (int k = 0; k < 4; ++k) d[k] += s[k];     // dw is a view into the parameter arena: 4-byte aligned only
}

// the patch-resident weight-grad applies: bf16, slab workspace, automatic split, 3x3 / stride 1
// / pad 1, one group, the stage-1 (22 x 22, 64 -> 64), stage-2 (11 x 11, 128 -> 128), stage-3
// (6 x 6, 256 -> 256) or stage-4 (3 x 3, 512 -> 512) geometry
static bool wpatch_ok(const avsr_conv_params* p) {
  if (!avsr_opt(AVSR_OPT_CONV_WPATCH) || p->dtype != AVSR_BF16 || !conv_glds_enabled() || p->groups != 1 || p->splitk > 0)
    return false;
  if (p->kh != 3 || p->kw != 3 || p->sh != 1 || p->sw != 1 || p->ph != 1 || p->pw != 1) return false;
  if (p->cin != p->cout || p->ldx != p->cin || p->ldy != p->cout || p->hin != p->hout || p->win != p->wout) return false;
  if (p->hin != p->win) return false;
  const int64_t bytes = (int64_t)p->nimg * p->hin * p->win * p->cin * 2;
  if (bytes <= 0 || bytes >= (int64_t)gemmg::OOB - (1 << 20)) return false;
  if ((p->cin == 256 && p->hin == 6) || (p->cin == 512 && p->hin == 3)) return AVSR_WP34 != 0;
  return (p->cin == 64 && p->hin == 22) || (p->cin == 128 && p->hin == 11);
}

static int wpatch_blocks(const avsr_conv_params* p) { return p->cin >= 256 ? WP34_BLOCKS : WP_BLOCKS; }

template <class G>
static int wpatch_launch_g(const avsr_conv_params* p, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_wgrad_patch_kernel<G>, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
    attr = true;
  }
  const uint32_t bytes = (uint32_t)((int64_t)p->nimg * p->hin * p->win * p->cin * 2);
  static_assert(G::NBLK % 8 == 0, "");
  const int nq = (p->cout / 64) * (p->cin / 64), S = G::NBLK / 8;
  if (nq <= S ? S % nq != 0 : (nq % S != 0 || 8 % (nq / S) != 0)) return AVSR_E_SHAPE;   // wp_block's mapping
  hipLaunchKernelGGL((conv_wgrad_patch_kernel<G>), dim3(G::NBLK), dim3(256), G::LDS, st, (const bf16*)p->x,
                     (const bf16*)p->dy, bytes, bytes, p->nimg, p->cin, p->cout, p->ws);
  AVSR_CHECK_LAUNCH();
  const unsigned gx = (64 * WP_COLS / 4 + 255) / 256;
  hipLaunchKernelGGL(wpatch_reduce_kernel, dim3(gx, (unsigned)nq, (unsigned)WPR_CHUNKS), dim3(256), 0, st, p->ws,
                     G::NBLK, p->cin, p->cout, p->dw, 0);
  AVSR_CHECK_LAUNCH();
  hipLaunchKernelGGL(wpatch_reduce_kernel, dim3(gx, (unsigned)nq, 1u), dim3(256), 0, st, p->ws, G::NBLK, p->cin,
                     p->cout, p->dw, 1);
  AVSR_CHECK_LAUNCH();
  return 0;
}

static int wpatch_launch(const avsr_conv_params* p, hipStream_t st) {
  if (p->cin == 64) return wpatch_launch_g<WPStage1>(p, st);
  if (p->cin == 128) return wpatch_launch_g<WPStage2>(p, st);
  if (p->cin == 256) return wpatch_launch_g<WPStage3>(p, st);
  return wpatch_launch_g<WPStage4>(p, st);
}

// ---------------------------------------------------------------- patch-resident stem weight-grad
// The stem conv's weight-gradient (Conv3d 1 -> 64, 5 x 7 x 7, stride (1, 2, 2), pad (2, 3, 3)) on
// the packed input xp [N][88][88][8] (the 5 frames t-2 .. t+2 of each pixel in channels 0-4,
// zeros after; ops.stem_pack): gp[co][kh][kw][c] += sum_p dy[p][co] * xp[p's image][2oy+kh-3]
// [2ox+kw-3][c] over the N x 44 x 44 output pixels. The general implicit GEMM computes an im2col
// address per 16-byte DMA slot and amortises its 256-column tiles over only 64 output channels
// (VALU-bound, MFMA busy 0.28: profiles/r05_stem_wgrad_counters.txt). Here persistent blocks
// (one per CU) walk tiles of 4 output rows of one image, 48 columns wide (44 real; the other dy
// rows are DMA zeros). Per tile the dy rows and the zero-padded 13 x 103 input patch (16 bytes
// per pixel) are DMA'd into LDS once, three buffers deep, and every tap of every pixel is an
// offset into the patch. A k-step's 32 pixels are a 4-row x 8-column block (dy rows stored in
// that order), so every LDS address of the main loop is a per-lane base fixed for the kernel plus
// a compile-time offset (no address arithmetic per k-step), and the DMA offsets are per-lane
// constants plus a per-tile scalar. The 64 x 392 gradient block stays in registers: columns are
// pairs of taps (t, t+1) x 8 channels (16 per MFMA tile; 25 pairs, the 49th tap's partner a
// discarded duplicate), pair P belongs to wave P mod 4, and waves 1-3 run a discarded 7th pair
// so that every wave has the same branch-free loop. The fragment reads of k-step kb+1 are issued
// between the two halves of k-step kb's MFMAs (scheduling barriers keep them there): the LDS
// latency hides behind the second half instead of an lgkmcnt drain in front of every k-step
// (lgkmcnt counts to 15; a step has 22 reads). Both operands are pixel-major, read
// transposed (ds_read_b64_tr_b16) with wgrad_patch's pixel order; a 16-lane group's patch read
// covers 4 pixels x 2 taps x 8 channels in 128 contiguous bytes modulo the banks (row stride
// 103 x 16 B keeps the pairs that straddle two kernel rows conflict-free too). Each block writes
// its fp32 partial to a slab [block][64][392]; wgrad_reduce_kernel sums the slabs in block order
// (deterministic).
constexpr int SWP_TR = 4, SWP_TC = 48, SWP_KS = SWP_TC / 8, SWP_TPI = 44 / SWP_TR;
constexpr int SWP_DYB = SWP_KS * 32 * 128, SWP_DYPIECE = SWP_DYB / 4096;
constexpr int SWP_PR = 2 * SWP_TR + 5, SWP_PC = 103, SWP_SLOTS = SWP_PR * SWP_PC, SWP_RB = SWP_PC * 16;
constexpr int SWP_PPIECE = (SWP_SLOTS + 255) / 256, SWP_PBYTES = SWP_PPIECE * 4096;
constexpr int SWP_BUF = SWP_DYB + SWP_PBYTES, SWP_NBUF = 3, SWP_LDS = SWP_NBUF * SWP_BUF;
constexpr int SWP_NP = SWP_DYPIECE + SWP_PPIECE, SWP_COLS = 392, SWP_PAIRS = 25;
constexpr int SWP_BLOCKS = 256;                  // persistent blocks, one per CU
constexpr int SWP_JW = (SWP_PAIRS + 3) / 4;     // pairs per wave (7; pairs >= 25 are discarded)
static_assert(SWP_LDS <= 160 * 1024 && SWP_DYB % 4096 == 0 && SWP_KS % 2 == 0, "stem weight-grad tile buffers");
static_assert(2 * (SWP_TC - 1) + 6 - 3 < SWP_PC - 3 + 1 && SWP_NP % SWP_KS == 0, "patch width / DMA spread");

AVSR_DEV int swp_toff(int t) {                 // patch byte offset of tap t = (kh, kw) (t > 48 -> 48)
  t = t > 48 ? 48 : t;
  const int kh = t / 7, kw = t - 7 * kh;
  return kh * SWP_RB + kw * 16;
}

__global__ __launch_bounds__(256, 1) void stem_wgrad_patch_kernel(const bf16* __restrict__ xp, const bf16* __restrict__ dy,
                                                                  uint32_t x_bytes, uint32_t dy_bytes, int nimg,
                                                                  float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntiles = nimg * SWP_TPI;
  const int ta = (int)((int64_t)ntiles * blockIdx.x / gridDim.x), tb = (int)((int64_t)ntiles * (blockIdx.x + 1) / gridDim.x);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(xp, x_bytes), rdy = make_rsrc(dy, dy_bytes);
  // per-lane DMA offsets relative to the tile's first dy pixel / input pixel (OOB: zeros)
  uint32_t vdy[SWP_DYPIECE];
  int vpt[SWP_PPIECE], ppr[SWP_PPIECE];
#pragma unroll
  for (int i = 0; i < SWP_DYPIECE; ++i) {
    const int sl = (wave + 4 * i) * 64 + lane, row = sl >> 3;          // dy LDS row = kb * 32 + r * 8 + c
    const int ch = (sl & 7) ^ whswz(row), k = row & 31, col = 8 * (row >> 5) + (k & 7);
    vdy[i] = col < 44 ? (uint32_t)(((k >> 3) * 44 + col) * 128 + ch * 16) : gemmg::OOB;
  }
#pragma unroll
  for (int i = 0; i < SWP_PPIECE; ++i) {
    const int sl = (wave + 4 * i) * 64 + lane, pr = sl / SWP_PC, pc = sl - pr * SWP_PC;
    const bool ok = sl < SWP_SLOTS && pc >= 3 && pc < 91;
    vpt[i] = ((pr - 3) * 88 + pc - 3) * 16;
    ppr[i] = ok ? pr - 3 : -1000;                   // input row offset of the slot (-1000: never valid)
  }
  auto issue = [&](int pc, int t, char* buf) {      // DMA piece pc of tile t (dy pieces, then patch)
    const int img = t / SWP_TPI, oy0 = (t - img * SWP_TPI) * SWP_TR;
    if (pc < SWP_DYPIECE) {
      gemmg::bglds16(rdy, vdy[pc], (uint32_t)(img * 1936 + oy0 * 44) * 128u, buf + (wave + 4 * pc) * 1024);
    } else {
      const int i = pc - SWP_DYPIECE, y = 2 * oy0 + ppr[i];
      const uint32_t vo = (uint32_t)y < 88u ? (uint32_t)(img * 123904 + oy0 * 2816 + vpt[i]) : gemmg::OOB;
      gemmg::bglds16(rx, vo, 0u, buf + SWP_DYB + (wave + 4 * i) * 1024);
    }
  };
  // fragment bases: lane group g holds k = 8g + j <-> pixel 16(g >> 1) + 4(g & 1) + (j & 3) + 8(j >> 2)
  // of the k-step = row k >> 3, column 8 kb + (k & 7) of the tile
  const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  const int pxa = 16 * (g >> 1) + 4 * (g & 1) + qq;
  const int sw = whswz(pxa);
  int dA[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dA[i] = pxa * 128 + (((2 * i + (pp >> 1)) ^ sw) << 4) + 8 * (pp & 1);
  const int pbase = SWP_DYB + (2 * (pxa >> 3) * SWP_PC + 2 * (pxa & 7)) * 16;
  int oB[SWP_JW];                                   // patch byte base of this lane per pair
#pragma unroll
  for (int j = 0; j < SWP_JW; ++j) oB[j] = pbase + swp_toff(2 * (wave + 4 * j) + (pp >> 1)) + 8 * (pp & 1);
  f32x4 acc[4][SWP_JW];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < SWP_JW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int PD = SWP_NBUF - 1, PER = SWP_NP / SWP_KS;
#pragma unroll
  for (int d = 0; d < PD; ++d)
    if (ta + d < tb)
#pragma unroll
      for (int pc = 0; pc < SWP_NP; ++pc) issue(pc, ta + d, smem + d * SWP_BUF);
  struct Fr { bf16x8 a[4], b[SWP_JW]; };
  // k-step kb: dy rows kb * 32 (+ 8: the next tile row), patch columns + 16 kb pixels (+ 2 rows)
  auto load = [&](Fr& f, const char* buf, int kb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) f.a[i] = trpair(buf + dA[i] + kb * 4096, buf + dA[i] + kb * 4096 + 1024);
#pragma unroll
    for (int j = 0; j < SWP_JW; ++j) f.b[j] = trpair(buf + oB[j] + kb * 256, buf + oB[j] + kb * 256 + 2 * SWP_RB);
  };
  auto mma = [&](const Fr& f, int h) {            // output-channel tiles 2h, 2h + 1
#pragma unroll
    for (int i = 2 * h; i < 2 * h + 2; ++i)
#pragma unroll
      for (int j = 0; j < SWP_JW; ++j) acc[i][j] = mfma16(f.a[i], f.b[j], acc[i][j]);
  };
  for (int t = ta; t < tb; ++t) {
    const char* buf = smem + ((t - ta) % SWP_NBUF) * SWP_BUF;
    char* nbuf = smem + ((t + PD - ta) % SWP_NBUF) * SWP_BUF;
    const bool more = t + PD < tb;
    if (t + 1 < tb) gemmg::wait_vmcnt<SWP_NP>();   // tile t landed; tile t+1's DMAs may fly
    else gemmg::wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();                  // ... for every wave; every wave is done with tile t-1
    asm volatile("" ::: "memory");
    // two fragment sets in fixed roles (even / odd k-steps): no register copies
    Fr f0, f1;
    load(f0, buf, 0);
#pragma unroll
    for (int kb = 0; kb < SWP_KS; kb += 2) {
      mma(f0, 0);
      __builtin_amdgcn_sched_barrier(0);
      load(f1, buf, kb + 1);
      __builtin_amdgcn_sched_barrier(0);
      mma(f0, 1);
      if (more)
#pragma unroll
        for (int d = 0; d < PER; ++d) issue(kb * PER + d, t + PD, nbuf);
      mma(f1, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (kb + 2 < SWP_KS) load(f0, buf, kb + 2);
      __builtin_amdgcn_sched_barrier(0);
      mma(f1, 1);
      if (more)
#pragma unroll
        for (int d = 0; d < PER; ++d) issue((kb + 1) * PER + d, t + PD, nbuf);
    }
  }
  // partial -> ws[block][co 64][392]: accumulator (i, j) register r = co 16i + 4g + r, column
  // 16 * pair + (lane & 15) = (tap 2 * pair + ((lane >> 3) & 1)) * 8 + channel (lane & 7)
  float* o = ws + (int64_t)blockIdx.x * 64 * SWP_COLS;
#pragma unroll
  for (int j = 0; j < SWP_JW; ++j) {
    const int col = 16 * (wave + 4 * j) + (lane & 15);
    if (col < SWP_COLS)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[(16 * i + 4 * g + r) * SWP_COLS + col] = acc[i][j][r];
  }
}

// the stem geometry on the packed input, bf16, slab workspace, both tensors below the 2 GiB
// buffer extent
static bool stem_wpatch_ok(const avsr_conv_params* p) {
  if (!avsr_opt(AVSR_OPT_STEM_WPATCH) || p->dtype != AVSR_BF16 || p->groups != 1 || p->splitk > 0) return false;
  if (p->cin != 8 || p->ldx != 8 || p->cout != 64 || p->ldy != 64 || p->kh != 7 || p->kw != 7) return false;
  if (p->sh != 2 || p->sw != 2 || p->ph != 3 || p->pw != 3 || p->hin != 88 || p->win != 88) return false;
  if (p->hout != 44 || p->wout != 44) return false;
  const int64_t dyb = (int64_t)p->nimg * 1936 * 128;
  return dyb > 0 && dyb < (int64_t)gemmg::OOB - (1 << 20);
}

static int stem_wpatch_launch(const avsr_conv_params* p, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)stem_wgrad_patch_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, SWP_LDS);
    attr = true;
  }
  const uint32_t xb = (uint32_t)((int64_t)p->nimg * 88 * 88 * 16), dyb = (uint32_t)((int64_t)p->nimg * 1936 * 128);
  hipLaunchKernelGGL(stem_wgrad_patch_kernel, dim3(SWP_BLOCKS), dim3(256), SWP_LDS, st, (const bf16*)p->x,
                     (const bf16*)p->dy, xb, dyb, p->nimg, p->ws);
  AVSR_CHECK_LAUNCH();
  const int64_t mn = 64 * SWP_COLS;
  const int xg = avsr_grid(mn / 4, 256, 1024);
  const int chunks = 8;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)xg, 1u, (unsigned)chunks), dim3(256), 0, st, p->ws, SWP_BLOCKS,
                     chunks, mn, p->dw, (int64_t)0);
  AVSR_CHECK_LAUNCH();
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)xg, 1u, 1u), dim3(256), 0, st, p->ws, SWP_BLOCKS, -chunks, mn,
                     p->dw, (int64_t)0);
  AVSR_CHECK_LAUNCH();
  return 0;
}

// the patch-resident stage-1 kernel applies (bf16, 3x3 / stride 1 / pad 1, 64 -> 64 channels)
static bool patch_ok(const avsr_conv_params* p, const ConvArgs& a) {
  if (!avsr_opt(AVSR_OPT_CONV_PATCH) || p->dtype != AVSR_BF16 || !conv_glds_enabled() || !a.a_bytes || p->groups != 1) return false;
  if (p->kh != 3 || p->kw != 3 || p->sh != 1 || p->sw != 1 || p->ph != 1 || p->pw != 1) return false;
  if (p->cin != 64 || p->cout != 64 || p->ldx != 64 || p->ldy != 64) return false;
  if (p->hin != p->hout || p->win != p->wout) return false;
  // worst-case padded span of 256 consecutive output pixels, plus the tap halo on both sides
  const int64_t W = p->win, HW = (int64_t)p->hin * p->win, Wp = W + 2;
  const int64_t span = (PCfg::BM - 1) + 2 * ((PCfg::BM - 1) / W + 1) + 2 * Wp * ((PCfg::BM - 1) / HW + 1) + 2 * (Wp + 1) + 1;
  return span <= PATCH_ROWS;
}

template <int KIND>
static int patch_launch(const ConvArgs& a, const avsr_conv_params* p, int sign, hipStream_t st) {
  PatchGeom pg;
  pg.nimg = p->nimg; pg.H = p->hin; pg.W = p->win; pg.Wp = p->win + 2; pg.PP = (p->hin + 2) * (p->win + 2);
  pg.f_pp = make_fastdiv((uint32_t)pg.PP); pg.f_wp = make_fastdiv((uint32_t)pg.Wp);
  pg.f_hw = make_fastdiv((uint32_t)(p->hin * p->win)); pg.f_w = make_fastdiv((uint32_t)p->win);
  pg.sign = sign;
  const int tm = (a.M + PCfg::BM - 1) / PCfg::BM;
  if (a.e.stats && a.e.stats_tiles != tm) return AVSR_E_SHAPE;
  hipLaunchKernelGGL((conv_patch_kernel<KIND>), dim3((unsigned)tm), dim3(PCfg::NTH), PATCH_LDS, st, a, pg);
  AVSR_CHECK_LAUNCH();
  return 0;
}

template <int KIND>
static int s2_launch(const ConvArgs& a0, const avsr_conv_params* p, hipStream_t st) {
  S2Class cl[4];
  s2_classes(p, cl);
  int64_t tile_off = 0;
  for (int q = 0; q < 4; ++q) {
    const S2Class& k = cl[q];
    const int Mc = p->nimg * k.hc * k.wc;
    if (Mc == 0) continue;
    ConvArgs a = a0;
    a.g.hin = k.hc; a.g.win = k.wc; a.g.kh = k.nkh; a.g.kw = k.nkw; a.g.sh = 1; a.g.sw = 1;
    a.g.ph = k.ci; a.g.pw = k.cj;
    a.g.f_hw_in = make_fastdiv((uint32_t)(k.hc * k.wc));
    a.g.f_w_in = make_fastdiv((uint32_t)k.wc);
    a.g.f_kw = make_fastdiv((uint32_t)(k.nkw > 0 ? k.nkw : 1));
    a.g.tap_kh0 = k.kh0; a.g.tap_kw0 = k.kw0; a.g.tap_step = 2;
    a.M = Mc; a.K = k.nkh * k.nkw * p->cout; a.kchunk = a.K;
    a.e.M = Mc;
    a.e.rm_wc = k.wc; a.e.rm_hc = k.hc; a.e.rm_hin = p->hin; a.e.rm_win = p->win; a.e.rm_a = k.a; a.e.rm_b = k.b;
    if (KIND >= K_DGRAD_BNR) a.bnr.ws = a0.bnr.ws + tile_off * 4 * a.N;
    tile_off += (Mc + tile_bm_k(Mc, a.N, AVSR_BF16) - 1) / tile_bm_k(Mc, a.N, AVSR_BF16);
    if (KIND == K_DGRAD && a.K == 0 && a.e.beta == 1.f) continue;   // dx += 0
    const int rc = glds_by_tile<bf16, KIND>(a, 1, st);
    if (rc) return rc;
  }
  return 0;
}

}  // namespace

extern "C" int avsr_conv_stat_tiles(const avsr_conv_params* p) {
  const int M = p->nimg * p->hout * p->wout;
  const int bm = tile_bm_k(M, p->cout, p->dtype);
  return (M + bm - 1) / bm;
}

extern "C" int avsr_conv_bnr_tiles(const avsr_conv_params* p) {
  if (s2_phase(p)) {
    S2Class cl[4];
    s2_classes(p, cl);
    int t = 0;
    for (int q = 0; q < 4; ++q) {
      const int Mc = p->nimg * cl[q].hc * cl[q].wc;
      if (Mc) t += (Mc + tile_bm_k(Mc, p->cin, p->dtype) - 1) / tile_bm_k(Mc, p->cin, p->dtype);
    }
    return t;
  }
  const int M = p->nimg * p->hin * p->win;
  const int bm = tile_bm_k(M, p->cin, p->dtype);
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
  a.splits = 1; a.kchunk = a.K; a.ws = nullptr;
  set_extents(a, p, (p->cin % 64) == 0,
              ((int64_t)p->nimg * p->hin * p->win - 1) * p->ldx + p->cin, (int64_t)p->cout * a.K);
  base_epi(a.e);
  a.e.M = a.M; a.e.N = a.N; a.e.C = p->y; a.e.ldc = p->ldy; a.e.stats = p->stats;
  a.e.stats_tiles = avsr_conv_stat_tiles(p);
  a.e.bias = p->bias; a.e.act = p->act; a.e.preact = p->preact; a.e.res = p->res; a.e.ldr = p->ldy;
  if (p->stats && (p->bias || p->act || p->res)) return AVSR_E_ARG;
  if (a.M == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (p->dtype == AVSR_F32) return by_tile<float, float, K_FWD>(a, p->groups, st);
  if (p->dtype == AVSR_BF16 && !p->bias && !p->act && !p->res && !p->preact && patch_ok(p, a))
    return patch_launch<K_FWD>(a, p, 1, st);
  if (p->dtype == AVSR_BF16)
    return conv_glds_enabled() ? glds_by_tile<bf16, K_FWD>(a, p->groups, st) : by_tile<bf16, bf16, K_FWD>(a, p->groups, st);
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
  a.splits = 1; a.kchunk = a.K; a.ws = nullptr;
  set_extents(a, p, (p->cout % 64) == 0 && (p->sh == 1 || p->sh == 2) && p->sw == p->sh,
              ((int64_t)p->nimg * p->hout * p->wout - 1) * p->ldy + p->cout, (int64_t)p->cout * a.K);
  base_epi(a.e);
  a.e.M = a.M; a.e.N = a.N; a.e.C = p->dx; a.e.ldc = p->ldx; a.e.alpha = p->alpha; a.e.beta = p->beta;
  if (p->bnr_h) {
    // BN-backward reduction in the epilogue: bf16 LDS-DMA path, one group, every operand of
    // the epilogue 16-byte aligned with the row stride of dx
    if (p->dtype != AVSR_BF16 || !conv_glds_enabled() || p->groups != 1 || !p->bnr_ws || !p->bnr_scale ||
        !p->bnr_shift || !p->bnr_prelu || !p->bnr_mean || !p->bnr_invstd || (p->bnr_scale2 && !p->bnr_res) ||
        (p->bnr_scale2 && (!p->bnr_shift2 || !p->bnr_mean2 || !p->bnr_invstd2)))
      return AVSR_E_ARG;
    if (!avsr_aligned16(p->bnr_h) || (p->bnr_res && !avsr_aligned16(p->bnr_res))) return AVSR_E_ALIGN;
    a.bnr.h = (const bf16*)p->bnr_h; a.bnr.res = (const bf16*)p->bnr_res;
    a.bnr.scale = p->bnr_scale; a.bnr.shift = p->bnr_shift; a.bnr.prelu = p->bnr_prelu;
    a.bnr.mean = p->bnr_mean; a.bnr.invstd = p->bnr_invstd; a.bnr.scale2 = p->bnr_scale2;
    a.bnr.shift2 = p->bnr_shift2; a.bnr.mean2 = p->bnr_mean2; a.bnr.invstd2 = p->bnr_invstd2; a.bnr.ws = p->bnr_ws;
    if (a.M == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    if (s2_phase(p)) {
      if (p->bnr_scale2) return s2_launch<K_DGRAD_BNR + 2>(a, p, st);
      if (p->bnr_res) return s2_launch<K_DGRAD_BNR + 1>(a, p, st);
      return s2_launch<K_DGRAD_BNR>(a, p, st);
    }
    if (patch_ok(p, a)) {
      if (p->bnr_scale2) return patch_launch<K_DGRAD_BNR + 2>(a, p, -1, st);
      if (p->bnr_res) return patch_launch<K_DGRAD_BNR + 1>(a, p, -1, st);
      return patch_launch<K_DGRAD_BNR>(a, p, -1, st);
    }
    if (p->bnr_scale2) return glds_by_tile<bf16, K_DGRAD_BNR + 2>(a, 1, st);
    if (p->bnr_res) return glds_by_tile<bf16, K_DGRAD_BNR + 1>(a, 1, st);
    return glds_by_tile<bf16, K_DGRAD_BNR>(a, 1, st);
  }
  if (a.M == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (p->dtype == AVSR_F32) return by_tile<float, float, K_DGRAD>(a, p->groups, st);
  if (s2_phase(p)) return s2_launch<K_DGRAD>(a, p, st);
  if (p->dtype == AVSR_BF16 && patch_ok(p, a)) return patch_launch<K_DGRAD>(a, p, -1, st);
  if (p->dtype == AVSR_BF16)
    return conv_glds_enabled() ? glds_by_tile<bf16, K_DGRAD>(a, p->groups, st)
                               : by_tile<bf16, bf16, K_DGRAD>(a, p->groups, st);
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
  if (p->ws && wpatch_ok(p)) return wpatch_launch(p, (hipStream_t)stream);   // patch-resident, ordered slab reduce
  if (p->ws && stem_wpatch_ok(p)) return stem_wpatch_launch(p, (hipStream_t)stream);
  set_extents(a, p, true, ((int64_t)p->nimg * p->hout * p->wout - 1) * p->ldy + p->cout,
              ((int64_t)p->nimg * p->hin * p->win - 1) * p->ldx + p->cin);
  const bool glds = p->dtype == AVSR_BF16 && conv_glds_enabled();
  const WgradPlan w = wgrad_plan(p, glds, p->ws != nullptr);
  a.splits = w.splits; a.kchunk = w.kchunk;
  a.ws = w.slab ? p->ws : nullptr;
  base_epi(a.e);
  a.e.M = a.M; a.e.N = a.N; a.e.C = p->dw; a.e.ldc = ktot; a.e.alpha = 1.f;
  if (w.slab) { a.e.ldc = a.N; }                       // plain stores into the slabs
  else if (w.splits == 1) { a.e.beta = 1.f; }          // dw += wgrad, one writer per element
  else { a.e.atomic = 1; }
  hipStream_t st = (hipStream_t)stream;
  if (p->dtype == AVSR_F32) rc = by_tile<float, float, K_WGRAD>(a, p->groups, st);
  else if (p->dtype != AVSR_BF16) return AVSR_E_DTYPE;
  else rc = !glds ? by_tile<bf16, float, K_WGRAD>(a, p->groups, st) : glds_by_tile<float, K_WGRAD>(a, p->groups, st);
  if (rc || !w.slab) return rc;
  const int64_t mn = (int64_t)a.M * a.N;
  const int xb = avsr_grid(mn / 4, 256, 1024);
  int chunks = (int)((65536 / 256 + (int64_t)xb * p->groups - 1) / ((int64_t)xb * p->groups));
  if (chunks > w.splits) chunks = w.splits;
  if (chunks < 1) chunks = 1;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)xb, (unsigned)p->groups, (unsigned)chunks), dim3(256), 0, st,
                     p->ws, w.splits, chunks, mn, p->dw, a.c_gstride);
  AVSR_CHECK_LAUNCH();
  if (chunks > 1) {
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)xb, (unsigned)p->groups, 1u), dim3(256), 0, st,
                       p->ws, w.splits, -chunks, mn, p->dw, a.c_gstride);
    AVSR_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int64_t avsr_conv_wgrad_ws(const avsr_conv_params* p) {
  if (!p || (p->dtype != AVSR_BF16 && p->dtype != AVSR_F32)) return 0;
  if (wpatch_ok(p)) return (int64_t)wpatch_blocks(p) * 64 * WP_COLS;
  if (stem_wpatch_ok(p)) return (int64_t)SWP_BLOCKS * 64 * SWP_COLS;
  const WgradPlan w = wgrad_plan(p, p->dtype == AVSR_BF16 && conv_glds_enabled(), true);
  if (!w.slab) return 0;
  return (int64_t)p->groups * w.splits * p->cout * ((int64_t)p->kh * p->kw * p->cin);
}
