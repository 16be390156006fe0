// Shared MFMA GEMM core for libavsr_hip.so (dense GEMM and implicit-GEMM convolution).
//
// Block tile (64*WM) x (64*WN) x 32, 256 threads = 4 waves laid out WM x WN, each wave a
// 64x64 sub-tile = 2x2 v_mfma_f32_32x32x16_bf16 accumulators (fp32). Operands are staged
// global -> registers -> LDS, double-buffered with one barrier per K-tile: the next tile's
// global loads are issued before the current tile's MFMAs. LDS rows are padded by one
// 16-byte vector (conflict-free ds_read_b128 fragment reads).
//
// Operand "loaders" describe how an (R x K) operand view maps to memory:
//   LdDenseK    elem(r,k) = p[r*ld + k]                     (k contiguous)
//   LdDenseR    elem(r,k) = p[k*ld + r]                     (r contiguous)
//   LdConvK     im2col gather of an NHWC activation, k = (kh, kw, c) with c contiguous
//               (conv forward A operand; with TRANSP, the data-grad A operand over dY)
//   LdConvR     im2col gather, r = (kh, kw, c) contiguous in c, k = output pixel
//               (conv weight-grad B operand)
//   LdWgtR      conv weight [cout][kh][kw][cin] viewed as (r = cin, k = (kh, kw, cout))
//               (conv data-grad B operand)
// fp32 storage runs the same tiles on bf16 hi/lo splits (3 MFMA products per step).
#pragma once
#include "common.h"

namespace gemmcore {

constexpr int BKE = 32, NT = 256;

template <typename T> struct V { static constexpr int VE = 16 / (int)sizeof(T); static constexpr int ROW = BKE + VE; };

AVSR_DEV void zero(v16& v) { v.w[0] = v.w[1] = v.w[2] = v.w[3] = 0u; }

// ---- convolution geometry (one group) ----------------------------------------------
struct ConvGeom {
  int nimg, hin, win, hout, wout;   // forward geometry (input x -> output y)
  int kh, kw, sh, sw, ph, pw;
  int cin, cout;                    // channels per group
  int64_t ldx, ldy;                 // pixel strides (total channels) of x and y
  FastDiv f_hw_out, f_w_out;        // division by hout*wout, wout
  FastDiv f_hw_in, f_w_in;          // division by hin*win, win
  FastDiv f_kw;                     // division by kw
  int cin_shift, cout_shift;        // log2(cin), log2(cout)
  // data-grad weight taps: K-tile tap t = (u, v) over the (kh, kw) grid above reads the weight
  // tap (tap_kh0 + tap_step*u, tap_kw0 + tap_step*v) of a tap_kfh x tap_kfw kernel whose rows
  // hold ktot_w = tap_kfh*tap_kfw*cin elements (tap_step 1: the plain kernel; 2: one parity
  // class of a stride-2 data-grad)
  int ktot_w, tap_kfw, tap_kh0, tap_kw0, tap_step;
};

// ---------------------------------------------------------------- dense loaders
template <typename T, int R> struct LdDenseK {
  static constexpr bool KMAJ = true;
  static constexpr int VE = V<T>::VE, VPT = R * BKE / VE / NT;
  const T* p; int64_t ld; int rext, K;
  AVSR_DEV void init(int, int) {}
  AVSR_DEV void load(int r0, int k0, v16 (&reg)[VPT], int tid) const {
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      int v = tid + i * NT, r = v / (BKE / VE), k = k0 + (v % (BKE / VE)) * VE;
      if (r0 + r < rext && k < K) reg[i] = *(const v16*)(p + (int64_t)(r0 + r) * ld + k);
      else zero(reg[i]);
    }
  }
};

template <typename T, int R> struct LdDenseR {
  static constexpr bool KMAJ = false;
  static constexpr int VE = V<T>::VE, VPT = R * BKE / VE / NT;
  const T* p; int64_t ld; int rext, K;
  AVSR_DEV void init(int, int) {}
  AVSR_DEV void load(int r0, int k0, v16 (&reg)[VPT], int tid) const {
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      int v = tid + i * NT, kk = v / (R / VE), rr = r0 + (v % (R / VE)) * VE, k = k0 + kk;
      if (k < K && rr < rext) reg[i] = *(const v16*)(p + (int64_t)k * ld + rr);
      else zero(reg[i]);
    }
  }
};

// ---------------------------------------------------------------- conv loaders
// A operand of conv forward (TRANSP=false: r = output pixel of y, gather x) or of conv
// data-grad (TRANSP=true: r = input pixel of x, gather dy at ((h+ph-kh)/sh, (w+pw-kw)/sw)).
// k = (kh, kw, c) with c fastest; c runs over cin (forward) or cout (data-grad).
template <typename T, int R, bool TRANSP> struct LdConvK {
  static constexpr bool KMAJ = true;
  static constexpr int VE = V<T>::VE, VPT = R * BKE / VE / NT;
  const T* p; ConvGeom g; int rext, K;
  int pn[VPT], ph_[VPT], pw_[VPT];  // per vector: image*pixels base, h origin, w origin (or -1e6 if row invalid)
  AVSR_DEV void init(int r0, int tid) {
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      int v = tid + i * NT, r = r0 + v / (BKE / VE);
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
  AVSR_DEV void load(int, int k0, v16 (&reg)[VPT], int tid) const {
    const int cs = TRANSP ? g.cout_shift : g.cin_shift;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      int v = tid + i * NT, k = k0 + (v % (BKE / VE)) * VE;
      int c = k & ((1 << cs) - 1), khw = k >> cs;
      int kh = fdiv(khw, g.f_kw), kw = khw - kh * g.f_kw.d;
      bool ok = k < K;
      int64_t off;
      if (!TRANSP) {
        int ih = ph_[i] + kh, iw = pw_[i] + kw;
        ok = ok && ih >= 0 && ih < g.hin && iw >= 0 && iw < g.win;
        off = (int64_t)(pn[i] + ih * g.win + iw) * g.ldx + c;
      } else {
        int th = ph_[i] - kh, tw = pw_[i] - kw;
        int oh = th / g.sh, ow = tw / g.sw;
        ok = ok && th >= 0 && tw >= 0 && oh * g.sh == th && ow * g.sw == tw && oh < g.hout && ow < g.wout;
        off = (int64_t)(pn[i] + oh * g.wout + ow) * g.ldy + c;
      }
      if (ok) reg[i] = *(const v16*)(p + off);
      else zero(reg[i]);
    }
  }
};

// B operand of conv weight-grad: r = (kh, kw, cin) (vectors along cin), k = output pixel.
template <typename T, int R> struct LdConvR {
  static constexpr bool KMAJ = false;
  static constexpr int VE = V<T>::VE, VPT = R * BKE / VE / NT;
  const T* p; ConvGeom g; int rext, K;
  int rk[VPT], rw[VPT], rc[VPT];   // per vector: kh, kw, c (kh = -1e6 if r invalid)
  AVSR_DEV void init(int r0, int tid) {
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      int v = tid + i * NT, r = r0 + (v % (R / VE)) * VE;
      if (r >= rext) { rk[i] = -1000000; rw[i] = 0; rc[i] = 0; continue; }
      int c = r & ((1 << g.cin_shift) - 1), khw = r >> g.cin_shift;
      int kh = fdiv(khw, g.f_kw);
      rk[i] = kh; rw[i] = khw - kh * g.f_kw.d; rc[i] = c;
    }
  }
  AVSR_DEV void load(int, int k0, v16 (&reg)[VPT], int tid) const {
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      int v = tid + i * NT, k = k0 + v / (R / VE);
      bool ok = k < K;
      uint32_t kk = ok ? k : 0;
      uint32_t n = fdiv(kk, g.f_hw_out); uint32_t rem = kk - n * g.f_hw_out.d;
      uint32_t oh = fdiv(rem, g.f_w_out); uint32_t ow = rem - oh * g.f_w_out.d;
      int ih = (int)oh * g.sh - g.ph + rk[i], iw = (int)ow * g.sw - g.pw + rw[i];
      ok = ok && ih >= 0 && ih < g.hin && iw >= 0 && iw < g.win;
      if (ok) reg[i] = *(const v16*)(p + (int64_t)(n * g.hin * g.win + ih * g.win + iw) * g.ldx + rc[i]);
      else zero(reg[i]);
    }
  }
};

// B operand of conv data-grad: weight stored [cout][kh][kw][cin] (one group), viewed as
// (r = cin, k = (kh, kw, cout) with cout fastest).
template <typename T, int R> struct LdWgtR {
  static constexpr bool KMAJ = false;
  static constexpr int VE = V<T>::VE, VPT = R * BKE / VE / NT;
  const T* p; ConvGeom g; int rext, K;
  AVSR_DEV void init(int, int) {}
  AVSR_DEV void load(int r0, int k0, v16 (&reg)[VPT], int tid) const {
    const int ktot = g.kh * g.kw * g.cin;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      int v = tid + i * NT, k = k0 + v / (R / VE), rr = r0 + (v % (R / VE)) * VE;
      int co = k & ((1 << g.cout_shift) - 1), khw = k >> g.cout_shift;
      if (k < K && rr < rext) reg[i] = *(const v16*)(p + (int64_t)co * ktot + khw * g.cin + rr);
      else zero(reg[i]);
    }
  }
};

// ---------------------------------------------------------------- LDS staging
// k-major operands: LDS image [R][BKE + VE] (row = r), fragments by ds_read_b128.
// r-contiguous operands: LDS image [BKE][R + PAD] (row = k) filled by plain 16-byte stores
// (no transpose on the write side); bf16 fragments come out of ds_read_b64_tr_b16 (the
// hardware transposing read, T10), fp32 (parity mode) by scalar reads. PAD makes the row
// stride 16 dwords mod 64, so a 32-lane half's four 4x16 transposed blocks hit 64 distinct
// banks.
template <typename T, int R, bool KMAJ> struct Img {
  static constexpr int VE = V<T>::VE;
  static constexpr int PADR = sizeof(T) == 2 ? 2 * ((16 - (R / 2) % 64 + 64) % 64) : 4;
  static constexpr int RROW = KMAJ ? (BKE + VE) : (R + PADR);     // row stride (elements)
  static constexpr int ELEMS = KMAJ ? R * RROW : BKE * RROW;     // one buffer
};

template <typename T, int R, bool KMAJ, int VPT>
AVSR_DEV void lstore(T* lds, const v16 (&reg)[VPT], int tid) {
  constexpr int VE = V<T>::VE, RROW = Img<T, R, KMAJ>::RROW;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    int v = tid + i * NT;
    if constexpr (KMAJ) {
      int r = v / (BKE / VE), kv = v % (BKE / VE);
      *(v16*)(lds + r * RROW + kv * VE) = reg[i];
    } else {
      int kk = v / (R / VE), rv = v % (R / VE);
      *(v16*)(lds + kk * RROW + rv * VE) = reg[i];
    }
  }
}

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

// MFMA operand fragment: rows rb..rb+31 (row = lane&31), k = s*16 + 8*(lane>>5) + 0..7
template <typename T, int R, bool KMAJ>
AVSR_DEV void frag(const T* lds, int rb, int s, int lane, bf16x8& hi, bf16x8& lo) {
  constexpr int RROW = Img<T, R, KMAJ>::RROW;
  if constexpr (KMAJ) {
    const T* p = lds + (rb + (lane & 31)) * RROW + s * 16 + 8 * (lane >> 5);
    if constexpr (sizeof(T) == 2) {
      hi = *(const bf16x8*)p;
    } else {
      f32x4 x0 = *(const f32x4*)p, x1 = *(const f32x4*)(p + 4);
      float x[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
      split8(x, hi, lo);
    }
  } else {
    const int k0 = s * 16 + 8 * (lane >> 5);
    if constexpr (sizeof(T) == 2) {
      // 16-lane group g supplies rows k0+q (q = (lane&15)>>2), columns 4p..4p+3 of the
      // 16-column block starting at rb + 16*(g&1); lane receives its column (= lane&31).
      const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
      const T* base = lds + rb + 16 * (g & 1) + 4 * p;
      const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + (k0 + q) * RROW));
      const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + (k0 + 4 + q) * RROW));
      union { v4i16 s4[2]; bf16x8 h; } u;
      u.s4[0] = a; u.s4[1] = b;
      hi = u.h;
    } else {
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = lds[(k0 + j) * RROW + rb + (lane & 31)];
      split8(x, hi, lo);
    }
  }
}

template <typename T, int WM, int WN, bool AK = true, bool BK = true> struct Tile {
  static constexpr int BM = 64 * WM, BN = 64 * WN;
  static constexpr int SA = Img<T, BM, AK>::ELEMS, SB = Img<T, BN, BK>::ELEMS;
  static constexpr int ML_BYTES = 2 * (SA + SB) * (int)sizeof(T);
  static constexpr int EP_BYTES = (BM / 2) * (BN + 4) * 4;
  static constexpr int LDS_BYTES = ML_BYTES > EP_BYTES ? ML_BYTES : EP_BYTES;
};

// Main loop over K-tiles [kbeg, kend): acc[i][j] is the wave's 2x2 block of 32x32 tiles.
template <typename T, int WM, int WN, class LA, class LB>
AVSR_DEV void mainloop(LA& la, LB& lb, int m0, int n0, int kbeg, int kend, f32x16 (&acc)[2][2], char* smem) {
  using TL = Tile<T, WM, WN, LA::KMAJ, LB::KMAJ>;
  T* lA = (T*)smem;
  T* lB = lA + 2 * TL::SA;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  if (kbeg >= kend) return;
  la.init(m0, tid);
  lb.init(n0, tid);
  v16 ra[LA::VPT], rb[LB::VPT];
  const int nk = (kend - kbeg + BKE - 1) / BKE;
  la.load(m0, kbeg, ra, tid);
  lb.load(n0, kbeg, rb, tid);
  lstore<T, TL::BM, LA::KMAJ>(lA, ra, tid);
  lstore<T, TL::BN, LB::KMAJ>(lB, rb, tid);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      la.load(m0, kbeg + (kt + 1) * BKE, ra, tid);
      lb.load(n0, kbeg + (kt + 1) * BKE, rb, tid);
    }
    const T* cA = lA + cur * TL::SA;
    const T* cB = lB + cur * TL::SB;
#pragma unroll
    for (int s = 0; s < BKE / 16; ++s) {
      bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) frag<T, TL::BM, LA::KMAJ>(cA, wm * 64 + i * 32, s, lane, ah[i], al[i]);
#pragma unroll
      for (int j = 0; j < 2; ++j) frag<T, TL::BN, LB::KMAJ>(cB, wn * 64 + j * 32, s, lane, bh[j], bl[j]);
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
      lstore<T, TL::BM, LA::KMAJ>(lA + (cur ^ 1) * TL::SA, ra, tid);
      lstore<T, TL::BN, LB::KMAJ>(lB + (cur ^ 1) * TL::SB, rb, tid);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- epilogue
struct Epi {
  int M, N;
  void* C; int64_t ldc;
  float alpha, beta;
  const float* bias;
  int act, bwd, atomic;
  void* preact;
  const void* res; int64_t ldr;
  const void* gate;
  float drop_p; uint64_t seed; uint64_t drop_base;
  float* stats;        // BN partials: [N][stats_tiles][3] = (count, mean, M2) of the stored values
  int stats_tiles;
  // output row map of a stride-2 data-grad parity class: GEMM row r = (n, i, j) over an
  // rm_hc x rm_wc grid stores to pixel (n, 2i + rm_a, 2j + rm_b) of an rm_hin x rm_win image;
  // rm_wc == 0: row r is stored at row r
  int rm_wc, rm_hc, rm_hin, rm_win, rm_a, rm_b;
  float* colsum;       // [row tiles][N]: per-tile column sums of the stored values (or nullptr)
};

AVSR_DEV int epi_row(const Epi& e, int r) {
  if (e.rm_wc == 0) return r;
  const int q = r / e.rm_wc, j = r - q * e.rm_wc;
  const int n = q / e.rm_hc, i = q - n * e.rm_hc;
  return (n * e.rm_hin + 2 * i + e.rm_a) * e.rm_win + 2 * j + e.rm_b;
}

// row/col of accumulator register r of tile (i, j)
AVSR_DEV int acc_row(int wm, int i, int r, int lane) { return wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }
AVSR_DEV int acc_col(int wn, int j, int lane) { return wn * 64 + j * 32 + (lane & 31); }

// apply the elementwise epilogue to NE consecutive columns [col, col+NE) of one row
template <typename T, typename OutT, int NE>
AVSR_DEV void epi_elems(const Epi& e, int row, int col, const float* v_in) {
  OutT* C = (OutT*)e.C;
  const T* R = (const T*)e.res;
  T* P = (T*)e.preact;
  const T* G = (const T*)e.gate;
  const int64_t off = (int64_t)row * e.ldc + col;
  if (e.atomic) {
#pragma unroll
    for (int q = 0; q < NE; ++q)
      if (col + q < e.N) atomicAdd((float*)C + off + q, e.alpha * v_in[q]);
    return;
  }
#pragma unroll
  for (int q = 0; q < NE; ++q) {
    if (col + q >= e.N) break;
    float v = e.alpha * v_in[q];
    const uint64_t didx = e.drop_base + (uint64_t)row * (uint64_t)e.N + col + q;
    if (!e.bwd) {
      if (e.bias) v += e.bias[col + q];
      if (P) P[off + q] = from_f<T>(v);
      v = act_fwd_t<T>(e.act, v);
      if (e.drop_p > 0.f) v *= drop_scale(e.drop_p, e.seed, didx);
      if (R) v += to_f(R[(int64_t)row * e.ldr + col + q]);
    } else {
      if (e.drop_p > 0.f) v *= drop_scale(e.drop_p, e.seed, didx);
      if (G) v *= act_bwd_t<T>(e.act, to_f(G[off + q]));
    }
    if (e.beta != 0.f) v += e.beta * to_f(C[off + q]);
    C[off + q] = from_f<OutT>(v);
  }
}

// Can the tile's stores use the 8-column vector path? (non-atomic; every row-major operand
// 16-byte aligned with a row stride that keeps 8-column groups aligned)
template <typename T, typename OutT>
AVSR_DEV bool epi_vec_ok(const Epi& e) {
  const uintptr_t a = (uintptr_t)e.C | (uintptr_t)e.preact | (uintptr_t)e.res | (uintptr_t)e.gate | (uintptr_t)e.bias;
  return !e.atomic && (a & 15u) == 0 && ((e.ldc * (int64_t)sizeof(OutT)) & 15) == 0 &&
         ((e.ldc * (int64_t)sizeof(T)) & 15) == 0 && ((e.ldr * (int64_t)sizeof(T)) & 15) == 0;
}

template <typename T> AVSR_DEV void ld8(const T* p, float (&o)[8]) {
  if constexpr (sizeof(T) == 2) {
    const bf16x8 x = *(const bf16x8*)p;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (float)x[j];
  } else {
    const f32x4 x0 = *(const f32x4*)p, x1 = *(const f32x4*)(p + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { o[j] = x0[j]; o[j + 4] = x1[j]; }
  }
}
template <typename T> AVSR_DEV void st8(T* p, const float (&o)[8]) {
  if constexpr (sizeof(T) == 2) {
    bf16x8 x;
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (bf16)o[j];
    *(bf16x8*)p = x;
  } else {
    *(f32x4*)p = f32x4{o[0], o[1], o[2], o[3]};
    *(f32x4*)(p + 4) = f32x4{o[4], o[5], o[6], o[7]};
  }
}

// epi_elems for 8 full columns [col, col+8) with 16-byte loads/stores (epi_vec_ok, col+8 <= N)
template <typename T, typename OutT>
AVSR_DEV void epi_vec8(const Epi& e, int row, int col, float (&v)[8]) {
  const int64_t off = (int64_t)row * e.ldc + col;
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] *= e.alpha;
  float t[8];
  const uint64_t d0 = e.drop_base + (uint64_t)row * (uint64_t)e.N + col;
  if (!e.bwd) {
    if (e.bias) {
      ld8(e.bias + col, t);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] += t[q];
    }
    if (e.preact) st8((T*)e.preact + off, v);
    if (e.act) {
      if (sizeof(T) == 2 && e.act == AVSR_ACT_GELU) {
#pragma unroll
        for (int q = 0; q < 8; q += 2) {
          const f32x2 r = gelu_fast2(f32x2{v[q], v[q + 1]});
          v[q] = r.x; v[q + 1] = r.y;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = act_fwd_t<T>(e.act, v[q]);
      }
    }
    if (e.drop_p > 0.f) drop8(e.drop_p, e.seed, d0, v);
    if (e.res) {
      ld8((const T*)e.res + (int64_t)row * e.ldr + col, t);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] += t[q];
    }
  } else {
    if (e.drop_p > 0.f) drop8(e.drop_p, e.seed, d0, v);
    if (e.gate) {
      ld8((const T*)e.gate + off, t);
      if (sizeof(T) == 2 && e.act == AVSR_ACT_GELU) {
#pragma unroll
        for (int q = 0; q < 8; q += 2) {
          const f32x2 r = gelu_fast_grad2(f32x2{t[q], t[q + 1]});
          v[q] *= r.x; v[q + 1] *= r.y;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] *= act_bwd_t<T>(e.act, t[q]);
      }
    }
  }
  if (e.beta != 0.f) {
    ld8((const OutT*)e.C + off, t);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] += e.beta * t[q];
  }
  st8((OutT*)e.C + off, v);
}

// Epilogue: (1) optional BN statistics straight from the accumulators; (2) the tile is
// staged through LDS in two halves (BM/2 rows each) and written row-major, 4 consecutive
// columns per thread (coalesced stores, vector residual/gate reads).
template <typename T, typename OutT, int WM, int WN>
AVSR_DEV void epilogue(const Epi& e, int m0, int n0, f32x16 (&acc)[2][2], char* smem) {
  constexpr int BM = 64 * WM, BN = 64 * WN, HR = BM / 2, LDR = BN + 4;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  float* st = (float*)smem;
  if (e.stats) {
    // per column: count / mean / M2 of alpha*acc over the tile's valid rows (the stored conv
    // output: no bias / activation on this path), merged across waves with Chan's formula
    __syncthreads();
    float* red = st;  // [WM][BN][3]
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float s = 0.f, c = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const bool ok = m0 + acc_row(wm, i, r, lane) < e.M;
          s += ok ? e.alpha * acc[i][j][r] : 0.f;
          c += ok ? 1.f : 0.f;
        }
      s += __shfl_xor(s, 32, 64);
      c += __shfl_xor(c, 32, 64);
      const float mean = c > 0.f ? s / c : 0.f;
      float m2 = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const bool ok = m0 + acc_row(wm, i, r, lane) < e.M;
          const float d = e.alpha * acc[i][j][r] - mean;
          m2 += ok ? d * d : 0.f;
        }
      m2 += __shfl_xor(m2, 32, 64);
      if (lane < 32) {
        const int lc = acc_col(wn, j, lane);
        red[(wm * BN + lc) * 3 + 0] = c;
        red[(wm * BN + lc) * 3 + 1] = mean;
        red[(wm * BN + lc) * 3 + 2] = m2;
      }
    }
    __syncthreads();
    for (int lc = tid; lc < BN; lc += NT) {
      const int col = n0 + lc;
      if (col < e.N) {
        float n = 0.f, mean = 0.f, m2 = 0.f;
        for (int w = 0; w < WM; ++w) {
          const float nb = red[(w * BN + lc) * 3 + 0], mb = red[(w * BN + lc) * 3 + 1], qb = red[(w * BN + lc) * 3 + 2];
          if (nb > 0.f) {
            const float nn = n + nb, d = mb - mean;
            mean += d * nb / nn;
            m2 += qb + d * d * n * nb / nn;
            n = nn;
          }
        }
        float* o = e.stats + ((int64_t)col * e.stats_tiles + m0 / BM) * 3;
        o[0] = n; o[1] = mean; o[2] = m2;
      }
    }
  }
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int lr = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        st[lr * LDR + wn * 64 + j * 32 + (lane & 31)] = acc[half][j][r];
      }
    __syncthreads();
    for (int c = tid; c < HR * BN / 4; c += NT) {
      const int lr = c / (BN / 4), lc = (c % (BN / 4)) * 4;
      const int row = m0 + (lr >> 5) * 64 + half * 32 + (lr & 31);
      const int col = n0 + lc;
      if (row < e.M && col < e.N) {
        const f32x4 v4 = *(const f32x4*)(st + lr * LDR + lc);
        const float v[4] = {v4[0], v4[1], v4[2], v4[3]};
        epi_elems<T, OutT, 4>(e, row, col, v);
      }
    }
  }
}

// split-K slab reduce: C[b] = alpha * sum_s ws[b][s] + beta * C[b]   (fp32, 4 columns/thread;
// slab s of batch b at ws + (b*splits + s)*sS)
static __global__ __launch_bounds__(256) void slab_reduce_kernel(const float* ws, int splits, int M, int N, int64_t sS,
                                                                 float* C, int64_t ldc, int64_t sC, float alpha,
                                                                 float beta) {
  const int nq = N / 4;
  const int64_t per = (int64_t)M * nq;
  const int b = blockIdx.y;
  // per = M * N/4 < 2^31 (host-checked): 32-bit index math (a 64-bit division per vector
  // made this kernel ALU-bound)
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < (uint32_t)per; i += gridDim.x * 256) {
    const int m = (int)(i / (uint32_t)nq), n = (int)(i - (uint32_t)m * nq) * 4;
    const float* w = ws + (int64_t)b * splits * sS + (int64_t)m * N + n;
    f32x4 s = *(const f32x4*)w;
    for (int q = 1; q < splits; ++q) s += *(const f32x4*)(w + q * sS);
    float* c = C + (int64_t)b * sC + (int64_t)m * ldc + n;
    f32x4 o = s * alpha;
    if (beta != 0.f) o += *(const f32x4*)c * beta;
    *(f32x4*)c = o;
  }
}

}  // namespace gemmcore
