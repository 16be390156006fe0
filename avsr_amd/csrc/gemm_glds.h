// bf16 MFMA GEMM core with LDS-DMA staging (global_load_lds_dwordx4) for libavsr_hip.so.
//
// Block tile (WM*32*FM) x (WN*32*FN) x 64 (GCfg), each wave a (32FM)x(32FN) sub-tile of
// v_mfma_f32_16x16x32_bf16 accumulators (the 16x16x32 shape holds a higher clock than
// 32x32x16 on random data at the same cycles per FLOP: MI355X_MICROARCH.md, DVFS item 7).
// Operand tiles go HBM/L2 -> LDS directly by global_load_lds (no register round trip, no
// ds_write pass) into a ring of S stages.
//
// LDS images are lane-linear (one wave instruction fills 1 KiB contiguously), so bank
// spreading is done by XOR-swizzling the 16-byte chunk index on the GLOBAL side:
//   k-major operand  [R][64] (128-B rows):  chunk' = chunk ^ ((row >> 1) & 7)
//       -> ds_read_b128 fragments, each 16-lane group hits 16 distinct 16-B bank slots;
//   r-contiguous     [64][R] (2R-B rows):   chunk' = chunk ^ rswz(k)
//       -> ds_read_b64_tr_b16 fragments, each 32-lane group covers 8 rows x 32 B = 256 B.
// Out-of-range vectors are DMA'd from a zero line (a masked lane would leave stale LDS).
#pragma once
#include "gemm_core.h"

namespace gemmg {
using namespace gemmcore;

constexpr int GBK = 64;

static __device__ __attribute__((aligned(16))) uint4 g_zero_line[64];

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

AVSR_DEV void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

// r-contiguous images: 16-byte chunk swizzle of k-row k (CPR chunks per row, always an even
// XOR so 32-byte chunk pairs stay together). One 32-lane group of a 16x16x32 fragment's
// ds_read_b64_tr_b16 reads rows {k0 + q, k0 + 8 + q : q < 4} x 32 B (k0 % 16 == 0). Rows of
// >= 256 B (CPR >= 16): 8 distinct 32-B windows from (k & 3, k & 8); rows of 128 B
// (CPR == 8): k & 1 picks the bank half, (k & 2, k & 8) the 32-B window in it.
template <int CPR> AVSR_DEV int rswz(int k) {
  return CPR >= 16 ? ((k & 3) | (((k >> 3) & 1) << 2)) << 1 : (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 1;
}

// ---------------------------------------------------------------- dense loaders
// k-major operand: elem(r, k) = p[r*ld + k]
template <int R, int NW> struct GDenseK {
  static constexpr bool KMAJ = true;
  static constexpr int SLOTS = R / 8 / NW;
  const bf16* p[SLOTS];
  int kc[SLOTS];
  int kend;
  AVSR_DEV void init(const bf16* base, int64_t ld, int r0, int rext, int kend_, int wave, int lane) {
    kend = kend_;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int pc = i * NW + wave, pr = pc * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((pr >> 1) & 7);
      kc[i] = c * 8;
      p[i] = (r0 + pr < rext) ? base + (int64_t)(r0 + pr) * ld + c * 8 : nullptr;
    }
  }
  AVSR_DEV void issue(char* img, int k0, int wave) const {
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const void* src = (p[i] && k0 + kc[i] < kend) ? (const void*)(p[i] + k0) : (const void*)g_zero_line;
      glds16(src, img + (i * NW + wave) * 1024);
    }
  }
};

// r-contiguous operand: elem(r, k) = p[k*ld + r]   (r extent a multiple of 8)
template <int R, int NW> struct GDenseR {
  static constexpr bool KMAJ = false;
  static constexpr int CPR = R / 8, RPP = 64 / CPR, SLOTS = GBK / RPP / NW;
  const bf16* p[SLOTS];
  int kr[SLOTS];
  int kend; int64_t ld;
  AVSR_DEV void init(const bf16* base, int64_t ld_, int r0, int rext, int kend_, int wave, int lane) {
    kend = kend_; ld = ld_;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int pc = i * NW + wave, pk = pc * RPP + lane / CPR;
      const int c = (lane % CPR) ^ rswz<CPR>(pk);
      const int r = r0 + c * 8;
      kr[i] = pk;
      p[i] = r < rext ? base + (int64_t)pk * ld + r : nullptr;
    }
  }
  AVSR_DEV void issue(char* img, int k0, int wave) const {
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const void* src = (p[i] && k0 + kr[i] < kend) ? (const void*)(p[i] + (int64_t)k0 * ld) : (const void*)g_zero_line;
      glds16(src, img + (i * NW + wave) * 1024);
    }
  }
};

// ---------------------------------------------------------------- buffer-DMA loaders
// Same images, but the DMA is buffer_load_dwordx4 ... lds on a buffer resource (base and
// byte extent in SGPRs): the per-lane part of the address is a 32-bit byte offset fixed at
// init, the per-K-tile advance is a scalar offset, and a lane with nothing valid to load
// gets offset OOB (>= the extent: the hardware returns zeros) instead of a 64-bit pointer
// select. This keeps the DMA issue path at a few VALU per piece (the pointer loaders cost
// ~20 VALU per piece, which made the convolutions VALU-bound). Extents must be < 2 GiB.
constexpr uint32_t OOB = 0x80000000u;

AVSR_DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
// buffer_load_dwordx4 ... lds as inline asm. The compiler then does not know that the
// instruction writes LDS: with __builtin_amdgcn_raw_ptr_buffer_load_lds its waitcnt pass puts
// an s_waitcnt vmcnt(0) in front of every later ds_read_b64_tr_b16 (an LDS read it cannot
// disambiguate from the pending DMA), which drained the prefetch of the NEXT K-tile before the
// current one was computed in every kernel with a transposed operand (data-grads,
// weight-grads). Callers order the DMAs against their LDS reads with explicit vmcnt waits and
// barriers (mainloop_glds, the conv patch kernels). M0 is written here and listed as clobbered,
// so the compiler re-materialises any value it keeps in M0 (LDS-DMA builtins, readlane, DS ops).
AVSR_DEV void bglds16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, char* lds_wave_base) {
  const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void_t*)lds_wave_base);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(m), "v"(voff), "s"(r),
               "s"(soff)
               : "memory", "m0");
}

// k-major: elem(r, k) = base[r*ld + k]
template <int R, int NW> struct BDenseK {
  static constexpr bool KMAJ = true;
  static constexpr int SLOTS = R / 8 / NW;
  __amdgpu_buffer_rsrc_t rs;
  uint32_t vo[SLOTS];
  int kc[SLOTS];
  int kend;
  AVSR_DEV void init(const bf16* base, uint32_t bytes, int64_t ld, int r0, int rext, int kend_, int wave, int lane) {
    rs = make_rsrc(base, bytes);
    kend = kend_;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int pc = i * NW + wave, pr = pc * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((pr >> 1) & 7);
      kc[i] = c * 8;
      vo[i] = r0 + pr < rext ? (uint32_t)(((int64_t)(r0 + pr) * ld + c * 8) * 2) : OOB;
    }
  }
  AVSR_DEV void issue(char* img, int k0, int wave) const {
    const bool full = k0 + GBK <= kend;        // wave-uniform: only a ragged last tile masks lanes
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const uint32_t v = (full || k0 + kc[i] < kend) ? vo[i] : OOB;
      bglds16(rs, v, (uint32_t)k0 * 2u, img + (i * NW + wave) * 1024);
    }
  }
};

// r-contiguous: elem(r, k) = base[k*ld + r]   (r extent a multiple of 8)
template <int R, int NW> struct BDenseR {
  static constexpr bool KMAJ = false;
  static constexpr int CPR = R / 8, RPP = 64 / CPR, SLOTS = GBK / RPP / NW;
  __amdgpu_buffer_rsrc_t rs;
  uint32_t vo[SLOTS];
  int kr[SLOTS];
  int kend; uint32_t ld2;
  AVSR_DEV void init(const bf16* base, uint32_t bytes, int64_t ld, int r0, int rext, int kend_, int wave, int lane) {
    rs = make_rsrc(base, bytes);
    kend = kend_; ld2 = (uint32_t)(ld * 2);
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int pc = i * NW + wave, pk = pc * RPP + lane / CPR;
      const int r = r0 + ((lane % CPR) ^ rswz<CPR>(pk)) * 8;
      kr[i] = pk;
      vo[i] = r < rext ? (uint32_t)(((int64_t)pk * ld + r) * 2) : OOB;
    }
  }
  AVSR_DEV void issue(char* img, int k0, int wave) const {
    const bool full = k0 + GBK <= kend;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const uint32_t v = (full || k0 + kr[i] < kend) ? vo[i] : OOB;
      bglds16(rs, v, (uint32_t)k0 * ld2, img + (i * NW + wave) * 1024);
    }
  }
};

// ---------------------------------------------------------------- fragments
// 16x16x32 operand fragment: rows rb..rb+15 (row = lane&15), k = 32kb + 8(lane>>4) + 0..7
template <int R, bool KMAJ>
AVSR_DEV bf16x8 gfrag(const char* img, int rb, int kb, int lane) {
  if constexpr (KMAJ) {
    const int row = rb + (lane & 15);
    const int c = (4 * kb + (lane >> 4)) ^ ((row >> 1) & 7);
    return *(const bf16x8*)(img + row * 128 + c * 16);
  } else {
    // 16-lane group g reads k-rows k0+q and k0+4+q (k0 = 32kb + 8g, q = (lane&15)>>2), 4
    // columns each from rb + 4p; the transposing read hands lane i its column rb + i.
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int k0 = 32 * kb + 8 * g;
    const int r = rb + 4 * pp;
    const int ka = k0 + q, kb2 = k0 + 4 + q;
    const char* pa = img + ka * (R * 2) + (((r >> 3) ^ rswz<R / 8>(ka)) << 4) + (r & 7) * 2;
    const char* pb = img + kb2 * (R * 2) + (((r >> 3) ^ rswz<R / 8>(kb2)) << 4) + (r & 7) * 2;
    const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)pa);
    const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)pb);
    union { v4i16 s4[2]; bf16x8 h; } u;
    u.s4[0] = a; u.s4[1] = b;
    return u.h;
  }
}

// S LDS stages: S-1 K-tiles in flight (the DMA of tile t+S-1 is issued at the top of t).
template <int WM_, int WN_, int FM_, int FN_, int S_ = 2> struct GCfg {
  static constexpr int WM = WM_, WN = WN_, FM = FM_, FN = FN_, S = S_;
  static constexpr int BM = WM * 32 * FM, BN = WN * 32 * FN, NW = WM * WN, NTH = 64 * NW;
  static constexpr int SA = BM * GBK * 2, SB = BN * GBK * 2, STAGE = SA + SB;
  static constexpr int GL = (BM + BN) * GBK * 2 / 1024 / NW;    // DMA instructions per wave per K-tile
  static constexpr int EP_BYTES = WM * 32 * (BN + 4) * 4;       // one 32-row strip per wave row
  static constexpr int LDS_BYTES = S * STAGE > EP_BYTES ? S * STAGE : EP_BYTES;
  static constexpr int MINB = LDS_BYTES <= 53 * 1024 ? 3 : LDS_BYTES <= 80 * 1024 ? 2 : 1;   // blocks per CU the LDS allows
  static constexpr int TM = 2 * FM, TN = 2 * FN;                 // 16x16 accumulator tiles per wave
};

template <int N> AVSR_DEV void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// K-tiles [0, nk) with k0 = kbeg + t*64; acc = the wave's FM x FN block of 32x32 tiles.
// Ring of S stages. Fragments are double-buffered in registers: the reads for k-step s+1
// are issued before the MFMAs of step s, and at the last k-step of tile t the ring
// advances first (counted vmcnt for tile t+1's DMAs, raw s_barrier that also retires every
// wave's reads of tile t, DMA of tile t+S into tile t's stage) so that tile t+1's first
// fragments are in flight behind tile t's last MFMAs.
template <class CF, bool AK, bool BK>
struct Frags {
  bf16x8 a[CF::TM], b[CF::TN];
  AVSR_DEV void load(const char* stage, int kb, int wm, int wn, int lane) {
#pragma unroll
    for (int i = 0; i < CF::TM; ++i) a[i] = gfrag<CF::BM, AK>(stage, (wm * CF::TM + i) * 16, kb, lane);
#pragma unroll
    for (int j = 0; j < CF::TN; ++j) b[j] = gfrag<CF::BN, BK>(stage + CF::SA, (wn * CF::TN + j) * 16, kb, lane);
  }
  AVSR_DEV void mma(f32x4 (&acc)[CF::TM][CF::TN]) const {
#pragma unroll
    for (int i = 0; i < CF::TM; ++i)
#pragma unroll
      for (int j = 0; j < CF::TN; ++j) acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
  }
};

template <class CF>
AVSR_DEV void wait_tiles_ahead(bool full) {   // tile t+1 retired: at most tiles t+2..t+S-1 in flight
  if (full) wait_vmcnt<CF::GL * (CF::S - 2)>();
  else wait_vmcnt<0>();
}

// `wave` = the wave's index inside its CF group (0 .. CF::NW-1): one group of waves per
// workgroup normally; the in-block split-K weight-gradient kernel runs two groups, each with its
// own LDS ring at `smem`, in lockstep (the same tile count, so the same barriers)
template <class CF, class LA, class LB>
AVSR_DEV void mainloop_glds(const LA& la, const LB& lb, int kbeg, int nk, f32x4 (&acc)[CF::TM][CF::TN], char* smem,
                            int wave) {
  constexpr int S = CF::S, KS = GBK / 32;
  const int lane = threadIdx.x & 63;
  const int wm = wave / CF::WN, wn = wave % CF::WN;
#pragma unroll
  for (int i = 0; i < CF::TM; ++i)
#pragma unroll
    for (int j = 0; j < CF::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nk <= 0) return;
#pragma unroll
  for (int p = 0; p < S; ++p)        // fill every stage: tiles 0..S-1
    if (p < nk) {
      la.issue(smem + p * CF::STAGE, kbeg + p * GBK, wave);
      lb.issue(smem + p * CF::STAGE + CF::SA, kbeg + p * GBK, wave);
    }
  if (nk >= S) wait_vmcnt<CF::GL * (S - 1)>();   // tile 0 retired, tiles 1..S-1 may be in flight
  else wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  // two fragment sets in fixed roles (KS == 2): f0 holds k-step 0 of a tile, f1 k-step 1, so the
  // register double-buffer needs no copies (a `cur = nxt` rotation compiled to 16 v_mov_b64 per
  // k-step on the 96x32 wave tile)
  static_assert(KS == 2, "the fragment sets alternate over two k-steps per K-tile");
  Frags<CF, LA::KMAJ, LB::KMAJ> f0, f1;
  f0.load(smem, 0, wm, wn, lane);
  int cs = 0;                       // stage of tile kt
  for (int kt = 0; kt < nk; ++kt) {
    const char* stage = smem + cs * CF::STAGE;
    const int ns = cs + 1 == S ? 0 : cs + 1;
    f1.load(stage, 1, wm, wn, lane);
    f0.mma(acc);
    if (kt + 1 < nk) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      wait_tiles_ahead<CF>(kt + S - 1 < nk);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + S < nk) {
        char* st = smem + cs * CF::STAGE;
        la.issue(st, kbeg + (kt + S) * GBK, wave);
        lb.issue(st + CF::SA, kbeg + (kt + S) * GBK, wave);
      }
      f0.load(smem + ns * CF::STAGE, 0, wm, wn, lane);
    }
    f1.mma(acc);
    cs = ns;
  }
  __syncthreads();
}

template <class CF, class LA, class LB>
AVSR_DEV void mainloop_glds(const LA& la, const LB& lb, int kbeg, int nk, f32x4 (&acc)[CF::TM][CF::TN], char* smem) {
  mainloop_glds<CF>(la, lb, kbeg, nk, acc, smem, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
}

// Epilogue for a GCfg tile: (1) optional BN column statistics from the accumulators;
// (2) FM passes, each staging one 32-row strip per wave row (accumulator tiles 2i, 2i+1)
// through LDS and writing it row-major, 8 consecutive columns per thread (one 16-byte store
// per bf16 output row segment; 16-byte preact/residual/gate reads). Accumulator tile (ti, tj) register r sits at wave-local row
// 16ti + 4(lane>>4) + r, column 16tj + (lane&15).
template <typename T, typename OutT, class CF>
AVSR_DEV void epilogue_g(const Epi& e, int m0, int n0, f32x4 (&acc)[CF::TM][CF::TN], char* smem) {
  constexpr int BN = CF::BN, LDR = BN + 4, SR = CF::WM * 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / CF::WN, wn = wave % CF::WN;
  float* st = (float*)smem;
  const bool vec = epi_vec_ok<T, OutT>(e);
  if (e.stats) {
    __syncthreads();
    float* red = st;  // [WM][BN][3]
#pragma unroll
    for (int j = 0; j < CF::TN; ++j) {
      float s = 0.f, c = 0.f;
#pragma unroll
      for (int i = 0; i < CF::TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wm * 32 * CF::FM + i * 16 + 4 * (lane >> 4) + r;
          const bool ok = m0 + row < e.M;
          s += ok ? e.alpha * acc[i][j][r] : 0.f;
          c += ok ? 1.f : 0.f;
        }
      s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
      c += __shfl_xor(c, 16, 64); c += __shfl_xor(c, 32, 64);
      const float mean = c > 0.f ? s / c : 0.f;
      float m2 = 0.f;
#pragma unroll
      for (int i = 0; i < CF::TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wm * 32 * CF::FM + i * 16 + 4 * (lane >> 4) + r;
          const float d = e.alpha * acc[i][j][r] - mean;
          m2 += m0 + row < e.M ? d * d : 0.f;
        }
      m2 += __shfl_xor(m2, 16, 64); m2 += __shfl_xor(m2, 32, 64);
      if (lane < 16) {
        const int lc = (wn * CF::TN + j) * 16 + lane;
        red[(wm * BN + lc) * 3 + 0] = c;
        red[(wm * BN + lc) * 3 + 1] = mean;
        red[(wm * BN + lc) * 3 + 2] = m2;
      }
    }
    __syncthreads();
    for (int lc = tid; lc < BN; lc += CF::NTH) {
      const int col = n0 + lc;
      if (col < e.N) {
        float n = 0.f, mean = 0.f, m2 = 0.f;
        for (int w = 0; w < CF::WM; ++w) {
          const float nb = red[(w * BN + lc) * 3 + 0], mb = red[(w * BN + lc) * 3 + 1], qb = red[(w * BN + lc) * 3 + 2];
          if (nb > 0.f) {
            const float nn = n + nb, d = mb - mean;
            mean += d * nb / nn;
            m2 += qb + d * d * n * nb / nn;
            n = nn;
          }
        }
        float* o = e.stats + ((int64_t)col * e.stats_tiles + m0 / CF::BM) * 3;
        o[0] = n; o[1] = mean; o[2] = m2;
      }
    }
  }
  static_assert(CF::NTH % (BN / 8) == 0, "a thread's column group must be fixed");
  float cs[8];          // column sums of this thread's stored values (e.colsum)
#pragma unroll
  for (int j = 0; j < 8; ++j) cs[j] = 0.f;
#pragma unroll
  for (int i = 0; i < CF::FM; ++i) {
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < CF::TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int lr = wm * 32 + h * 16 + 4 * (lane >> 4) + r;
          st[lr * LDR + (wn * CF::TN + j) * 16 + (lane & 15)] = acc[2 * i + h][j][r];
        }
    __syncthreads();
    for (int c = tid; c < SR * BN / 8; c += CF::NTH) {
      const int lr = c / (BN / 8), lc = (c % (BN / 8)) * 8;
      const int row = m0 + ((lr >> 5) * CF::FM + i) * 32 + (lr & 31);
      const int col = n0 + lc;
      if (row < e.M && col < e.N) {
        const f32x4 v0 = *(const f32x4*)(st + lr * LDR + lc), v1 = *(const f32x4*)(st + lr * LDR + lc + 4);
        float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        const int orow = epi_row(e, row);
        if (vec && col + 8 <= e.N) {
          epi_vec8<T, OutT>(e, orow, col, v);
          if (e.colsum) {
#pragma unroll
            for (int j = 0; j < 8; ++j) cs[j] += v[j];
          }
        } else {
          epi_elems<T, OutT, 4>(e, orow, col, v);
          if (col + 4 < e.N) epi_elems<T, OutT, 4>(e, orow, col + 4, v + 4);
        }
      }
    }
  }
  if (e.colsum) {       // (host-checked: vector path, N % 8 == 0) block reduction per column
    constexpr int CG = BN / 8, RP = 9;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) st[tid * RP + j] = cs[j];
    __syncthreads();
    for (int t = tid; t < BN; t += CF::NTH) {
      const int g = t >> 3, j = t & 7;
      float s = 0.f;
      for (int k = g; k < CF::NTH; k += CG) s += st[k * RP + j];
      if (n0 + t < e.N) e.colsum[(int64_t)(m0 / CF::BM) * e.N + n0 + t] = s;
    }
  }
}

// BatchNorm(+PReLU) backward reduction fused into a data-gradient epilogue. The tile's
// values v (alpha*acc + beta*C) are the gradient of y = prelu(z), z = h*scale + shift
// (+ res | + res*scale2 + shift2); the epilogue stores dz = prelu'(z)*v instead of v and
// writes the tile's per-column partial sums
//   ws[tile_m][0][col] = sum dz, [1] = sum dz*xhat, [2] = sum dz*xhat2, [3] = sum v*z*[z<=0]
// (xhat = (h-mean)*invstd, xhat2 the same for res under its BN) over the tile's valid rows.
// h / res are laid out like C (row stride ldc). Requires N % 8 == 0 and the vector path.
struct BnrArgs {
  const bf16* h; const bf16* res;
  const float *scale, *shift, *prelu, *mean, *invstd, *scale2, *shift2, *mean2, *invstd2;
  float* ws;
};

// RES: 0 no residual, 1 identity residual, 2 residual under its own BN (downsample)
template <class CF, int RES>
AVSR_DEV void epilogue_bnr(const Epi& e, const BnrArgs& b, int m0, int n0, f32x4 (&acc)[CF::TM][CF::TN], char* smem) {
  constexpr int BN = CF::BN, LDR = BN + 4, SR = CF::WM * 32, CG = BN / 8, RP = 33, IT = SR * CG / CF::NTH;
  static_assert(CF::NTH % CG == 0 && (SR * CG) % CF::NTH == 0, "a thread's column group must be fixed");
  static_assert(CF::NTH * RP * 4 <= CF::LDS_BYTES, "partials staging exceeds LDS");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / CF::WN, wn = wave % CF::WN;
  float* st = (float*)smem;
  const int lc = (tid % CG) * 8, col = n0 + lc;
  const bool colok = col < e.N;
  const bool beta = e.beta != 0.f, alpha1 = e.alpha == 1.f;
  float sc[8], sh[8], pw[8], mu[8], is[8], sc2[8], sh2[8], mu2[8], is2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = colok ? col + j : 0;
    sc[j] = b.scale[c]; sh[j] = b.shift[c]; pw[j] = b.prelu[c]; mu[j] = b.mean[c]; is[j] = b.invstd[c];
    if constexpr (RES == 2) { sc2[j] = b.scale2[c]; sh2[j] = b.shift2[c]; mu2[j] = b.mean2[c]; is2[j] = b.invstd2[c]; }
  }
  float s0[8], s1[8], s2[8], s3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s0[j] = s1[j] = s2[j] = s3[j] = 0.f;
  bf16* C = (bf16*)e.C;
#pragma unroll
  for (int i = 0; i < CF::FM; ++i) {
    // this pass's epilogue operands (h, residual, old dx) are requested before the LDS
    // staging barrier so their latency overlaps it
    bf16x8 ph[IT], pr[IT], pc[IT];
    int64_t off[IT];
    bool ok[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int lr = (tid + it * CF::NTH) / CG;
      const int row = m0 + ((lr >> 5) * CF::FM + i) * 32 + (lr & 31);
      ok[it] = row < e.M && colok;
      off[it] = ok[it] ? (int64_t)epi_row(e, row) * e.ldc + col : 0;
      ph[it] = *(const bf16x8*)(b.h + off[it]);
      if constexpr (RES != 0) pr[it] = *(const bf16x8*)(b.res + off[it]);
      if (beta) pc[it] = *(const bf16x8*)(C + off[it]);
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < CF::TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int lr = wm * 32 + h * 16 + 4 * (lane >> 4) + r;
          st[lr * LDR + (wn * CF::TN + j) * 16 + (lane & 15)] = acc[2 * i + h][j][r];
        }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      if (!ok[it]) continue;
      const int lr = (tid + it * CF::NTH) / CG;
      const f32x4 v0 = *(const f32x4*)(st + lr * LDR + lc), v1 = *(const f32x4*)(st + lr * LDR + lc + 4);
      float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      if (alpha1) {
        if (beta)
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = fmaf(e.beta, (float)pc[it][j], v[j]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = beta ? fmaf(e.beta, (float)pc[it][j], v[j] * e.alpha) : v[j] * e.alpha;
      }
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float vj = v[j];
        const float hh = (float)ph[it][j];
        float z = hh * sc[j] + sh[j];
        float rr = 0.f;
        if constexpr (RES != 0) rr = (float)pr[it][j];
        if constexpr (RES == 1) z += rr;
        if constexpr (RES == 2) z += rr * sc2[j] + sh2[j];
        const bool pos = z > 0.f;
        const float d = pos ? vj : vj * pw[j];
        s3[j] = fmaf(vj, pos ? 0.f : z, s3[j]);
        s0[j] += d;
        s1[j] = fmaf(d, hh - mu[j], s1[j]);                 // x invstd once per column, below
        if constexpr (RES == 2) s2[j] = fmaf(d, rr - mu2[j], s2[j]);
        o[j] = (bf16)d;
      }
      *(bf16x8*)(C + off[it]) = o;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s1[j] *= is[j];
    if constexpr (RES == 2) s2[j] *= is2[j];
  }
  // per-column sums over the block: thread partials -> LDS (padded rows), then one thread per
  // (sum, column) adds the NTH/CG threads that own that column group
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    st[tid * RP + j] = s0[j]; st[tid * RP + 8 + j] = s1[j];
    st[tid * RP + 16 + j] = s2[j]; st[tid * RP + 24 + j] = s3[j];
  }
  __syncthreads();
  for (int t = tid; t < 4 * BN; t += CF::NTH) {
    const int q = t / BN, cc = t % BN, g = cc >> 3, j = cc & 7;
    float s = 0.f;
    for (int k = g; k < CF::NTH; k += CG) s += st[k * RP + q * 8 + j];
    if (n0 + cc < e.N) b.ws[((int64_t)(m0 / CF::BM) * 4 + q) * e.N + n0 + cc] = s;
  }
}

// XCD-aware block order: consecutive remapped ids run on one XCD (shared L2), bijective for
// any grid size (nwg need not be a multiple of 8)
AVSR_DEV int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// Tile of a remapped block id: batches outermost, then groups of GM tile-rows; inside a group
// the tile-row runs fastest, so the ~64 blocks an XCD holds at once cover about 8 x 8 tiles
// (A and B panels ~2 MiB each at K = 1024: both stay in that XCD's 4 MiB L2) instead of
// 2 rows x all columns (the whole B operand streamed through L2 for every pair of rows).
AVSR_DEV void tile_of(int id, int tiles_m, int tiles_n, int& tm, int& tn, int& z) {
  constexpr int GM = 8;
  const int per = tiles_m * tiles_n;
  z = id / per;
  const int t = id - z * per;
  const int grp = t / (GM * tiles_n), first = grp * GM;
  const int gsz = min(tiles_m - first, GM);
  const int r = t - grp * GM * tiles_n;
  tm = first + r % gsz;
  tn = r / gsz;
}

}  // namespace gemmg
