// bf16 MFMA GEMM core with LDS-DMA staging (global_load_lds_dwordx4) for libavsr_hip.so.
//
// Block tile (64*WM) x (64*WN) x 64, 64*WM*WN threads, each wave a 64x64 sub-tile (2x2
// v_mfma_f32_32x32x16_bf16 accumulators). Operand tiles go HBM/L2 -> LDS directly by
// global_load_lds (no register round trip, no ds_write pass), two LDS stages: the DMA of
// K-tile t+1 is issued right after the barrier that opens K-tile t and lands while t's 16
// MFMAs per wave run. Two blocks per CU (64 KiB LDS each) cover each other's barrier.
//
// LDS images are lane-linear (one wave instruction fills 1 KiB contiguously), so bank
// spreading is done by XOR-swizzling the 16-byte chunk index on the GLOBAL side:
//   k-major operand  [R][64] (128-B rows):  chunk' = chunk ^ ((row >> 1) & 7)
//       -> ds_read_b128 fragments, each 16-lane group hits 16 distinct 16-B bank slots;
//   r-contiguous     [64][R] (2R-B rows):   chunk' = chunk ^ ((k & 3) << 2)
//       -> ds_read_b64_tr_b16 fragments, each 32-lane group covers 4 rows x 64 B = 256 B.
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

// r-contiguous images: 16-byte chunk swizzle of k-row k (CPR chunks per row). Rows of >= 256 B
// (CPR >= 16): shift by (k & 3) * 64 B; rows of 128 B (CPR == 8): rows k, k+1 already sit in
// opposite bank halves, so only k & 2 shifts by 64 B. Either way one 32-lane group of a
// ds_read_b64_tr_b16 (4 consecutive k-rows x 64 B) covers all 64 banks.
template <int CPR> AVSR_DEV int rswz(int k) { return CPR >= 16 ? (k & 3) << 2 : ((k >> 1) & 1) << 2; }

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

// ---------------------------------------------------------------- fragments
// rows rb..rb+31 (row = lane&31), k = 16s + 8(lane>>5) + 0..7
template <int R, bool KMAJ>
AVSR_DEV bf16x8 gfrag(const char* img, int rb, int s, int lane) {
  if constexpr (KMAJ) {
    const int row = rb + (lane & 31);
    const int c = (2 * s + (lane >> 5)) ^ ((row >> 1) & 7);
    return *(const bf16x8*)(img + row * 128 + c * 16);
  } else {
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int k0 = 16 * s + 8 * (lane >> 5);
    const int r = rb + 16 * (g & 1) + 4 * pp;
    const int off = (((r >> 3) ^ rswz<R / 8>(q)) << 4) + (r & 7) * 2;   // k0 % 4 == 0: swizzle of k0+q, k0+4+q = of q
    const char* base = img + off;
    const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + (k0 + q) * (R * 2)));
    const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + (k0 + 4 + q) * (R * 2)));
    union { v4i16 s4[2]; bf16x8 h; } u;
    u.s4[0] = a; u.s4[1] = b;
    return u.h;
  }
}

// Block tile BM x BN = (WM*32*FM) x (WN*32*FN): WM x WN waves, each owning FM x FN
// accumulators of 32x32 (fp32, 16 registers each).
// S LDS stages: S-1 K-tiles in flight (the DMA of tile t+S-1 is issued at the top of t).
template <int WM_, int WN_, int FM_, int FN_, int S_ = 2> struct GCfg {
  static constexpr int WM = WM_, WN = WN_, FM = FM_, FN = FN_, S = S_;
  static constexpr int BM = WM * 32 * FM, BN = WN * 32 * FN, NW = WM * WN, NTH = 64 * NW;
  static constexpr int SA = BM * GBK * 2, SB = BN * GBK * 2, STAGE = SA + SB;
  static constexpr int GL = (BM + BN) * GBK * 2 / 1024 / NW;    // DMA instructions per wave per K-tile
  static constexpr int EP_BYTES = WM * 32 * (BN + 4) * 4;       // one 32-row strip per wave row
  static constexpr int LDS_BYTES = S * STAGE > EP_BYTES ? S * STAGE : EP_BYTES;
  static constexpr int MINB = LDS_BYTES <= 80 * 1024 ? 2 : 1;    // blocks per CU the LDS allows
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
  bf16x8 a[CF::FM], b[CF::FN];
  AVSR_DEV void load(const char* stage, int s, int wm, int wn, int lane) {
#pragma unroll
    for (int i = 0; i < CF::FM; ++i) a[i] = gfrag<CF::BM, AK>(stage, (wm * CF::FM + i) * 32, s, lane);
#pragma unroll
    for (int j = 0; j < CF::FN; ++j) b[j] = gfrag<CF::BN, BK>(stage + CF::SA, (wn * CF::FN + j) * 32, s, lane);
  }
  AVSR_DEV void mma(f32x16 (&acc)[CF::FM][CF::FN]) const {
#pragma unroll
    for (int i = 0; i < CF::FM; ++i)
#pragma unroll
      for (int j = 0; j < CF::FN; ++j) acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
  }
};

template <class CF>
AVSR_DEV void wait_tiles_ahead(bool full) {   // tile t+1 retired: at most tiles t+2..t+S-1 in flight
  if (full) wait_vmcnt<CF::GL * (CF::S - 2)>();
  else wait_vmcnt<0>();
}

template <class CF, class LA, class LB>
AVSR_DEV void mainloop_glds(const LA& la, const LB& lb, int kbeg, int nk, f32x16 (&acc)[CF::FM][CF::FN], char* smem) {
  constexpr int S = CF::S, KS = GBK / 16;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / CF::WN, wn = wave % CF::WN;
#pragma unroll
  for (int i = 0; i < CF::FM; ++i)
#pragma unroll
    for (int j = 0; j < CF::FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
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
  Frags<CF, LA::KMAJ, LB::KMAJ> cur, nxt;
  cur.load(smem, 0, wm, wn, lane);
  int cs = 0;                       // stage of tile kt
  for (int kt = 0; kt < nk; ++kt) {
    const char* stage = smem + cs * CF::STAGE;
    const int ns = cs + 1 == S ? 0 : cs + 1;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (s + 1 < KS) {
        nxt.load(stage, s + 1, wm, wn, lane);
      } else if (kt + 1 < nk) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        wait_tiles_ahead<CF>(kt + S - 1 < nk);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (kt + S < nk) {
          char* st = smem + cs * CF::STAGE;
          la.issue(st, kbeg + (kt + S) * GBK, wave);
          lb.issue(st + CF::SA, kbeg + (kt + S) * GBK, wave);
        }
        nxt.load(smem + ns * CF::STAGE, 0, wm, wn, lane);
      }
      cur.mma(acc);
      cur = nxt;
    }
    cs = ns;
  }
  __syncthreads();
}

// Epilogue for a GCfg tile: (1) optional BN column statistics from the accumulators;
// (2) FM passes, each staging one 32-row strip per wave row through LDS and writing it
// row-major, 4 consecutive columns per thread (coalesced stores, vector residual reads).
template <typename T, typename OutT, class CF>
AVSR_DEV void epilogue_g(const Epi& e, int m0, int n0, f32x16 (&acc)[CF::FM][CF::FN], char* smem) {
  constexpr int BN = CF::BN, LDR = BN + 4, SR = CF::WM * 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / CF::WN, wn = wave % CF::WN;
  float* st = (float*)smem;
  if (e.stats) {
    __syncthreads();
    float* red = st;  // [WM][BN][3]
#pragma unroll
    for (int j = 0; j < CF::FN; ++j) {
      float s = 0.f, c = 0.f;
#pragma unroll
      for (int i = 0; i < CF::FM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (wm * CF::FM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const bool ok = m0 + row < e.M;
          s += ok ? e.alpha * acc[i][j][r] : 0.f;
          c += ok ? 1.f : 0.f;
        }
      s += __shfl_xor(s, 32, 64);
      c += __shfl_xor(c, 32, 64);
      const float mean = c > 0.f ? s / c : 0.f;
      float m2 = 0.f;
#pragma unroll
      for (int i = 0; i < CF::FM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (wm * CF::FM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const float d = e.alpha * acc[i][j][r] - mean;
          m2 += m0 + row < e.M ? d * d : 0.f;
        }
      m2 += __shfl_xor(m2, 32, 64);
      if (lane < 32) {
        const int lc = (wn * CF::FN + j) * 32 + lane;
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
#pragma unroll
  for (int i = 0; i < CF::FM; ++i) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < CF::FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int lr = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        st[lr * LDR + (wn * CF::FN + j) * 32 + (lane & 31)] = acc[i][j][r];
      }
    __syncthreads();
    for (int c = tid; c < SR * BN / 4; c += CF::NTH) {
      const int lr = c / (BN / 4), lc = (c % (BN / 4)) * 4;
      const int row = m0 + ((lr >> 5) * CF::FM + i) * 32 + (lr & 31);
      const int col = n0 + lc;
      if (row < e.M && col < e.N) {
        const f32x4 v4 = *(const f32x4*)(st + lr * LDR + lc);
        const float v[4] = {v4[0], v4[1], v4[2], v4[3]};
        epi_elems<T, OutT, 4>(e, row, col, v);
      }
    }
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
