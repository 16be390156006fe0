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
      const int c = (lane % CPR) ^ ((pk & 3) << 2);
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
    const int off = (((r >> 3) ^ (q << 2)) << 4) + (r & 7) * 2;   // (k0 + q) & 3 == q
    const char* base = img + off;
    const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + (k0 + q) * (R * 2)));
    const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + (k0 + 4 + q) * (R * 2)));
    union { v4i16 s4[2]; bf16x8 h; } u;
    u.s4[0] = a; u.s4[1] = b;
    return u.h;
  }
}

template <int WM, int WN> struct GTile {
  static constexpr int BM = 64 * WM, BN = 64 * WN, NW = WM * WN, NTH = 64 * NW;
  static constexpr int SA = BM * GBK * 2, SB = BN * GBK * 2, STAGE = SA + SB;
  static constexpr int EP_BYTES = (BM / 2) * (BN + 4) * 4;
  static constexpr int LDS_BYTES = 2 * STAGE > EP_BYTES ? 2 * STAGE : EP_BYTES;
};

// K-tiles [0, nk) with k0 = kbeg + t*64; acc = the wave's 2x2 block of 32x32 tiles
template <int WM, int WN, class LA, class LB>
AVSR_DEV void mainloop_glds(const LA& la, const LB& lb, int kbeg, int nk, f32x16 (&acc)[2][2], char* smem) {
  using TL = GTile<WM, WN>;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  if (nk <= 0) return;
  la.issue(smem, kbeg, wave);
  lb.issue(smem + TL::SA, kbeg, wave);
  for (int kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nk) {
      char* nx = smem + ((kt + 1) & 1) * TL::STAGE;
      la.issue(nx, kbeg + (kt + 1) * GBK, wave);
      lb.issue(nx + TL::SA, kbeg + (kt + 1) * GBK, wave);
    }
    const char* cA = smem + (kt & 1) * TL::STAGE;
    const char* cB = cA + TL::SA;
#pragma unroll
    for (int s = 0; s < GBK / 16; ++s) {
      bf16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = gfrag<TL::BM, LA::KMAJ>(cA, wm * 64 + i * 32, s, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = gfrag<TL::BN, LB::KMAJ>(cB, wn * 64 + j * 32, s, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
    }
  }
  __syncthreads();
}

// XCD-aware block order: consecutive remapped ids run on one XCD (shared L2), bijective for
// any grid size (nwg need not be a multiple of 8)
AVSR_DEV int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

}  // namespace gemmg
