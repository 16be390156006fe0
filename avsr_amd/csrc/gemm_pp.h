// 256x256 bf16 MFMA GEMM core with two wave groups in ping-pong (gfx950).
//
// Block = 8 waves as 2 (rows) x 4 (cols), each wave a 128x64 output (8x4 accumulators of
// v_mfma_f32_16x16x32_bf16, 128 VGPRs). A K-tile (64) is processed in 4 phases, one per
// 64x32 quadrant of the wave's output (16 MFMAs each); every phase is
//     [LDS fragment reads | one half-tile DMA | counted vmcnt]  s_barrier
//     [lgkmcnt(0), setprio 1, 8 MFMAs, setprio 0]              s_barrier
// and wave row 1 runs one barrier behind wave row 0, so on every SIMD (one wave of each
// group) one wave issues MFMAs while the other issues its reads and DMAs.
//
// LDS: 2 stages (K-tile t in stage t&1) x 4 half-images of 16 KiB:
//   A half h = rows {wr*128 + h*64 + [0,64)} of both wave rows  (read in quadrants m-half h)
//   B half h = cols {wc*64 + h*32 + [0,32)} of all wave columns (read in quadrants n-half h)
// in the swizzled layouts of gemm_glds.h (k-major [128][64] or r-contiguous [64][128]).
// Quadrant order per tile: (m0,n0) (m0,n1) (m1,n1) (m1,n0) -> reads A0+B0, B1, A1, B0.
// DMA order per phase of tile u: A1(u+1), B0(u+1), A0(u+2), B1(u+2): every half-tile is
// rewritten two phases after its last read (WAR-safe with the one-barrier group offset)
// and retired by a counted vmcnt in the phase before its first read (RAW).
#pragma once
#include "gemm_glds.h"

namespace gemmpp {
using namespace gemmcore;
using gemmg::GBK;
using gemmg::glds16;
using gemmg::g_zero_line;

constexpr int BM = 256, BN = 256, NW = 8, NTH = 512;
constexpr int HALF = 128 * GBK * 2;                 // 16 KiB
constexpr int STAGE = 4 * HALF;                     // A0 A1 B0 B1
constexpr int EP_BYTES = 2 * 32 * (BN + 4) * 4;     // epilogue_g strips (WM = 2)
constexpr int LDS_BYTES = 2 * STAGE > EP_BYTES ? 2 * STAGE : EP_BYTES;
using CF = gemmg::GCfg<2, 4, 4, 2, 2>;              // wave / accumulator layout for epilogue_g

// image position rho (0..127) of half h -> tile row/col, groups of G (A: 64, B: 32)
template <int G> AVSR_DEV int half_map(int rho, int h) { return (rho / G) * (2 * G) + h * G + rho % G; }

// k-major operand elem(r, k) = p[r*ld + k]: 2 DMA pieces per wave per half-image
template <int G> struct HalfK {
  static constexpr bool KMAJ = true;
  const bf16* p[2][2];          // [slot][half]
  int kc[2];
  int kend;
  AVSR_DEV void init(const bf16* base, int64_t ld, int r0, int rext, int kend_, int wave, int lane) {
    kend = kend_;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int pc = i * NW + wave, rho = pc * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((rho >> 1) & 7);
      kc[i] = c * 8;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = r0 + half_map<G>(rho, h);
        p[i][h] = r < rext ? base + (int64_t)r * ld + c * 8 : nullptr;
      }
    }
  }
  AVSR_DEV void issue(char* img, int h, int k0, int wave) const {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bf16* q = p[i][h];
      glds16((q && k0 + kc[i] < kend) ? (const void*)(q + k0) : (const void*)g_zero_line, img + (i * NW + wave) * 1024);
    }
  }
};

// r-contiguous operand elem(r, k) = p[k*ld + r]
template <int G> struct HalfR {
  static constexpr bool KMAJ = false;
  const bf16* p[2][2];
  int kr[2];
  int kend; int64_t ld;
  AVSR_DEV void init(const bf16* base, int64_t ld_, int r0, int rext, int kend_, int wave, int lane) {
    kend = kend_; ld = ld_;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int pc = i * NW + wave, pk = pc * 4 + lane / 16;
      const int rho = ((lane % 16) ^ gemmg::rswz<16>(pk)) * 8;
      kr[i] = pk;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = r0 + half_map<G>(rho, h);
        p[i][h] = r < rext ? base + (int64_t)pk * ld + r : nullptr;
      }
    }
  }
  AVSR_DEV void issue(char* img, int h, int k0, int wave) const {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bf16* q = p[i][h];
      glds16((q && k0 + kr[i] < kend) ? (const void*)(q + (int64_t)k0 * ld) : (const void*)g_zero_line,
             img + (i * NW + wave) * 1024);
    }
  }
};

AVSR_DEV void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <class LA, class LB>
AVSR_DEV void mainloop_pp(const LA& la, const LB& lb, int kbeg, int nk, f32x4 (&acc)[8][4], char* smem) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // part: 0 = A0, 1 = A1, 2 = B0, 3 = B1
  auto dma = [&](int t, int part) {
    char* img = smem + (t & 1) * STAGE + part * HALF;
    const int k0 = kbeg + t * GBK;
    if (part < 2) la.issue(img, part, k0, wave);
    else lb.issue(img, part - 2, k0, wave);
  };
  // prologue = phases -5..0 of the steady-state DMA order
  dma(0, 0); dma(0, 3); dma(0, 1); dma(0, 2); dma(1, 0); dma(1, 3);
  gemmg::wait_vmcnt<4>();                  // A0(0), B0(0) retired
  bar();
  if (wr == 1) bar();                      // wave row 1 runs one barrier behind
  bf16x8 af[4][2], bfr[2][2];               // [row|col tile][kb]
  for (int u = 0; u < nk; ++u) {
    const char* st = smem + (u & 1) * STAGE;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int mh = p < 2 ? 0 : 1, nh = (p == 0 || p == 3) ? 0 : 1;
      // ---- reads + DMA + counted wait
      if (p == 0 || p == 2) {
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
          for (int kb = 0; kb < 2; ++kb)
            af[ii][kb] = gemmg::gfrag<128, LA::KMAJ>(st + mh * HALF, wr * 64 + ii * 16, kb, lane);
      }
      if (p != 2) {                        // (m1,n1) reuses the B1 fragments of (m0,n1)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int kb = 0; kb < 2; ++kb)
            bfr[jj][kb] = gemmg::gfrag<128, LB::KMAJ>(st + (2 + nh) * HALF, wc * 32 + jj * 16, kb, lane);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (p == 0) dma(u + 1, 1);
      else if (p == 1) dma(u + 1, 2);
      else if (p == 2) dma(u + 2, 0);
      else dma(u + 2, 3);
      if (p == 0 || p == 1) gemmg::wait_vmcnt<10>();
      else if (p == 3) gemmg::wait_vmcnt<4>();
      bar();
      // ---- MFMA
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
            acc[4 * mh + ii][2 * nh + jj] = mfma16(af[ii][kb], bfr[jj][kb], acc[4 * mh + ii][2 * nh + jj]);
      __builtin_amdgcn_s_setprio(0);
      bar();
    }
  }
  if (wr == 0) bar();                      // rebalance the barrier count
  gemmg::wait_vmcnt<0>();
  __syncthreads();
}

}  // namespace gemmpp
