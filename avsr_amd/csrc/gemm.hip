// Dense GEMM with fused epilogue (C-ABI avsr_gemm). Mainloop/epilogue: gemm_core.h.
// Replaces every torch.nn.Linear on the AVSR hot path (forward, data-grad, weight-grad);
// see include/avsr_hip.h for the reference call sites.
#include "gemm_core.h"
#include "gemm_glds.h"
#include "gemm_pp.h"
#include <algorithm>
#include <cstring>

using namespace gemmcore;

namespace {

struct DenseArgs {
  int M, N, K, splits, kchunk;
  uint32_t a_bytes, b_bytes;   // buffer extents of one batch's A / B (buffer-DMA loaders); 0 = pointer loaders
  int64_t sSplit;      // slab mode: C offset between K splits (0: atomics / no split)
  const void* A; int64_t lda, sA;
  const void* B; int64_t ldb, sB;
  int64_t sC, sR;
  Epi e;
  unsigned long long* stamp;   // diagnostic {min start, max end} (avsr_gemm_params.stamp) or null
  unsigned* cnt;               // wgrad_dual_kernel slab mode: per-tile arrival counters (zeroed) or null
  float* fC; int64_t fldc;     // ... its final output C (the slabs' reduction target)
  float falpha, fbeta;
  const float* ln_c1; float ln_eps;   // skinny_mma_kernel LayerNorm prologue (avsr_gemm_params.ln_c1)
  float* lnst;                        // ... its per-chunk row statistics (split launches)
  float* kvk; float* kvv; const int* kvpos; int kvrows;   // KV-cache append (avsr_gemm_params.kv_k)
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
  e.C = (OutT*)e.C + (int64_t)bz * a.sC + sp * a.sSplit;
  if (e.res) e.res = (const T*)e.res + (int64_t)bz * a.sR;
  if (e.preact) e.preact = (T*)e.preact + (int64_t)bz * a.sC;
  if (e.gate) e.gate = (const T*)e.gate + (int64_t)bz * a.sC;
  e.drop_base = (uint64_t)bz * (uint64_t)a.M * (uint64_t)a.N;
  epilogue<T, OutT, WM, WN>(e, m0, n0, acc, smem);
}

// bf16 LDS-DMA path (gemm_glds.h): GCfg tiles, 1-D XCD-remapped grid
template <typename OutT, bool AK, bool BK, class CF>
__global__ __launch_bounds__(CF::NTH, CF::MINB) void dense_glds_kernel(DenseArgs a, int tiles_m, int tiles_n) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (a.stamp != nullptr && threadIdx.x == 0) atomicMin(a.stamp, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  const int id = gemmg::xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn, z;
  gemmg::tile_of(id, tiles_m, tiles_n, tm, tn, z);
  const int bz = z / a.splits, sp = z % a.splits;
  const int m0 = tm * CF::BM, n0 = tn * CF::BN;
  const int kbeg = sp * a.kchunk, kend = min(a.K, kbeg + a.kchunk);
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  f32x4 acc[CF::TM][CF::TN];
  const int nk = (kend - kbeg + gemmg::GBK - 1) / gemmg::GBK;
  if (a.a_bytes) {   // buffer-DMA loaders (operands < 2 GiB)
    using LA = typename std::conditional<AK, gemmg::BDenseK<CF::BM, CF::NW>, gemmg::BDenseR<CF::BM, CF::NW>>::type;
    using LB = typename std::conditional<BK, gemmg::BDenseK<CF::BN, CF::NW>, gemmg::BDenseR<CF::BN, CF::NW>>::type;
    LA la; la.init((const bf16*)a.A + (int64_t)bz * a.sA, a.a_bytes, a.lda, m0, a.M, kend, wave, lane);
    LB lb; lb.init((const bf16*)a.B + (int64_t)bz * a.sB, a.b_bytes, a.ldb, n0, a.N, kend, wave, lane);
    gemmg::mainloop_glds<CF>(la, lb, kbeg, nk, acc, smem);
  } else {
    using LA = typename std::conditional<AK, gemmg::GDenseK<CF::BM, CF::NW>, gemmg::GDenseR<CF::BM, CF::NW>>::type;
    using LB = typename std::conditional<BK, gemmg::GDenseK<CF::BN, CF::NW>, gemmg::GDenseR<CF::BN, CF::NW>>::type;
    LA la; la.init((const bf16*)a.A + (int64_t)bz * a.sA, a.lda, m0, a.M, kend, wave, lane);
    LB lb; lb.init((const bf16*)a.B + (int64_t)bz * a.sB, a.ldb, n0, a.N, kend, wave, lane);
    gemmg::mainloop_glds<CF>(la, lb, kbeg, nk, acc, smem);
  }
  Epi e = a.e;
  e.C = (OutT*)e.C + (int64_t)bz * a.sC + sp * a.sSplit;
  if (e.res) e.res = (const bf16*)e.res + (int64_t)bz * a.sR;
  if (e.preact) e.preact = (bf16*)e.preact + (int64_t)bz * a.sC;
  if (e.gate) e.gate = (const bf16*)e.gate + (int64_t)bz * a.sC;
  e.drop_base = (uint64_t)bz * (uint64_t)a.M * (uint64_t)a.N;
  gemmg::epilogue_g<bf16, OutT, CF>(e, m0, n0, acc, smem);
  if (a.stamp != nullptr) {   // uniform: every wave's stores issued before the end stamp
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(a.stamp + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
}

// Weight-gradient GEMM (both operands r-contiguous, fp32 out, plain epilogue) with an in-block
// K split: 8 waves = two groups of 4, each group a 128x128 Cfg tile over its own half of the
// block's K range with its own LDS ring (2 x 2 x 32 KiB), both groups in lockstep. Group 0 stages
// its accumulators in LDS, group 1 adds its own (fp32 addition commutes: fixed result), then all
// 8 waves write the tile: C = alpha*sum + beta*C, or the raw partial into split `sp`'s slab when
// the block grid also splits K (out-proj: 64 tiles x 4 splits). Two groups per block replace the
// two-blocks-per-CU split-K of the plain core without a slab round trip through HBM.
// With arrival counters (a.cnt) the grid split reduces in the kernel: a tile's splits are adjacent
// block ids (one XCD, one L2), each writes its partial slab write-through (sc1: relaxed agent-scope
// atomic stores), drains its stores (s_waitcnt vmcnt(0)) before the barrier that precedes its
// counter add, and the last of the tile's splits to arrive sums the slabs in split order (its own
// from LDS, the others with sc1 loads), writes C = alpha*sum + beta*C — the arithmetic of
// slab_reduce_kernel, which this replaces — and resets the counter (cdna_hip_programming.md
// Guideline 16, counter form).
template <class CF, bool FR>     // FR: the in-kernel slab reduction (its own register budget)
__device__ __forceinline__ void wgrad_dual_body(const DenseArgs& a, int tiles_m, int tiles_n, int id, char* smem) {
  static_assert(CF::BM * (CF::BN + 4) * 4 <= 2 * CF::S * CF::STAGE, "reduction tile exceeds the two rings");
  if (a.stamp != nullptr && threadIdx.x == 0) atomicMin(a.stamp, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  int tm, tn, sp;
  if (a.cnt) {                                      // splits innermost: a tile's splits share an XCD
    int z;
    gemmg::tile_of(id / a.splits, tiles_m, tiles_n, tm, tn, z);
    sp = id % a.splits;
  } else {
    gemmg::tile_of(id, tiles_m, tiles_n, tm, tn, sp);
  }
  const int m0 = tm * CF::BM, n0 = tn * CF::BN;
  const int kbeg = sp * a.kchunk, kend = min(a.K, kbeg + a.kchunk);
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wv >> 2, wave = wv & 3;
  const int ntile = (kend - kbeg + gemmg::GBK - 1) / gemmg::GBK;
  const int nk = (ntile + 1) >> 1;                  // per group; group 1's last tile may be empty (zeros)
  const int gbeg = kbeg + grp * nk * gemmg::GBK, gend = min(kend, gbeg + nk * gemmg::GBK);
  f32x4 acc[CF::TM][CF::TN];
  char* ring = smem + grp * (CF::S * CF::STAGE);
  if (a.a_bytes) {
    gemmg::BDenseR<CF::BM, CF::NW> la; la.init((const bf16*)a.A, a.a_bytes, a.lda, m0, a.M, gend, wave, lane);
    gemmg::BDenseR<CF::BN, CF::NW> lb; lb.init((const bf16*)a.B, a.b_bytes, a.ldb, n0, a.N, gend, wave, lane);
    gemmg::mainloop_glds<CF>(la, lb, gbeg, nk, acc, ring, wave);
  } else {
    gemmg::GDenseR<CF::BM, CF::NW> la; la.init((const bf16*)a.A, a.lda, m0, a.M, gend, wave, lane);
    gemmg::GDenseR<CF::BN, CF::NW> lb; lb.init((const bf16*)a.B, a.ldb, n0, a.N, gend, wave, lane);
    gemmg::mainloop_glds<CF>(la, lb, gbeg, nk, acc, ring, wave);
  }
  // (mainloop_glds ends with a barrier: both rings are free)
  constexpr int LDR = CF::BN + 4;
  float* st = (float*)smem;
  const int wm = wave / CF::WN, wn = wave % CF::WN;
#pragma unroll
  for (int i = 0; i < CF::TM; ++i)
#pragma unroll
    for (int j = 0; j < CF::TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 32 * CF::FM + 16 * i + 4 * (lane >> 4) + r, col = wn * 32 * CF::FN + 16 * j + (lane & 15);
        if (grp == 0) st[row * LDR + col] = acc[i][j][r];
      }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < CF::TM; ++i)
#pragma unroll
    for (int j = 0; j < CF::TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 32 * CF::FM + 16 * i + 4 * (lane >> 4) + r, col = wn * 32 * CF::FN + 16 * j + (lane & 15);
        if (grp == 1) st[row * LDR + col] += acc[i][j][r];
      }
  __syncthreads();
  const bool slab = a.sSplit != 0;
  constexpr int Q = CF::BN / 4;                      // float4 per tile row
  if constexpr (FR) {
    // 16-byte write-through (sc1) buffer stores / loads: the vector form of the agent-scope
    // relaxed atomic store / load (global_store_dword ... sc1), one instruction per 4 columns
    float* W = (float*)a.e.C;                        // slab 0; split q's at W + q * sSplit
    const int64_t ldw = a.e.ldc;
    const __amdgpu_buffer_rsrc_t rs = gemmg::make_rsrc(W, (uint32_t)((int64_t)a.splits * a.sSplit * 4));
    for (int c = threadIdx.x; c < CF::BM * Q; c += 2 * CF::NTH) {
      const int lr = c / Q, lc = (c % Q) * 4, row = m0 + lr, col = n0 + lc;
      if (row >= a.M || col >= a.N) continue;        // N % 4 == 0 in slab mode (host-checked)
      const f32x4 v = *(const f32x4*)(st + lr * LDR + lc);
      const uint32_t off = (uint32_t)((sp * a.sSplit + (int64_t)row * ldw + col) * 4);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i32, v), rs, off, 0, 16 /* sc1 */);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its partial is out
    __shared__ int last;
    __syncthreads();
    const int tile = tm * tiles_n + tn;
    if (threadIdx.x == 0)
      last = __hip_atomic_fetch_add(&a.cnt[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)a.splits - 1;
    __syncthreads();
    if (last) {
      // every load of the tail in flight at once (the tile's NI vectors per thread x the other
      // splits, and C for beta), then the sums in split order
      constexpr int NI = CF::BM * Q / (2 * CF::NTH), SMAX = 4;
      static_assert(NI * 2 * CF::NTH == CF::BM * Q, "tile vectors per thread");
      if (a.splits <= SMAX) {
        f32x4 pv[NI][SMAX], cv[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const int c = threadIdx.x + i * 2 * CF::NTH;
          const int lr = c / Q, lc = (c % Q) * 4, row = m0 + lr, col = n0 + lc;
          const bool ok = row < a.M && col < a.N;
          const int64_t w = (int64_t)row * ldw + col;
#pragma unroll
          for (int q = 0; q < SMAX; ++q)
            if (ok && q < a.splits && q != sp)
              pv[i][q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                             rs, (uint32_t)((q * a.sSplit + w) * 4), 0, 16 /* sc1 */));
          if (ok && a.fbeta != 0.f) cv[i] = *(const f32x4*)(a.fC + (int64_t)row * a.fldc + col);
        }
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const int c = threadIdx.x + i * 2 * CF::NTH;
          const int lr = c / Q, lc = (c % Q) * 4, row = m0 + lr, col = n0 + lc;
          if (row >= a.M || col >= a.N) continue;
          const f32x4 own = *(const f32x4*)(st + lr * LDR + lc);
          f32x4 sum = sp == 0 ? own : pv[i][0];
#pragma unroll
          for (int q = 1; q < SMAX; ++q)
            if (q < a.splits) sum += (q == sp ? own : pv[i][q]);
          f32x4 y = sum * a.falpha;
          if (a.fbeta != 0.f) y += cv[i] * a.fbeta;
          *(f32x4*)(a.fC + (int64_t)row * a.fldc + col) = y;
        }
      } else {
        for (int c = threadIdx.x; c < CF::BM * Q; c += 2 * CF::NTH) {
          const int lr = c / Q, lc = (c % Q) * 4, row = m0 + lr, col = n0 + lc;
          if (row >= a.M || col >= a.N) continue;
          const int64_t w = (int64_t)row * ldw + col;
          const f32x4 own = *(const f32x4*)(st + lr * LDR + lc);
          f32x4 sum;
          for (int q = 0; q < a.splits; ++q) {
            f32x4 v;
            if (q == sp) v = own;
            else v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                         rs, (uint32_t)((q * a.sSplit + w) * 4), 0, 16 /* sc1 */));
            if (q == 0) sum = v; else sum += v;
          }
          float* o = a.fC + (int64_t)row * a.fldc + col;
          f32x4 y = sum * a.falpha;
          if (a.fbeta != 0.f) y += *(const f32x4*)o * a.fbeta;
          *(f32x4*)o = y;
        }
      }
      if (threadIdx.x == 0) __hip_atomic_store(&a.cnt[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (a.stamp != nullptr) {
      __syncthreads();
      if (threadIdx.x == 0) atomicMax(a.stamp + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
    return;
  }
  float* C = slab ? (float*)a.e.C + sp * a.sSplit : (float*)a.e.C;
  const int64_t ldc = a.e.ldc;
  const float alpha = slab ? 1.f : a.e.alpha, beta = slab ? 0.f : a.e.beta;
  for (int c = threadIdx.x; c < CF::BM * Q; c += 2 * CF::NTH) {
    const int lr = c / Q, lc = (c % Q) * 4, row = m0 + lr, col = n0 + lc;
    if (row >= a.M || col >= a.N) continue;
    const f32x4 v = *(const f32x4*)(st + lr * LDR + lc);
    float* o = C + (int64_t)row * ldc + col;
    if (col + 4 <= a.N) {
      f32x4 y = v * alpha;
      if (beta != 0.f) y += *(const f32x4*)o * beta;
      *(f32x4*)o = y;
    } else {
      for (int q = 0; q < a.N - col; ++q) o[q] = beta != 0.f ? alpha * v[q] + beta * o[q] : alpha * v[q];
    }
  }
  if (a.stamp != nullptr) {
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(a.stamp + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
}

template <class CF, bool FR = false>
__global__ __launch_bounds__(2 * CF::NTH, 1) void wgrad_dual_kernel(DenseArgs a, int tiles_m, int tiles_n) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  wgrad_dual_body<CF, FR>(a, tiles_m, tiles_n, gemmg::xcd_remap(blockIdx.x, gridDim.x), smem);
}

// several weight-gradients in one grid (avsr_gemm_wgrad_group): block ids [start[q], start[q+1])
// are problem q's output tiles, each block the whole K range (no split). Two problems that leave
// part of the chip idle alone fill it together (encoder out-proj 64 + QKV 192 tiles = 256 = one
// block per CU).
constexpr int WG_MAX = 4;
struct WgGroup {
  DenseArgs a[WG_MAX];
  int tm[WG_MAX], tn[WG_MAX], start[WG_MAX + 1];
};
template <class CF>
__global__ __launch_bounds__(2 * CF::NTH, 1) void wgrad_group_kernel(WgGroup g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int id = gemmg::xcd_remap(blockIdx.x, gridDim.x);
  int q = 0;
#pragma unroll
  for (int i = 1; i < WG_MAX; ++i) q += id >= g.start[i];
  q = __builtin_amdgcn_readfirstlane(q);
  wgrad_dual_body<CF, false>(g.a[q], g.tm[q], g.tn[q], id - g.start[q], smem);
}

// 256x256 ping-pong core (gemm_pp.h)
template <typename OutT, bool AK, bool BK>
__global__ __launch_bounds__(gemmpp::NTH, 1) void dense_pp_kernel(DenseArgs a, int tiles_m, int tiles_n) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int id = gemmg::xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn, z;
  gemmg::tile_of(id, tiles_m, tiles_n, tm, tn, z);
  const int bz = z / a.splits, sp = z % a.splits;
  const int m0 = tm * gemmpp::BM, n0 = tn * gemmpp::BN;
  const int kbeg = sp * a.kchunk, kend = min(a.K, kbeg + a.kchunk);
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  using LA = typename std::conditional<AK, gemmpp::HalfK<64>, gemmpp::HalfR<64>>::type;
  using LB = typename std::conditional<BK, gemmpp::HalfK<32>, gemmpp::HalfR<32>>::type;
  LA la; la.init((const bf16*)a.A + (int64_t)bz * a.sA, a.lda, m0, a.M, kend, wave, lane);
  LB lb; lb.init((const bf16*)a.B + (int64_t)bz * a.sB, a.ldb, n0, a.N, kend, wave, lane);
  f32x4 acc[8][4];
  gemmpp::mainloop_pp(la, lb, kbeg, (kend - kbeg + gemmg::GBK - 1) / gemmg::GBK, acc, smem);
  Epi e = a.e;
  e.C = (OutT*)e.C + (int64_t)bz * a.sC + sp * a.sSplit;
  if (e.res) e.res = (const bf16*)e.res + (int64_t)bz * a.sR;
  if (e.preact) e.preact = (bf16*)e.preact + (int64_t)bz * a.sC;
  if (e.gate) e.gate = (const bf16*)e.gate + (int64_t)bz * a.sC;
  e.drop_base = (uint64_t)bz * (uint64_t)a.M * (uint64_t)a.N;
  gemmg::epilogue_g<bf16, OutT, gemmpp::CF>(e, m0, n0, acc, smem);
}

template <typename OutT, bool AK, bool BK>
int launch_pp(const DenseArgs& a, int batch, hipStream_t st) {
  const int tm = (a.M + 255) / 256, tn = (a.N + 255) / 256;
  const long nwg = (long)tm * tn * batch * a.splits;
  if (nwg > 0x7fffffffL) return AVSR_E_SHAPE;
  hipLaunchKernelGGL((dense_pp_kernel<OutT, AK, BK>), dim3((unsigned)nwg), dim3(gemmpp::NTH), gemmpp::LDS_BYTES, st, a,
                     tm, tn);
  AVSR_CHECK_LAUNCH();
  return 0;
}

template <typename OutT, bool AK, bool BK, class CF>
int launch_glds(const DenseArgs& a, int batch, hipStream_t st) {
  const int tm = (a.M + CF::BM - 1) / CF::BM, tn = (a.N + CF::BN - 1) / CF::BN;
  const long nwg = (long)tm * tn * batch * a.splits;
  if (nwg > 0x7fffffffL) return AVSR_E_SHAPE;
  hipLaunchKernelGGL((dense_glds_kernel<OutT, AK, BK, CF>), dim3((unsigned)nwg), dim3(CF::NTH), CF::LDS_BYTES, st, a,
                     tm, tn);
  AVSR_CHECK_LAUNCH();
  return 0;
}

using Cfg128 = gemmg::GCfg<2, 2, 2, 2, 2>;       // 128x128, 4 waves, 2 stages, 2 blocks/CU
using Cfg256 = gemmg::GCfg<2, 4, 4, 2, 2>;       // 256x256, 8 waves, 2 stages (128 KiB)
using Cfg256x128 = gemmg::GCfg<4, 2, 2, 2, 3>;   // 256x128, 8 waves, 3 stages (144 KiB)
using Cfg128x256 = gemmg::GCfg<2, 4, 2, 2, 3>;   // 128x256, 8 waves, 3 stages
using Cfg128s3 = gemmg::GCfg<2, 2, 2, 2, 3>;     // 128x128, 4 waves, 3 stages (96 KiB)
using Cfg128s4 = gemmg::GCfg<2, 2, 2, 2, 4>;     // 128x128, 4 waves, 4 stages (128 KiB)
using Cfg128w8s3 = gemmg::GCfg<2, 4, 2, 1, 3>;   // 128x128, 8 waves (64x32 each), 3 stages
using Cfg128w8s4 = gemmg::GCfg<2, 4, 2, 1, 4>;   // 128x128, 8 waves, 4 stages
using Cfg96 = gemmg::GCfg<3, 2, 1, 2, 2>;        // 96x128, 6 waves (32x64 each), 2 stages, 2 blocks/CU
using Cfg128x64 = gemmg::GCfg<4, 1, 1, 2, 2>;    // 128x64, 4 waves (32x64 each), 2 stages, 3 blocks/CU
using Cfg192 = gemmg::GCfg<2, 2, 3, 2, 2>;       // 192x128, 4 waves (96x64 each), 2 stages (80 KiB), 2 blocks/CU
using Cfg192x256 = gemmg::GCfg<2, 4, 3, 2, 2>;   // 192x256, 8 waves (96x64 each), 2 stages (112 KiB)
using Cfg192s3 = gemmg::GCfg<2, 2, 3, 2, 3>;     // 192x128, 4 waves, 3 stages (120 KiB)
using Cfg192w8 = gemmg::GCfg<2, 4, 3, 1, 2>;     // 192x128, 8 waves (96x32 each), 2 stages (80 KiB)
using Cfg192w8s3 = gemmg::GCfg<2, 4, 3, 1, 3>;   // 192x128, 8 waves, 3 stages (120 KiB)
using Cfg64 = gemmg::GCfg<2, 2, 1, 1, 2>;        // 64x64, 4 waves (32x32 each), 2 stages (32 KiB)
using Cfg64s4 = gemmg::GCfg<2, 2, 1, 1, 4>;      // 64x64, 4 stages (64 KiB: 3 K-tiles in flight)
using Cfg192w8s4 = gemmg::GCfg<2, 4, 3, 1, 4>;   // 192x128, 8 waves, 4 stages (160 KiB: 3 K-tiles in flight)

// tile choice: AVSR_OPT_GEMM_TILE = k + 1 forces configuration k (AVSR_TILE_*, benchmarks);
// otherwise the configuration with the fewest block rounds x per-tile work (wave quantisation
// over 256 CUs)
#ifndef AVSR_AB_FWD2      // A/B builds only (tools/build_variant.py): tile of the multi-round shapes
#define AVSR_AB_FWD2 11
#endif
#ifndef AVSR_AB_ROUND1    // ... and of the one-round (N = 1024) shapes
#define AVSR_AB_ROUND1 15
#endif
int tile_cfg(const avsr_gemm_params* p, int splits) {
  const int forced = (int)avsr_opt(AVSR_OPT_GEMM_TILE) - 1;
  if (forced >= 0) return forced;
  // 128x128 at two blocks per CU is the default (tools/gemm_table.py, profiles/r02_gemm_table.*:
  // the 256x256 ping-pong core loses 8-36 % at M = 6000, the 3-stage / 8-wave variants are
  // slower). The 192x128 tile (96x64 per wave: 48 MFMAs per 20 fragment reads and 10 DMAs
  // instead of 32 per 16 and 8) wins where it still runs >= 2 blocks per CU and its rounds
  // carry no more work than 128x128's: the M = 6000 encoder GEMMs with N >= 3072 (QKV / FFN1
  // fwd, FFN2 dgrad: -7..-15 %, profiles/r02_gemm_table192.txt). With one block per CU
  // (N = 1024) it loses 4-18 %. k-major A only (r-contiguous A images need BM % 64 == 0).
  if (p->a_kmajor) {
    const long tiles_z = (long)p->batch * splits;
    const long t128 = (long)((p->M + 127) / 128) * ((p->N + 127) / 128) * tiles_z;
    const long t192 = (long)((p->M + 191) / 192) * ((p->N + 127) / 128) * tiles_z;
    const long n128 = (t128 + 255) / 256, n192 = (t192 + 255) / 256;   // blocks on the busiest CU
    if (n192 >= 2 && 3 * n192 * 50 <= 2 * n128 * 51) return AVSR_AB_FWD2;      // 1.5 n192 <= 1.02 n128
    // one round of 192-row tiles that fills at least half the chip (the M = 6000, N = 1024
    // encoder GEMMs: 256 tiles): one block per CU, so 8 waves (two per SIMD, one's MFMAs cover
    // the other's LDS-DMA issue) and 3 stages: -10..-15 % vs 128x128 (profiles/r03_gemm_table_192w8.txt)
    if (t192 > 128 && t192 <= 256) return AVSR_AB_ROUND1;
  }
  // grids of fewer 128x128 tiles than CUs (the teacher-forced decoder: M = 16 x 41 rows, N = 1024:
  // 48 tiles) leave most of the chip idle: 64x64 tiles (4x the workgroups, several per CU)
  {
    const long tiles_z = (long)p->batch * splits;
    const long t128 = (long)((p->M + 127) / 128) * ((p->N + 127) / 128) * tiles_z;
    const long t64 = (long)((p->M + 63) / 64) * ((p->N + 63) / 64) * tiles_z;
    // with at most one 64x64 block per CU and a long K (>= 32 K-tiles) the K loop is DMA-latency
    // bound: 4 stages keep 3 K-tiles in flight (decoder K = 3072 / 5056 GEMMs 26 -> 20 us,
    // 41 -> 30 us; with 2+ blocks per CU or K = 1024 the 2-stage tile stays ahead,
    // profiles/r05_dec_gemm_stages.txt)
    if (t128 < 256 && t64 >= 2 * t128) return (t64 <= 256 && p->K >= 2048) ? 18 : 16;
  }
  return 0;
}

// row-tile height of a configuration (the fused column-sum partials are per row tile)
int cfg_bm(int cfg, bool ak) {
  switch (cfg) {
    case 1: return Cfg256::BM;
    case 2: return Cfg256x128::BM;
    case 3: return Cfg128x256::BM;
    case 4: return Cfg128s3::BM;
    case 5: return Cfg128s4::BM;
    case 6: return Cfg128w8s3::BM;
    case 7: return Cfg128w8s4::BM;
    case 8: return gemmpp::BM;
    case 9: return ak ? Cfg96::BM : Cfg128::BM;   // as launch_cfg
    case 10: return Cfg128x64::BM;
    case 16: return Cfg64::BM;
    case 18: return Cfg64s4::BM;
    case 11: return ak ? Cfg192::BM : Cfg128::BM;
    case 12: return ak ? Cfg192x256::BM : Cfg128::BM;
    case 13: return ak ? Cfg192s3::BM : Cfg128::BM;
    case 14: return ak ? Cfg192w8::BM : Cfg128::BM;
    case 15: return ak ? Cfg192w8s3::BM : Cfg128::BM;
    case 17: return ak ? Cfg192w8s4::BM : Cfg128::BM;
    default: return Cfg128::BM;
  }
}

template <typename OutT, bool AK, bool BK>
int launch_cfg(int cfg, const DenseArgs& a, int batch, hipStream_t st) {
  switch (cfg) {
    case 1: return launch_glds<OutT, AK, BK, Cfg256>(a, batch, st);
    case 2: return launch_glds<OutT, AK, BK, Cfg256x128>(a, batch, st);
    case 3: return launch_glds<OutT, AK, BK, Cfg128x256>(a, batch, st);
    case 4: return launch_glds<OutT, AK, BK, Cfg128s3>(a, batch, st);
    case 5: return launch_glds<OutT, AK, BK, Cfg128s4>(a, batch, st);
    case 6: return launch_glds<OutT, AK, BK, Cfg128w8s3>(a, batch, st);
    case 7: return launch_glds<OutT, AK, BK, Cfg128w8s4>(a, batch, st);
    case 8: return launch_pp<OutT, AK, BK>(a, batch, st);
    case 9:
      if constexpr (AK) return launch_glds<OutT, AK, BK, Cfg96>(a, batch, st);   // r-contiguous A needs BM % 64 == 0
      else return launch_glds<OutT, AK, BK, Cfg128>(a, batch, st);
    case 10: return launch_glds<OutT, AK, BK, Cfg128x64>(a, batch, st);
    case 16: return launch_glds<OutT, AK, BK, Cfg64>(a, batch, st);
    case 18: return launch_glds<OutT, AK, BK, Cfg64s4>(a, batch, st);
    case 11:   // BM = 192: r-contiguous A needs BM % 64 == 0 (weight-grads stay on 128x128)
      if constexpr (AK) return launch_glds<OutT, AK, BK, Cfg192>(a, batch, st);
      else return launch_glds<OutT, AK, BK, Cfg128>(a, batch, st);
    case 12:
      if constexpr (AK) return launch_glds<OutT, AK, BK, Cfg192x256>(a, batch, st);
      else return launch_glds<OutT, AK, BK, Cfg128>(a, batch, st);
    case 13:
      if constexpr (AK) return launch_glds<OutT, AK, BK, Cfg192s3>(a, batch, st);
      else return launch_glds<OutT, AK, BK, Cfg128>(a, batch, st);
    case 14:
      if constexpr (AK) return launch_glds<OutT, AK, BK, Cfg192w8>(a, batch, st);
      else return launch_glds<OutT, AK, BK, Cfg128>(a, batch, st);
    case 15:
      if constexpr (AK) return launch_glds<OutT, AK, BK, Cfg192w8s3>(a, batch, st);
      else return launch_glds<OutT, AK, BK, Cfg128>(a, batch, st);
    case 17:
      if constexpr (AK) return launch_glds<OutT, AK, BK, Cfg192w8s4>(a, batch, st);
      else return launch_glds<OutT, AK, BK, Cfg128>(a, batch, st);
    default: return launch_glds<OutT, AK, BK, Cfg128>(a, batch, st);
  }
}

template <typename OutT>
int glds_by_layout(const avsr_gemm_params* p, const DenseArgs& a, hipStream_t st) {
  const int cfg = tile_cfg(p, a.splits);
  if (p->a_kmajor && p->b_kmajor) return launch_cfg<OutT, true, true>(cfg, a, p->batch, st);
  if (p->a_kmajor) return launch_cfg<OutT, true, false>(cfg, a, p->batch, st);
  if (p->b_kmajor) return launch_cfg<OutT, false, true>(cfg, a, p->batch, st);
  return launch_cfg<OutT, false, false>(cfg, a, p->batch, st);
}

// the LDS-DMA path needs whole 16-byte vectors along every operand's contiguous dimension
bool glds_ok(const avsr_gemm_params* p) {
  if (p->dtype != AVSR_BF16 || p->M < 128 || p->N < 128) return false;
  if (!p->a_kmajor && (p->M % 8)) return false;
  if (!p->b_kmajor && (p->N % 8)) return false;
  return true;
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

// ---------------------------------------------------------------- skinny (M <= 64) linears
// The decoder's per-step linears during beam search have n = utterances x beam rows (<= 40 at
// C5). The tiled cores put one 64 x 256 tile per 256 columns on them (4 workgroups for
// N = 1024, each streaming a 1 MiB weight slab; 63 us per call in fp32 parity mode). Here the
// work is spread over N / 16 workgroups and done with fp32 FMAs on the vector ALUs (exact
// fp32 products and sums, fixed order): a workgroup stages the A rows of a 256-wide K chunk in
// LDS (as fp32), thread (column pair cg, K lane kl) keeps partial sums of 2 columns for every
// row over k = 4kl + 128j .. +3 (one 16-byte weight load per column and k group, 4 FMAs per
// row), then the 32 K lanes are reduced (shuffles within a wave, LDS across the 4 waves) and
// the usual elementwise epilogue (bias / activation / residual / beta) writes the tile.
constexpr int SK_NB = 16;

template <typename T> AVSR_DEV f32x4 ld4f(const T* p) {
  if constexpr (sizeof(T) == 2) {
    const bf16x4 v = *(const bf16x4*)p;
    return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
  } else {
    return *(const f32x4*)p;
  }
}

// K split (part != nullptr): block row blockIdx.y sums k in [y * kchunk, (y + 1) * kchunk) and
// writes the raw sums to part[y][m][n] (N / 16 workgroups alone leave most CUs idle at
// N = 1024); the last of the S workgroups of a column block to arrive (agent-scope counter
// cnt[blockIdx.x]) adds the S partials in a fixed order and runs the epilogue. Hand-off:
// partials stored write-through (sc1, relaxed agent-scope atomic stores), every storing wave
// drains its stores (s_waitcnt vmcnt(0)) before the barrier that precedes the counter add, the
// reducer reads them with sc1 loads (cdna_hip_programming.md Guideline 16, counter form) — no
// fence, no second launch; the reducer resets the counter (zero-initialised by the caller).
template <typename T, typename OutT, int MR>
__global__ __launch_bounds__(256) void skinny_kernel(DenseArgs a, float* part, int kchunk, unsigned* cnt) {
  constexpr int SK_KC = MR <= 32 ? 256 : 128;        // K chunk staged per pass (<= 33 KiB of LDS)
  constexpr int XPT = MR * SK_KC / 4 / 256;           // A vectors per thread per chunk
  constexpr int WJ = SK_KC / 128;                     // k groups per thread per chunk
  __shared__ __attribute__((aligned(16))) float xs[MR][SK_KC + 4];
  static_assert(4 * MR * (SK_NB + 1) <= MR * (SK_KC + 4), "reduction slab reuses the staging buffer");
  float (*red)[MR][SK_NB + 1] = (float (*)[MR][SK_NB + 1])&xs[0][0];
  const int tid = threadIdx.x, cg = tid & 7, kl = tid >> 3, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * SK_NB, c0 = n0 + 2 * cg, c1 = c0 + 1;
  const T* A = (const T*)a.A;
  const T* B0 = (const T*)a.B + (int64_t)min(c0, a.N - 1) * a.ldb;
  const T* B1 = (const T*)a.B + (int64_t)min(c1, a.N - 1) * a.ldb;
  const bool ok0 = c0 < a.N, ok1 = c1 < a.N;
  float acc0[MR], acc1[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) acc0[m] = acc1[m] = 0.f;
  const int kbeg = part ? blockIdx.y * kchunk : 0;
  const int kend = part ? min(a.K, kbeg + kchunk) : a.K;
  // the next chunk's A rows and weights are loaded into registers while this chunk computes
  f32x4 xr[XPT], w0[WJ], w1[WJ];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int idx = tid + 256 * i, m = idx / (SK_KC / 4), q = idx - m * (SK_KC / 4), k = k0 + 4 * q;
      xr[i] = (m < a.M && k < kend) ? ld4f(A + (int64_t)m * a.lda + k) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < WJ; ++j) {
      const int k = k0 + 4 * (kl + 32 * j);
      w0[j] = (ok0 && k < kend) ? ld4f(B0 + k) : f32x4{0.f, 0.f, 0.f, 0.f};
      w1[j] = (ok1 && k < kend) ? ld4f(B1 + k) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  load(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += SK_KC) {
    __syncthreads();                                // the previous chunk's reads of xs are done
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int idx = tid + 256 * i, m = idx / (SK_KC / 4), q = idx - m * (SK_KC / 4);
      *(f32x4*)&xs[m][4 * q] = xr[i];
    }
    f32x4 wc0[WJ], wc1[WJ];
#pragma unroll
    for (int j = 0; j < WJ; ++j) { wc0[j] = w0[j]; wc1[j] = w1[j]; }
    __syncthreads();
    if (k0 + SK_KC < kend) load(k0 + SK_KC);
#pragma unroll
    for (int j = 0; j < WJ; ++j) {
      const int g = kl + 32 * j;
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        const f32x4 x = *(const f32x4*)&xs[m][4 * g];
        acc0[m] = fmaf(x[0], wc0[j][0], acc0[m]); acc0[m] = fmaf(x[1], wc0[j][1], acc0[m]);
        acc0[m] = fmaf(x[2], wc0[j][2], acc0[m]); acc0[m] = fmaf(x[3], wc0[j][3], acc0[m]);
        acc1[m] = fmaf(x[0], wc1[j][0], acc1[m]); acc1[m] = fmaf(x[1], wc1[j][1], acc1[m]);
        acc1[m] = fmaf(x[2], wc1[j][2], acc1[m]); acc1[m] = fmaf(x[3], wc1[j][3], acc1[m]);
      }
    }
  }
  // sum over the 8 K lanes of a wave (lane bits 3-5), then over the 4 waves
#pragma unroll
  for (int m = 0; m < MR; ++m) {
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) {
      acc0[m] += __shfl_xor(acc0[m], o, 64);
      acc1[m] += __shfl_xor(acc1[m], o, 64);
    }
  }
  __syncthreads();                                  // staging buffer -> reduction slab
  if (lane < 8) {
#pragma unroll
    for (int m = 0; m < MR; ++m) { red[wave][m][2 * cg] = acc0[m]; red[wave][m][2 * cg + 1] = acc1[m]; }
  }
  __syncthreads();
  for (int o = tid; o < MR * SK_NB; o += 256) {
    const int m = o / SK_NB, c = o - m * SK_NB, col = n0 + c;
    if (m < a.M && col < a.N) {
      const float v = (red[0][m][c] + red[1][m][c]) + (red[2][m][c] + red[3][m][c]);
      if (part) __hip_atomic_store(&part[((int64_t)blockIdx.y * a.M + m) * a.N + col], v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
      else epi_elems<T, OutT, 1>(a.e, m, col, &v);
    }
  }
  if (!part) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave: its partials are out
  __shared__ int last;
  __syncthreads();
  if (tid == 0)
    last = __hip_atomic_fetch_add(&cnt[blockIdx.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.y - 1;
  __syncthreads();
  if (!last) return;
  const int S = gridDim.y;
  const int64_t MN = (int64_t)a.M * a.N;
  for (int o = tid; o < MR * SK_NB; o += 256) {
    const int m = o / SK_NB, c = o - m * SK_NB, col = n0 + c;
    if (m < a.M && col < a.N) {
      const float* pp = part + (int64_t)m * a.N + col;
      float v = __hip_atomic_load(pp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int s = 1; s < S; ++s) v += __hip_atomic_load(pp + s * MN, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      epi_elems<T, OutT, 1>(a.e, m, col, &v);
    }
  }
  if (tid == 0) __hip_atomic_store(&cnt[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// fp32 few-row linears on the fp32-input matrix cores (v_mfma_f32_16x16x4_f32: exact fp32
// products, fp32 accumulation): a workgroup = SKM_WAVES waves over one 16-column block and one K
// chunk; wave w takes the 16-k groups w, w + SKM_WAVES, ... of the chunk; per group a lane loads the
// 4 consecutive weights of its column (16 B) and, per 16-row tile, its row's 4 activations (16 B,
// L2-resident: no LDS staging), then 4 MFMAs per row tile; the chunk is one load batch (all loads
// in flight at once), and the waves' partials are summed in LDS in a fixed order. The decoder's
// weights arrive cold from HBM every step, so the grid is sized to occupy every CU
// (skinny_mma_splits: K chunks until N/16 x S >= 256); the S partials of a column block go
// through the last-arriver hand-off of skinny_kernel. A row's result never depends on M (rows are
// independent in the MFMA, the k order is fixed).
// The epilogue's bias / residual operands are read at the start, beside the weight loads.
// UNR = 4 where the grid exceeds one workgroup per CU (fewer registers, two per CU).
// LNP (LayerNorm prologue, a.ln_c1): the batch holds whole rows of the chunk, so each row's chunk
// mean and M2 (two passes over the registers, partials over the 4 lanes of a row and the 8 waves in
// a fixed order) come for free; split launches hand them over with the partial sums (a.lnst) and
// the last arriver combines them (Chan et al.'s pairwise formula, split order). Everything runs on
// x' = x - s with s = x[m][0], a per-row shift every chunk knows (x - s is exact in fp32 for values
// within a factor 2): the statistics give mean' = mean - s, the MFMAs x' against gamma o W, and the
// epilogue applies rstd * (acc - mean' * c1[n]). Without the shift a row whose |mean| is large next
// to its spread would subtract two large terms (acc ~ mean * c1) and lose the digits the
// reference's normalise-then-project keeps.
constexpr int SKM_WAVES = 8;
template <typename OutT, int MT, int UNR, bool LNP = false>
__global__ __launch_bounds__(64 * SKM_WAVES) void skinny_mma_kernel(DenseArgs a, float* part, int kchunk, unsigned* cnt) {
  constexpr int NW = SKM_WAVES, NE = (16 * MT * SK_NB + 64 * NW - 1) / (64 * NW);
  __shared__ __attribute__((aligned(16))) float red[NW][16 * MT][SK_NB + 1];
  __shared__ float st1[LNP ? NW : 1][16 * MT], st2[LNP ? NW : 1][16 * MT];
  __shared__ float rmean[LNP ? 16 * MT : 1], rrstd[LNP ? 16 * MT : 1];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, c = lane & 15;
  const int n0 = blockIdx.x * SK_NB, col = n0 + c;
  const Epi& e = a.e;
  const bool fast = !e.bwd && !e.preact && e.drop_p == 0.f && e.beta == 0.f && !e.atomic;
  float pb[NE], pr[NE];
  if (fast) {
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int o = tid + 64 * NW * i, m = o / SK_NB, cl = n0 + (o - m * SK_NB);
      const bool ok = o < 16 * MT * SK_NB && m < a.M && cl < a.N;
      pb[i] = ok && e.bias ? e.bias[cl] : 0.f;
      pr[i] = ok && e.res ? ((const float*)e.res)[(int64_t)m * e.ldr + cl] : 0.f;
    }
  }
  const bool cok = col < a.N;
  const float* Wr = (const float*)a.B + (int64_t)min(col, a.N - 1) * a.ldb + 4 * g;
  const float* Ar[MT];
  bool rok[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int m = 16 * t + c;
    rok[t] = m < a.M;
    Ar[t] = (const float*)a.A + (int64_t)min(m, a.M - 1) * a.lda + 4 * g;
  }
  const int kbeg = part ? blockIdx.y * kchunk : 0, kend = part ? min(a.K, kbeg + kchunk) : a.K;
  const int ng = (kend - kbeg) / 16;                  // K % 16 == 0 (host-checked); kchunk % 16 == 0
  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // LNP: exactly one pass for every wave (ng <= NW * UNR, host-checked), so all reach its barrier
  for (int q0 = w; LNP ? q0 == w : q0 < ng; q0 += NW * UNR) {
    f32x4 b[UNR], x[UNR][MT];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int q = q0 + NW * u;
      const bool ok = q < ng;
      const int k = kbeg + 16 * (ok ? q : 0);
      b[u] = (ok && cok) ? *(const f32x4*)(Wr + k) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < MT; ++t) x[u][t] = (ok && rok[t]) ? *(const f32x4*)(Ar[t] + k) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (LNP) {       // the batch holds the chunk's rows: chunk mean and M2 per row of x - s
      float sft[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t) sft[t] = ((const float*)a.A)[(int64_t)min(16 * t + c, a.M - 1) * a.lda];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {   // loads past the chunk stay 0 (they meet b = 0 and no statistic)
        const bool ok = q0 + NW * u < ng;
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
          for (int e2 = 0; e2 < 4; ++e2) x[u][t][e2] = ok ? x[u][t][e2] - sft[t] : 0.f;
      }
      const float inv_n = 1.f / (float)(kend - kbeg);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        float s1 = 0.f;
#pragma unroll
        for (int u = 0; u < UNR; ++u) s1 += (x[u][t][0] + x[u][t][1]) + (x[u][t][2] + x[u][t][3]);
        s1 += __shfl_xor(s1, 16, 64);
        s1 += __shfl_xor(s1, 32, 64);
        if (g == 0) st1[w][16 * t + c] = s1;
      }
      __syncthreads();
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        float sm = 0.f;
#pragma unroll
        for (int v = 0; v < NW; ++v) sm += st1[v][16 * t + c];
        const float mu = sm * inv_n;
        float s2 = 0.f;
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          if (q0 + NW * u >= ng) continue;
#pragma unroll
          for (int e2 = 0; e2 < 4; ++e2) { const float d = x[u][t][e2] - mu; s2 += d * d; }
        }
        s2 += __shfl_xor(s2, 16, 64);
        s2 += __shfl_xor(s2, 32, 64);
        if (g == 0) st2[w][16 * t + c] = s2;
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[u][t][e2], b[u][e2], acc[t], 0, 0, 0);
  }
  // acc[t][r] = this wave's partial of y[16t + 4g + r][n0 + c]; the waves' in a fixed order
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][16 * t + 4 * g + r][c] = acc[t][r];
  __syncthreads();
  // row statistics of this chunk (LNP): mean and M2 over the waves' partials in a fixed order
  auto chunk_stats = [&](int m, float& mean, float& m2) {
    float sm = 0.f, sq = 0.f;
#pragma unroll
    for (int v = 0; v < NW; ++v) { sm += st1[v][m]; sq += st2[v][m]; }
    mean = sm / (float)(kend - kbeg);
    m2 = sq;
  };
  const int kvD = a.N / 3;
  auto epi = [&](int i, int m, int cl, float v) {
    if (fast) {                // epi_elems' arithmetic, operands already in registers
      float y = e.alpha * v;
      if (e.bias) y += pb[i];
      y = act_fwd_t<float>(e.act, y);
      if (e.res) y += pr[i];
      if (a.kvk && cl >= kvD) {  // K / V columns: appended to the cache at this step's rows
        const int64_t row = (int64_t)(*a.kvpos) * a.kvrows + m;
        float* dst = cl < 2 * kvD ? a.kvk : a.kvv;
        dst[row * kvD + (cl < 2 * kvD ? cl - kvD : cl - 2 * kvD)] = y;
      } else {
        ((OutT*)e.C)[(int64_t)m * e.ldc + cl] = from_f<OutT>(y);
      }
    } else {
      epi_elems<float, OutT, 1>(a.e, m, cl, &v);
    }
  };
  if (!part) {
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int o = tid + 64 * NW * i;
      if (o >= 16 * MT * SK_NB) break;
      const int m = o / SK_NB, cc = o - m * SK_NB, cl = n0 + cc;
      if (m < a.M && cl < a.N) {
        float v = (red[0][m][cc] + red[1][m][cc]) + (red[2][m][cc] + red[3][m][cc]);
        v += (red[4][m][cc] + red[5][m][cc]) + (red[6][m][cc] + red[7][m][cc]);
        if constexpr (LNP) {
          float mean, m2;
          chunk_stats(m, mean, m2);
          v = (1.f / sqrtf(m2 / (float)a.K + a.ln_eps)) * (v - mean * a.ln_c1[cl]);
        }
        epi(i, m, cl, v);
      }
    }
    return;
  }
  for (int o = tid; o < 16 * MT * SK_NB; o += 64 * NW) {
    const int m = o / SK_NB, cc = o - m * SK_NB, cl = n0 + cc;
    if (m < a.M && cl < a.N) {
      float v = (red[0][m][cc] + red[1][m][cc]) + (red[2][m][cc] + red[3][m][cc]);
      v += (red[4][m][cc] + red[5][m][cc]) + (red[6][m][cc] + red[7][m][cc]);
      __hip_atomic_store(&part[((int64_t)blockIdx.y * a.M + m) * a.N + cl], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if constexpr (LNP) {         // this chunk's (mean, M2) per row, per column block and split
    if (tid < a.M) {
      float mean, m2;
      chunk_stats(tid, mean, m2);
      float* sp = a.lnst + (((int64_t)blockIdx.x * gridDim.y + blockIdx.y) * a.M + tid) * 2;
      __hip_atomic_store(sp, mean, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sp + 1, m2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave: its partials are out
  __syncthreads();
  if (tid == 0)
    last = __hip_atomic_fetch_add(&cnt[blockIdx.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.y - 1;
  __syncthreads();
  if (!last) return;
  const int S = gridDim.y;
  if constexpr (LNP) {         // combine the S chunks' (n, mean, M2) in split order
    if (tid < a.M) {
      const float* sp = a.lnst + ((int64_t)blockIdx.x * S * a.M + tid) * 2;
      float n = 0.f, mean = 0.f, m2 = 0.f;
      for (int q = 0; q < S; ++q) {
        const float nq = (float)(min(a.K, (q + 1) * kchunk) - q * kchunk);
        const float mq = __hip_atomic_load(sp + (int64_t)q * a.M * 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const float vq = __hip_atomic_load(sp + (int64_t)q * a.M * 2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const float nn = n + nq, d = mq - mean;
        mean += d * (nq / nn);
        m2 += vq + d * d * (n * nq / nn);
        n = nn;
      }
      rmean[tid] = mean;
      rrstd[tid] = 1.f / sqrtf(m2 / (float)a.K + a.ln_eps);
    }
    __syncthreads();
  }
  const int64_t MN = (int64_t)a.M * a.N;
#pragma unroll
  for (int i = 0; i < NE; ++i) {
    const int o = tid + 64 * NW * i;
    if (o >= 16 * MT * SK_NB) break;
    const int m = o / SK_NB, cc = o - m * SK_NB, cl = n0 + cc;
    if (m < a.M && cl < a.N) {
      const float* pp = part + (int64_t)m * a.N + cl;
      float v = __hip_atomic_load(pp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int q = 1; q < S; ++q) v += __hip_atomic_load(pp + q * MN, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if constexpr (LNP) v = rrstd[m] * (v - rmean[m] * a.ln_c1[cl]);
      epi(i, m, cl, v);
    }
  }
  if (tid == 0) __hip_atomic_store(&cnt[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// K split count: enough block rows for >= 512 workgroups, chunks of >= 256 k, and S * 64 * N
// partials within AVSR_SKINNY_WS (S depends on N and K only, never on M: a row's result does
// not depend on how many rows share the launch).
int skinny_splits(int N, int K, int& kchunk) {
  const int nb = (N + SK_NB - 1) / SK_NB;
  int S = (512 + nb - 1) / nb;
  S = std::min(S, std::max(1, K / 256));
  S = std::min(S, (int)std::max<int64_t>(1, AVSR_SKINNY_WS / (64 * (int64_t)N)));
  kchunk = ((K + S - 1) / S + 255) / 256 * 256;
  return (K + kchunk - 1) / kchunk;
}

// the matrix-core kernel's split: enough K chunks for N/16 x S >= 256 workgroups (every CU pulls
// weights from HBM) and chunks of <= 1024 k (one load batch), chunks of >= 256 k, the partials
// plus the LayerNorm chunk statistics within AVSR_SKINNY_WS
int skinny_mma_splits(int N, int K, int& kchunk) {
  const int nb = (N + SK_NB - 1) / SK_NB;
  int S = std::max((256 + nb - 1) / nb, (K + 1023) / 1024);
  S = std::min(S, std::max(1, K / 256));
  while (S > 1 && (int64_t)S * 64 * N + (int64_t)nb * S * 64 * 2 > AVSR_SKINNY_WS) --S;
  kchunk = ((K + S - 1) / S + 15) / 16 * 16;
  return (K + kchunk - 1) / kchunk;
}

bool skinny_mma_ok(const DenseArgs& a) {
  return a.K % 16 == 0 && a.lda % 4 == 0 && a.ldb % 4 == 0;
}

template <typename T, typename OutT>
int skinny_launch(const DenseArgs& a, float* ws, hipStream_t st) {
  int kchunk = a.K;
  const bool mma = sizeof(T) == 4 && skinny_mma_ok(a);
  const int S = ws ? (mma ? skinny_mma_splits(a.N, a.K, kchunk) : skinny_splits(a.N, a.K, kchunk)) : 1;
  float* part = S > 1 ? ws : nullptr;
  unsigned* cnt = S > 1 ? (unsigned*)(ws + AVSR_SKINNY_WS) : nullptr;   // AVSR_SKINNY_CNT counters
  const int nb = (a.N + SK_NB - 1) / SK_NB;
  if (S > 1 && nb > AVSR_SKINNY_CNT) return AVSR_E_SHAPE;
  const dim3 g((unsigned)nb, (unsigned)S);
  const int unr = nb * S > 256 ? 4 : 8;
  if (a.kvk && !(sizeof(T) == 4 && mma && !a.e.bwd && !a.e.preact && a.e.drop_p == 0.f && a.e.beta == 0.f &&
                 !a.e.atomic))
    return AVSR_E_ARG;                   // the cache append is the matrix-core kernel's fast epilogue
  if (a.ln_c1) {                       // LayerNorm prologue: fp32, every chunk one load batch
    if (!(sizeof(T) == 4 && mma && kchunk <= SKM_WAVES * unr * 16 && !a.e.bwd && !a.e.preact &&
          a.e.drop_p == 0.f && a.e.beta == 0.f && !a.e.atomic))
      return AVSR_E_ARG;
    if constexpr (sizeof(T) == 4) {
      DenseArgs al = a;
      al.lnst = S > 1 ? ws + (int64_t)S * a.M * a.N : nullptr;   // chunk statistics after the partials
#define SKL_LN(T_) do { if (unr == 4) hipLaunchKernelGGL((skinny_mma_kernel<OutT, T_, 4, true>), g, dim3(64 * SKM_WAVES), 0, st, al, part, kchunk, cnt); \
                        else hipLaunchKernelGGL((skinny_mma_kernel<OutT, T_, 8, true>), g, dim3(64 * SKM_WAVES), 0, st, al, part, kchunk, cnt); } while (0)
      // one row-tile count for every M: the per-row statistics / shift / epilogue arithmetic of the
      // MT = 1..3 instantiations compiled to different roundings (a row's result then depended on
      // how many rows shared the launch: batched decode != per-utterance by 1e-5, and
      // test_skinny_layernorm_prologue_every_row_alone failed); MT = 4 for all is batch-invariant
      SKL_LN(4);
#undef SKL_LN
      AVSR_CHECK_LAUNCH();
      return 0;
    }
  }
  if constexpr (sizeof(T) == 4) {       // fp32: the matrix-core form (16-byte rows, 16-k groups)
    if (mma) {
#define SKM(T_) do { if (unr == 4) hipLaunchKernelGGL((skinny_mma_kernel<OutT, T_, 4>), g, dim3(64 * SKM_WAVES), 0, st, a, part, kchunk, cnt); \
                      else hipLaunchKernelGGL((skinny_mma_kernel<OutT, T_, 8>), g, dim3(64 * SKM_WAVES), 0, st, a, part, kchunk, cnt); } while (0)
      if (a.M <= 16) SKM(1);
      else if (a.M <= 32) SKM(2);
      else if (a.M <= 48) SKM(3);
      else SKM(4);
#undef SKM
      AVSR_CHECK_LAUNCH();
      return 0;
    }
  }
#define SKL(R) hipLaunchKernelGGL((skinny_kernel<T, OutT, R>), g, dim3(256), 0, st, a, part, kchunk, cnt)
  if (a.M <= 8) SKL(8);
  else if (a.M <= 16) SKL(16);
  else if (a.M <= 24) SKL(24);
  else if (a.M <= 32) SKL(32);
  else if (a.M <= 40) SKL(40);
  else if (a.M <= 48) SKL(48);
  else SKL(64);
#undef SKL
  AVSR_CHECK_LAUNCH();
  return 0;
}

using CfgDual = gemmg::GCfg<2, 2, 2, 2, 2>;       // per wave group of wgrad_dual_kernel (8 waves, 128 KiB)

// weight-gradient shape (dy^T x: both operands r-contiguous, fp32 C, plain epilogue, one batch):
// the in-block split-K kernel (AVSR_OPT_WGRAD_DUAL = 0 keeps the 4-wave core: A/B runs)
bool wgrad_dual_ok(const avsr_gemm_params* p, int splits, bool slab) {
  const bool off = avsr_opt(AVSR_OPT_WGRAD_DUAL) == 0;
  return !off && !p->a_kmajor && !p->b_kmajor && p->c_f32 && p->batch == 1 && (splits == 1 || slab) && !p->bias &&
         !p->act && !p->preact && !p->res && !p->gate && p->drop_p == 0.f && !p->epi_bwd && !p->db &&
         (p->ldc % 4) == 0 && avsr_aligned16(p->C);
}

template <class CF>
int launch_wgrad_dual(const DenseArgs& a, hipStream_t st) {
  const int tm = (a.M + CF::BM - 1) / CF::BM, tn = (a.N + CF::BN - 1) / CF::BN;
  const long nwg = (long)tm * tn * a.splits;
  if (nwg > 0x7fffffffL) return AVSR_E_SHAPE;
  if (a.cnt)
    hipLaunchKernelGGL((wgrad_dual_kernel<CF, true>), dim3((unsigned)nwg), dim3(2 * CF::NTH), 2 * CF::S * CF::STAGE,
                       st, a, tm, tn);
  else
    hipLaunchKernelGGL((wgrad_dual_kernel<CF, false>), dim3((unsigned)nwg), dim3(2 * CF::NTH), 2 * CF::S * CF::STAGE,
                       st, a, tm, tn);
  AVSR_CHECK_LAUNCH();
  return 0;
}

// forward linears with few rows
bool skinny_ok(const avsr_gemm_params* p, int splits) {
  const int esz = p->dtype == AVSR_BF16 ? 2 : 4;
  return p->M <= 64 && p->a_kmajor && p->b_kmajor && p->batch == 1 && splits == 1 && !p->epi_bwd && !p->db &&
         (p->K % 4) == 0 && (p->lda % 4) == 0 && (p->ldb % 4) == 0 && ((uintptr_t)p->A % (4 * esz)) == 0 &&
         ((uintptr_t)p->B % (4 * esz)) == 0;
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
  const bool slab = splits > 1 && p->ws != nullptr;
  if (slab && (p->bias || p->act || p->preact || p->res || p->gate || p->drop_p > 0.f || p->epi_bwd || (p->N % 4) ||
               (p->ldc % 4) || (p->strideC % 4) || !avsr_aligned16(p->C)))
    return AVSR_E_ARG;
  DenseArgs a;
  a.M = p->M; a.N = p->N; a.K = p->K;
  a.splits = splits;
  const bool glds = glds_ok(p);
  const int kq = glds ? gemmg::GBK : BKE;
  a.kchunk = ((p->K + splits - 1) / splits + kq - 1) / kq * kq;
  a.A = p->A; a.lda = p->lda; a.sA = p->strideA;
  {   // operand extents in bytes (last element touched + 1) for the buffer-DMA loaders
    const int esz = p->dtype == AVSR_BF16 ? 2 : 4;
    const int64_t ea = (p->a_kmajor ? ((int64_t)(p->M - 1) * p->lda + p->K) : ((int64_t)(p->K - 1) * p->lda + p->M)) * esz;
    const int64_t eb = (p->b_kmajor ? ((int64_t)(p->N - 1) * p->ldb + p->K) : ((int64_t)(p->K - 1) * p->ldb + p->N)) * esz;
    const int64_t lim = (int64_t)gemmg::OOB - (1 << 20);
    const bool ok = ea > 0 && eb > 0 && ea < lim && eb < lim;
    a.a_bytes = ok ? (uint32_t)ea : 0u;
    a.b_bytes = ok ? (uint32_t)eb : 0u;
  }
  a.B = p->B; a.ldb = p->ldb; a.sB = p->strideB;
  a.sC = p->strideC; a.sR = p->strideR;
  a.stamp = p->stamp;
  a.cnt = nullptr; a.fC = nullptr; a.fldc = 0; a.falpha = 1.f; a.fbeta = 0.f;
  a.ln_c1 = p->ln_c1; a.ln_eps = p->ln_eps; a.lnst = nullptr;
  a.kvk = (float*)p->kv_k; a.kvv = (float*)p->kv_v; a.kvpos = p->kv_pos; a.kvrows = p->kv_rows;
  if (p->kv_k && (p->dtype != AVSR_F32 || p->M > 64 || splits > 1 || (p->N % 3) || !p->kv_v || !p->kv_pos ||
                  p->kv_rows < p->M))
    return AVSR_E_ARG;
  if (p->kv_k && (glds || slab || !skinny_ok(p, splits))) return AVSR_E_ARG;
  if (p->ln_c1 && (p->dtype != AVSR_F32 || p->M > 64 || splits > 1)) return AVSR_E_ARG;
  Epi& e = a.e;
  e.M = p->M; e.N = p->N; e.C = p->C; e.ldc = p->ldc;
  e.alpha = p->alpha; e.beta = p->beta; e.bias = p->bias;
  e.act = p->act; e.bwd = p->epi_bwd; e.atomic = splits > 1 && !slab;
  a.sSplit = 0;
  if (slab) {   // partial tiles -> ws[b][split][M][N], reduced below
    e.C = p->ws; e.ldc = p->N; e.alpha = 1.f; e.beta = 0.f;
    a.sSplit = (int64_t)p->M * p->N + AVSR_GEMM_SLAB_PAD; a.sC = (int64_t)splits * a.sSplit;
  }
  e.preact = p->preact; e.res = p->res; e.ldr = p->ldr; e.gate = p->gate;
  e.drop_p = p->drop_p; e.seed = p->seed; e.drop_base = 0; e.stats = nullptr; e.stats_tiles = 0;
  e.rm_wc = 0; e.rm_hc = 0; e.rm_hin = 0; e.rm_win = 0; e.rm_a = 0; e.rm_b = 0;
  e.colsum = nullptr;
  int colsum_bm = 0;
  if (p->db) {   // fused bias gradient: the LDS-DMA bf16 path's vector epilogue, one K pass
    if (!glds || p->dtype != AVSR_BF16 || p->c_f32 || splits > 1 || p->batch != 1 || !p->db_ws || (p->N % 8) ||
        (p->ldc % 8) || (p->ldr % 8) || !avsr_aligned16(p->C) || (p->gate && !avsr_aligned16(p->gate)) ||
        (p->preact && !avsr_aligned16(p->preact)) || (p->res && (!avsr_aligned16(p->res) || (p->ldr % 8))) ||
        (p->bias && !avsr_aligned16(p->bias)))
      return AVSR_E_ARG;
    colsum_bm = cfg_bm(tile_cfg(p, splits), p->a_kmajor != 0);
    e.colsum = p->db_ws;
  }
  hipStream_t st = (hipStream_t)stream;
  if (p->K == 0) return AVSR_E_SHAPE;
  int rc;
  if (p->ln_c1 && (glds || slab || !skinny_ok(p, splits))) return AVSR_E_ARG;   // the prologue is the few-row kernel's
  if (!glds && !slab && skinny_ok(p, splits)) {
    float* sws = p->skinny_ws;          // optional K-split partials (AVSR_SKINNY_WS floats)
    if (p->dtype == AVSR_F32) return skinny_launch<float, float>(a, sws, st);
    return p->c_f32 ? skinny_launch<bf16, float>(a, sws, st) : skinny_launch<bf16, bf16>(a, sws, st);
  }
  if (glds && wgrad_dual_ok(p, splits, slab)) {
    const int tiles = ((p->M + CfgDual::BM - 1) / CfgDual::BM) * ((p->N + CfgDual::BN - 1) / CfgDual::BN);
    if (slab && p->slab_cnt && tiles <= AVSR_SLAB_CNT &&
        (int64_t)splits * a.sSplit * 4 < (1ll << 31)) {   // in-kernel slab reduction (no slab_reduce pass)
      a.cnt = p->slab_cnt;
      a.fC = (float*)p->C; a.fldc = p->ldc; a.falpha = p->alpha; a.fbeta = p->beta;
      return launch_wgrad_dual<CfgDual>(a, st);
    }
    rc = launch_wgrad_dual<CfgDual>(a, st);
  }
  else if (glds) rc = p->c_f32 ? glds_by_layout<float>(p, a, st) : glds_by_layout<bf16>(p, a, st);
  else if (p->dtype == AVSR_F32) rc = by_tile<float, float>(p, a, st);
  else if (p->c_f32) rc = by_tile<bf16, float>(p, a, st);
  else rc = by_tile<bf16, bf16>(p, a, st);
  if (rc) return rc;
  if (colsum_bm) {
    const int tiles = (p->M + colsum_bm - 1) / colsum_bm;
    rc = colsum_launch((const float*)p->db_ws, tiles, (int64_t)p->N, p->N, p->db, 0, nullptr, st);
    if (rc) return rc;
  }
  if (!slab) return 0;
  const int64_t per = (int64_t)p->M * (p->N / 4);
  if (per >= (1ll << 31)) return AVSR_E_SHAPE;
  const dim3 g((unsigned)avsr_grid(per, 256, 4096), p->batch);
  hipLaunchKernelGGL(slab_reduce_kernel, g, dim3(256), 0, st, (const float*)p->ws, splits, p->M, p->N,
                     (int64_t)p->M * p->N + AVSR_GEMM_SLAB_PAD, (float*)p->C, p->ldc, p->strideC, p->alpha, p->beta);
  AVSR_CHECK_LAUNCH();
  return 0;
}

// grouped weight-gradients: each problem must be the plain wgrad_dual shape (bf16 operands, both
// r-contiguous, fp32 C, no epilogue, no split); otherwise the problems run one by one
extern "C" int avsr_gemm_wgrad_group(const avsr_gemm_params* ps, int n, void* stream) {
  if (!ps || n < 1 || n > WG_MAX) return AVSR_E_ARG;
  bool grouped = true;
  for (int i = 0; i < n; ++i) {
    const avsr_gemm_params* p = ps + i;
    if (p->M <= 0 || p->N <= 0 || p->K <= 0 || p->batch != 1) return AVSR_E_SHAPE;
    grouped = grouped && glds_ok(p) && p->splitk <= 1 && !p->ws && !p->stamp && wgrad_dual_ok(p, 1, false) &&
              avsr_aligned16(p->A) && avsr_aligned16(p->B) && (p->lda % 8) == 0 && (p->ldb % 8) == 0;
  }
  if (!grouped) {
    for (int i = 0; i < n; ++i) {
      const int rc = avsr_gemm(ps + i, stream);
      if (rc) return rc;
    }
    return 0;
  }
  using CF = CfgDual;
  WgGroup g;
  std::memset(&g, 0, sizeof(g));
  int total = 0;
  for (int i = 0; i < n; ++i) {
    const avsr_gemm_params* p = ps + i;
    DenseArgs& a = g.a[i];
    a.M = p->M; a.N = p->N; a.K = p->K; a.splits = 1;
    a.kchunk = (p->K + gemmg::GBK - 1) / gemmg::GBK * gemmg::GBK;
    const int64_t ea = ((int64_t)(p->K - 1) * p->lda + p->M) * 2, eb = ((int64_t)(p->K - 1) * p->ldb + p->N) * 2;
    const int64_t lim = (int64_t)gemmg::OOB - (1 << 20);
    const bool ok = ea < lim && eb < lim;
    a.a_bytes = ok ? (uint32_t)ea : 0u;
    a.b_bytes = ok ? (uint32_t)eb : 0u;
    a.A = p->A; a.lda = p->lda; a.B = p->B; a.ldb = p->ldb;
    a.e.M = p->M; a.e.N = p->N; a.e.C = p->C; a.e.ldc = p->ldc; a.e.alpha = p->alpha; a.e.beta = p->beta;
    g.tm[i] = (p->M + CF::BM - 1) / CF::BM;
    g.tn[i] = (p->N + CF::BN - 1) / CF::BN;
    g.start[i] = total;
    total += g.tm[i] * g.tn[i];
  }
  for (int i = n; i <= WG_MAX; ++i) g.start[i] = total;
  hipLaunchKernelGGL(wgrad_group_kernel<CF>, dim3((unsigned)total), dim3(2 * CF::NTH), 2 * CF::S * CF::STAGE,
                     (hipStream_t)stream, g);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_gemm_skinny_splits(int dtype, int N, int K) {
  if (N <= 0 || K <= 0) return 1;
  int kchunk;
  if (dtype == AVSR_F32 && K % 16 == 0) return skinny_mma_splits(N, K, kchunk);
  return skinny_splits(N, K, kchunk);
}
