// Lip-ROI stem convolution straight from the video (C-ABI avsr_stem_conv_fwd): the
// Conv3d(1 -> 64, kernel 5x7x7, stride 1x2x2, pad 2x3x3, no bias) of
// src/nets/backend/backbones/resnet.py:132 (ResEncoder.frontend3D), bf16 MFMA.
//
// The general path packs the 5 frames of every output frame into an 8-channel NHWC tensor
// (743 MB at C2) and runs a 7x7 implicit GEMM over it with K = 49 taps x 8 channels = 392, of
// which 3/8 multiply zero channels. Here K is ordered as 36 groups of 8 = (frame dt, row kh) x
// (column kw 0..6 + one zero weight) = 288 (K = 245 is the minimum; group 35 has zero weights),
// and each group is 8 CONSECUTIVE pixels of one input row: for output column ow the stride-2
// window starts at input column 2ow - 3. A block stages the 13 input rows x 5 frames its band of
// 4 output rows needs (fp32 video -> bf16) in two copies shifted by one pixel pair, so every
// window starts 8-byte aligned in one of them: an A fragment is two ds_read_b64 per lane, no
// gather, no packed tensor. The 64 x 288 weight sits in LDS with padded rows (conflict-free
// ds_read_b128). The epilogue writes the NHWC output and BN partial statistics (count, mean,
// M2) in the general conv epilogue's format.
#include "common.h"

namespace {

constexpr int SC_R = 4;                    // output rows per band (44 = 11 bands)
constexpr int SC_BANDS = 44 / SC_R;
constexpr int SC_VW = 48;                  // virtual output width (columns 44..47 computed and dropped)
constexpr int SC_ROWS = 2 * SC_R + 5;      // input rows per band
constexpr int SC_CW = 96;                  // elements per staged copy of an input row
constexpr int SC_ND = SC_CW / 2 + 1;       // pixel pairs staged per input row (49)
constexpr int SC_K = 288;
constexpr int SC_ROWB = 2 * SC_CW * 2;     // one staged input row, both copies (384 B)
constexpr int SC_SLOT = SC_ROWS * SC_ROWB; // one frame's band (4,992 B)
constexpr int SC_LDS = 5 * SC_SLOT + 64;   // ring of the 5 frames a step reads (24,960 B) + the dropped columns' overrun
constexpr int SC_BLOCKS_PER_CU = 2;

typedef int v2i32 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void sc_lds_t;

// B fragment i of a step: two 8-byte LDS reads at the lane's window base + the fragment's
// compile-time offset (fragment i = pixel row i / 3 of the wave, 16-column block i % 3), as
// inline asm: two ds_read_b64 (2 cycles each) with the offset in the instruction, which the
// compiler would otherwise pair into ds_read2_b64 (8 cycles). The compiler does not see these
// LDS reads, so the consumer waits with sc_lgkm_wait (which also pins the registers).
template <int I>
AVSR_DEV bf16x8 sc_frag(uint32_t a) {
  constexpr int off = 2 * (I / 3) * (2 * 2 * 96) + 64 * (I % 3);
  union { uint2 u[2]; bf16x8 h; } x;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(x.u[0]) : "v"(a), "i"(off));
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(x.u[1]) : "v"(a), "i"(off + 8));
  return x.h;
}
template <int N>
AVSR_DEV void sc_lgkm_wait(bf16x8 (&b)[6]) {
  asm volatile("s_waitcnt lgkmcnt(%6)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]) : "n"(N));
}

AVSR_DEV uint32_t pack_bf16(float a, float b) {
  union { bf16 h[2]; uint32_t u; } v;
  v.h[0] = (bf16)a; v.h[1] = (bf16)b;
  return v.u;
}

// Stage input frame tt of clip b (rows ir0 .. ir0 + 12 of the band) into ring slot tt mod 5:
// pair k of a row is D_k = (x[2k - 3], x[2k - 2]); copy A dword d = D_d (an even ow's window
// starts at element 2ow), copy B dword d = D_(d+1) (an odd ow's starts at 2ow - 2). Frames,
// rows and columns outside the clip come back as zeros from the buffer's range check (the
// conv padding). Split in two so the loads of the next frame fly during a step's MFMAs.
constexpr int SC_NT = 256;
constexpr int SC_NI = (SC_ROWS * SC_ND + SC_NT - 1) / SC_NT;
struct StageRegs { float xa[SC_NI], xb[SC_NI]; };

AVSR_DEV void stem_stage_load(StageRegs& g, __amdgpu_buffer_rsrc_t rs, int b, int T, int tt, int ir0, int tid) {
  constexpr uint32_t OOB = 0x80000000u;
  const bool fok = tt >= 0 && tt < T;
#pragma unroll
  for (int u = 0; u < SC_NI; ++u) {
    const int i = tid + u * SC_NT;
    const int r = i / SC_ND, k = i - r * SC_ND;
    const int ir = ir0 + r, c0 = 2 * k - 3;
    const bool rok = fok && i < SC_ROWS * SC_ND && ir >= 0 && ir < 88;
    const uint32_t row = (uint32_t)(((b * T + tt) * 88 + ir) * 88);
    const uint32_t oa = rok && c0 >= 0 && c0 < 88 ? (row + c0) * 4u : OOB;
    const uint32_t ob = rok && c0 + 1 >= 0 && c0 + 1 < 88 ? (row + c0 + 1) * 4u : OOB;
    g.xa[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, oa, 0, 0));
    g.xb[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, ob, 0, 0));
  }
}

AVSR_DEV void stem_stage_store(const StageRegs& g, char* ring, int tt, int tid) {
  char* slot = ring + ((tt + 10) % 5) * SC_SLOT;
#pragma unroll
  for (int u = 0; u < SC_NI; ++u) {
    const int i = tid + u * SC_NT;
    if (i < SC_ROWS * SC_ND) {
      const int r = i / SC_ND, k = i - r * SC_ND;
      const uint32_t dk = pack_bf16(g.xa[u], g.xb[u]);
      char* base = slot + r * SC_ROWB;
      if (k < SC_ND - 1) *(uint32_t*)(base + k * 4) = dk;                  // copy A
      if (k > 0) *(uint32_t*)(base + SC_CW * 2 + (k - 1) * 4) = dk;       // copy B
    }
  }
}

// Persistent blocks, one per (clip, band of 4 output rows, run of frames): consecutive frames
// of a band share 4 of their 5 input frames, so each step stages ONE new frame into a 5-slot
// ring (13 rows x 2 copies) instead of five. 4 waves: wave (wm, wn) = 96 pixels x 32 output
// channels. The MFMA computes C[co][px] (A = weights, held in registers for the whole run: the
// wave's 32 channels x 288 k; B = the input windows from the ring), so a lane's accumulator is
// 4 consecutive channels of one pixel -> 8-byte NHWC stores, no staging. BN statistics (count,
// mean, M2) per channel are merged over the block's whole run (Chan), one partial per block.
__global__ __launch_bounds__(256, SC_BLOCKS_PER_CU) void stem_conv_kernel(
    int B, int T, int chunks, int fpc, const float* __restrict__ video, uint32_t vbytes, const bf16* __restrict__ wk,
    bf16* __restrict__ h, float* __restrict__ stats, int tiles) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float red[2][64][3];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int blk = blockIdx.x;
  const int stream = blk / chunks, chunk = blk - stream * chunks;
  const int b = stream / SC_BANDS, band = stream - b * SC_BANDS;
  const int t0 = chunk * fpc, t1 = min(T, t0 + fpc);
  const int oh0 = band * SC_R, ir0 = 2 * oh0 - 3;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(video), (short)0,
                                                                        (int)vbytes, 0x00020000);
  // this wave's weights: rows co = 32wn + 16j + (lane & 15), k-chunk (lane >> 4) of each step
  bf16x8 wr[SC_K / 32][2];
#pragma unroll
  for (int ks = 0; ks < SC_K / 32; ++ks)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      wr[ks][j] = *(const bf16x8*)(wk + (wn * 32 + j * 16 + (lane & 15)) * SC_K + ks * 32 + (lane >> 4) * 8);
  // this lane's pixel (B column) in each of the wave's 6 pixel fragments: fragment i is pixel
  // (ob, ow) = (2wm + i/3, 16(i%3) + l), l = lane & 15 (3 fragments = one 48-wide row), so its
  // LDS window is the lane's base pbase0 plus a compile-time offset (LDS instruction offset
  // field, no per-fragment address VALU). Columns 44..47 (fragments 2 and 5, l >= 12) are
  // computed from whatever follows the row in LDS (in range; out of the allocation reads as 0)
  // and dropped.
  const int l16 = lane & 15;
  const int pbase0 = 4 * wm * SC_ROWB + (l16 & 1) * (SC_CW * 2) + 4 * l16 - 4 * (l16 & 1);
  const bool tail_ok = l16 < 12;                         // fragments 2 and 5: ow = 32 + l < 44
  const uint32_t sbase = (uint32_t)(uintptr_t)(sc_lds_t*)smem;
  bool pvalid[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) pvalid[i] = i % 3 != 2 || tail_ok;
  float shift[8], s1[8], s2[8], cnt = 0.f;               // this lane's 8 channels: shifted sums
  float pv_count = 0.f;
#pragma unroll
  for (int i = 0; i < 6; ++i) pv_count += pvalid[i] ? 1.f : 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) shift[q] = s1[q] = s2[q] = 0.f;
  // the ring's first 5 frames: every load issued before the first store (one latency)
  if (t0 < t1) {
    StageRegs p[5];
#pragma unroll
    for (int f = 0; f < 5; ++f) stem_stage_load(p[f], rs, b, T, t0 - 2 + f, ir0, tid);
#pragma unroll
    for (int f = 0; f < 5; ++f) stem_stage_store(p[f], smem, t0 - 2 + f, tid);
  }
  // frames t + 3 and t + 4 stay in flight in registers (two sets, alternating): a frame's loads
  // are issued two steps before it is stored into the ring. Loads past the clip return zeros
  // (range check) and are issued unconditionally, and the output goes out through buffer
  // stores with out-of-range offsets for the dropped columns, so the step has no divergent
  // memory operations and the ring store waits only for its own frame's loads
  StageRegs sa, sb;
  stem_stage_load(sb, rs, b, T, t0 + 3, ir0, tid);
  __syncthreads();
  const int g0 = lane >> 4;
  int ooff[6][2];                                         // byte offsets in the band (OOB: dropped)
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int v = wm * 96 + i * 16 + (lane & 15);
    const int ob = v / SC_VW, ow = v - ob * SC_VW;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      ooff[i][j] = pvalid[i] ? ((ob * 44 + ow) * 64 + wn * 32 + j * 16 + 4 * g0) * 2 : (int)0x80000000u;
  }
  auto step = [&](int t, StageRegs& ld, const StageRegs& st) {
    stem_stage_load(ld, rs, b, T, t + 4, ir0, tid);       // frame t + 4: stored at the end of step t + 1
    f32x4 acc[6][2];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // B fragments of K-step ks (the lane's 8 k = group 4ks + g0 of its pixel), double-buffered:
    // step ks + 1's reads are issued before step ks's MFMAs
    // k group g = 4ks + g0 -> (frame dt, row kh) = divmod(g, 7), from compile-time 4ks / 7 and
    // 4ks % 7 (group 35 has zero weights: its window is any in-range row)
    const int t5 = (t + 8) % 5;
    auto rdB = [&](int ks, bf16x8 (&xb)[6]) {
      const int q7 = (4 * ks) / 7, r7 = (4 * ks) % 7;
      const int c = g0 >= 7 - r7 ? 1 : 0;
      const int dt = q7 + c, kh = r7 + g0 - 7 * c;
      int slot = t5 + dt;
      slot = slot >= 5 ? slot - 5 : slot;
      slot = slot >= 5 ? slot - 5 : slot;
      const uint32_t a = sbase + (uint32_t)(pbase0 + slot * SC_SLOT + kh * SC_ROWB);
      xb[0] = sc_frag<0>(a); xb[1] = sc_frag<1>(a); xb[2] = sc_frag<2>(a);
      xb[3] = sc_frag<3>(a); xb[4] = sc_frag<4>(a); xb[5] = sc_frag<5>(a);
    };
    bf16x8 bb[2][6];                                      // ping-pong by k-step parity (no register copies)
    rdB(0, bb[0]);
#pragma unroll
    for (int ks = 0; ks < SC_K / 32; ++ks) {
      if (ks + 1 < SC_K / 32) {
        rdB(ks + 1, bb[(ks + 1) & 1]);
        sc_lgkm_wait<12>(bb[ks & 1]);                      // step ks's reads are done, step ks + 1's fly
      } else {
        sc_lgkm_wait<0>(bb[ks & 1]);
      }
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(wr[ks][j], bb[ks & 1][i], acc[i][j]);
    }
    // output: lane holds channels co0 .. co0+3 of pixel (ob, ow) in tile (i, j)
    const int n = b * T + t;
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        h + ((int64_t)n * 44 * 44 + (int64_t)oh0 * 44) * 64, (short)0, SC_R * 44 * 64 * 2, 0x00020000);
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        union { bf16x4 v4; v2i32 u; } o;
        o.v4 = bf16x4{(bf16)acc[i][j][0], (bf16)acc[i][j][1], (bf16)acc[i][j][2], (bf16)acc[i][j][3]};
        __builtin_amdgcn_raw_buffer_store_b64(o.u, ro, (uint32_t)ooff[i][j], 0, 0);
      }
    if (stats != nullptr) {   // per-lane shifted sums of the lane's 8 channels (no cross-lane work per step)
      if (t == t0) {
#pragma unroll
        for (int q = 0; q < 8; ++q) shift[q] = acc[0][q >> 2][q & 3];   // pixel fragment 0 is always valid
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const float d = acc[i][q >> 2][q & 3] - shift[q];
          const float x = i % 3 != 2 ? d : (tail_ok ? d : 0.f);
          s1[q] += x;
          s2[q] = fmaf(x, x, s2[q]);
        }
      cnt += pv_count;
    }
    __syncthreads();                                      // every wave is done with frame t - 2's slot
    if (t + 1 < t1) {
      stem_stage_store(st, smem, t + 3, tid);
      __syncthreads();
    }
  };
  for (int t = t0; t < t1; t += 2) {
    step(t, sa, sb);
    if (t + 1 < t1) step(t + 1, sb, sa);
  }
  if (stats != nullptr) {
    // per lane (count, mean, M2) from the shifted sums, Chan-merged over the 16 pixel lanes of
    // the lane group (fixed butterfly: every lane ends with the same bits), then over the two
    // pixel halves (wm) in LDS: the block's partial per channel
    float rn[8], rmean[8], rm2[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      rn[q] = cnt;
      rmean[q] = cnt > 0.f ? shift[q] + s1[q] / cnt : 0.f;
      rm2[q] = cnt > 0.f ? fmaxf(s2[q] - s1[q] * s1[q] / cnt, 0.f) : 0.f;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const float nb = __shfl_xor(rn[q], o, 64), mb = __shfl_xor(rmean[q], o, 64), qb = __shfl_xor(rm2[q], o, 64);
        // symmetric merge (a, b) -> same bits on both lanes: order the pair by lane bit
        const bool lo = (lane & o) == 0;
        const float na = lo ? rn[q] : nb, ma = lo ? rmean[q] : mb, qa = lo ? rm2[q] : qb;
        const float nc = lo ? nb : rn[q], mc = lo ? mb : rmean[q], qc = lo ? qb : rm2[q];
        const float nn = na + nc;
        if (nn > 0.f) {
          const float d = mc - ma;
          rmean[q] = ma + d * nc / nn;
          rm2[q] = qa + qc + d * d * na * nc / nn;
        }
        rn[q] = nn;
      }
    }
    if ((lane & 15) == 0) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int co = wn * 32 + (q >> 2) * 16 + 4 * g0 + (q & 3);
        red[wm][co][0] = rn[q]; red[wm][co][1] = rmean[q]; red[wm][co][2] = rm2[q];
      }
    }
    __syncthreads();
    if (tid < 64) {
      const float n0 = red[0][tid][0], m0 = red[0][tid][1], q0 = red[0][tid][2];
      const float n1 = red[1][tid][0], m1 = red[1][tid][1], q1 = red[1][tid][2];
      const float nn = n0 + n1;
      float* o = stats + ((int64_t)tid * tiles + blk) * 3;
      if (nn > 0.f) {
        const float dd = m1 - m0;
        o[0] = nn; o[1] = m0 + dd * n1 / nn; o[2] = q0 + q1 + dd * dd * n0 * n1 / nn;
      } else {
        o[0] = 0.f; o[1] = 0.f; o[2] = 0.f;
      }
    }
  }
}

static void stem_grid(int B, int T, int& chunks, int& fpc, int& nblk) {
  const int streams = B * SC_BANDS;
  const long target = 8L * 256 * SC_BLOCKS_PER_CU;
  chunks = (int)((target + streams - 1) / streams);
  const int maxc = T / 16 > 0 ? T / 16 : 1;
  if (chunks > maxc) chunks = maxc;
  if (chunks < 1) chunks = 1;
  fpc = (T + chunks - 1) / chunks;
  chunks = (T + fpc - 1) / fpc;
  nblk = streams * chunks;
}

// Conv3d weight (64, 1, 5, 7, 7) fp32 -> [64][36 groups][8] bf16, group = dt*7 + kh, entry kw
// (kw = 7 and group 35 are zeros)
__global__ void stem_wpack2_kernel(const float* w, bf16* wk) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= 64 * SC_K) return;
  const int co = i / SC_K, k = i - co * SC_K, g = k >> 3, kw = k & 7;
  const bool ok = g < 35 && kw < 7;
  wk[i] = (bf16)(ok ? w[co * 245 + g * 7 + kw] : 0.f);
}

}  // namespace

extern "C" int avsr_stem_conv_tiles(int B, int T) {
  int chunks, fpc, nblk;
  stem_grid(B, T, chunks, fpc, nblk);
  return nblk;
}

extern "C" int avsr_stem_wpack2(const float* w, void* wk, void* stream) {
  if (!w || !wk || !avsr_aligned16(wk)) return AVSR_E_ARG;
  hipLaunchKernelGGL(stem_wpack2_kernel, dim3((64 * SC_K + 255) / 256), dim3(256), 0, (hipStream_t)stream, w,
                     (bf16*)wk);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_stem_conv_fwd(int B, int T, const float* video, const void* wk, void* h, float* stats,
                                  void* stream) {
  if (B <= 0 || T <= 0) return B == 0 || T == 0 ? 0 : AVSR_E_SHAPE;
  if (!video || !wk || !h) return AVSR_E_ARG;
  if (!avsr_aligned16(wk) || !avsr_aligned16(h) || !avsr_aligned16(video)) return AVSR_E_ALIGN;
  const int64_t vbytes = (int64_t)B * T * 88 * 88 * 4;
  if (vbytes >= 0x7fffffffLL) return AVSR_E_SHAPE;
  int chunks, fpc, nblk;
  stem_grid(B, T, chunks, fpc, nblk);
  hipLaunchKernelGGL(stem_conv_kernel, dim3((unsigned)nblk), dim3(256), SC_LDS, (hipStream_t)stream, B, T, chunks, fpc,
                     video, (uint32_t)vbytes, (const bf16*)wk, (bf16*)h, stats, nblk);
  AVSR_CHECK_LAUNCH();
  return 0;
}
