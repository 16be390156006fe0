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
// ds_read_b128). The epilogue writes the NHWC output through an LDS staging tile and the BN
// partial statistics (count, mean, M2) of the block (the general conv epilogue's format).
#include "common.h"

namespace {

constexpr int SC_R = 4;                    // output rows per block (44 = 11 bands)
constexpr int SC_BANDS = 44 / SC_R;
constexpr int SC_VW = 48;                  // virtual output width (columns 44..47 computed and dropped)
constexpr int SC_PX = SC_R * SC_VW;        // 192 pixels per block
constexpr int SC_ROWS = 2 * SC_R + 5;      // input rows per band
constexpr int SC_CW = 96;                  // elements per staged copy of an input row
constexpr int SC_IMG = 5 * SC_ROWS * 2 * SC_CW * 2;      // 24,960 B
constexpr int SC_K = 288, SC_WROW = SC_K + 8;            // weight row: 592 B (conflict-free)
constexpr int SC_WB = 64 * SC_WROW * 2;                  // 37,888 B
constexpr int SC_LDS = SC_IMG + SC_WB;                   // 62,848 B: two blocks per CU
constexpr int SC_SROW = 64 + 8;                          // staging row (bf16), 144 B
static_assert(SC_PX * SC_SROW * 2 + 2 * 64 * 3 * 4 <= SC_LDS, "epilogue staging exceeds LDS");

AVSR_DEV uint32_t pack_bf16(float a, float b) {
  union { bf16 h[2]; uint32_t u; } v;
  v.h[0] = (bf16)a; v.h[1] = (bf16)b;
  return v.u;
}

// XCD-aware block order (gemm_glds.h xcd_remap): consecutive bands / frames share input rows
AVSR_DEV int sc_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

__global__ __launch_bounds__(256, 2) void stem_conv_kernel(int B, int T, const float* __restrict__ video,
                                                           const bf16* __restrict__ wk, bf16* __restrict__ h,
                                                           float* __restrict__ stats, int tiles) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* img = smem;
  char* wl = smem + SC_IMG;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int blk = sc_remap(blockIdx.x, gridDim.x);
  const int n = blk / SC_BANDS, band = blk - n * SC_BANDS;
  const int b = n / T, t = n - b * T;
  const int oh0 = band * SC_R, ir0 = 2 * oh0 - 3;
  // weights -> LDS (16-B pieces of the [64][288] packed weight into 592-B rows) and the input
  // band -> LDS: every global load of the block is issued before any LDS write (a loop that
  // waits for each load in turn made this prologue latency-bound: 1.7 ms at C2)
  constexpr int WP = 64 * SC_K / 8 / 256;                  // 9 weight pieces per thread
  constexpr int ND = SC_CW / 2 + 1;                        // 49 pixel pairs per input row
  constexpr int NI = (5 * SC_ROWS * ND + 255) / 256;       // 13 pairs per thread
  uint4 wv[WP];
#pragma unroll
  for (int u = 0; u < WP; ++u) {
    const int i = tid + u * 256, co = i / (SC_K / 8), c = i - co * (SC_K / 8);
    wv[u] = *(const uint4*)(wk + co * SC_K + c * 8);
  }
  // pair k of staged row rr: D_k = (x[2k - 3], x[2k - 2]); copy A dword d = D_d (an even ow's
  // window starts at element 2ow), copy B dword d = D_(d+1) (an odd ow's starts at 2ow - 2);
  // frames / rows / columns outside the clip read as zero (the conv padding)
  float xa[NI], xb[NI];
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int i = tid + u * 256;
    const int rr = i / ND, k = i - rr * ND;
    const int r = rr % SC_ROWS, dt = rr / SC_ROWS;
    const int tt = t + dt - 2, ir = ir0 + r, c0 = 2 * k - 3;
    const bool rowok = i < 5 * SC_ROWS * ND && tt >= 0 && tt < T && ir >= 0 && ir < 88;
    const float* row = video + (((int64_t)b * T + (rowok ? tt : 0)) * 88 + (rowok ? ir : 0)) * 88;
    xa[u] = (rowok && c0 >= 0 && c0 < 88) ? row[c0] : 0.f;
    xb[u] = (rowok && c0 + 1 >= 0 && c0 + 1 < 88) ? row[c0 + 1] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < WP; ++u) {
    const int i = tid + u * 256, co = i / (SC_K / 8), c = i - co * (SC_K / 8);
    *(uint4*)(wl + co * SC_WROW * 2 + c * 16) = wv[u];
  }
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int i = tid + u * 256;
    if (i < 5 * SC_ROWS * ND) {
      const int rr = i / ND, k = i - rr * ND;
      const uint32_t dk = pack_bf16(xa[u], xb[u]);
      char* base = img + (rr * 2) * (SC_CW * 2);
      if (k < ND - 1) *(uint32_t*)(base + k * 4) = dk;                    // copy A
      if (k > 0) *(uint32_t*)(base + SC_CW * 2 + (k - 1) * 4) = dk;       // copy B
    }
  }
  __syncthreads();
  // wave tile: 96 pixels (wm) x 32 output channels (wn); 16x16x32 MFMA, K-step = 4 groups
  const int wm = wave >> 1, wn = wave & 1;
  int abase[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int v = wm * 96 + i * 16 + (lane & 15);
    const int ob = v / SC_VW, ow = min(v - ob * SC_VW, 43);
    const int cp = ow & 1, j0 = 2 * ow - 2 * cp;
    abase[i] = (2 * ob * 2 + cp) * (SC_CW * 2) + j0 * 2;    // row 2*ob of frame 0; + (dt*13 + kh) rows below
  }
  f32x4 acc[6][2];
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g0 = lane >> 4;
#pragma unroll 1
  for (int ks = 0; ks < SC_K / 32; ++ks) {
    const int g = 4 * ks + g0;                              // (dt, kh) group of this lane's 8 k
    const int dt = g < 35 ? g / 7 : 0, kh = g < 35 ? g - 7 * (g / 7) : 0;
    const int roff = (dt * SC_ROWS + kh) * 2 * (SC_CW * 2);
    bf16x8 a[6], bw[2];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const char* p = img + abase[i] + roff;
      union { uint2 u[2]; bf16x8 h; } x;
      x.u[0] = *(const uint2*)p;
      x.u[1] = *(const uint2*)(p + 8);
      a[i] = x.h;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int co = wn * 32 + j * 16 + (lane & 15);
      bw[j] = *(const bf16x8*)(wl + co * SC_WROW * 2 + (4 * ks + g0) * 16);
    }
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(a[i], bw[j], acc[i][j]);
  }
  __syncthreads();
  // ---- epilogue 1: BN partial statistics of the block's 176 valid pixels, per channel
  float* red = (float*)(smem + SC_PX * SC_SROW * 2);       // [2 (wm)][64][3]
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    float s = 0.f, c = 0.f;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int v = wm * 96 + i * 16 + 4 * (lane >> 4) + r;
        const bool ok = v % SC_VW < 44;
        s += ok ? acc[i][j][r] : 0.f;
        c += ok ? 1.f : 0.f;
      }
    s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
    c += __shfl_xor(c, 16, 64); c += __shfl_xor(c, 32, 64);
    const float mean = s / c;
    float m2 = 0.f;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int v = wm * 96 + i * 16 + 4 * (lane >> 4) + r;
        const float dd = acc[i][j][r] - mean;
        m2 += v % SC_VW < 44 ? dd * dd : 0.f;
      }
    m2 += __shfl_xor(m2, 16, 64); m2 += __shfl_xor(m2, 32, 64);
    if (lane < 16) {
      const int co = wn * 32 + j * 16 + lane;
      red[(wm * 64 + co) * 3 + 0] = c;
      red[(wm * 64 + co) * 3 + 1] = mean;
      red[(wm * 64 + co) * 3 + 2] = m2;
    }
  }
  // ---- epilogue 2: bf16 tile -> LDS staging [192 px][64 co]
  bf16* stg = (bf16*)smem;
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int v = wm * 96 + i * 16 + 4 * (lane >> 4) + r;
        stg[v * SC_SROW + wn * 32 + j * 16 + (lane & 15)] = (bf16)acc[i][j][r];
      }
  __syncthreads();
  if (stats != nullptr && tid < 64) {                      // Chan's merge of the two pixel halves
    const float n0 = red[tid * 3], m0 = red[tid * 3 + 1], q0 = red[(tid) * 3 + 2];
    const float n1 = red[(64 + tid) * 3], m1 = red[(64 + tid) * 3 + 1], q1 = red[(64 + tid) * 3 + 2];
    const float nn = n0 + n1, dd = m1 - m0;
    float* o = stats + ((int64_t)tid * tiles + blk) * 3;
    o[0] = nn;
    o[1] = m0 + dd * n1 / nn;
    o[2] = q0 + q1 + dd * dd * n0 * n1 / nn;
  }
  // ---- 16-byte stores of the 176 valid pixel rows (NHWC, 128 B each)
  bf16* out = h + ((int64_t)n * 44 * 44 + (int64_t)oh0 * 44) * 64;
  for (int i = tid; i < SC_R * 44 * 8; i += 256) {
    const int c = i & 7, pxi = i >> 3;                     // pixel (ob, ow) with ow < 44
    const int ob = pxi / 44, ow = pxi - ob * 44;
    const uint4 v = *(const uint4*)(stg + (ob * SC_VW + ow) * SC_SROW + c * 8);
    *(uint4*)(out + (int64_t)pxi * 64 + c * 8) = v;
  }
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

extern "C" int avsr_stem_conv_tiles(int nimg) { return nimg * SC_BANDS; }

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
  const int64_t nblk = (int64_t)B * T * SC_BANDS;
  if (nblk > 0x7fffffff) return AVSR_E_SHAPE;
  hipLaunchKernelGGL(stem_conv_kernel, dim3((unsigned)nblk), dim3(256), SC_LDS, (hipStream_t)stream, B, T, video,
                     (const bf16*)wk, (bf16*)h, stats, (int)nblk);
  AVSR_CHECK_LAUNCH();
  return 0;
}
