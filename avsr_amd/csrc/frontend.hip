// Input front end on device: log mel filterbank + 4-frame stacking + per-row
// LayerNorm of the audio stream, and crop/normalise of the uint8 lip frames.
//
// fbank_stack_kernel: one 256-thread block per (clip, output row) = 4 consecutive 25 ms frames.
// The 4 x 400 preemphasised samples are staged in LDS with a 512-entry twiddle table; each
// thread forms power-spectrum bins of the 4 frames as direct 400-term DFTs (4 x 257 bins =
// 1028 dot products, ~0.8 MFLOP per row -- the whole C2 batch is ~5 GFLOP of fp32 VALU, far
// below any roofline that matters next to the encoder), then 4 x 26 threads apply the
// triangular mel filters (sparse: bins[j]..bins[j+2]), take the log, and one wave normalises
// the 104 features of the row (two-pass mean / variance in fp32).
#include "common.h"

namespace {

constexpr int FLEN = 400, FSTEP = 160, NFFT = 512, NBIN = NFFT / 2 + 1, NFILT = 26, STK = 4;
constexpr int NF = STK * NFILT;   // 104 features per row

__global__ __launch_bounds__(256) void fbank_stack_kernel(avsr_fbank_params p) {
  __shared__ float sig[STK][FLEN];
  __shared__ float cs[NFFT], sn[NFFT];
  __shared__ float pw[STK][NBIN + 3];
  __shared__ float feat[NF];
  const int b = blockIdx.y, r = blockIdx.x, tid = threadIdx.x;
  const int64_t n = p.n_samples[b];
  const int nfr = n <= FLEN ? 1 : 1 + (int)((n - FLEN + FSTEP - 1) / FSTEP);
  const int rows = (nfr + STK - 1) / STK;
  float* out = p.out + (int64_t)b * NF * p.T + r;
  if (r >= rows) {                                   // collate_pad rows
    for (int c = tid; c < NF; c += 256) out[(int64_t)c * p.T] = 0.f;
    return;
  }
  const float* w = p.wav + (int64_t)b * p.ldw;
  for (int i = tid; i < NFFT; i += 256) {
    float s, c;
    sincospif((float)i / (NFFT / 2), &s, &c);        // angle 2*pi*i/512
    cs[i] = c; sn[i] = s;
  }
  for (int e = tid; e < STK * FLEN; e += 256) {
    const int f = e / FLEN, i = e - f * FLEN;
    const int64_t s = (int64_t)(r * STK + f) * FSTEP + i;
    float v = 0.f;
    if (s < n) v = s == 0 ? w[0] : w[s] - p.preemph * w[s - 1];
    sig[f][i] = v;
  }
  __syncthreads();
  for (int e = tid; e < STK * NBIN; e += 256) {
    const int f = e / NBIN, k = e - f * NBIN;
    float re = 0.f, im = 0.f;
    int ph = 0;
    for (int i = 0; i < FLEN; ++i) {
      const float v = sig[f][i];
      re += v * cs[ph];
      im += v * sn[ph];
      ph = (ph + k) & (NFFT - 1);
    }
    pw[f][k] = (re * re + im * im) * (1.f / NFFT);
  }
  __syncthreads();
  if (tid < NF) {
    const int f = tid / NFILT, j = tid - f * NFILT;
    float v = 0.f;
    if (r * STK + f < nfr) {
      const int b0 = p.bins[j], b1 = p.bins[j + 1], b2 = p.bins[j + 2];
      float acc = 0.f;
      for (int i = b0; i < b1; ++i) acc += pw[f][i] * ((float)(i - b0) / (float)(b1 - b0));
      for (int i = b1; i < b2; ++i) acc += pw[f][i] * ((float)(b2 - i) / (float)(b2 - b1));
      v = logf(acc == 0.f ? 2.220446049250313e-16f : acc);
    }                                                // stacker's zero rows stay 0 (post-log)
    feat[tid] = v;
  }
  __syncthreads();
  if (tid < 64) {
    const float a0 = feat[tid], a1 = tid + 64 < NF ? feat[tid + 64] : 0.f;
    const float mu = wave_sum(a0 + a1) * (1.f / NF);
    const float d0 = a0 - mu, d1 = tid + 64 < NF ? a1 - mu : 0.f;
    const float var = wave_sum(d0 * d0 + d1 * d1) * (1.f / NF);
    const float rs = rsqrtf(var + p.ln_eps);
    out[(int64_t)tid * p.T] = d0 * rs;
    if (tid + 64 < NF) out[(int64_t)(tid + 64) * p.T] = d1 * rs;
  }
}

// 4 output pixels per thread; rows of the crop are contiguous in the output
__global__ __launch_bounds__(256) void video_norm_kernel(avsr_video_norm_params p, int64_t total4) {
  const int q = p.crop / 4;
  const float sc = 1.f / (255.f * p.std), sh = p.mean / p.std;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total4; i += (int64_t)gridDim.x * 256) {
    const int64_t row = i / q;                       // (b, t, y)
    const int x4 = (int)(i - row * q) * 4;
    const int y = (int)(row % p.crop);
    const int64_t bt = row / p.crop;
    const uint8_t* src = p.frames + (bt * p.H + p.oy + y) * p.W + p.ox + x4;
    f32x4 v;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = (float)src[k] * sc - sh;
    *(f32x4*)(p.out + i * 4) = v;
  }
}

}  // namespace

extern "C" int avsr_fbank_stack(const avsr_fbank_params* p, void* stream) {
  if (!p || !p->wav || !p->n_samples || !p->out) return AVSR_E_ARG;
  if (p->B < 0 || p->T < 0 || p->ldw < 1) return AVSR_E_SHAPE;
  if (p->B == 0 || p->T == 0) return 0;
  for (int j = 0; j < NFILT + 1; ++j)
    if (p->bins[j] < 0 || p->bins[j + 1] < p->bins[j] || p->bins[j + 1] > NBIN) return AVSR_E_ARG;
  if (p->B > 65535) return AVSR_E_SHAPE;
  hipLaunchKernelGGL(fbank_stack_kernel, dim3((unsigned)p->T, (unsigned)p->B), dim3(256), 0, (hipStream_t)stream, *p);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_video_normalize(const avsr_video_norm_params* p, void* stream) {
  if (!p || !p->frames || !p->out) return AVSR_E_ARG;
  if (p->B < 0 || p->T < 0 || p->crop <= 0 || (p->crop % 4) || p->oy < 0 || p->ox < 0 || p->oy + p->crop > p->H ||
      p->ox + p->crop > p->W)
    return AVSR_E_SHAPE;
  if (!avsr_aligned16(p->out)) return AVSR_E_ALIGN;
  if (p->std == 0.f) return AVSR_E_ARG;
  const int64_t total4 = (int64_t)p->B * p->T * p->crop * (p->crop / 4);
  if (total4 == 0) return 0;
  hipLaunchKernelGGL(video_norm_kernel, dim3((unsigned)avsr_grid(total4, 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, *p, total4);
  AVSR_CHECK_LAUNCH();
  return 0;
}
