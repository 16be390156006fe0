// Train-time augmentation on device: time masking, noise / interferer mixing
// at a target SNR, RGB -> gray. Byte / HBM work: vector loads and stores, no MFMA.
// C-ABI and reference call sites in include/avsr_hip.h.
#include <algorithm>

#include "common.h"

namespace {

// zero the masked time steps: grid (vector blocks of one clip, clip); a thread owns 16-byte
// vectors (4-byte when the row length is not a multiple of 16) and tests its row against the
// clip's spans (a few dozen at most)
template <int VB>
__global__ __launch_bounds__(256) void time_mask_kernel(avsr_time_mask_params p) {
  const int b = blockIdx.y;
  const int64_t nv = (int64_t)p.L * p.row_bytes / VB;
  char* x = (char*)p.x + (int64_t)b * p.clip_stride_bytes;
  const int* sp = p.spans + (int64_t)b * p.nspan * 2;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nv; v += (int64_t)gridDim.x * 256) {
    const int64_t row = v * VB / p.row_bytes;
    bool hit = false;
    for (int s = 0; s < p.nspan; ++s) hit |= row >= sp[2 * s] && row < sp[2 * s + 1];
    if (hit) {
      if constexpr (VB == 16) *(uint4*)(x + v * 16) = make_uint4(0u, 0u, 0u, 0u);
      else *(uint32_t*)(x + v * 4) = 0u;
    }
  }
}

// per (chunk, clip): partial energies of signal and noise over the clip's first len samples
constexpr int NCH = 64;
__global__ __launch_bounds__(256) void noise_energy_kernel(avsr_add_noise_params p) {
  const int b = blockIdx.y, ch = blockIdx.x;
  const int len = p.lengths ? min(p.lengths[b], p.L) : p.L;
  const int per = (len + NCH - 1) / NCH, i0 = ch * per, i1 = min(len, i0 + per);
  const float* x = p.x + (int64_t)b * p.ldx;
  const float* n = p.noise + (int64_t)b * p.ldn;
  double es = 0.0, en = 0.0;
  for (int i = i0 + threadIdx.x; i < i1; i += 256) {
    const double a = x[i], c = n[i];
    es += a * a; en += c * c;
  }
  __shared__ double rs[256], rn[256];
  rs[threadIdx.x] = es; rn[threadIdx.x] = en;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) { rs[threadIdx.x] += rs[threadIdx.x + o]; rn[threadIdx.x] += rn[threadIdx.x + o]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) { p.ws[(b * NCH + ch) * 2] = rs[0]; p.ws[(b * NCH + ch) * 2 + 1] = rn[0]; }
}

// y = x + scale * noise over the clip's first len samples (beyond len: y = x)
__global__ __launch_bounds__(256) void noise_mix_kernel(avsr_add_noise_params p) {
  const int b = blockIdx.y;
  __shared__ float scale_s;
  if (threadIdx.x == 0) {
    double es = 0.0, en = 0.0;
    for (int c = 0; c < NCH; ++c) { es += p.ws[(b * NCH + c) * 2]; en += p.ws[(b * NCH + c) * 2 + 1]; }
    const double snr0 = 10.0 * (log10(es) - log10(en));
    scale_s = (float)pow(10.0, (snr0 - (double)p.snr_db[b]) / 20.0);
  }
  __syncthreads();
  const float sc = scale_s;
  const int len = p.lengths ? min(p.lengths[b], p.L) : p.L;
  const float* x = p.x + (int64_t)b * p.ldx;
  const float* n = p.noise + (int64_t)b * p.ldn;
  float* y = p.y + (int64_t)b * p.ldy;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < p.L; i += gridDim.x * 256) y[i] = i < len ? x[i] + sc * n[i] : x[i];
}

__global__ __launch_bounds__(256) void rgb_gray_kernel(const uint8_t* rgb, uint8_t* gray, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint32_t r = rgb[3 * i], g = rgb[3 * i + 1], bl = rgb[3 * i + 2];
    gray[i] = (uint8_t)((r * 4899u + g * 9617u + bl * 1868u + 8192u) >> 14);
  }
}

}  // namespace

extern "C" int avsr_time_mask(const avsr_time_mask_params* p, void* stream) {
  if (!p || !p->x || (p->nspan > 0 && !p->spans) || p->row_bytes <= 0) return AVSR_E_ARG;
  if (p->B == 0 || p->L == 0 || p->nspan == 0) return 0;
  if (p->B > 65535) return AVSR_E_SHAPE;
  const bool v16 = ((uintptr_t)p->x & 15) == 0 && p->row_bytes % 16 == 0 && p->clip_stride_bytes % 16 == 0;
  if (!v16 && (((uintptr_t)p->x & 3) || p->row_bytes % 4 || p->clip_stride_bytes % 4)) return AVSR_E_ALIGN;
  const int vb = v16 ? 16 : 4;
  const int64_t nv = (int64_t)p->L * p->row_bytes / vb;
  const dim3 g((unsigned)std::min<int64_t>((nv + 255) / 256, 1024), p->B);
  if (v16) hipLaunchKernelGGL(time_mask_kernel<16>, g, dim3(256), 0, (hipStream_t)stream, *p);
  else hipLaunchKernelGGL(time_mask_kernel<4>, g, dim3(256), 0, (hipStream_t)stream, *p);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_add_noise(const avsr_add_noise_params* p, void* stream) {
  if (!p || !p->x || !p->noise || !p->y || !p->snr_db || !p->ws) return AVSR_E_ARG;
  if (p->B == 0 || p->L == 0) return 0;
  if (p->B > 65535) return AVSR_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(noise_energy_kernel, dim3(NCH, p->B), dim3(256), 0, st, *p);
  hipLaunchKernelGGL(noise_mix_kernel, dim3((unsigned)std::min((p->L + 255) / 256, 256), p->B), dim3(256), 0, st, *p);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_rgb_to_gray(const uint8_t* rgb, uint8_t* gray, int64_t n, void* stream) {
  if (!rgb || !gray) return AVSR_E_ARG;
  if (n == 0) return 0;
  hipLaunchKernelGGL(rgb_gray_kernel, dim3(avsr_grid(n, 256, 4096)), dim3(256), 0, (hipStream_t)stream, rgb, gray, n);
  AVSR_CHECK_LAUNCH();
  return 0;
}
