// Loss kernels of the joint CTC / attention objective (include/avsr_hip.h):
// row log-sum-exp, label-smoothing KL (+argmax accuracy), CTC alpha/beta/occupancy and
// the logits gradients, plus the on-device loss combination. One 256-thread block per row
// for the V = 5049 row reductions; one block per utterance for the CTC recursions (the
// T-loop is sequential, states are spread over the block's threads, one barrier per step).
#include "common.h"

namespace {

constexpr float NEG = -1e30f;

AVSR_DEV float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  return m <= NEG ? NEG : m + logf(expf(a - m) + expf(b - m));
}
AVSR_DEV float lse3(float a, float b, float c) {
  const float m = fmaxf(a, fmaxf(b, c));
  return m <= NEG ? NEG : m + logf(expf(a - m) + expf(b - m) + expf(c - m));
}

// CTC recursion step: hardware exp2 / log2 (v_exp_f32 / v_log_f32, ~1 ulp) instead of the
// libm sequences on the recursion's dependent chain (measured 408 -> 352 us per C2 batch);
// the max term contributes exp(0) = 1 exactly
AVSR_DEV float lse3_fast(float a, float b, float c) {
  const float m = fmaxf(a, fmaxf(b, c));
  return m <= NEG ? NEG : m + __logf(__expf(a - m) + __expf(b - m) + __expf(c - m));
}

// block-wide reductions (256 threads)
AVSR_DEV float block_max(float v, float* sh) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  v = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
  __syncthreads();
  return v;
}
AVSR_DEV float block_sum(float v, float* sh) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  v = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  return v;
}

// per-row statistics: max, sum exp (relative to max), sum x, argmax (first index)
template <typename T>
AVSR_DEV void row_stats(const T* x, int V, float* sh, float& mx, float& se, float& sx, int& amax) {
  constexpr int VE = VecW<T>::VE;
  float m = NEG, s = 0.f, t = 0.f, bv = NEG;
  int bi = 0x7fffffff;
  for (int c0 = threadIdx.x * VE; c0 < V; c0 += 256 * VE) {
    float v[VE];
    ldv(x + c0, v);
#pragma unroll
    for (int j = 0; j < VE; ++j) {
      if (c0 + j < V) {
        const float xv = v[j];
        if (xv > m) { s = s * expf(m - xv) + 1.f; m = xv; }
        else s += expf(xv - m);
        t += xv;
        if (xv > bv) { bv = xv; bi = c0 + j; }
      }
    }
  }
  mx = block_max(m, sh);
  se = block_sum(s * expf(m - mx), sh);
  sx = block_sum(t, sh);
  // argmax: max value, smallest index among ties
  const float gv = mx;
  int cand = bv == gv ? bi : 0x7fffffff;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o, 64));
  __shared__ int shi[4];
  if ((threadIdx.x & 63) == 0) shi[threadIdx.x >> 6] = cand;
  __syncthreads();
  amax = min(min(shi[0], shi[1]), min(shi[2], shi[3]));
  __syncthreads();
}

template <typename T, int MODE>  // MODE 0: lse only; 1: label smoothing fwd
__global__ __launch_bounds__(256) void xent_fwd_kernel(avsr_xent_params p) {
  __shared__ float sh[4];
  const int row = blockIdx.x;
  const T* x = (const T*)p.x + (int64_t)row * p.ldx;
  float mx, se, sx;
  int am;
  row_stats<T>(x, p.V, sh, mx, se, sx, am);
  const float lse = mx + logf(se);
  if (threadIdx.x == 0) {
    p.lse[row] = lse;
    if (MODE == 1) {
      const int tg = p.target[row];
      if (tg < 0) {
        p.row_loss[row] = 0.f;
        if (p.row_correct) p.row_correct[row] = -1;
      } else {
        const float V = (float)p.V, sm = p.smoothing;
        const float e = sm / (V - 1.f), conf = 1.f - sm;
        const float xt = to_f(x[tg]);
        const float cst = (e > 0.f ? (V - 1.f) * e * logf(e) : 0.f) + (conf > 0.f ? conf * logf(conf) : 0.f);
        p.row_loss[row] = cst + lse - (e * (sx - xt) + conf * xt);
        if (p.row_correct) p.row_correct[row] = am == tg ? 1 : 0;
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void lsm_bwd_kernel(avsr_xent_params p) {
  constexpr int VE = VecW<T>::VE;
  const int row = blockIdx.x;
  const T* x = (const T*)p.x + (int64_t)row * p.ldx;
  T* dx = (T*)p.dx + (int64_t)row * p.lddx;
  const int tg = p.target[row];
  const float scale = tg < 0 ? 0.f : (*p.dloss) * p.coef;
  const float lse = p.lse[row];
  const float e = p.smoothing / (float)(p.V - 1), conf = 1.f - p.smoothing;
  for (int c0 = threadIdx.x * VE; c0 < p.lddx; c0 += 256 * VE) {
    float v[VE], o[VE];
    if (c0 < p.V) ldv(x + c0, v);
#pragma unroll
    for (int j = 0; j < VE; ++j) {
      const int c = c0 + j;
      o[j] = c < p.V ? scale * (expf(v[j] - lse) - (c == tg ? conf : e)) : 0.f;
    }
    stv(dx + c0, o);
  }
}

// ------------------------------------------------------------------------------- CTC
AVSR_DEV int ext_label(const int* lab, int s) { return (s & 1) ? lab[s >> 1] : 0; }

// One block per utterance; the recursions are sequential in t, so every global access is
// taken off the per-step critical path: extended labels / skip flags live in LDS, and the
// emissions lp(t, s) = x[t][l'(s)] - lse[t] (and, for the beta pass, alpha) are gathered
// cooperatively into LDS in chunks of CH time steps -- one exposed memory latency per chunk
// instead of one per step.
constexpr int CTC_CHUNK = 6144;   // floats per LDS chunk buffer

template <typename T>
__global__ __launch_bounds__(256) void ctc_fwd_kernel(avsr_ctc_params p) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const int L = p.label_len[b], Tb = min(p.in_len[b], p.T), S = 2 * L + 1;
  const int SS = 2 * p.Lmax + 1;
  const int* lab = p.labels + (int64_t)b * p.Lmax;
  const T* X = (const T*)p.x + (int64_t)b * p.T * p.ldx;
  const float* LSE = p.lse + (int64_t)b * p.T;
  float* A = p.alpha + (int64_t)b * p.T * SS;
  float* G = p.gamma + (int64_t)b * p.T * SS;
  __shared__ float buf[2][1024];
  __shared__ float E[CTC_CHUNK], AC[CTC_CHUNK];
  __shared__ int kl[1024];
  __shared__ unsigned char sk[1024];
  __shared__ float logp_s;
  if (S > 1024 || Tb <= 0) {   // unsupported label length or empty input: zero_infinity semantics
    for (int i = tid; i < p.T * SS; i += 256) G[i] = 0.f;
    if (tid == 0) p.nll[b] = 0.f;
    return;
  }
  const int CH = max(1, min(64, CTC_CHUNK / S));
  for (int s = tid; s < S; s += 256) kl[s] = ext_label(lab, s);
  __syncthreads();
  for (int s = tid; s < S; s += 256) sk[s] = s >= 2 && (s & 1) && kl[s] != kl[s - 2];
  // E[(t - t0) * S + s] = lp(t, s) for t in [t0, t0 + n); optionally AC = alpha of the same range
  auto load = [&](int t0, int n, bool with_alpha) {
    for (int i = tid; i < n * S; i += 256) {
      const int dt = i / S, s = i - dt * S, t = t0 + dt;
      E[i] = to_f(X[(int64_t)t * p.ldx + kl[s]]) - LSE[t];
      if (with_alpha) AC[i] = A[(int64_t)t * SS + s];
    }
  };
  __syncthreads();
  // alpha
  int t0 = 0;
  load(0, min(CH, Tb), false);
  __syncthreads();
  for (int s = tid; s < S; s += 256) {
    const float a0 = s < 2 ? E[s] : NEG;
    buf[0][s] = a0;
    A[s] = a0;
  }
  __syncthreads();
  for (int t = 1; t < Tb; ++t) {
    if (t - t0 >= CH) {
      t0 = t;
      load(t0, min(CH, Tb - t0), false);
      __syncthreads();
    }
    const float* prev = buf[(t - 1) & 1];
    float* cur = buf[t & 1];
    const float* e = E + (t - t0) * S;
    for (int s = tid; s < S; s += 256) {
      const float a1 = s >= 1 ? prev[s - 1] : NEG;
      const float a2 = sk[s] ? prev[s - 2] : NEG;
      const float v = lse3_fast(prev[s], a1, a2);
      const float r = v <= NEG ? NEG : v + e[s];
      cur[s] = r;
      A[(int64_t)t * SS + s] = r;
    }
    __syncthreads();
  }
  if (tid == 0) {
    const float* last = buf[(Tb - 1) & 1];
    logp_s = S > 1 ? lse2(last[S - 1], last[S - 2]) : last[S - 1];
  }
  __syncthreads();
  const float logp = logp_s;
  const bool feasible = logp > NEG * 0.5f;
  if (tid == 0) p.nll[b] = feasible ? -logp : 0.f;
  // beta (reuse buf), occupancy gamma_t(s) = exp(alpha + beta - lp - logP)
  for (int i = tid; i < p.T * SS; i += 256) {
    const int t = i / SS;
    if (t >= Tb || !feasible || (i % SS) >= S) G[i] = 0.f;
  }
  if (!feasible) return;
  __syncthreads();                       // alpha in global memory visible to the whole block
  t0 = max(0, Tb - CH);
  load(t0, Tb - t0, true);
  __syncthreads();
  for (int s = tid; s < S; s += 256) {
    const int i = (Tb - 1 - t0) * S + s;
    const float l = E[i];
    const float b0 = s >= S - 2 ? l : NEG;
    buf[(Tb - 1) & 1][s] = b0;
    const float a = AC[i];
    G[(int64_t)(Tb - 1) * SS + s] = (a <= NEG || b0 <= NEG) ? 0.f : expf(a + b0 - l - logp);
  }
  __syncthreads();
  for (int t = Tb - 2; t >= 0; --t) {
    if (t < t0) {
      t0 = max(0, t - CH + 1);
      load(t0, t + 1 - t0, true);
      __syncthreads();
    }
    const float* nxt = buf[(t + 1) & 1];
    float* cur = buf[t & 1];
    const int base = (t - t0) * S;
    for (int s = tid; s < S; s += 256) {
      const float b1 = s + 1 < S ? nxt[s + 1] : NEG;
      const float b2 = (s + 2 < S && sk[s + 2]) ? nxt[s + 2] : NEG;
      const float v = lse3_fast(nxt[s], b1, b2);
      const float l = E[base + s];
      const float r = v <= NEG ? NEG : v + l;
      cur[s] = r;
      const float a = AC[base + s];
      G[(int64_t)t * SS + s] = (a <= NEG || r <= NEG) ? 0.f : expf(a + r - l - logp);
    }
    __syncthreads();
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ctc_bwd_kernel(avsr_ctc_params p) {
  constexpr int VE = VecW<T>::VE;
  const int row = blockIdx.x, b = row / p.T, t = row % p.T;
  const int L = p.label_len[b], Tb = min(p.in_len[b], p.T), S = 2 * L + 1;
  const int SS = 2 * p.Lmax + 1;
  const int* lab = p.labels + (int64_t)b * p.Lmax;
  const bool active = t < Tb && p.nll[b] != 0.f && S <= 1024;
  const float scale = active ? (*p.dloss) * p.coef : 0.f;
  const T* x = (const T*)p.x + (int64_t)row * p.ldx;
  T* dx = (T*)p.dx + (int64_t)row * p.lddx;
  const float lse = p.lse[row];
  const float* G = p.gamma + ((int64_t)b * p.T + t) * SS;
  __shared__ float gsum_blank;
  __shared__ float sh[4];
  float gb = 0.f;
  if (active)
    for (int s = threadIdx.x * 2; s < S; s += 512) gb += G[s];
  gb = block_sum(gb, sh);
  if (threadIdx.x == 0) gsum_blank = gb;
  __syncthreads();
  for (int c0 = threadIdx.x * VE; c0 < p.lddx; c0 += 256 * VE) {
    float v[VE], o[VE];
    if (c0 < p.V) ldv(x + c0, v);
#pragma unroll
    for (int j = 0; j < VE; ++j) {
      const int c = c0 + j;
      o[j] = c < p.V ? scale * (expf(v[j] - lse) - (c == 0 ? gsum_blank : 0.f)) : 0.f;
    }
    stv(dx + c0, o);
  }
  __syncthreads();
  if (!active) return;
  // label columns: softmax - sum of the occupancies of every state carrying that label
  for (int i = threadIdx.x; i < L; i += 256) {
    const int k = lab[i];
    float g = 0.f;
    for (int j = 0; j < L; ++j)
      if (lab[j] == k) g += G[2 * j + 1];
    const float sm = expf(to_f(x[k]) - lse);
    dx[k] = from_f<T>(scale * (sm - g));
  }
}

__global__ void loss_finalize_kernel(int B, const float* nll, int rows, const float* row_loss,
                                     const int* row_correct, float mtl, int per_token, float* out) {
  __shared__ float sh[4];
  float a = 0.f, c = 0.f, n = 0.f, v = 0.f;
  for (int i = threadIdx.x; i < B; i += 256) a += nll[i];
  for (int i = threadIdx.x; i < rows; i += 256) {
    c += row_loss[i];
    if (row_correct) { const int rc = row_correct[i]; if (rc >= 0) { v += 1.f; n += (float)rc; } }
  }
  a = block_sum(a, sh); c = block_sum(c, sh); n = block_sum(n, sh); v = block_sum(v, sh);
  if (threadIdx.x == 0) {
    const float lc = a / (float)B, la = c / (per_token ? fmaxf(v, 1.f) : (float)B);
    out[0] = mtl * lc + (1.f - mtl) * la;
    out[1] = lc; out[2] = la; out[3] = v > 0.f ? n / v : 0.f;
  }
}

}  // namespace

extern "C" int avsr_row_lse(const avsr_xent_params* p, void* stream) {
  if (!p || p->ldx % 8) return AVSR_E_ALIGN;
  if (p->rows == 0) return 0;
  if (p->dtype == AVSR_BF16) hipLaunchKernelGGL((xent_fwd_kernel<bf16, 0>), dim3(p->rows), dim3(256), 0, (hipStream_t)stream, *p);
  else hipLaunchKernelGGL((xent_fwd_kernel<float, 0>), dim3(p->rows), dim3(256), 0, (hipStream_t)stream, *p);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_lsm_fwd(const avsr_xent_params* p, void* stream) {
  if (!p || p->ldx % 8 || !p->target || !p->row_loss) return AVSR_E_ARG;
  if (p->rows == 0) return 0;
  if (p->dtype == AVSR_BF16) hipLaunchKernelGGL((xent_fwd_kernel<bf16, 1>), dim3(p->rows), dim3(256), 0, (hipStream_t)stream, *p);
  else hipLaunchKernelGGL((xent_fwd_kernel<float, 1>), dim3(p->rows), dim3(256), 0, (hipStream_t)stream, *p);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_lsm_bwd(const avsr_xent_params* p, void* stream) {
  if (!p || p->lddx % 8 || !p->dloss || !p->dx) return AVSR_E_ARG;
  if (p->rows == 0) return 0;
  if (p->dtype == AVSR_BF16) hipLaunchKernelGGL(lsm_bwd_kernel<bf16>, dim3(p->rows), dim3(256), 0, (hipStream_t)stream, *p);
  else hipLaunchKernelGGL(lsm_bwd_kernel<float>, dim3(p->rows), dim3(256), 0, (hipStream_t)stream, *p);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_ctc_fwd(const avsr_ctc_params* p, void* stream) {
  if (!p || p->ldx % 8) return AVSR_E_ARG;
  if (2 * p->Lmax + 1 > 1024) return AVSR_E_SHAPE;
  if (p->B == 0) return 0;
  if (p->dtype == AVSR_BF16) hipLaunchKernelGGL(ctc_fwd_kernel<bf16>, dim3(p->B), dim3(256), 0, (hipStream_t)stream, *p);
  else hipLaunchKernelGGL(ctc_fwd_kernel<float>, dim3(p->B), dim3(256), 0, (hipStream_t)stream, *p);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_ctc_bwd(const avsr_ctc_params* p, void* stream) {
  if (!p || p->lddx % 8 || !p->dloss || !p->dx) return AVSR_E_ARG;
  if (p->B * p->T == 0) return 0;
  if (p->dtype == AVSR_BF16) hipLaunchKernelGGL(ctc_bwd_kernel<bf16>, dim3(p->B * p->T), dim3(256), 0, (hipStream_t)stream, *p);
  else hipLaunchKernelGGL(ctc_bwd_kernel<float>, dim3(p->B * p->T), dim3(256), 0, (hipStream_t)stream, *p);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_loss_finalize(int B, const float* nll, int rows, const float* row_loss, const int* row_correct,
                                  float mtlalpha, int att_per_token, float* out, void* stream) {
  if (att_per_token && !row_correct) return AVSR_E_ARG;
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, B, nll, rows, row_loss,
                     row_correct, mtlalpha, att_per_token, out);
  AVSR_CHECK_LAUNCH();
  return 0;
}
