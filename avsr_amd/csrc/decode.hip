// Joint CTC / attention beam-search kernels (declarations and the
// reference call sites in include/avsr_hip.h):
//   avsr_log_softmax_rows  log_softmax over V (decoder output layer, CTC log-probs)
//   avsr_dec_attn          one-query multi-head attention per hypothesis over a K/V cache
//   avsr_row_topk          pre-beam: top-P decoder tokens per hypothesis
//   avsr_ctc_prefix        CTC prefix scores of the pre-beam tokens (T recursion)
//   avsr_beam_select       weighted scores + flat top-beam over (hyps x V)
//   avsr_gather_rows       reorder per-hypothesis state (K/V caches, CTC variables)
// All fp32 math; decode runs at batch 1 utterance x beam hypotheses, so these kernels are
// latency-bound: one block per row / hypothesis, no host round trip inside a step.
#include "common.h"

namespace {

constexpr float LOGZERO = -10000000000.0f;   // CTCPrefixScoreTH.logzero (ctc_prefix_score.py:29)

// torch.logsumexp of two finite values: m + log(exp(a-m) + exp(b-m)). One of the two terms is
// exp(0) = 1 exactly, so m + log(1 + exp(min - m)) is the same float computation with one
// transcendental less (bit-identical; the CTC prefix recursion's serial chain is two of these)
AVSR_DEV float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  return m + logf(1.f + expf(fminf(a, b) - m));
}
// the same with the hardware exp2 / log2 (v_exp_f32 / v_log_f32, ~1 ulp): the CTC prefix
// recursion's dependent chain (two of these per frame, T frames in sequence), as in loss.hip's
// CTC recursion; the correction term is <= log 2, so the result differs from lse2 by a few ulp
// of that term
AVSR_DEV float lse2_fast(float a, float b) {
  const float m = fmaxf(a, b);
  return m + __logf(1.f + __expf(fminf(a, b) - m));
}

// Cross-lane reductions on DPP row rotations (common.h): the __shfl_xor butterflies they replace
// are ds_bpermute round trips through the LDS unit (~2 us per block arg-max: the pre-beam's 7
// rounds took 12 us of an 18 us kernel).
// (value, index) arg-max over the wave, ties -> smaller index (a total order: exact, uniform)
AVSR_DEV void dwave_argmax(float& v, int& i) {
#define DA_STEP(R_) { const float ov = rorf<R_>(v); const int oi = rori<R_>(i); \
                      if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; } }
  DA_STEP(8) DA_STEP(4) DA_STEP(2) DA_STEP(1)
#undef DA_STEP
  float bv = lanef(v, 0); int bi = __builtin_amdgcn_readlane(i, 0);
#pragma unroll
  for (int r = 1; r < 4; ++r) {
    const float ov = lanef(v, 16 * r); const int oi = __builtin_amdgcn_readlane(i, 16 * r);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  v = bv; i = bi;
}

AVSR_DEV float block_max256(float v, float* sh) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  v = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
  __syncthreads();
  return v;
}
AVSR_DEV float block_sum256(float v, float* sh) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  v = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  return v;
}

// (value, index) arg-max across the 256-thread block; ties -> smaller index
AVSR_DEV void block_argmax256(float& v, int& i, float* shv, int* shi) {
  dwave_argmax(v, i);
  if ((threadIdx.x & 63) == 0) { shv[threadIdx.x >> 6] = v; shi[threadIdx.x >> 6] = i; }
  __syncthreads();
  v = shv[0]; i = shi[0];
#pragma unroll
  for (int w = 1; w < 4; ++w)
    if (shv[w] > v || (shv[w] == v && shi[w] < i)) { v = shv[w]; i = shi[w]; }
  __syncthreads();
}

// ---------------------------------------------------------------- log_softmax rows
template <typename T>
__global__ __launch_bounds__(256) void log_softmax_kernel(int V, const T* x, int64_t ldx, float* out, int64_t ldo) {
  __shared__ float sh[4];
  const T* r = x + (int64_t)blockIdx.x * ldx;
  float m = -INFINITY;
  for (int c = threadIdx.x; c < V; c += 256) m = fmaxf(m, to_f(r[c]));
  m = block_max256(m, sh);
  float s = 0.f;
  for (int c = threadIdx.x; c < V; c += 256) s += expf(to_f(r[c]) - m);
  s = block_sum256(s, sh);
  const float ls = logf(s);
  float* o = out + (int64_t)blockIdx.x * ldo;
  for (int c = threadIdx.x; c < V; c += 256) o[c] = to_f(r[c]) - m - ls;
}

// ---------------------------------------------------------------- one-query attention
// block (hyp i, head h), 4 waves: a wave reads 4 keys per instruction (16 lanes x 4 elements
// per 64-wide row: coalesced 256-B rows), scores by 16-lane butterfly sums into LDS, block
// softmax, then o = sum_j p_j v_j with the same row-per-16-lanes reads, reduced over the 4 key
// slots of a wave (shuffles) and the 4 waves (LDS). Rows come through kmap (ancestry-indexed
// self-attention cache), kidx (batched memories) or directly.
template <typename T> AVSR_DEV f32x4 ld4(const T* p) {
  if constexpr (sizeof(T) == 2) {
    const bf16x4 v = *(const bf16x4*)p;
    return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
  } else {
    return *(const f32x4*)p;
  }
}

// G hypotheses per workgroup (p.group; G = 1 for per-hypothesis keys): every key / value row is
// read once for the G queries of the group. 8 waves; key j of iteration it is handled by wave
// (j / 4) % 8, key slot j % 4 (16 lanes x 4 elements); each lane issues DA_UNROLL row loads
// back to back before using them, so a 375-key memory takes two load round trips per phase
// (the one-load-per-iteration loop was latency-bound: 51 us per call at 375 keys, G = 5).
constexpr int DA_WAVES = 8, DA_UNROLL = 8;
// Key split (p.ksplit >= 2, blockIdx.z): workgroup z of a (group, head) takes keys
// [z * chunk, (z + 1) * chunk) of its rows' klen, with nz = min(ksplit, ceil(klen / 192)) chunks
// (a function of klen alone, so a hypothesis's result never depends on the batch); it writes its
// per-query (max, sum of exp, unnormalised o) to p.ws and the last of the nz to arrive merges them
// in split order (write-through partials, drained before the counter add; Guideline 16).
constexpr int DA_SPLIT_KEYS = 192;
template <typename T, int G>
__global__ __launch_bounds__(64 * DA_WAVES) void dec_attn_kernel(avsr_dec_attn_params p) {
  constexpr int NW = DA_WAVES, U = DA_UNROLL, KS = 4 * NW;
  extern __shared__ float sc[];           // [G][kpad] scores, then [NW][G][64] partials
  __shared__ float shr[G][NW];
  __shared__ int last;
  const int h = blockIdx.x, i0 = blockIdx.y * G;
  const int klen = p.klen ? min(p.klen[i0], p.klen_max) : p.klen_max;
  const int kpad = (p.klen_max + 3) & ~3;
  const int nz = p.ksplit > 1 ? max(1, min(p.ksplit, (klen + DA_SPLIT_KEYS - 1) / DA_SPLIT_KEYS)) : 1;
  const int z = blockIdx.z;
  if (z >= nz) return;                    // (no arrival: the merge counts nz workgroups)
  const int chunk = (klen + nz - 1) / nz;
  const int jbeg = z * chunk, jend = min(klen, jbeg + chunk), jn = jend - jbeg;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, sub = lane >> 4, d0 = (lane & 15) * 4;
  const int kb = p.kmap ? 0 : (p.kidx ? p.kidx[i0] : i0);
  const T* K = (const T*)p.k + (int64_t)kb * p.k_bstride + h * 64 + d0;
  const T* Vv = (const T*)p.v + (int64_t)kb * p.v_bstride + h * 64 + d0;
  const int* km = p.kmap ? p.kmap + (int64_t)i0 * p.ldmap : nullptr;  // key j -> row km[j] (G == 1)
  const int ng = min(G, p.n - i0);
  const int jl = 4 * w + sub;             // this lane's key offset within an iteration
  auto rows_of = [&](int it0, int (&row)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = jbeg + (it0 + u) * KS + jl;
      row[u] = j < jend ? (km ? km[j] : j) : 0;
    }
  };
  f32x4 q[G];
#pragma unroll
  for (int g = 0; g < G; ++g) q[g] = ld4((const T*)p.q + (int64_t)(i0 + min(g, ng - 1)) * p.ldq + h * 64 + d0);
  float m[G];
#pragma unroll
  for (int g = 0; g < G; ++g) m[g] = -INFINITY;
  for (int it0 = 0; it0 * KS < jn; it0 += U) {
    int row[U];
    rows_of(it0, row);
    f32x4 k[U];
#pragma unroll
    for (int u = 0; u < U; ++u) k[u] = ld4(K + (int64_t)row[u] * p.ldk);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = jbeg + (it0 + u) * KS + jl;
      const bool ok = j < jend;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float s = q[g][0] * k[u][0] + q[g][1] * k[u][1] + q[g][2] * k[u][2] + q[g][3] * k[u][3];
        s = row_sum16(s);               // over the key's 16 lanes (one DPP row)
        s *= p.scale;
        if (ok) {
          if ((lane & 15) == 0) sc[g * kpad + j] = s;
          m[g] = fmaxf(m[g], s);
        }
      }
    }
  }
  // block max of every group row (one barrier pair for all G)
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float v = wave_max(m[g]);
    if (lane == 0) shr[g][w] = v;
  }
  __syncthreads();
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float v = shr[g][0];
#pragma unroll
    for (int x = 1; x < NW; ++x) v = fmaxf(v, shr[g][x]);
    m[g] = v;
  }
  __syncthreads();
  float l[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float lg = 0.f;
    for (int j = jbeg + threadIdx.x; j < jend; j += 64 * NW) {
      const float e = expf(sc[g * kpad + j] - m[g]);
      sc[g * kpad + j] = e;
      lg += e;
    }
    lg = wave_sum(lg);
    if (lane == 0) shr[g][w] = lg;
  }
  __syncthreads();                         // every score is final, every wave sum written
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float v = shr[g][0];
#pragma unroll
    for (int x = 1; x < NW; ++x) v += shr[g][x];
    l[g] = v;
  }
  f32x4 acc[G];
#pragma unroll
  for (int g = 0; g < G; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it0 = 0; it0 * KS < jn; it0 += U) {
    int row[U];
    rows_of(it0, row);
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld4(Vv + (int64_t)row[u] * p.ldv);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = jbeg + (it0 + u) * KS + jl;
      const bool ok = j < jend;
#pragma unroll
      for (int g = 0; g < G; ++g) acc[g] += (ok ? sc[g * kpad + j] : 0.f) * v[u];
    }
  }
  float* part = sc + G * kpad;
#pragma unroll
  for (int g = 0; g < G; ++g) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[g][e] += __shfl_xor(acc[g][e], 16, 64);
      acc[g][e] += __shfl_xor(acc[g][e], 32, 64);
    }
    if (sub == 0) *(f32x4*)&part[(w * G + g) * 64 + d0] = acc[g];
  }
  __syncthreads();
  if (nz == 1) {
    for (int t = threadIdx.x; t < ng * 64; t += 64 * NW) {
      const int g = t >> 6, d = t & 63;
      float o = 0.f;
#pragma unroll
      for (int x = 0; x < NW; ++x) o += part[(x * G + g) * 64 + d];
      ((T*)p.o)[(int64_t)(i0 + g) * p.ldo + h * 64 + d] = from_f<T>(o / l[g]);
    }
    return;
  }
  // split: this chunk's (o[64], max, sum) per query -> ws[(group, head)][z][g][66]
  const int64_t slot = (int64_t)blockIdx.y * gridDim.x + h;
  float* wz = p.ws + (slot * p.ksplit) * G * 66;
  for (int t = threadIdx.x; t < ng * 64; t += 64 * NW) {
    const int g = t >> 6, d = t & 63;
    float o = 0.f;
#pragma unroll
    for (int x = 0; x < NW; ++x) o += part[(x * G + g) * 64 + d];
    __hip_atomic_store(wz + ((int64_t)z * G + g) * 66 + d, o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x < ng) {
    const int g = threadIdx.x;
#pragma unroll
    for (int gg = 0; gg < G; ++gg)
      if (gg == g) {
        __hip_atomic_store(wz + ((int64_t)z * G + g) * 66 + 64, m[gg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(wz + ((int64_t)z * G + g) * 66 + 65, l[gg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave: its partials are out
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(&p.cnt[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)nz - 1;
  __syncthreads();
  if (!last) return;
  for (int t = threadIdx.x; t < ng * 64; t += 64 * NW) {
    const int g = t >> 6, d = t & 63;
    auto ld = [&](int q, int e) {
      return __hip_atomic_load(wz + ((int64_t)q * G + g) * 66 + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    float mx = -INFINITY;
    for (int q = 0; q < nz; ++q) mx = fmaxf(mx, ld(q, 64));
    float lsum = 0.f, o = 0.f;
    for (int q = 0; q < nz; ++q) {
      const float f = expf(ld(q, 64) - mx);
      lsum += ld(q, 65) * f;
      o += ld(q, d) * f;
    }
    ((T*)p.o)[(int64_t)(i0 + g) * p.ldo + h * 64 + d] = from_f<T>(o / lsum);
  }
  if (threadIdx.x == 0) __hip_atomic_store(&p.cnt[slot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- pre-beam top-P
// one block per hypothesis row; P rounds of block arg-max over per-thread sorted candidate
// lists (each thread keeps its own top-P of a strided slice)
constexpr int KMAX = 16;

__global__ __launch_bounds__(256) void row_topk_kernel(avsr_topk_params p) {
  __shared__ float shv[4];
  __shared__ int shi[4];
  const float* x = p.x + (int64_t)blockIdx.x * p.ldx;   // one row per block
  float tv[KMAX];
  int ti[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) { tv[k] = -INFINITY; ti[k] = 0x7fffffff; }
  for (int c = threadIdx.x; c < p.V; c += 256) {
    float v = x[c];
    int id = c;
    // insertion into the descending list (ties keep the smaller index first)
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k < p.K && (v > tv[k] || (v == tv[k] && id < ti[k]))) {
        const float t = tv[k]; const int u = ti[k];
        tv[k] = v; ti[k] = id; v = t; id = u;
      }
    }
  }
  int head = 0;
  for (int r = 0; r < p.K; ++r) {
    float v = -INFINITY; int id = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) if (k == head) { v = tv[k]; id = ti[k]; }
    const int mine = id;
    block_argmax256(v, id, shv, shi);
    if (threadIdx.x == 0) p.ids[(int64_t)blockIdx.x * p.K + r] = id;
    if (mine == id && id != 0x7fffffff) ++head;
  }
}

// log_softmax_rows + row_topk of the decoder output in one pass (decode steps): the row stays
// in registers (<= 24 values per thread, V <= 6144), the log-probs are written once and the
// top-K runs on the same register values. Per-thread element order, the block reductions and
// top-K order (value desc, index asc) equal the two separate kernels', so the output is
// identical to them.
constexpr int LSM_TOPK_NV = 24;
template <typename T>
__global__ __launch_bounds__(256) void log_softmax_topk_kernel(int V, int K, const T* x, int64_t ldx, float* out,
                                                               int64_t ldo, int* ids) {
  __shared__ float sh[4];
  __shared__ float shv[4];
  __shared__ int shi[4];
  const T* r = x + (int64_t)blockIdx.x * ldx;
  float v[LSM_TOPK_NV];
#pragma unroll
  for (int q = 0; q < LSM_TOPK_NV; ++q) {
    const int c = threadIdx.x + q * 256;
    v[q] = c < V ? to_f(r[c]) : -INFINITY;
  }
  float m = -INFINITY;
#pragma unroll
  for (int q = 0; q < LSM_TOPK_NV; ++q) m = fmaxf(m, v[q]);
  m = block_max256(m, sh);
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < LSM_TOPK_NV; ++q)
    if (threadIdx.x + q * 256 < V) s += expf(v[q] - m);
  s = block_sum256(s, sh);
  const float ls = logf(s);
  float* o = out + (int64_t)blockIdx.x * ldo;
#pragma unroll
  for (int q = 0; q < LSM_TOPK_NV; ++q) {
    const int c = threadIdx.x + q * 256;
    if (c < V) { v[q] = v[q] - m - ls; o[c] = v[q]; }
  }
  // top-K by K rounds of "largest element below the previous pick" in the order (value desc,
  // index asc) -- the order row_topk's insertion lists produce, so the ids are the same; a
  // round is one register scan plus a block arg-max (the unrolled 24 x 16 insertion network
  // with its divergent swaps took ~30 us per call)
  // Each wave first takes the top-K of its own elements (rounds of wave arg-max, DPP only, no
  // barrier); the block's top-K is among those 4K candidates, which wave 0 then ranks the same way
  // (one barrier instead of two per round).
  __shared__ float cv[4 * KMAX];
  __shared__ int ci[4 * KMAX];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float pv = INFINITY;
  int pi = -1;
  for (int rr = 0; rr < K; ++rr) {
    float bv = -INFINITY; int bi = 0x7fffffff;
#pragma unroll
    for (int q = 0; q < LSM_TOPK_NV; ++q) {
      const int c = threadIdx.x + q * 256;
      const bool below = c < V && (v[q] < pv || (v[q] == pv && c > pi));
      if (below && (v[q] > bv || bi == 0x7fffffff)) { bv = v[q]; bi = c; }
    }
    dwave_argmax(bv, bi);
    if (lane == 0) { cv[wv * KMAX + rr] = bv; ci[wv * KMAX + rr] = bi; }
    pv = bv; pi = bi;
  }
  __syncthreads();
  if (wv != 0) return;
  const bool have = lane < 4 * KMAX && (lane % KMAX) < K;
  const float mv = have ? cv[lane] : -INFINITY;
  const int mi = have ? ci[lane] : 0x7fffffff;
  pv = INFINITY; pi = -1;
  for (int rr = 0; rr < K; ++rr) {
    const bool below = have && mi != 0x7fffffff && (mv < pv || (mv == pv && mi > pi));
    float bv = below ? mv : -INFINITY; int bi = below ? mi : 0x7fffffff;
    dwave_argmax(bv, bi);
    if (lane == 0) ids[(int64_t)blockIdx.x * K + rr] = bi;
    pv = bv; pi = bi;
  }
}

// ---------------------------------------------------------------- CTC prefix scores
// CTCPrefixScoreTH.__call__ (ctc_prefix_score.py:65-187) for one utterance: block = one
// hypothesis, lane j = its j-th scored token; the T recursion is sequential per lane.
__global__ __launch_bounds__(64) void ctc_prefix_kernel(avsr_ctc_prefix_params p) {
  const int h = blockIdx.x, j = threadIdx.x;
  if (p.out_len_dev) p.out_len = p.out_len_dev[0];
  const int V = p.V;
  const int u = p.uidx ? p.uidx[h] : 0;
  const int T = p.uidx ? p.tlen[u] : p.T;         // this utterance's frames
  const int TS = p.T;                              // row stride of r_prev / r_new
  if (p.uidx) p.logp += (int64_t)u * p.logp_ustride;
  const bool act = j < p.P;
  const int id = act ? p.ids[h * p.P + j] : 0;
  const bool same = act && id == p.last[h];
  const float* rp = p.r_prev ? p.r_prev + (int64_t)h * TS * 2 : nullptr;
  float* rn = act ? p.r_new + ((int64_t)h * p.P + j) * TS * 2 : nullptr;
  // r_prev at the first step: (logzero, cumsum of blank log-probs)
  auto rprev = [&](int t, int q, float cum) -> float { return rp ? rp[t * 2 + q] : (q == 0 ? LOGZERO : cum); };
  const int start = max(p.out_len, 1);
  // values of r for t < start
  float r0 = LOGZERO, r1 = LOGZERO;
  float cum = 0.f;          // running cumsum of logp[t][blank] (first step only)
  for (int t = 0; t < start; ++t) {
    const float xb = p.logp[(int64_t)t * V + p.blank];
    cum += xb;
    float a0 = LOGZERO;
    if (t == 0 && p.out_len == 0) a0 = act ? p.logp[id] : LOGZERO;
    if (act) { rn[t * 2 + 0] = a0; rn[t * 2 + 1] = LOGZERO; }
    if (t == start - 1) { r0 = a0; r1 = LOGZERO; }
  }
  // psi accumulates logsumexp over { phi(t-1) + x0(t) : t in [start, T) } U { r0(start-1) }
  float pm = r0;            // running max
  float ps = 1.f;           // sum of exp(. - pm)
  // phi(t-1) needs r_prev at t-1: carry the previous frame's values
  float prev_r0 = rprev(start - 1, 0, 0.f);
  float prev_r1 = rprev(start - 1, 1, cum);   // cum = cumsum of blank log-probs through start-1
  float cur_cum = cum;
  for (int t = start; t < T; ++t) {
    const float rsum_prev = lse2(prev_r0, prev_r1);
    const float phi = same ? prev_r1 : rsum_prev;
    const float x0 = act ? p.logp[(int64_t)t * V + id] : LOGZERO;
    const float xb = p.logp[(int64_t)t * V + p.blank];
    const float n0 = lse2_fast(r0, phi) + x0;
    const float n1 = lse2_fast(r0, r1) + xb;
    r0 = n0; r1 = n1;
    if (act) { rn[t * 2 + 0] = r0; rn[t * 2 + 1] = r1; }
    const float term = phi + x0;
    if (term > pm) { ps = ps * expf(pm - term) + 1.f; pm = term; }
    else ps += expf(term - pm);
    cur_cum += xb;
    prev_r0 = rprev(t, 0, 0.f);
    prev_r1 = rprev(t, 1, cur_cum);
  }
  // r_sum at the last frame (for eos): logsumexp of r_prev[T-1]
  const float rsum_last = lse2(prev_r0, prev_r1);
  float psi = pm + logf(ps);
  if (act) {
    if (id == p.blank) psi = LOGZERO;
    if (id == p.eos) psi = rsum_last;
    p.psi[h * (p.P + 1) + j] = psi;
  }
  if (j == 0) p.psi[h * (p.P + 1) + p.P] = rsum_last;
}

// The same recursion with its inputs staged in LDS first: the P scored tokens' and the blank's
// log-probs over all T frames ([T][P + 1], 4 independent gathers in flight per lane, the token
// ids read once) and phi(t) for both cases of a candidate ([T][2]: logsumexp(r_prev[t]) and
// r_prev[t][1] for a repeated label; at the first step the blank cumsum). Only the r recursion is
// sequential (wave 0, LDS reads issued ahead by the unrolled loop, hardware exp2 / log2 on the
// chain): psi = logsumexp({r0(start-1)} U {phi(t-1) + x0(t)}) does not depend on r, so waves 1-3
// reduce it meanwhile (a wave per candidate, lanes over t).
__global__ __launch_bounds__(256) void ctc_prefix_lds_kernel(avsr_ctc_prefix_params p) {
  extern __shared__ float sm[];
  __shared__ int sid[65];
  const int h = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int out_len = p.out_len_dev ? p.out_len_dev[0] : p.out_len;
  const int V = p.V, P = p.P, W = P + 1;
  const int u = p.uidx ? p.uidx[h] : 0;
  const int T = p.uidx ? p.tlen[u] : p.T;
  const int TS = p.T;
  const float* __restrict__ logp = p.logp + (p.uidx ? (int64_t)u * p.logp_ustride : 0);
  float* xs = sm;                           // [T][W]: ids then blank
  float* ph = sm + (int64_t)TS * W;         // [T][2]: phi for a new label, phi for a repeated one
  const int* __restrict__ ids = p.ids + h * P;
  if (tid < P) sid[tid] = ids[tid];
  if (tid == P) sid[P] = p.blank;
  const float* __restrict__ rp = p.r_prev ? p.r_prev + (int64_t)h * TS * 2 : nullptr;
  if (rp)
    for (int t = tid; t < T; t += 256) {
      const float a0 = rp[2 * t], a1 = rp[2 * t + 1];
      ph[2 * t] = lse2(a0, a1);
      ph[2 * t + 1] = a1;
    }
  __syncthreads();
  const int n = T * W;
  for (int base = tid; base < n; base += 4 * 256) {
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = base + q * 256;
      if (idx < n) {
        const int t = idx / W, c = idx - t * W;
        v[q] = logp[(int64_t)t * V + sid[c]];
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (base + q * 256 < n) xs[base + q * 256] = v[q];
  }
  __syncthreads();
  if (!rp && tid == 0) {                    // first step: r_prev = (logzero, cumsum of blank)
    float cum = 0.f;
    for (int t = 0; t < T; ++t) {
      cum += xs[t * W + P];
      ph[2 * t] = lse2(LOGZERO, cum);
      ph[2 * t + 1] = cum;
    }
  }
  if (!rp) __syncthreads();
  const int start = max(out_len, 1);
  const float* __restrict__ pc = ph;
  if (w == 0) {
    const int j = lane;
    const bool act = j < P;
    const int id = act ? sid[j] : 0;
    const int q = (act && id == p.last[h]) ? 1 : 0;     // repeated label: phi = r_prev[t][1]
    float* __restrict__ rn = act ? p.r_new + ((int64_t)h * P + j) * TS * 2 : nullptr;
    const int jj = act ? j : 0;
    float r0 = LOGZERO, r1 = LOGZERO;
    for (int t = 0; t < min(start, T); ++t) {
      float a0 = LOGZERO;
      if (t == 0 && out_len == 0) a0 = act ? xs[jj] : LOGZERO;
      if (act) { rn[t * 2 + 0] = a0; rn[t * 2 + 1] = LOGZERO; }
      r0 = a0;
    }
#pragma unroll 4
    for (int t = start; t < T; ++t) {
      const float phi = pc[2 * (t - 1) + q];
      const float x0 = xs[t * W + jj];
      const float xb = xs[t * W + P];
      const float n0 = lse2_fast(r0, phi) + x0;
      const float n1 = lse2_fast(r0, r1) + xb;
      r0 = n0; r1 = n1;
      if (act) { rn[t * 2 + 0] = r0; rn[t * 2 + 1] = r1; }
    }
  }
  // psi of candidate j (waves 1-3, beside wave 0's recursion): logsumexp over {r0(start-1)} U
  // {phi(t-1) + x0(t), t in [start, T)}
  const float rsum_last = pc[2 * (T - 1)];          // logsumexp(r_prev[T-1]) (the eos score)
  for (int j = w - 1; w > 0 && j < P; j += 3) {
    const int id = sid[j];
    const int q = id == p.last[h] ? 1 : 0;
    const float r0i = (out_len == 0) ? xs[j] : LOGZERO;  // r0 at frame start - 1 (= 0 when out_len == 0)
    float m = lane == 0 ? r0i : -INFINITY;
    for (int t = start + lane; t < T; t += 64) m = fmaxf(m, pc[2 * (t - 1) + q] + xs[t * W + j]);
    m = wave_max(m);
    float sum = lane == 0 ? expf(r0i - m) : 0.f;
    for (int t = start + lane; t < T; t += 64) sum += expf(pc[2 * (t - 1) + q] + xs[t * W + j] - m);
    sum = wave_sum(sum);
    if (lane == 0) {
      float psi = m + logf(sum);
      if (id == p.blank) psi = LOGZERO;
      if (id == p.eos) psi = rsum_last;
      p.psi[h * (P + 1) + j] = psi;
    }
  }
  if (tid == 0) p.psi[h * (P + 1) + P] = rsum_last;
}

// ---------------------------------------------------------------- beam selection
// weighted[h][v] = w_dec * dec[h][v] + w_ctc * (psi[h][v] - s_prev[h]) + score[h]
// (psi = LOGZERO for tokens outside the pre-beam, r_sum[T-1] for eos; batch_beam_search.py
// :228-260), flat top-`beam` over h*V + v; ties -> smaller flat index.
// Tokens outside a row's pre-beam have psi = LOGZERO, i.e. a weighted score below
// w_ctc * (LOGZERO - s_prev[h]) + score[h] (dec <= 0). The selection first runs over the
// candidates only (each row's P pre-beam tokens and eos: <= 256 per segment) and keeps that
// result when its beam-th score is above that bound for every row of the segment — then no
// other token can enter the top beam and the result equals the full scan; otherwise (fewer
// than `beam` finite candidates) it scans all rows x V as before.
__global__ __launch_bounds__(256) void beam_select_kernel(avsr_beam_select_params p) {
  __shared__ float shv[4];
  __shared__ int shi[4];
  __shared__ int use_full;
  float tv[KMAX];
  int ti[KMAX];
  // segment (utterance) of this block: rows [r0, r0 + nrow); flat ids are segment-local
  const int u = blockIdx.x;
  const int r0 = p.nseg ? p.seg[u] : 0, nrow = p.nseg ? p.seg[u + 1] - r0 : p.n;
  const int beam = min(p.beam, nrow * p.V);
  const int total = nrow * p.V;
  const int W = p.P + 1;
  auto weighted = [&](int f) -> float {
    const int h = r0 + f / p.V, v = f - (f / p.V) * p.V;
    if (p.score[h] == -INFINITY) return -INFINITY;      // a dead row of the device-side search
    float psi = LOGZERO;
    if (v == p.eos) psi = p.psi[h * (p.P + 1) + p.P];
    else if (v != p.blank)
      for (int c = 0; c < p.P; ++c)
        if (p.ids[h * p.P + c] == v) { psi = p.psi[h * (p.P + 1) + c]; break; }
    float w = 0.f;
    w += p.w_dec * (p.dec[(int64_t)h * p.ld + v]);
    w += p.w_ctc * (psi - p.s_prev[h]);
    w += p.score[h];
    return w;
  };
  auto insert = [&](float val, int id) {
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k < beam && (val > tv[k] || (val == tv[k] && id < ti[k]))) {
        const float t = tv[k]; const int w = ti[k];
        tv[k] = val; ti[k] = id; val = t; id = w;
      }
    }
  };
  // top-beam of the block's per-thread lists (written to out_*); returns the beam-th score
  auto select = [&]() -> float {
    int head = 0;
    float last = INFINITY;
    for (int r = 0; r < beam; ++r) {
      float v = -INFINITY; int id = 0x7fffffff;
#pragma unroll
      for (int k = 0; k < KMAX; ++k) if (k == head) { v = tv[k]; id = ti[k]; }
      const int mine = id;
      block_argmax256(v, id, shv, shi);
      if (mine == id && id != 0x7fffffff) ++head;
      last = v;
      if (threadIdx.x == 0 && id != 0x7fffffff) {     // (fewer candidates than beam: left to the full scan)
        const int h = r0 + id / p.V, tok = id - (id / p.V) * p.V;
        int col = p.P - 1;                       // scoring_idmap == -1 -> python index -1
        for (int c = 0; c < p.P; ++c)
          if (p.ids[h * p.P + c] == tok) { col = c; break; }
        float psi = LOGZERO;
        if (tok == p.eos) psi = p.psi[h * (p.P + 1) + p.P];
        else if (tok != p.blank && p.ids[h * p.P + col] == tok) psi = p.psi[h * (p.P + 1) + col];
        const int o = u * p.beam + r;
        p.out_prev[o] = h;
        p.out_tok[o] = tok;
        p.out_col[o] = col;
        p.out_score[o] = v;
        p.out_dec[o] = p.dec[(int64_t)h * p.ld + tok];
        p.out_ctc[o] = psi - p.s_prev[h];
        p.out_s[o] = psi;
      }
    }
    return last;
  };
  auto reset = [&]() {
#pragma unroll
    for (int k = 0; k < KMAX; ++k) { tv[k] = -INFINITY; ti[k] = 0x7fffffff; }
  };
  bool full = !(nrow * W <= 256 && p.w_ctc > 0.f);     // block-uniform
  {   // a segment with no live row (a finished utterance of the device-side search): nothing to select
    bool any = false;
    for (int hl = 0; hl < nrow; ++hl) any |= p.score[r0 + hl] != -INFINITY;
    if (!any) {
      for (int r = threadIdx.x; r < p.beam; r += 256) {
        const int o = u * p.beam + r;
        p.out_prev[o] = r0; p.out_tok[o] = p.eos; p.out_col[o] = p.P - 1; p.out_score[o] = -INFINITY;
        p.out_dec[o] = 0.f; p.out_ctc[o] = 0.f; p.out_s[o] = 0.f;
      }
      return;
    }
  }
  if (!full) {
    reset();
    const int c = threadIdx.x;
    if (c < nrow * W) {
      const int hl = c / W, k = c - hl * W, h = r0 + hl;
      const int v = k < p.P ? p.ids[h * p.P + k] : p.eos;
      // eos once per row: as the extra candidate, not again as a pre-beam id
      if (!(k < p.P && v == p.eos)) insert(weighted(hl * p.V + v), hl * p.V + v);
    }
    const float last = select();
    if (threadIdx.x == 0) {
      // bound on any non-candidate's score (dec <= 0), with a relative margin for rounding
      float bound = -INFINITY;
      for (int hl = 0; hl < nrow; ++hl) {
        const int h = r0 + hl;
        bound = fmaxf(bound, p.w_ctc * (LOGZERO - p.s_prev[h]) + p.score[h]);
      }
      use_full = !(last > bound + 1e-3f * fabsf(bound));
    }
    __syncthreads();
    full = use_full != 0;
  }
  if (full) {
    reset();
    for (int f = threadIdx.x; f < total; f += 256) insert(weighted(f), f);
    select();
  }
}

// ---------------------------------------------------------------- state gather
template <typename W>
__global__ __launch_bounds__(256) void gather_rows_kernel(int groups, int n, int64_t vecs, const W* src,
                                                          int64_t sg, int64_t sr, W* dst, int64_t dg, int64_t dr,
                                                          const int* idx) {
  const int64_t total = (int64_t)groups * n * vecs;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t v = e % vecs, gi = e / vecs;
    const int i = (int)(gi % n), g = (int)(gi / n);
    dst[g * dg + i * dr + v] = src[g * sg + (int64_t)idx[i] * sr + v];
  }
}

}  // namespace

extern "C" int avsr_log_softmax_rows(int dtype, int rows, int V, const void* x, int64_t ldx, float* out, int64_t ldo,
                                     void* stream) {
  if (rows <= 0) return 0;
  if (V <= 0 || !x || !out) return AVSR_E_ARG;
  if (dtype == AVSR_BF16)
    hipLaunchKernelGGL(log_softmax_kernel<bf16>, dim3(rows), dim3(256), 0, (hipStream_t)stream, V, (const bf16*)x, ldx, out, ldo);
  else if (dtype == AVSR_F32)
    hipLaunchKernelGGL(log_softmax_kernel<float>, dim3(rows), dim3(256), 0, (hipStream_t)stream, V, (const float*)x, ldx, out, ldo);
  else return AVSR_E_DTYPE;
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_log_softmax_topk(int dtype, int rows, int V, const void* x, int64_t ldx, float* out,
                                     int64_t ldo, int K, int* ids, void* stream) {
  if (rows <= 0) return 0;
  if (V <= 0 || !x || !out || !ids) return AVSR_E_ARG;
  if (K < 1 || K > KMAX || K > V) return AVSR_E_SHAPE;
  if (V > LSM_TOPK_NV * 256) {             // row does not fit the registers: the two passes
    const int e = avsr_log_softmax_rows(dtype, rows, V, x, ldx, out, ldo, stream);
    if (e) return e;
    avsr_topk_params tp{rows, V, K, out, ldo, ids};
    return avsr_row_topk(&tp, stream);
  }
  if (dtype == AVSR_BF16)
    hipLaunchKernelGGL(log_softmax_topk_kernel<bf16>, dim3(rows), dim3(256), 0, (hipStream_t)stream, V, K,
                       (const bf16*)x, ldx, out, ldo, ids);
  else if (dtype == AVSR_F32)
    hipLaunchKernelGGL(log_softmax_topk_kernel<float>, dim3(rows), dim3(256), 0, (hipStream_t)stream, V, K,
                       (const float*)x, ldx, out, ldo, ids);
  else return AVSR_E_DTYPE;
  AVSR_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------- device-side bookkeeping
__global__ __launch_bounds__(256) void beam_step_prep_kernel(int R, int Lmax, const int* pos_p, int* anc, int* klen) {
  const int pos = pos_p[0];
  for (int r = blockIdx.x * 256 + threadIdx.x; r < R; r += gridDim.x * 256) {
    anc[(int64_t)r * Lmax + pos] = pos * R + r;
    klen[r] = pos + 1;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void beam_kv_put_kernel(int R, int D, const T* qkv, int64_t ld, T* ck, T* cv,
                                                          const int* pos_p) {
  const int pos = pos_p[0];
  const int nv = D / VecW<T>::VE;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < R * nv; e += gridDim.x * 256) {
    const int r = e / nv, c = (e - r * nv) * VecW<T>::VE;
    const int64_t dst = ((int64_t)pos * R + r) * D + c;
    *(v16*)(ck + dst) = *(const v16*)(qkv + (int64_t)r * ld + D + c);
    *(v16*)(cv + dst) = *(const v16*)(qkv + (int64_t)r * ld + 2 * D + c);
  }
}

// one workgroup: rows of the step (R <= 1024), then one thread per utterance
__global__ __launch_bounds__(256) void beam_post_kernel(avsr_beam_post_params p) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  double* od = (double*)sm;                   // [R] old decoder sums
  double* oc = od + p.R;                      // [R] old CTC sums
  int* ended = (int*)(oc + p.R);              // [R] 0 running, 1 eos, 2 forced eos at maxlen
  const int pos = p.pos[0];
  for (int r = threadIdx.x; r < p.R; r += 256) { od[r] = p.sdec[r]; oc[r] = p.sctc[r]; }
  __syncthreads();
  const int64_t so = (int64_t)pos * p.R;
  for (int r = threadIdx.x; r < p.R; r += 256) {
    const int u = r / p.beam;
    ended[r] = 0;
    if (p.done[u]) {                          // finished before this step: stays dead
      p.score[r] = -INFINITY;
      p.src[r] = r; p.src[p.R + r] = r * p.P;
      p.bp_prev[so + r] = r; p.bp_tok[so + r] = p.eos; p.end_flag[so + r] = 0;
      continue;
    }
    const int h = p.sel_prev[r], t = p.sel_tok[r];
    const float sc = p.sel_score[r];
    const double nd = od[h] + (double)p.sel_dec[r], nc = oc[h] + (double)p.sel_ctc[r];
    const bool forced = pos == p.maxlen[u] - 1;   // eos appended to every hypothesis at the last step
    const int e = forced ? 2 : (t == p.eos ? 1 : 0);
    ended[r] = e;
    p.bp_prev[so + r] = h; p.bp_tok[so + r] = t; p.end_flag[so + r] = e;
    if (e) { p.end_score[so + r] = sc; p.end_dec[so + r] = nd; p.end_ctc[so + r] = nc; }
    p.tok[r] = t;
    p.score[r] = e ? -INFINITY : sc;
    p.sdec[r] = nd; p.sctc[r] = nc; p.s_prev[r] = p.sel_s[r];
    p.src[r] = h; p.src[p.R + r] = h * p.P + p.sel_col[r];
  }
  __syncthreads();
  const int LB = p.Lmax + 3;
  for (int u = threadIdx.x; u < p.U; u += 256) {
    if (p.done[u]) continue;
    bool any_live = false;
    float* bl = p.best_len + (int64_t)u * LB;
    for (int k = 0; k < p.beam; ++k) {         // this step's ended hypotheses, in selection order
      const int r = u * p.beam + k;
      if (!ended[r]) { any_live = true; continue; }
      const int len = pos + 2 + (ended[r] == 2 ? 1 : 0);     // sos + pos+1 tokens (+ the forced eos)
      const float s = p.end_score[so + r];
      if (len < LB && s > bl[len]) bl[len] = s;
      if (s > p.best_end[u]) p.best_end[u] = s;
    }
    bool det = false;
    if (p.end_detect && p.best_end[u] != -INFINITY) {
      int count = 0;
      for (int m = 0; m < 3; ++m) {
        const int len = pos - m;
        if (len >= 0 && len < LB && bl[len] != -INFINITY && (double)bl[len] - (double)p.best_end[u] < p.d_end) ++count;
      }
      det = count == 3;
    }
    if (det || !any_live || pos >= p.maxlen[u] - 1) {
      p.done[u] = 1;
      for (int k = 0; k < p.beam; ++k) p.score[u * p.beam + k] = -INFINITY;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int n = 0;
    for (int u = 0; u < p.U; ++u) n += p.done[u];
    p.done[p.U] = n;
    p.pos[0] = pos + 1;
  }
}

extern "C" int avsr_beam_step_prep(int R, int Lmax, const int* pos, int* anc, int* klen, void* stream) {
  if (R <= 0 || Lmax <= 0 || !pos || !anc || !klen) return AVSR_E_ARG;
  hipLaunchKernelGGL(beam_step_prep_kernel, dim3((R + 255) / 256), dim3(256), 0, (hipStream_t)stream, R, Lmax, pos, anc,
                     klen);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_beam_kv_put(int dtype, int R, int D, const void* qkv, int64_t ldqkv, void* cache_k, void* cache_v,
                                const int* pos, void* stream) {
  const int ve = dtype == AVSR_BF16 ? 8 : 4;
  if (R <= 0 || D % ve || ldqkv % ve || !pos) return AVSR_E_ARG;
  if (!avsr_aligned16(qkv) || !avsr_aligned16(cache_k) || !avsr_aligned16(cache_v)) return AVSR_E_ALIGN;
  const int g = avsr_grid((int64_t)R * D / ve, 256, 1024);
  if (dtype == AVSR_BF16)
    hipLaunchKernelGGL(beam_kv_put_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, R, D, (const bf16*)qkv, ldqkv,
                       (bf16*)cache_k, (bf16*)cache_v, pos);
  else if (dtype == AVSR_F32)
    hipLaunchKernelGGL(beam_kv_put_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, R, D, (const float*)qkv,
                       ldqkv, (float*)cache_k, (float*)cache_v, pos);
  else return AVSR_E_DTYPE;
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_beam_post(const avsr_beam_post_params* p, void* stream) {
  if (!p || p->U <= 0 || p->beam <= 0 || p->R != p->U * p->beam || p->R > 2048) return AVSR_E_ARG;
  const size_t lds = (size_t)p->R * (2 * sizeof(double) + sizeof(int));
  hipLaunchKernelGGL(beam_post_kernel, dim3(1), dim3(256), lds, (hipStream_t)stream, *p);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_dec_attn(const avsr_dec_attn_params* p, void* stream) {
  if (!p || p->n <= 0 || p->H <= 0) return AVSR_E_ARG;
  if (p->klen_max <= 0 || p->klen_max > 16384) return AVSR_E_SHAPE;
  if (p->ldq % 4 || p->ldk % 4 || p->ldv % 4 || p->k_bstride % 4 || p->v_bstride % 4) return AVSR_E_ALIGN;
  const int G = p->group > 1 ? p->group : 1;
  if (G > 8 || (G > 1 && p->kmap)) return AVSR_E_ARG;
  const int kpad = (p->klen_max + 3) & ~3;
  const size_t lds = ((size_t)G * kpad + (size_t)DA_WAVES * G * 64) * sizeof(float);
  if (lds > 64 * 1024) return AVSR_E_SHAPE;
  const int ks = p->ksplit > 1 ? p->ksplit : 1;
  if (ks > 8 || (ks > 1 && (!p->ws || !p->cnt))) return AVSR_E_ARG;
  const dim3 g(p->H, (p->n + G - 1) / G, ks);
  hipStream_t st = (hipStream_t)stream;
#define DA(T_, G_) hipLaunchKernelGGL((dec_attn_kernel<T_, G_>), g, dim3(64 * DA_WAVES), lds, st, *p)
#define DAG(T_) switch (G) { case 1: DA(T_, 1); break; case 2: DA(T_, 2); break; case 3: DA(T_, 3); break;   \
                              case 4: DA(T_, 4); break; case 5: DA(T_, 5); break; case 6: DA(T_, 6); break;   \
                              case 7: DA(T_, 7); break; default: DA(T_, 8); }
  if (p->dtype == AVSR_BF16) { DAG(bf16) }
  else if (p->dtype == AVSR_F32) { DAG(float) }
  else return AVSR_E_DTYPE;
#undef DAG
#undef DA
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_row_topk(const avsr_topk_params* p, void* stream) {
  if (!p || p->rows <= 0) return p ? 0 : AVSR_E_ARG;
  if (p->K < 1 || p->K > KMAX || p->K > p->V) return AVSR_E_SHAPE;
  hipLaunchKernelGGL(row_topk_kernel, dim3(p->rows), dim3(256), 0, (hipStream_t)stream, *p);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_ctc_prefix(const avsr_ctc_prefix_params* p, void* stream) {
  if (!p || p->n <= 0) return AVSR_E_ARG;
  if (p->P < 1 || p->P > 64 || p->T < 1) return AVSR_E_SHAPE;
  const size_t lds = (size_t)p->T * (p->P + 1 + 2) * sizeof(float);
  if (lds <= 64 * 1024)
    hipLaunchKernelGGL(ctc_prefix_lds_kernel, dim3(p->n), dim3(256), lds, (hipStream_t)stream, *p);
  else
    hipLaunchKernelGGL(ctc_prefix_kernel, dim3(p->n), dim3(64), 0, (hipStream_t)stream, *p);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_beam_select(const avsr_beam_select_params* p, void* stream) {
  if (!p || p->n <= 0) return AVSR_E_ARG;
  if (p->beam < 1 || p->beam > KMAX || p->P < 1 || p->nseg < 0) return AVSR_E_SHAPE;
  if (!p->nseg && p->beam > p->n * p->V) return AVSR_E_SHAPE;
  if (p->nseg && !p->seg) return AVSR_E_ARG;
  hipLaunchKernelGGL(beam_select_kernel, dim3(p->nseg ? p->nseg : 1), dim3(256), 0, (hipStream_t)stream, *p);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_gather_rows(int groups, int n, int64_t row_bytes, const void* src, int64_t src_gstride,
                                int64_t src_rstride, void* dst, int64_t dst_gstride, int64_t dst_rstride,
                                const int* idx, void* stream) {
  if (groups <= 0 || n <= 0 || row_bytes <= 0) return 0;
  const int64_t all = row_bytes | src_gstride | src_rstride | dst_gstride | dst_rstride;
  if (all % 16 == 0 && avsr_aligned16(src) && avsr_aligned16(dst)) {   // 16-byte words
    const int64_t vecs = row_bytes / 16;
    const int g = avsr_grid((int64_t)groups * n * vecs, 256, 2048);
    hipLaunchKernelGGL(gather_rows_kernel<uint4>, dim3(g), dim3(256), 0, (hipStream_t)stream, groups, n, vecs,
                       (const uint4*)src, src_gstride / 16, src_rstride / 16, (uint4*)dst, dst_gstride / 16,
                       dst_rstride / 16, idx);
  } else if (all % 4 == 0 && ((uintptr_t)src & 3) == 0 && ((uintptr_t)dst & 3) == 0) {   // 4-byte words
    const int64_t vecs = row_bytes / 4;
    const int g = avsr_grid((int64_t)groups * n * vecs, 256, 2048);
    hipLaunchKernelGGL(gather_rows_kernel<uint32_t>, dim3(g), dim3(256), 0, (hipStream_t)stream, groups, n, vecs,
                       (const uint32_t*)src, src_gstride / 4, src_rstride / 4, (uint32_t*)dst, dst_gstride / 4,
                       dst_rstride / 4, idx);
  } else {
    return AVSR_E_ALIGN;
  }
  AVSR_CHECK_LAUNCH();
  return 0;
}
