// Fused multi-head attention (head dim 64) forward / backward on bf16 MFMA 32x32x16 tiles.
// C-ABI: avsr_attn_fwd / avsr_attn_bwd_prep / avsr_attn_bwd (include/avsr_hip.h).
//
// Forward (one workgroup = 4 waves = 128 queries of one (batch, head); K/V tiles of 32 keys
// staged in LDS and shared by the 4 waves):
//   S^T = K Q^T with the query on the MFMA lane, so each lane owns one query row of the
//   online softmax (16 of the 32 keys in registers, the other 16 on lane^32); P^T is then
//   already the B operand of O^T += V^T P^T (accumulator-as-operand, no LDS round trip);
//   V is staged transposed so its A fragments are two 8-byte LDS reads.
// Backward (one workgroup = 4 waves = 128 keys; each wave owns 32 keys and keeps dK^T,
//   dV^T in accumulators while sweeping all query tiles): S and dP are computed with the
//   key on the lane so they feed dV^T += dO^T P' and dK^T += Q^T dS directly; dS crosses
//   LDS once for dQ = dS K, which is summed over the 4 waves in LDS and added to an fp32
//   accumulator with one atomic per element per workgroup.
// fp32 storage ("parity mode") runs the same tiles on bf16 hi/lo splits (3 products).
#include "common.h"
#include <algorithm>
#include <type_traits>
#include <cstdlib>

namespace {

constexpr int DH = 64;
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

struct Frag { bf16x8 hi, lo; };

template <typename T> AVSR_DEV Frag mkfrag(const float* x) {
  Frag f;
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { f.hi[j] = (bf16)x[j]; f.lo[j] = (bf16)0.f; }
  } else {
    split8(x, f.hi, f.lo);
  }
  return f;
}
template <typename T> AVSR_DEV Frag zfrag() {
  float z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  return mkfrag<T>(z);
}
// 8 contiguous elements
template <typename T> AVSR_DEV Frag ld8(const T* p) {
  if constexpr (sizeof(T) == 2) {
    Frag f; f.hi = *(const bf16x8*)p; return f;
  } else {
    f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
    float x[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    return mkfrag<T>(x);
  }
}
// two groups of 4 contiguous elements
template <typename T> AVSR_DEV Frag ld4x2(const T* p0, const T* p1) {
  if constexpr (sizeof(T) == 2) {
    bf16x4 a = *(const bf16x4*)p0, b = *(const bf16x4*)p1;
    Frag f;
    f.hi = bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    return f;
  } else {
    f32x4 a = *(const f32x4*)p0, b = *(const f32x4*)p1;
    float x[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    return mkfrag<T>(x);
  }
}
// registers 8s..8s+7 of an accumulator as an operand fragment
template <typename T, int S> AVSR_DEV Frag accfrag(const f32x16& x) {
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = x[8 * S + j];
  return mkfrag<T>(v);
}
template <typename T> AVSR_DEV void mm(f32x16& acc, const Frag& a, const Frag& b) {
  acc = mfma32(a.hi, b.hi, acc);
  if constexpr (sizeof(T) == 4) {
    acc = mfma32(a.hi, b.lo, acc);
    acc = mfma32(a.lo, b.hi, acc);
  }
}
AVSR_DEV int qrow(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }
AVSR_DEV void zacc(f32x16& x) {
#pragma unroll
  for (int r = 0; r < 16; ++r) x[r] = 0.f;
}

// ---- attention-probability dropout ------------------------------------------------------
// One 32-bit hash per (query, key pair) supplies the 16-bit uniforms of both keys of the pair
// (half the hash work of a per-element stream; the hash, two multiply-xorshift rounds, is the
// VALU-dominant cost of the attention kernels). Key k of query q of head (b, h) reads pair
//   g = ((b*H + h) * Lq + q) * ceil(Lk / 2) + k / 2,  u = (k odd ? hi : lo) 16 bits of hash(g),
// dropped iff u < thr = round(p * 65536) (p_eff within 8e-6 of p), kept values scaled by
// 65536 / (65536 - thr) so that E[mask] = 1 exactly. Every attention kernel (forward, dK/dV,
// dQ; bf16 and fp32) evaluates this same function: masks are recomputed, never stored.
struct AttnDrop {
  uint64_t seed; uint32_t pre, thr, npair; float scale; bool small;
  AVSR_DEV AttnDrop(float p, uint64_t seed_, int B, int H, int Lq, int Lk) {
    seed = seed_;
    thr = (uint32_t)(p * 65536.f + 0.5f);
    scale = thr < 65536u ? 65536.f / (float)(65536u - thr) : 0.f;
    npair = (uint32_t)((Lk + 1) >> 1);
    small = (uint64_t)B * H * Lq * npair <= 0xFFFFFFFFull;
    pre = mix32_hi(seed, 0u);
  }
  AVSR_DEV uint64_t index(int bh, int Lq, int q, int k) const {
    return ((uint64_t)bh * Lq + q) * npair + (uint32_t)(k >> 1);
  }
  AVSR_DEV uint32_t hash(uint64_t g) const { return small ? mix32_lo(pre, (uint32_t)g) : mix32(seed, g); }
  AVSR_DEV float keep(uint32_t h, int k) const {
    const uint32_t u = (k & 1) ? (h >> 16) : (h & 0xFFFFu);
    return u >= thr ? scale : 0.f;
  }
  AVSR_DEV float at(int bh, int Lq, int q, int k) const { return keep(hash(index(bh, Lq, q, k)), k); }
};

struct AttnArgs {
  int B, H, Lq, Lk; float scale;
  const void* q; int64_t ldq; const void* k; int64_t ldk; const void* v; int64_t ldv;
  void* o; int64_t ldo; float* lse; const int* klen; int causal; float drop_p; uint64_t seed;
  const void* dout; int64_t lddo; float* delta; float* dq; int64_t lddq;
  void* dk; int64_t lddk; void* dv; int64_t lddv;
  const uint64_t* mq;           // dropout keep masks (avsr_attn_dropmask, query on the lane) or null
  int mnqb, mnkb;               // their 32-row query blocks / (even) 32-row key blocks per head
};

template <typename T> struct L {
  static constexpr int VE = 16 / (int)sizeof(T);
  static constexpr int KROW = DH + VE;                       // [rows][64] tiles, b128-aligned rows
  static constexpr int VROW = 32 + (sizeof(T) == 2 ? 8 : 4); // [64][32] transposed tiles
};

// write a pair of accumulator tiles X[dt] (rows d = dt*32 + qrow, column = lane&31) transposed
// (out row = column index) through the wave's LDS slab st[32][65]; rows r0.. of out
template <typename T>
AVSR_DEV void store_t(const f32x16& x0, const f32x16& x1, float mul, float* st, T* out, int64_t ld, int nvalid) {
  const int l = threadIdx.x & 63, c = l & 31, hh = l >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    st[c * 65 + qrow(r, hh)] = x0[r] * mul;
    st[c * 65 + 32 + qrow(r, hh)] = x1[r] * mul;
  }
  __syncthreads();
  // each store instruction writes whole 128-byte (bf16) / 256-byte (fp32) output rows: lane l
  // takes row i0 + l / LPR, elements (l % LPR) * VE ..; the slab reads are conflict-free (row
  // stride 65 floats)
  constexpr int VE = 16 / (int)sizeof(T), LPR = 64 / VE, RPI = 64 / LPR;
  const int rr = l / LPR, ch = (l % LPR) * VE;
#pragma unroll
  for (int i0 = 0; i0 < 32; i0 += RPI) {
    const int i = i0 + rr;
    if (i < nvalid) {
      float v[VE];
#pragma unroll
      for (int j = 0; j < VE; ++j) v[j] = st[i * 65 + ch + j];
      stv(out + (int64_t)i * ld + ch, v);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs a) {
  constexpr int VE = L<T>::VE, KROW = L<T>::KROW, VROW = L<T>::VROW;
  __shared__ __attribute__((aligned(16))) T Ks[32 * KROW];
  __shared__ __attribute__((aligned(16))) T Vt[DH * VROW];
  __shared__ __attribute__((aligned(16))) float Os[4 * 32 * 65];
  const int b = blockIdx.y / a.H, h = blockIdx.y % a.H;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, c = l & 31, hh = l >> 5;
  const int q0 = blockIdx.x * 128 + w * 32, qi = q0 + c;
  const T* Q = (const T*)a.q + (int64_t)b * a.Lq * a.ldq + h * DH;
  const T* K = (const T*)a.k + (int64_t)b * a.Lk * a.ldk + h * DH;
  const T* V = (const T*)a.v + (int64_t)b * a.Lk * a.ldv + h * DH;
  Frag qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = qi < a.Lq ? ld8<T>(Q + (int64_t)qi * a.ldq + s * 16 + 8 * hh) : zfrag<T>();
  f32x16 o0, o1;
  zacc(o0); zacc(o1);
  float m = -INFINITY, lsum = 0.f;
  const int klen = a.klen ? min(a.klen[b], a.Lk) : a.Lk;
  int kend = klen;
  if (a.causal) kend = min(kend, (int)blockIdx.x * 128 + 128);
  const float sl2 = a.scale * LOG2E;
  const AttnDrop drop(a.drop_p, a.seed, a.B, a.H, a.Lq, a.Lk);
  for (int kt0 = 0; kt0 < kend; kt0 += 32) {
    __syncthreads();
    for (int v = tid; v < 32 * DH / VE; v += 256) {
      const int key = v / (DH / VE), dv = (v % (DH / VE)) * VE;
      v16 kv, vv;
      if (kt0 + key < a.Lk) {
        kv = *(const v16*)(K + (int64_t)(kt0 + key) * a.ldk + dv);
        vv = *(const v16*)(V + (int64_t)(kt0 + key) * a.ldv + dv);
      } else {
        kv.w[0] = kv.w[1] = kv.w[2] = kv.w[3] = 0u; vv = kv;
      }
      *(v16*)&Ks[key * KROW + dv] = kv;
      const T* ve = (const T*)&vv;
#pragma unroll
      for (int e = 0; e < VE; ++e) Vt[(dv + e) * VROW + key] = ve[e];
    }
    __syncthreads();
    f32x16 st;
    zacc(st);
#pragma unroll
    for (int s = 0; s < 4; ++s) mm<T>(st, ld8<T>(&Ks[c * KROW + s * 16 + 8 * hh]), qf[s]);
    float mt = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kt0 + qrow(r, hh);
      const bool ok = key < klen && (!a.causal || key <= qi);
      st[r] = ok ? st[r] * sl2 : -INFINITY;
      mt = fmaxf(mt, st[r]);
    }
    mt = xor32_max(mt);
    const float mn = fmaxf(m, mt);
    const float alpha = mn == -INFINITY ? 1.f : exp2f(m - mn);
    float ps = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = st[r] == -INFINITY ? 0.f : exp2f(st[r] - mn);
      ps += p;
      st[r] = p;
    }
    ps = xor32_sum(ps);
    lsum = lsum * alpha + ps;
    m = mn;
#pragma unroll
    for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
    if (a.drop_p > 0.f) {
#pragma unroll
      for (int r = 0; r < 16; ++r) st[r] *= drop.at(b * a.H + h, a.Lq, qi, kt0 + qrow(r, hh));
    }
    const Frag pf0 = accfrag<T, 0>(st), pf1 = accfrag<T, 1>(st);
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      const T* row = &Vt[(dt * 32 + c) * VROW + 4 * hh];
      const Frag v0 = ld4x2<T>(row, row + 8), v1 = ld4x2<T>(row + 16, row + 24);
      if (dt == 0) { mm<T>(o0, v0, pf0); mm<T>(o0, v1, pf1); }
      else { mm<T>(o1, v0, pf0); mm<T>(o1, v1, pf1); }
    }
  }
  const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
  if (hh == 0 && qi < a.Lq) a.lse[(int64_t)(b * a.H + h) * a.Lq + qi] = lsum > 0.f ? (m + log2f(lsum)) * LN2 : -INFINITY;
  T* O = (T*)a.o + ((int64_t)b * a.Lq + q0) * a.ldo + h * DH;
  store_t<T>(o0, o1, inv, Os + w * 32 * 65, O, a.ldo, a.Lq - q0);
}

// delta[b][h][i] = sum_d dO * O
template <typename T>
__global__ __launch_bounds__(256) void attn_prep_kernel(AttnArgs a) {
  constexpr int VE = L<T>::VE;
  const int64_t n = (int64_t)a.B * a.Lq * a.H;
  for (int64_t t = blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    const int h = (int)(t % a.H);
    const int64_t row = t / a.H;                 // b*Lq + i
    const T* o = (const T*)a.o + row * a.ldo + h * DH;
    const T* d = (const T*)a.dout + row * a.lddo + h * DH;
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < DH; e += VE) {
      float x[VE], y[VE];
      ldv(o + e, x); ldv(d + e, y);
#pragma unroll
      for (int j = 0; j < VE; ++j) s += x[j] * y[j];
    }
    const int64_t b = row / a.Lq, i = row % a.Lq;
    a.delta[(b * a.H + h) * a.Lq + i] = s;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void attn_bwd_kernel(AttnArgs a) {
  constexpr int VE = L<T>::VE, KROW = L<T>::KROW, VROW = L<T>::VROW, SROW = 32 + VE;
  __shared__ __attribute__((aligned(16))) T Qs[32 * KROW];
  __shared__ __attribute__((aligned(16))) T QsT[DH * VROW];
  __shared__ __attribute__((aligned(16))) T dOs[32 * KROW];
  __shared__ __attribute__((aligned(16))) T dOsT[DH * VROW];
  __shared__ __attribute__((aligned(16))) T dSs[4 * 32 * SROW];
  __shared__ __attribute__((aligned(16))) float red[4 * 32 * 65];
  __shared__ float lse_s[32], dl_s[32];
  const int b = blockIdx.y / a.H, h = blockIdx.y % a.H;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, c = l & 31, hh = l >> 5;
  const int kb0 = blockIdx.x * 128 + w * 32, key = kb0 + c;
  const T* Q = (const T*)a.q + (int64_t)b * a.Lq * a.ldq + h * DH;
  const T* K = (const T*)a.k + (int64_t)b * a.Lk * a.ldk + h * DH;
  const T* V = (const T*)a.v + (int64_t)b * a.Lk * a.ldv + h * DH;
  const T* dO = (const T*)a.dout + (int64_t)b * a.Lq * a.lddo + h * DH;
  const float* LSE = a.lse + (int64_t)(b * a.H + h) * a.Lq;
  const float* DL = a.delta + (int64_t)(b * a.H + h) * a.Lq;
  Frag kf[4], vf[4], ktf[2][2];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = key < a.Lk ? ld8<T>(K + (int64_t)key * a.ldk + s * 16 + 8 * hh) : zfrag<T>();
    vf[s] = key < a.Lk ? ld8<T>(V + (int64_t)key * a.ldv + s * 16 + 8 * hh) : zfrag<T>();
  }
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kk = kb0 + s * 16 + 8 * hh + j;
        x[j] = kk < a.Lk ? to_f(K[(int64_t)kk * a.ldk + dt * 32 + c]) : 0.f;
      }
      ktf[dt][s] = mkfrag<T>(x);
    }
  f32x16 dv0, dv1, dk0, dk1;
  zacc(dv0); zacc(dv1); zacc(dk0); zacc(dk1);
  const int klen = a.klen ? min(a.klen[b], a.Lk) : a.Lk;
  const float sl2 = a.scale * LOG2E;
  const int qstart = a.causal ? (int)blockIdx.x * 128 : 0;
  const AttnDrop drop(a.drop_p, a.seed, a.B, a.H, a.Lq, a.Lk);
  T* dsw = dSs + w * 32 * SROW;
  float* rw = red + w * 32 * 65;
  for (int qt0 = qstart; qt0 < a.Lq; qt0 += 32) {
    __syncthreads();
    for (int v = tid; v < 32 * DH / VE; v += 256) {
      const int qq = v / (DH / VE), dv = (v % (DH / VE)) * VE;
      v16 qv, ov;
      if (qt0 + qq < a.Lq) {
        qv = *(const v16*)(Q + (int64_t)(qt0 + qq) * a.ldq + dv);
        ov = *(const v16*)(dO + (int64_t)(qt0 + qq) * a.lddo + dv);
      } else {
        qv.w[0] = qv.w[1] = qv.w[2] = qv.w[3] = 0u; ov = qv;
      }
      *(v16*)&Qs[qq * KROW + dv] = qv;
      *(v16*)&dOs[qq * KROW + dv] = ov;
      const T* qe = (const T*)&qv;
      const T* oe = (const T*)&ov;
#pragma unroll
      for (int e = 0; e < VE; ++e) {
        QsT[(dv + e) * VROW + qq] = qe[e];
        dOsT[(dv + e) * VROW + qq] = oe[e];
      }
    }
    if (tid < 32) lse_s[tid] = qt0 + tid < a.Lq ? LSE[qt0 + tid] : 0.f;
    else if (tid < 64) dl_s[tid - 32] = qt0 + tid - 32 < a.Lq ? DL[qt0 + tid - 32] : 0.f;
    __syncthreads();
    f32x16 sc, dp;
    zacc(sc); zacc(dp);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      mm<T>(sc, ld8<T>(&Qs[c * KROW + s * 16 + 8 * hh]), kf[s]);
      mm<T>(dp, ld8<T>(&dOs[c * KROW + s * 16 + 8 * hh]), vf[s]);
    }
    f32x16 pp, ds;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ql = qrow(r, hh), q = qt0 + ql;
      const bool ok = q < a.Lq && key < klen && (!a.causal || key <= q);
      const float p = ok ? exp2f(sc[r] * sl2 - lse_s[ql] * LOG2E) : 0.f;
      const float keep = (a.drop_p > 0.f && ok) ? drop.at(b * a.H + h, a.Lq, q, key) : 1.f;
      ds[r] = p * (dp[r] * keep - dl_s[ql]) * a.scale;
      pp[r] = p * keep;
    }
    const Frag pf0 = accfrag<T, 0>(pp), pf1 = accfrag<T, 1>(pp);
    const Frag sf0 = accfrag<T, 0>(ds), sf1 = accfrag<T, 1>(ds);
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      const T* ro = &dOsT[(dt * 32 + c) * VROW + 4 * hh];
      const T* rq = &QsT[(dt * 32 + c) * VROW + 4 * hh];
      const Frag a0 = ld4x2<T>(ro, ro + 8), a1 = ld4x2<T>(ro + 16, ro + 24);
      const Frag b0 = ld4x2<T>(rq, rq + 8), b1 = ld4x2<T>(rq + 16, rq + 24);
      if (dt == 0) { mm<T>(dv0, a0, pf0); mm<T>(dv0, a1, pf1); mm<T>(dk0, b0, sf0); mm<T>(dk0, b1, sf1); }
      else { mm<T>(dv1, a0, pf0); mm<T>(dv1, a1, pf1); mm<T>(dk1, b0, sf0); mm<T>(dk1, b1, sf1); }
    }
    // dQ = dS K : dS through LDS (row q, column key)
#pragma unroll
    for (int r = 0; r < 16; ++r) dsw[qrow(r, hh) * SROW + c] = from_f<T>(ds[r]);
    __syncthreads();
    f32x16 dq0, dq1;
    zacc(dq0); zacc(dq1);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const Frag sa = ld8<T>(&dsw[c * SROW + s * 16 + 8 * hh]);
      mm<T>(dq0, sa, ktf[0][s]);
      mm<T>(dq1, sa, ktf[1][s]);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      rw[qrow(r, hh) * 64 + c] = dq0[r];
      rw[qrow(r, hh) * 64 + 32 + c] = dq1[r];
    }
    __syncthreads();
    for (int e = tid; e < 32 * 64; e += 256) {
      const int qq = e >> 6, d = e & 63;
      const float v = red[e] + red[32 * 65 + e] + red[2 * 32 * 65 + e] + red[3 * 32 * 65 + e];
      if (qt0 + qq < a.Lq && v != 0.f) atomicAdd(a.dq + ((int64_t)b * a.Lq + qt0 + qq) * a.lddq + h * DH + d, v);
    }
  }
  __syncthreads();
  T* DK = (T*)a.dk + ((int64_t)b * a.Lk + kb0) * a.lddk + h * DH;
  store_t<T>(dk0, dk1, 1.f, rw, DK, a.lddk, a.Lk - kb0);
  __syncthreads();
  T* DV = (T*)a.dv + ((int64_t)b * a.Lk + kb0) * a.lddv + h * DH;
  store_t<T>(dv0, dv1, 1.f, rw, DV, a.lddv, a.Lk - kb0);
}

// =====================================================================================
// bf16 streaming kernels. Each workgroup (4 waves x 32 rows of its own dimension) streams
// 64-row tiles of the other operand pair through a double-buffered LDS ring: the next
// tile's global loads are issued into registers before the current tile's MFMAs and
// written to the other ring slot after them, so one barrier per tile covers both hazards.
// Images are row-major [64][ROW]; transposed operand fragments come straight from them
// through ds_read_b64_tr_b16 (no transposed LDS stores). The backward is split in two
// kernels, dK/dV per key block and dQ per query block (each recomputes P): no atomics,
// no cross-wave reduction, dQ written once in its final dtype.
namespace v2 {
typedef short s4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v lds_s4v;

constexpr int ROW = 72;          // 144-B rows: b128 reads of 16 rows at one column hit distinct banks
constexpr int IMG = 64 * ROW;    // elements of one [64][64] tile image

struct Pref { v16 x[2]; };       // this thread's two 16-byte chunks of a tile (chunk id tid + 256 i)

AVSR_DEV void pref_load(Pref& r, const bf16* base, int64_t ld, int row0, int nrows, int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = tid + 256 * i, row = row0 + (id >> 3);
    if (row < nrows) {
      r.x[i] = *(const v16*)(base + (int64_t)row * ld + (id & 7) * 8);
    } else {
      r.x[i].w[0] = r.x[i].w[1] = r.x[i].w[2] = r.x[i].w[3] = 0u;
    }
  }
}
AVSR_DEV void pref_store(const Pref& r, bf16* img, int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = tid + 256 * i;
    *(v16*)&img[(id >> 3) * ROW + (id & 7) * 8] = r.x[i];
  }
}
// A/B fragment of mfma32 with the operand row on the lane: X[row][col .. col+7]
AVSR_DEV bf16x8 rd8(const bf16* img, int row, int col) { return *(const bf16x8*)&img[row * ROW + col]; }
// Transposed A fragment of mfma32 from a row-major image: lane l gets X^T[c0 + (l&31)][r]
// for r = r0 + 4*(l>>5) + {0..3, 8..11} — the row order of accumulator registers
// 8S..8S+7 used as a B operand (accb), so r0 = (row block of the accumulator) + 16 S.
AVSR_DEV bf16x8 rdT(const bf16* img, int r0, int c0, int lane) {
  const int hh = lane >> 5, g = (lane >> 4) & 1, i = lane & 15;
  const bf16* pa = img + (r0 + 4 * hh + (i >> 2)) * ROW + c0 + 16 * g + 4 * (i & 3);
  union { s4v s[2]; bf16x8 h; } u;
  u.s[0] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)pa);
  u.s[1] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(pa + 8 * ROW));
  return u.h;
}
// accumulator registers 8S..8S+7 as a bf16 operand fragment
AVSR_DEV bf16x8 accb(const f32x16& x, int S) {
  bf16x8 h;
#pragma unroll
  for (int j = 0; j < 8; ++j) h[j] = (bf16)x[8 * S + j];
  return h;
}
AVSR_DEV bf16x8 ldrow(const bf16* p, bool ok) {
  if (ok) return *(const bf16x8*)p;
  bf16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (bf16)0.f;
  return z;
}

// forward: per wave 32 queries on the lanes; S^T = K Q^T and O^T += V^T P^T over 64-key tiles
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 sm[4 * IMG];          // [slot][K | V]
  const int b = blockIdx.y / a.H, h = blockIdx.y % a.H;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, c = l & 31, hh = l >> 5;
  const int q0 = blockIdx.x * 128 + w * 32, qi = q0 + c;
  const bf16* Q = (const bf16*)a.q + (int64_t)b * a.Lq * a.ldq + h * DH;
  const bf16* K = (const bf16*)a.k + (int64_t)b * a.Lk * a.ldk + h * DH;
  const bf16* V = (const bf16*)a.v + (int64_t)b * a.Lk * a.ldv + h * DH;
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = ldrow(Q + (int64_t)qi * a.ldq + s * 16 + 8 * hh, qi < a.Lq);
  f32x16 o0, o1;
  zacc(o0); zacc(o1);
  float m = -INFINITY, lsum = 0.f;
  const int klen = a.klen ? min(a.klen[b], a.Lk) : a.Lk;
  int kend = klen;
  if (a.causal) kend = min(kend, (int)blockIdx.x * 128 + 128);
  const int nt = (kend + 63) / 64;
  const float sl2 = a.scale * LOG2E;
  const AttnDrop drop(a.drop_p, a.seed, a.B, a.H, a.Lq, a.Lk);
  Pref pk, pv;
  if (nt > 0) {
    pref_load(pk, K, a.ldk, 0, a.Lk, tid); pref_load(pv, V, a.ldv, 0, a.Lk, tid);
    pref_store(pk, sm, tid); pref_store(pv, sm + IMG, tid);
  }
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int kt0 = t * 64;
    const bf16* Ks = sm + (t & 1) * 2 * IMG;
    const bf16* Vs = Ks + IMG;
    if (t + 1 < nt) { pref_load(pk, K, a.ldk, kt0 + 64, a.Lk, tid); pref_load(pv, V, a.ldv, kt0 + 64, a.Lk, tid); }
    f32x16 s0, s1;
    zacc(s0); zacc(s1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      s0 = mfma32(rd8(Ks, c, s * 16 + 8 * hh), qf[s], s0);
      s1 = mfma32(rd8(Ks, 32 + c, s * 16 + 8 * hh), qf[s], s1);
    }
    const bool full = kt0 + 64 <= klen && !a.causal;
    float mt = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float x0 = s0[r] * sl2, x1 = s1[r] * sl2;
      if (!full) {
        const int k0 = kt0 + qrow(r, hh), k1 = k0 + 32;
        if (!(k0 < klen && (!a.causal || k0 <= qi))) x0 = -INFINITY;
        if (!(k1 < klen && (!a.causal || k1 <= qi))) x1 = -INFINITY;
      }
      s0[r] = x0; s1[r] = x1;
      mt = fmaxf(mt, fmaxf(x0, x1));
    }
    mt = xor32_max(mt);
    const float mn = fmaxf(m, mt);
    const float mb = mn == -INFINITY ? 0.f : mn;
    const float alpha = exp2f(m - mb);
    float ps = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p0 = exp2f(s0[r] - mb), p1 = exp2f(s1[r] - mb);
      ps += p0 + p1;
      s0[r] = p0; s1[r] = p1;
    }
    ps = xor32_sum(ps);
    lsum = lsum * alpha + ps;
    m = mn;
#pragma unroll
    for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
    if (a.drop_p > 0.f) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s0[r] *= drop.at(b * a.H + h, a.Lq, qi, kt0 + qrow(r, hh));
        s1[r] *= drop.at(b * a.H + h, a.Lq, qi, kt0 + 32 + qrow(r, hh));
      }
    }
    const bf16x8 p0a = accb(s0, 0), p0b = accb(s0, 1), p1a = accb(s1, 0), p1b = accb(s1, 1);
    o0 = mfma32(rdT(Vs, 0, 0, l), p0a, o0);
    o0 = mfma32(rdT(Vs, 16, 0, l), p0b, o0);
    o0 = mfma32(rdT(Vs, 32, 0, l), p1a, o0);
    o0 = mfma32(rdT(Vs, 48, 0, l), p1b, o0);
    o1 = mfma32(rdT(Vs, 0, 32, l), p0a, o1);
    o1 = mfma32(rdT(Vs, 16, 32, l), p0b, o1);
    o1 = mfma32(rdT(Vs, 32, 32, l), p1a, o1);
    o1 = mfma32(rdT(Vs, 48, 32, l), p1b, o1);
    if (t + 1 < nt) {
      bf16* nx = sm + ((t + 1) & 1) * 2 * IMG;
      pref_store(pk, nx, tid); pref_store(pv, nx + IMG, tid);
    }
    __syncthreads();
  }
  const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
  if (hh == 0 && qi < a.Lq) a.lse[(int64_t)(b * a.H + h) * a.Lq + qi] = lsum > 0.f ? (m + log2f(lsum)) * LN2 : -INFINITY;
  bf16* O = (bf16*)a.o + ((int64_t)b * a.Lq + q0) * a.ldo + h * DH;
  store_t<bf16>(o0, o1, inv, (float*)sm + w * 32 * 65, O, a.ldo, a.Lq - q0);
}

// dK / dV: per wave 32 keys on the lanes (K, V rows in registers); 64-query tiles of Q, dO
// (+ lse, delta) streamed; S = Q K^T, dP = dO V^T, dV^T += dO^T P', dK^T += Q^T dS
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 sm[4 * IMG];          // [slot][Q | dO]
  __shared__ float lss[2][64], dls[2][64];
  const int b = blockIdx.y / a.H, h = blockIdx.y % a.H;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, c = l & 31, hh = l >> 5;
  const int kb0 = blockIdx.x * 128 + w * 32, key = kb0 + c;
  const bf16* Q = (const bf16*)a.q + (int64_t)b * a.Lq * a.ldq + h * DH;
  const bf16* K = (const bf16*)a.k + (int64_t)b * a.Lk * a.ldk + h * DH;
  const bf16* V = (const bf16*)a.v + (int64_t)b * a.Lk * a.ldv + h * DH;
  const bf16* dO = (const bf16*)a.dout + (int64_t)b * a.Lq * a.lddo + h * DH;
  const float* LSE = a.lse + (int64_t)(b * a.H + h) * a.Lq;
  const float* DL = a.delta + (int64_t)(b * a.H + h) * a.Lq;
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = ldrow(K + (int64_t)key * a.ldk + s * 16 + 8 * hh, key < a.Lk);
    vf[s] = ldrow(V + (int64_t)key * a.ldv + s * 16 + 8 * hh, key < a.Lk);
  }
  f32x16 dv0, dv1, dk0, dk1;
  zacc(dv0); zacc(dv1); zacc(dk0); zacc(dk1);
  const int klen = a.klen ? min(a.klen[b], a.Lk) : a.Lk;
  const float sl2 = a.scale * LOG2E;
  const int qstart = a.causal ? (int)blockIdx.x * 128 : 0;
  const int nt = a.Lq > qstart ? (a.Lq - qstart + 63) / 64 : 0;
  const AttnDrop drop(a.drop_p, a.seed, a.B, a.H, a.Lq, a.Lk);
  Pref pq, po;
  float lsr = 0.f, dlr = 0.f;
  auto fetch = [&](int qt0) {
    pref_load(pq, Q, a.ldq, qt0, a.Lq, tid); pref_load(po, dO, a.lddo, qt0, a.Lq, tid);
    if (tid < 64) {
      const int q = qt0 + tid;
      lsr = q < a.Lq ? LSE[q] * LOG2E : 0.f;
      dlr = q < a.Lq ? DL[q] : 0.f;
    }
  };
  auto stash = [&](int slot) {
    bf16* img = sm + slot * 2 * IMG;
    pref_store(pq, img, tid); pref_store(po, img + IMG, tid);
    if (tid < 64) { lss[slot][tid] = lsr; dls[slot][tid] = dlr; }
  };
  if (nt > 0) { fetch(qstart); stash(0); }
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int qt0 = qstart + t * 64, slot = t & 1;
    const bf16* Qs = sm + slot * 2 * IMG;
    const bf16* dOs = Qs + IMG;
    if (t + 1 < nt) fetch(qt0 + 64);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      f32x16 sc, dp;
      zacc(sc); zacc(dp);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sc = mfma32(rd8(Qs, 32 * u + c, s * 16 + 8 * hh), kf[s], sc);
        dp = mfma32(rd8(dOs, 32 * u + c, s * 16 + 8 * hh), vf[s], dp);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ql = 32 * u + qrow(r, hh), q = qt0 + ql;
        const bool ok = q < a.Lq && key < klen && (!a.causal || key <= q);
        const float p = ok ? exp2f(sc[r] * sl2 - lss[slot][ql]) : 0.f;
        const float keep = (a.drop_p > 0.f && ok) ? drop.at(b * a.H + h, a.Lq, q, key) : 1.f;
        sc[r] = p * keep;                                       // P' = dropout(P)
        dp[r] = p * (dp[r] * keep - dls[slot][ql]) * a.scale;   // dS (scaled)
      }
      const bf16x8 pa = accb(sc, 0), pb = accb(sc, 1), sa = accb(dp, 0), sb = accb(dp, 1);
      dv0 = mfma32(rdT(dOs, 32 * u, 0, l), pa, dv0);
      dv0 = mfma32(rdT(dOs, 32 * u + 16, 0, l), pb, dv0);
      dv1 = mfma32(rdT(dOs, 32 * u, 32, l), pa, dv1);
      dv1 = mfma32(rdT(dOs, 32 * u + 16, 32, l), pb, dv1);
      dk0 = mfma32(rdT(Qs, 32 * u, 0, l), sa, dk0);
      dk0 = mfma32(rdT(Qs, 32 * u + 16, 0, l), sb, dk0);
      dk1 = mfma32(rdT(Qs, 32 * u, 32, l), sa, dk1);
      dk1 = mfma32(rdT(Qs, 32 * u + 16, 32, l), sb, dk1);
    }
    if (t + 1 < nt) stash((t + 1) & 1);
    __syncthreads();
  }
  float* scr = (float*)sm + w * 32 * 65;
  bf16* DK = (bf16*)a.dk + ((int64_t)b * a.Lk + kb0) * a.lddk + h * DH;
  store_t<bf16>(dk0, dk1, 1.f, scr, DK, a.lddk, a.Lk - kb0);
  __syncthreads();
  bf16* DV = (bf16*)a.dv + ((int64_t)b * a.Lk + kb0) * a.lddv + h * DH;
  store_t<bf16>(dv0, dv1, 1.f, scr, DV, a.lddv, a.Lk - kb0);
}

// dQ: per wave 32 queries on the lanes (Q, dO rows in registers, lse / delta per lane);
// 64-key tiles of K, V streamed; S^T = K Q^T, dP^T = V dO^T, dQ^T += K^T dS^T
template <typename OutT>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnArgs a, OutT* dq, int64_t lddq) {
  __shared__ __attribute__((aligned(16))) bf16 sm[4 * IMG];          // [slot][K | V]
  const int b = blockIdx.y / a.H, h = blockIdx.y % a.H;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, c = l & 31, hh = l >> 5;
  const int q0 = blockIdx.x * 128 + w * 32, qi = q0 + c;
  const bf16* Q = (const bf16*)a.q + (int64_t)b * a.Lq * a.ldq + h * DH;
  const bf16* K = (const bf16*)a.k + (int64_t)b * a.Lk * a.ldk + h * DH;
  const bf16* V = (const bf16*)a.v + (int64_t)b * a.Lk * a.ldv + h * DH;
  const bf16* dO = (const bf16*)a.dout + (int64_t)b * a.Lq * a.lddo + h * DH;
  const bool qok = qi < a.Lq;
  bf16x8 qf[4], of[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = ldrow(Q + (int64_t)qi * a.ldq + s * 16 + 8 * hh, qok);
    of[s] = ldrow(dO + (int64_t)qi * a.lddo + s * 16 + 8 * hh, qok);
  }
  const int64_t bhq = (int64_t)(b * a.H + h) * a.Lq + qi;
  const float lq = qok ? a.lse[bhq] * LOG2E : 0.f;
  const float dl = qok ? a.delta[bhq] : 0.f;
  f32x16 dq0, dq1;
  zacc(dq0); zacc(dq1);
  const int klen = a.klen ? min(a.klen[b], a.Lk) : a.Lk;
  int kend = klen;
  if (a.causal) kend = min(kend, (int)blockIdx.x * 128 + 128);
  const int nt = (kend + 63) / 64;
  const float sl2 = a.scale * LOG2E;
  const AttnDrop drop(a.drop_p, a.seed, a.B, a.H, a.Lq, a.Lk);
  Pref pk, pv;
  if (nt > 0) {
    pref_load(pk, K, a.ldk, 0, a.Lk, tid); pref_load(pv, V, a.ldv, 0, a.Lk, tid);
    pref_store(pk, sm, tid); pref_store(pv, sm + IMG, tid);
  }
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int kt0 = t * 64;
    const bf16* Ks = sm + (t & 1) * 2 * IMG;
    const bf16* Vs = Ks + IMG;
    if (t + 1 < nt) { pref_load(pk, K, a.ldk, kt0 + 64, a.Lk, tid); pref_load(pv, V, a.ldv, kt0 + 64, a.Lk, tid); }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      f32x16 st, dpt;
      zacc(st); zacc(dpt);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        st = mfma32(rd8(Ks, 32 * u + c, s * 16 + 8 * hh), qf[s], st);
        dpt = mfma32(rd8(Vs, 32 * u + c, s * 16 + 8 * hh), of[s], dpt);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kk = kt0 + 32 * u + qrow(r, hh);
        const bool ok = kk < klen && (!a.causal || kk <= qi);
        const float p = ok ? exp2f(st[r] * sl2 - lq) : 0.f;
        const float keep = (a.drop_p > 0.f && ok) ? drop.at(b * a.H + h, a.Lq, qi, kk) : 1.f;
        dpt[r] = p * (dpt[r] * keep - dl) * a.scale;
      }
      const bf16x8 sa = accb(dpt, 0), sb = accb(dpt, 1);
      dq0 = mfma32(rdT(Ks, 32 * u, 0, l), sa, dq0);
      dq0 = mfma32(rdT(Ks, 32 * u + 16, 0, l), sb, dq0);
      dq1 = mfma32(rdT(Ks, 32 * u, 32, l), sa, dq1);
      dq1 = mfma32(rdT(Ks, 32 * u + 16, 32, l), sb, dq1);
    }
    if (t + 1 < nt) {
      bf16* nx = sm + ((t + 1) & 1) * 2 * IMG;
      pref_store(pk, nx, tid); pref_store(pv, nx + IMG, tid);
    }
    __syncthreads();
  }
  OutT* DQ = dq + ((int64_t)b * a.Lq + q0) * lddq + h * DH;
  store_t<OutT>(dq0, dq1, 1.f, (float*)sm + w * 32 * 65, DQ, lddq, a.Lq - q0);
}
}  // namespace v2


// =====================================================================================
// Resident kernels (bf16; Lk or Lq <= 384: the encoder's 375-frame attention, the decoder's
// self / source attention). One workgroup per (batch, head) and 32-row block range: the
// whole streamed operand pair of that head (K and V for the forward / dQ, Q and dO for
// dK / dV) is loaded into LDS ONCE (<= 2 x 384 x 144 B), then every wave (32 rows of its own
// dimension on the MFMA lanes) sweeps it with no further barrier — nothing to pipeline, waves
// drift freely, 3 waves per SIMD hide each other's MFMA / VALU / LDS latency.
//   forward: exact two-pass softmax per 32-query block (pass 1: row max of S = Q K^T; pass 2:
//            P = exp2(S - max), row sum, dropout, O^T += V^T P^T) — no running-max rescale of O;
//   dK/dV:   per 32-key wave: S, dP with the key on the lane, dV^T += dO^T P', dK^T += Q^T dS;
//            delta = rowsum(dO * O) is computed here (Q/dO already in LDS) and published for dQ;
//   dQ:      per 32-query wave: S^T, dP^T, dQ^T += K^T dS^T.
// Dropout: AttnDrop pairs — in the forward / dQ layout a lane holds 4 consecutive keys of one
// query per register quad (2 hashes); in the dK/dV layout the key pair sits on lanes c, c^1,
// which split the 16 queries' hashes and swap halves (__shfl_xor 1).
namespace res {
using namespace v2;

// diagnostic only (avsr_debug_attn_stamps): per workgroup [start, after loads, after compute,
// end] s_memrealtime ticks (100 MHz) and the hardware id, written by lane 0 of wave 0 to a
// buffer of its own; no output depends on it
__device__ unsigned long long* g_stamps = nullptr;
AVSR_DEV void stamp(int slot) {
  unsigned long long* st = g_stamps;
  if (st != nullptr && threadIdx.x == 0) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    st[(blockIdx.y * gridDim.x + blockIdx.x) * 6 + slot] = t;
    if (slot == 0) {
      st[(blockIdx.y * gridDim.x + blockIdx.x) * 6 + 4] = (unsigned long long)__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
      st[(blockIdx.y * gridDim.x + blockIdx.x) * 6 + 5] = (unsigned long long)__builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11));
    }
  }
}
// the same per workgroup for a 1-D grid at buffer offset `part` x (6 x gridDim.x): the encoder
// backward's dQ (part 0) and dK / dV (part 1) kernels
AVSR_DEV void stamp_part(int slot, int part) {
  unsigned long long* st = g_stamps;
  if (st != nullptr && threadIdx.x == 0) {
    unsigned long long* o = st + ((unsigned long long)part * gridDim.x + blockIdx.x) * 6;
    o[slot] = __builtin_amdgcn_s_memrealtime();
    if (slot == 0) {
      o[4] = (unsigned long long)__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
      o[5] = (unsigned long long)__builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11));
    }
  }
}
constexpr int MAXR = 384;           // resident rows per (b, h)
constexpr int MAXW = MAXR / 32;     // waves per workgroup (768 threads)
constexpr uint32_t GOLD = 0x9E3779B1u;

AVSR_DEV void load_img(bf16* img, const bf16* src, int64_t ld, int n, int nz, int tid, int nthr) {
  for (int id = tid; id < nz * 8; id += nthr) {
    const int row = id >> 3, ch = (id & 7) * 8;
    v16 x;
    if (row < n) x = *(const v16*)(src + (int64_t)row * ld + ch);
    else x.w[0] = x.w[1] = x.w[2] = x.w[3] = 0u;
    *(v16*)&img[row * ROW + ch] = x;
  }
}

// Two [n][64] row-major operands -> two padded LDS images (rows >= n zero), every global load
// of a pass issued before any LDS write (one HBM round trip per pass of 4 vectors per thread
// per image instead of one per vector); out-of-range rows load a clamped valid row and are
// zeroed by a select, so no load sits behind a branch
constexpr int LD_IT = 4;
AVSR_DEV void load_pair(bf16* i1, const bf16* s1, int64_t ld1, bf16* i2, const bf16* s2, int64_t ld2, int n, int nz,
                        int tid, int nthr) {
  for (int base = 0; base < nz * 8; base += LD_IT * nthr) {
    v16 x1[LD_IT], x2[LD_IT];
#pragma unroll
    for (int it = 0; it < LD_IT; ++it) {
      const int id = base + it * nthr + tid, row = id >> 3, ch = (id & 7) * 8;
      const int rr = min(row, n - 1);
      x1[it] = *(const v16*)(s1 + (int64_t)rr * ld1 + ch);
      x2[it] = *(const v16*)(s2 + (int64_t)rr * ld2 + ch);
    }
#pragma unroll
    for (int it = 0; it < LD_IT; ++it) {
      const int id = base + it * nthr + tid, row = id >> 3, ch = (id & 7) * 8;
      if (id < nz * 8) {
        const bool ok = row < n;
#pragma unroll
        for (int j = 0; j < 4; ++j) { x1[it].w[j] = ok ? x1[it].w[j] : 0u; x2[it].w[j] = ok ? x2[it].w[j] : 0u; }
        *(v16*)&i1[row * ROW + ch] = x1[it];
        *(v16*)&i2[row * ROW + ch] = x2[it];
      }
    }
  }
}

// fragment row load without a branch: row index clamped by the caller's `ok`, value selected
AVSR_DEV bf16x8 ldrow_sel(const bf16* base, int64_t ld, int row, int nrows, int col) {
  const v16 x = *(const v16*)(base + (int64_t)min(row, nrows - 1) * ld + col);
  v16 y;
#pragma unroll
  for (int j = 0; j < 4; ++j) y.w[j] = row < nrows ? x.w[j] : 0u;
  return *(const bf16x8*)&y;
}

// AttnDrop's 32-bit-index form (the dispatcher guarantees B*H*Lq*ceil(Lk/2) < 2^32) with the
// golden-ratio premultiply distributed over the index: hash(g) = fmix32(g*G ^ pre) and
// g*G = rowG + (k/2)*G (mod 2^32), so per pair only an add, a xor and the finaliser remain
AVSR_DEV uint32_t hashG(uint32_t gG, uint32_t pre) { return fmix32(gG ^ pre); }
AVSR_DEV float keep16(uint32_t h, bool odd, uint32_t thr, float scale) {
  const uint32_t u = odd ? (h >> 16) : (h & 0xFFFFu);
  return u >= thr ? scale : 0.f;
}

// keep factors of a score tile held as (query on the lane, keys k0 + qrow(r, hh)): registers
// r, r+1 (r even) are keys 2j, 2j+1 of one pair; tG = ((bh*Lq + q) * npair + k0/2) * G
AVSR_DEV void drop_tile(f32x16& x, uint32_t tG, const AttnDrop& d, int hh) {
#pragma unroll
  for (int r = 0; r < 16; r += 2) {
    const uint32_t kp = (uint32_t)(((r & 3) >> 1) + 4 * (r >> 2) + 2 * hh);     // (qrow(r, hh) >> 1)
    const uint32_t h = hashG(tG + kp * GOLD, d.pre);
    x[r] *= keep16(h, false, d.thr, d.scale);
    x[r + 1] *= keep16(h, true, d.thr, d.scale);
  }
}
// same mask, selection form: dropped elements -> 0, kept ones unscaled (the 1/(1-p) factor is
// applied once to the tile's output sums by the caller)
AVSR_DEV void drop_tile_sel(f32x16& x, uint32_t tG, const AttnDrop& d, int hh) {
#pragma unroll
  for (int r = 0; r < 16; r += 2) {
    const uint32_t kp = (uint32_t)(((r & 3) >> 1) + 4 * (r >> 2) + 2 * hh);     // (qrow(r, hh) >> 1)
    const uint32_t h = hashG(tG + kp * GOLD, d.pre);
    x[r] = (h & 0xFFFFu) >= d.thr ? x[r] : 0.f;
    x[r + 1] = (h >> 16) >= d.thr ? x[r + 1] : 0.f;
  }
}

// stored dropout masks (avsr_attn_dropmask): 16 lane masks per 32 x 32 tile, read through the
// constant address space so that a wave-uniform tile address becomes scalar loads
typedef const __attribute__((address_space(4))) uint64_t* smask_t;
AVSR_DEV smask_t mask_tile(const uint64_t* base, int64_t tile) { return (smask_t)(base + tile * 16); }
// x on the lanes whose bit of m is set, else 0: one v_cndmask with the scalar mask as condition
AVSR_DEV float msel(float x, uint64_t m) {
  float r;
  asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(r) : "v"(x), "s"(m));
  return r;
}

__global__ __launch_bounds__(768) void attn_fwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) bf16 sm[];
  stamp(0);
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const int tid = threadIdx.x, nthr = blockDim.x, w = tid >> 6, l = tid & 63, c = l & 31, hh = l >> 5;
  const int nk = (a.Lk + 31) & ~31;
  bf16* Ks = sm;
  bf16* Vs = sm + nk * ROW;
  const int q0 = (blockIdx.y * (nthr >> 6) + w) * 32, qi = q0 + c;
  const bf16* Q = (const bf16*)a.q + (int64_t)b * a.Lq * a.ldq + h * DH;
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = ldrow_sel(Q, a.ldq, qi, a.Lq, s * 16 + 8 * hh);
  // K/V images: when one pass of LD_IT vectors per thread covers them, all loads are issued
  // here and the images are written round by round inside the tile loop (round r = rows
  // [r*nthr/8, (r+1)*nthr/8)), so later rounds' HBM latency hides behind the first tiles'
  // compute (one workgroup per head per CU leaves nothing else to hide it); the barriers are
  // raw s_barrier after lgkmcnt(0), which do not drain the outstanding loads
  const bf16* Kg = (const bf16*)a.k + (int64_t)b * a.Lk * a.ldk + h * DH;
  const bf16* Vg = (const bf16*)a.v + (int64_t)b * a.Lk * a.ldv + h * DH;
  const bool pipe = nk * 8 <= LD_IT * nthr;
  const int rtot = pipe ? (nk * 8 + nthr - 1) / nthr : 0;     // rounds to write (uniform)
  const int rpr = nthr >> 3;                                    // image rows per round
  v16 xk[LD_IT], xv[LD_IT];
  if (pipe) {
#pragma unroll
    for (int it = 0; it < LD_IT; ++it) {
      const int id = it * nthr + tid, rr = min(id >> 3, a.Lk - 1), ch = (id & 7) * 8;
      xk[it] = *(const v16*)(Kg + (int64_t)rr * a.ldk + ch);
      xv[it] = *(const v16*)(Vg + (int64_t)rr * a.ldv + ch);
    }
  } else {
    load_pair(Ks, Kg, a.ldk, Vs, Vg, a.ldv, a.Lk, nk, tid, nthr);
  }
  const int klen = a.klen ? min(a.klen[b], a.Lk) : a.Lk;
  const int kend = a.causal ? min(klen, q0 + 32) : klen;
  const int nt = (kend + 31) >> 5;
  const float sl2 = a.scale * LOG2E;
  const AttnDrop drop(a.drop_p, a.seed, a.B, a.H, a.Lq, a.Lk);
  const uint32_t rowG = ((uint32_t)bh * (uint32_t)a.Lq + (uint32_t)min(qi, a.Lq - 1)) * drop.npair * GOLD;
  if (!pipe) __syncthreads();
  f32x16 o0, o1;
  zacc(o0); zacc(o1);
  float lsum = 0.f;
  // reference max (log2 units, scale * log2(e) applied): -inf until the row sees a key; it only
  // moves when a tile's max exceeds it by more than 8, so P = exp2(s - mb) <= 256 and the
  // rescale of O / the row sum (exact: softmax does not depend on the reference) is rare
  float mb = -INFINITY;
  int t = 0;                                    // next key tile
#pragma unroll
  for (int it = 0; it < LD_IT; ++it) {
    if (pipe && it < rtot) {
      const int id = it * nthr + tid, row = id >> 3, ch = (id & 7) * 8;
      if (id < nk * 8) {
        const bool ok = row < a.Lk;
#pragma unroll
        for (int j = 0; j < 4; ++j) { xk[it].w[j] = ok ? xk[it].w[j] : 0u; xv[it].w[j] = ok ? xv[it].w[j] : 0u; }
        *(v16*)&Ks[row * ROW + ch] = xk[it];
        *(v16*)&Vs[row * ROW + ch] = xv[it];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (it == 0) stamp(1);
    }
    // tiles whose 32 keys are all in LDS after this round
    const int tend = (!pipe || it + 1 >= rtot) ? nt : min(nt, ((it + 1) * rpr) >> 5);
    if (q0 >= a.Lq) continue;
    // one pass, online softmax: per 32-key tile S^T = K Q^T, the row max over the tile (the
    // two lane halves hold the same query, different keys), rescale of the running O^T / row
    // sum when the max grows (per-lane scalar: the lane's accumulator column is its query),
    // P = exp2(S*scale*log2e - max), dropout, O^T += V^T P^T
    for (; t < tend; ++t) {
      f32x16 st;
      zacc(st);
#pragma unroll
      for (int s = 0; s < 4; ++s) st = mfma32(rd8(Ks, t * 32 + c, s * 16 + 8 * hh), qf[s], st);
      const bool full = t * 32 + 32 <= klen && (!a.causal || t * 32 + 31 <= q0);
      if (!full) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int k = t * 32 + qrow(r, hh);
          const bool ok = (k < klen) & (!a.causal | (k <= qi));
          st[r] = ok ? st[r] : -INFINITY;
        }
      }
      float mx[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) mx[r] = fmaxf(st[r], st[r + 8]);
#pragma unroll
      for (int w2 = 4; w2 > 0; w2 >>= 1)
#pragma unroll
        for (int r = 0; r < w2; ++r) mx[r] = fmaxf(mx[r], mx[r + w2]);
      float mt = xor32_max(mx[0]) * sl2;
      // a query with no visible key so far keeps mb = -inf (exponent reference 0) and
      // contributes exp2(-inf) = 0; the MFMAs below run for the whole wave
      const bool grow = mt > mb + 8.f;
      if (__any(grow)) {                            // wave-uniform: rare after the first tile
        const float alpha = grow ? (mb == -INFINITY ? 0.f : fexp2(mb - mt)) : 1.f;
        mb = grow ? mt : mb;
        lsum *= alpha;
#pragma unroll
        for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
      }
      const float mbu = mb == -INFINITY ? 0.f : mb;
      float ts[8];
#pragma unroll
      for (int r = 0; r < 16; ++r) st[r] = fexp2(fmaf(st[r], sl2, -mbu));     // masked keys: exp2(-inf) = 0
#pragma unroll
      for (int r = 0; r < 8; ++r) ts[r] = st[r] + st[r + 8];
#pragma unroll
      for (int w2 = 4; w2 > 0; w2 >>= 1)
#pragma unroll
        for (int r = 0; r < w2; ++r) ts[r] += ts[r + w2];
      lsum += ts[0];
      if (a.drop_p > 0.f) drop_tile_sel(st, rowG + (uint32_t)(t * 16) * GOLD, drop, hh);
      const bf16x8 pa = accb(st, 0), pb = accb(st, 1);
      o0 = mfma32(rdT(Vs, t * 32, 0, l), pa, o0);
      o0 = mfma32(rdT(Vs, t * 32 + 16, 0, l), pb, o0);
      o1 = mfma32(rdT(Vs, t * 32, 32, l), pa, o1);
      o1 = mfma32(rdT(Vs, t * 32 + 16, 32, l), pb, o1);
    }
  }
  if (q0 < a.Lq) {
    lsum = xor32_sum(lsum);
    if (hh == 0 && qi < a.Lq)
      a.lse[(int64_t)bh * a.Lq + qi] = lsum > 0.f ? (mb + log2f(lsum)) * LN2 : -INFINITY;
  }
  __syncthreads();                         // K/V images no longer read: reuse LDS as store slabs
  stamp(2);
  if (q0 < a.Lq) {
    const float inv = lsum > 0.f ? (a.drop_p > 0.f ? drop.scale : 1.f) / lsum : 0.f;
    bf16* O = (bf16*)a.o + ((int64_t)b * a.Lq + q0) * a.ldo + h * DH;
    store_t<bf16>(o0, o1, inv, (float*)sm + w * 32 * 65, O, a.ldo, a.Lq - q0);
  }
  __syncthreads();
  stamp(3);
}

// dK / dV (decoder shapes: causal self-attention, source attention), one workgroup per (b, h)
// and up to 12 waves of 32 keys; dropout hashed per key pair
__global__ __launch_bounds__(768) void attn_bwd_dkdv_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) bf16 sm[];
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const int tid = threadIdx.x, nthr = blockDim.x, l = tid & 63, c = l & 31, hh = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nq = (a.Lq + 31) & ~31;
  bf16* Qs = sm;
  bf16* dOs = sm + nq * ROW;
  float* lss = (float*)(sm + 2 * nq * ROW);          // lse * log2(e) (0 past Lq)
  float* dls = lss + nq;                              // delta (0 past Lq)
  const bf16* Q = (const bf16*)a.q + (int64_t)b * a.Lq * a.ldq + h * DH;
  const bf16* dO = (const bf16*)a.dout + (int64_t)b * a.Lq * a.lddo + h * DH;
  const int kb0 = (blockIdx.y * (nthr >> 6) + w) * 32, key = kb0 + c;
  const bf16* K = (const bf16*)a.k + (int64_t)b * a.Lk * a.ldk + h * DH;
  const bf16* V = (const bf16*)a.v + (int64_t)b * a.Lk * a.ldv + h * DH;
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = ldrow_sel(K, a.ldk, key, a.Lk, s * 16 + 8 * hh);
    vf[s] = ldrow_sel(V, a.ldv, key, a.Lk, s * 16 + 8 * hh);
  }
  // Q / dO images and delta[q] = sum_d dO * O in one pass: every load of a pass is issued
  // first; 8 consecutive lanes hold one query row (one 16-byte chunk each)
  {
    const bf16* O = (const bf16*)a.o + (int64_t)b * a.Lq * a.ldo + h * DH;
    for (int base = 0; base < nq * 8; base += LD_IT * nthr) {
      v16 xq[LD_IT], xd[LD_IT], xo[LD_IT];
      float ls[LD_IT];
#pragma unroll
      for (int it = 0; it < LD_IT; ++it) {
        const int id = base + it * nthr + tid, rr = min(id >> 3, a.Lq - 1), ch = (id & 7) * 8;
        xq[it] = *(const v16*)(Q + (int64_t)rr * a.ldq + ch);
        xd[it] = *(const v16*)(dO + (int64_t)rr * a.lddo + ch);
        xo[it] = *(const v16*)(O + (int64_t)rr * a.ldo + ch);
        ls[it] = a.lse[(int64_t)bh * a.Lq + rr];
      }
#pragma unroll
      for (int it = 0; it < LD_IT; ++it) {
        const int id = base + it * nthr + tid, q = id >> 3, ch = (id & 7) * 8;
        const bool ok = q < a.Lq;
        float sacc = 0.f;
        const bf16x8 ov = *(const bf16x8*)&xo[it], dv = *(const bf16x8*)&xd[it];
#pragma unroll
        for (int j = 0; j < 8; ++j) sacc += (float)ov[j] * (float)dv[j];
        sacc = ok ? sacc : 0.f;
        sacc += __shfl_xor(sacc, 1, 64);
        sacc += __shfl_xor(sacc, 2, 64);
        sacc += __shfl_xor(sacc, 4, 64);
        if (id < nq * 8) {
#pragma unroll
          for (int j = 0; j < 4; ++j) { xq[it].w[j] = ok ? xq[it].w[j] : 0u; xd[it].w[j] = ok ? xd[it].w[j] : 0u; }
          *(v16*)&Qs[q * ROW + ch] = xq[it];
          *(v16*)&dOs[q * ROW + ch] = xd[it];
          if ((id & 7) == 0) {
            dls[q] = sacc;
            lss[q] = ok ? ls[it] * LOG2E : 0.f;
            if (blockIdx.y == 0 && ok) a.delta[(int64_t)bh * a.Lq + q] = sacc;
          }
        }
      }
    }
  }
  const int klen = a.klen ? min(a.klen[b], a.Lk) : a.Lk;
  const float sl2 = a.scale * LOG2E;
  const bool drop_on = a.drop_p > 0.f;
  uint32_t thr = 0, pre = 0, nG = 0, keyG = 0;
  float dscale = 1.f;
  if (drop_on) {
    const AttnDrop drop(a.drop_p, a.seed, a.B, a.H, a.Lq, a.Lk);
    dscale = drop.scale;
    thr = drop.thr; pre = drop.pre; nG = drop.npair * GOLD;
    keyG = ((uint32_t)bh * (uint32_t)a.Lq * drop.npair + (uint32_t)(min(key, a.Lk - 1) >> 1)) * GOLD;
  }
  const bool odd = c & 1;
  __syncthreads();
  f32x16 dv0, dv1, dk0, dk1;
  zacc(dv0); zacc(dv1); zacc(dk0); zacc(dk1);
  if (kb0 < a.Lk && kb0 < klen) {
    const int qstart = a.causal ? kb0 : 0;
    const int nt = (a.Lq - qstart + 31) >> 5;
    const bool kok = key < klen;
    for (int t = 0; t < nt; ++t) {
      const int qt0 = qstart + t * 32;
      f32x16 sc, dp;
      zacc(sc); zacc(dp);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sc = mfma32(rd8(Qs, qt0 + c, s * 16 + 8 * hh), kf[s], sc);
        dp = mfma32(rd8(dOs, qt0 + c, s * 16 + 8 * hh), vf[s], dp);
      }
      const uint32_t tG = keyG + (uint32_t)(qt0 + 4 * hh) * nG;
      const bool full = kok && qt0 + 32 <= a.Lq && (!a.causal || key <= qt0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {                 // registers 4i..4i+3 = queries qt0 + 8i + 4hh + 0..3
        const f32x4 ls = *(const f32x4*)&lss[qt0 + 8 * i + 4 * hh];
        const f32x4 ds = *(const f32x4*)&dls[qt0 + 8 * i + 4 * hh];
        // P' = dropout(P) is stored unscaled (the 1/(1-p) factor goes on dV at the store),
        // dP' = dropout(dP) scaled; the softmax scale of dS goes on dK at the store
        {
          // hashed dropout: this lane pair (keys 2j, 2j+1) splits the 4 queries' hashes: even
          // lanes hash queries 0, 1, odd lanes 2, 3, then the two swap (static registers only)
          bool kb[4] = {true, true, true, true};
          if (drop_on) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              const uint32_t mine = hashG(tG + (uint32_t)(8 * i + (odd ? 2 : 0) + u) * nG, pre);
              const uint32_t other = __shfl_xor(mine, 1, 64);
              const uint32_t h0 = odd ? other : mine, h1 = odd ? mine : other;
              kb[u] = (odd ? (h0 >> 16) : (h0 & 0xFFFFu)) >= thr;
              kb[u + 2] = (odd ? (h1 >> 16) : (h1 & 0xFFFFu)) >= thr;
            }
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 4 * i + e, ql = qt0 + 8 * i + 4 * hh + e;
            const bool ok = full || (kok & (ql < a.Lq) & (!a.causal | (key <= ql)));
            const float p = ok ? fexp2(fmaf(sc[r], sl2, -ls[e])) : 0.f;
            sc[r] = kb[e] ? p : 0.f;
            dp[r] = p * fmaf(kb[e] ? dp[r] : 0.f, dscale, -ds[e]);
          }
        }
      }
      const bf16x8 pa = accb(sc, 0), pb = accb(sc, 1), sa = accb(dp, 0), sb = accb(dp, 1);
      dv0 = mfma32(rdT(dOs, qt0, 0, l), pa, dv0);
      dv0 = mfma32(rdT(dOs, qt0 + 16, 0, l), pb, dv0);
      dv1 = mfma32(rdT(dOs, qt0, 32, l), pa, dv1);
      dv1 = mfma32(rdT(dOs, qt0 + 16, 32, l), pb, dv1);
      dk0 = mfma32(rdT(Qs, qt0, 0, l), sa, dk0);
      dk0 = mfma32(rdT(Qs, qt0 + 16, 0, l), sb, dk0);
      dk1 = mfma32(rdT(Qs, qt0, 32, l), sa, dk1);
      dk1 = mfma32(rdT(Qs, qt0 + 16, 32, l), sb, dk1);
    }
  }
  __syncthreads();
  if (kb0 < a.Lk) {
    float* scr = (float*)sm + w * 32 * 65;
    bf16* DK = (bf16*)a.dk + ((int64_t)b * a.Lk + kb0) * a.lddk + h * DH;
    store_t<bf16>(dk0, dk1, a.scale, scr, DK, a.lddk, a.Lk - kb0);
    bf16* DV = (bf16*)a.dv + ((int64_t)b * a.Lk + kb0) * a.lddv + h * DH;
    store_t<bf16>(dv0, dv1, dscale, scr, DV, a.lddv, a.Lk - kb0);
  }
}

// dQ (decoder shapes), one workgroup per (b, h) and up to 12 waves of 32 queries
template <typename OutT>
__global__ __launch_bounds__(768) void attn_bwd_dq_kernel(AttnArgs a, OutT* dq, int64_t lddq) {
  extern __shared__ __attribute__((aligned(16))) bf16 sm[];
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const int tid = threadIdx.x, nthr = blockDim.x, l = tid & 63, c = l & 31, hh = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nk = (a.Lk + 31) & ~31;
  bf16* Ks = sm;
  bf16* Vs = sm + nk * ROW;
  const int q0 = (blockIdx.y * (nthr >> 6) + w) * 32, qi = q0 + c;
  const bool qok = qi < a.Lq;
  const bf16* Q = (const bf16*)a.q + (int64_t)b * a.Lq * a.ldq + h * DH;
  const bf16* dO = (const bf16*)a.dout + (int64_t)b * a.Lq * a.lddo + h * DH;
  bf16x8 qf[4], of[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = ldrow_sel(Q, a.ldq, qi, a.Lq, s * 16 + 8 * hh);
    of[s] = ldrow_sel(dO, a.lddo, qi, a.Lq, s * 16 + 8 * hh);
  }
  const int64_t bhq = (int64_t)bh * a.Lq + min(qi, a.Lq - 1);
  const float lq0 = a.lse[bhq], dl0 = a.delta[bhq];
  load_pair(Ks, (const bf16*)a.k + (int64_t)b * a.Lk * a.ldk + h * DH, a.ldk,
            Vs, (const bf16*)a.v + (int64_t)b * a.Lk * a.ldv + h * DH, a.ldv, a.Lk, nk, tid, nthr);
  const float lq = qok ? lq0 * LOG2E : 0.f;
  const float dl = qok ? dl0 : 0.f;
  const int klen = a.klen ? min(a.klen[b], a.Lk) : a.Lk;
  const int kend = a.causal ? min(klen, q0 + 32) : klen;
  const int nt = (kend + 31) >> 5;
  const float sl2 = a.scale * LOG2E;
  const AttnDrop drop(a.drop_p, a.seed, a.B, a.H, a.Lq, a.Lk);
  const uint32_t rowG = ((uint32_t)bh * (uint32_t)a.Lq + (uint32_t)min(qi, a.Lq - 1)) * drop.npair * GOLD;
  const float dscale = drop.scale;
  __syncthreads();
  f32x16 dq0, dq1;
  zacc(dq0); zacc(dq1);
  if (q0 < a.Lq) {
    for (int t = 0; t < nt; ++t) {
      f32x16 st, dpt;
      zacc(st); zacc(dpt);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        st = mfma32(rd8(Ks, t * 32 + c, s * 16 + 8 * hh), qf[s], st);
        dpt = mfma32(rd8(Vs, t * 32 + c, s * 16 + 8 * hh), of[s], dpt);
      }
      // dP' = dropout(dP): kept elements scaled by 1/(1-p) (dscale), dropped ones 0; the
      // softmax scale of dS is applied to dQ once, at the store
      if (a.drop_p > 0.f) {
#pragma unroll
        for (int r = 0; r < 16; ++r) dpt[r] *= dscale;
        drop_tile_sel(dpt, rowG + (uint32_t)(t * 16) * GOLD, drop, hh);
      }
      if (t * 32 + 32 <= klen && (!a.causal || t * 32 + 31 <= q0)) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fexp2(fmaf(st[r], sl2, -lq));
          dpt[r] = p * (dpt[r] - dl);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int k = t * 32 + qrow(r, hh);
          const bool ok = (k < klen) & (!a.causal | (k <= qi));
          const float p = ok ? fexp2(fmaf(st[r], sl2, -lq)) : 0.f;
          dpt[r] = p * (dpt[r] - dl);
        }
      }
      const bf16x8 sa = accb(dpt, 0), sb = accb(dpt, 1);
      dq0 = mfma32(rdT(Ks, t * 32, 0, l), sa, dq0);
      dq0 = mfma32(rdT(Ks, t * 32 + 16, 0, l), sb, dq0);
      dq1 = mfma32(rdT(Ks, t * 32, 32, l), sa, dq1);
      dq1 = mfma32(rdT(Ks, t * 32 + 16, 32, l), sb, dq1);
    }
  }
  __syncthreads();
  if (q0 < a.Lq) {
    OutT* DQ = dq + ((int64_t)b * a.Lq + q0) * lddq + h * DH;
    store_t<OutT>(dq0, dq1, a.scale, (float*)sm + w * 32 * 65, DQ, lddq, a.Lq - q0);
  }
}

// the keep masks of avsr_attn_dropmask: workgroup (qb, bh) of 4 waves, wave w writes the lane
// masks of the tiles (bh, qb, kb = w, w + 4, ..), query on the lane (AttnDrop's bits, 0 past Lq /
// Lk). Register pair (r, r + 1) of a lane holds keys 2j, 2j + 1: one hash per pair, 32-bit
// index arithmetic, no divisions.
__global__ __launch_bounds__(256) void attn_mask_kernel(AttnArgs a, uint64_t* mq) {
  const int l = threadIdx.x & 63, c = l & 31, hh = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int qb = blockIdx.x, bh = blockIdx.y;
  const AttnDrop d(a.drop_p, a.seed, a.B, a.H, a.Lq, a.Lk);
  const int q = qb * 32 + c;
  // pair index of register pair (r, r + 1): row (bh, q), pair kb * 16 + ((r & 3) >> 1) + 4 (r >> 2) + 2 hh
  const uint32_t rowG = (((uint32_t)bh * (uint32_t)a.Lq + (uint32_t)min(q, a.Lq - 1)) * d.npair + (uint32_t)(2 * hh)) * GOLD;
  uint64_t* out = mq + ((int64_t)bh * a.mnqb + qb) * a.mnkb * 16;
  auto tile = [&](int kb, auto edge) {
    const uint32_t gG = rowG + (uint32_t)(kb * 16) * GOLD;
    // edge tiles: thresholds that reject keys past Lk and every key of a query past Lq
    const int klim = q < a.Lq ? a.Lk - kb * 32 - 4 * hh : -1;
    uint32_t wlo = 0, whi = 0;                         // lane r < 16: lane mask r
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const uint32_t hv = hashG(gG + (uint32_t)(((r & 3) >> 1) + 4 * (r >> 2)) * GOLD, d.pre);
      bool k0 = (hv & 0xFFFFu) >= d.thr, k1 = (hv >> 16) >= d.thr;
      if (edge) {
        const int kr = (r & 3) + 8 * (r >> 2);        // key offset in the tile, minus 4 hh
        k0 = k0 & (kr < klim);
        k1 = k1 & (kr + 1 < klim);
      }
      const uint64_t b0 = __ballot(k0), b1 = __ballot(k1);
      wlo = l == r ? (uint32_t)b0 : wlo;
      whi = l == r ? (uint32_t)(b0 >> 32) : whi;
      wlo = l == r + 1 ? (uint32_t)b1 : wlo;
      whi = l == r + 1 ? (uint32_t)(b1 >> 32) : whi;
    }
    if (l < 16) out[kb * 16 + l] = ((uint64_t)whi << 32) | wlo;
  };
  for (int kb = w; kb < a.mnkb; kb += 4) {
    if (qb * 32 + 32 <= a.Lq && kb * 32 + 32 <= a.Lk) tile(kb, std::false_type());
    else tile(kb, std::true_type());
  }
}

// launch geometry: waves per workgroup (<= 12) covering `rows` 32-row blocks, grid.y chunks
inline int nwaves(int rows) { const int n = (rows + 31) / 32; return n < MAXW ? n : MAXW; }
inline size_t img_lds(int rows) { return (size_t)2 * ((rows + 31) & ~31) * ROW * sizeof(bf16); }
inline size_t slab_lds(int nw) { return (size_t)nw * 32 * 65 * sizeof(float); }
inline bool small_index(const avsr_attn_params* p) {
  return (uint64_t)p->B * p->H * p->Lq * (uint64_t)((p->Lk + 1) / 2) <= 0xFFFFFFFFull;
}

// XCD-aware block order (blocks b, b + 8 share an XCD): consecutive ids on one XCD
AVSR_DEV int xcd_id(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

template <typename F> void allow_lds(F* f) {
  static bool done = false;                     // once per kernel instantiation
  if (!done) {
    (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    done = true;
  }
}
}  // namespace res

// =====================================================================================
// Tiled kernels with the streamed operand pair going through an LDS-DMA ring (bf16, non-causal,
// Lq, Lk >= 128: the encoder's self-attention). One workgroup = 4 waves x 32 rows of its own
// dimension of one (batch, head); grid = B*H x ceil(rows / 128) in XCD-remapped order (the
// blocks of one head adjacent: they share its streamed operands in one L2). 64-row tiles of the
// other dimension go HBM/L2 -> LDS by buffer_load ... lds (no staging registers, no VALU) into
// a 3-stage ring (two tiles in flight), ~48 KiB per workgroup, so three workgroups share a CU
// (12 waves) and one's load / store phases run beside the others' compute (the resident
// kernels hold a whole head, 110 KiB, per CU and serialise load -> compute -> store).
//   forward: stream K, V;   dQ: stream K, V (computes delta = rowsum(dO * O), runs first);
//   dK / dV: stream Q, dO and the 64 lse / delta values of each tile.
// LDS images are unpadded [64][64] bf16 (128-B rows) whose 16-byte chunk c of row r sits at
// c ^ swz(r), swz(r) = g ^ ((g & 1) << 2), g = (r >> 1) & 7 (applied on the DMA's global side):
// conflict-free for both fragment forms — ds_read_b128 rows on the lanes (every 16-lane bank
// group meets each (row parity, swz) once) and ds_read_b64_tr_b16 transposed reads (rows
// 4m, 4m + 2 land in opposite 64-B halves) — and every lane's fragment offsets are
// loop-invariant (tile base + compile-time row-block offsets).
namespace sq {
using namespace res;
constexpr int KT = 64;                   // rows per streamed tile
constexpr int NS = 3;                    // ring stages
constexpr int IMGB = KT * 128;           // bytes of one [64][64] bf16 image
constexpr int STAGEB = 2 * IMGB;         // two images (K | V, or Q | dO)
constexpr int STAGEB_F = STAGEB + 2 * KT * 4;   // + lse | delta of the tile (dK / dV kernel)
static_assert(4 * 32 * 65 * 4 <= NS * STAGEB, "store slabs exceed the ring");

typedef __attribute__((address_space(3))) void lds_void_t;
typedef short s4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v lds_s4v;

AVSR_DEV int swz(int row) { const int g = (row >> 1) & 7; return g ^ ((g & 1) << 2); }
// base and extent are wave-uniform at every call; readfirstlane states it, so the descriptor
// always lands in SGPRs (the DMA asm requires them)
AVSR_DEV __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  const uint64_t b = (uint64_t)(uintptr_t)base;
  const uint64_t ub = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)ub, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes),
                                           0x00020000);
}
// one wave-instruction: 64 lanes x 16 B (x4: 4 B) -> 1 KiB (256 B) of LDS at lds_wave_base.
// Inline asm as gemm_glds.h bglds16: the compiler's waitcnt pass would otherwise drain the
// ring before each transposed LDS read; the ring is ordered by explicit vmcnt waits + barriers.
AVSR_DEV void dma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, char* lds_wave_base) {
  const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void_t*)lds_wave_base);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m), "v"(voff), "s"(r)
               : "memory", "m0");
}
AVSR_DEV void dma4(__amdgpu_buffer_rsrc_t r, uint32_t voff, char* lds_wave_base) {
  const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void_t*)lds_wave_base);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds" ::"s"(m), "v"(voff), "s"(r)
               : "memory", "m0");
}
template <int N> AVSR_DEV void vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// per-lane byte offsets of the two fragment forms inside an image
struct FragOff {
  uint32_t row[4];       // b128 fragment, row on the lane: row c (+4096: rows 32..63), d-chunk 2s + hh
  uint32_t tr[2][2];     // transposed fragment of a 16-row block (+ r0 * 128): [d half][second 8 rows]
  AVSR_DEV void init(int l) {
    const int c = l & 31, hh = l >> 5, i = l & 15, gl = (l >> 4) & 1;
#pragma unroll
    for (int s = 0; s < 4; ++s) row[s] = c * 128 + (((2 * s + hh) ^ swz(c)) << 4);
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int R = 4 * hh + (i >> 2) + 8 * e, ch = 4 * cb + 2 * gl + ((i & 3) >> 1);
        tr[cb][e] = R * 128 + ((ch ^ swz(R)) << 4) + (i & 1) * 8;
      }
  }
};
AVSR_DEV bf16x8 ldA(const char* img, uint32_t off) { return *(const bf16x8*)(img + off); }
// lane l: X^T[d = 32 cb + (l & 31)][rows r0 + 4hh + {0..3, 8..11}] (see v2::rdT)
AVSR_DEV bf16x8 ldT(const char* img, int r0, const FragOff& f, int cb) {
  union { s4v s[2]; bf16x8 x; } u;
  u.s[0] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(img + r0 * 128 + f.tr[cb][0]));
  u.s[1] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(img + r0 * 128 + f.tr[cb][1]));
  return u.x;
}

// the DMA pieces of one tile: wave w moves 8-row pieces 2w, 2w+1 of both images; with fp32
// row arrays (lse, delta) waves 0 / 1 also move the tile's 64 values of one each
struct Ring {
  const bf16* s0; const bf16* s1; int64_t ld0, ld1; int n;
  const float* f0; const float* f1;
  uint32_t o0[2], o1[2];
  static constexpr int DMAS = 4;         // per wave per tile (+1 on waves 0, 1 with arrays)
  AVSR_DEV void init(const bf16* a, int64_t la, const bf16* b, int64_t lb, int n_, const float* fa, const float* fb,
                     int w, int l) {
    s0 = a; s1 = b; ld0 = la; ld1 = lb; n = n_; f0 = fa; f1 = fb;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = 8 * (2 * w + i) + (l >> 3), ch = (l & 7) ^ swz(row);
      o0[i] = (uint32_t)((row * ld0 + ch * 8) * 2);
      o1[i] = (uint32_t)((row * ld1 + ch * 8) * 2);
    }
  }
  // rows of tile t past n lie outside the buffer extent: the DMA writes zeros for them
  AVSR_DEV void issue(char* stage, int t, int w, int l) const {
    const int r0 = t * KT, nr = min(KT, n - r0);
    const __amdgpu_buffer_rsrc_t ra = rsrc(s0 + (int64_t)r0 * ld0, (uint32_t)(((nr - 1) * ld0 + DH) * 2));
    const __amdgpu_buffer_rsrc_t rb = rsrc(s1 + (int64_t)r0 * ld1, (uint32_t)(((nr - 1) * ld1 + DH) * 2));
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      dma16(ra, o0[i], stage + (2 * w + i) * 1024);
      dma16(rb, o1[i], stage + IMGB + (2 * w + i) * 1024);
    }
    if (f0 != nullptr && w < 2) {
      const float* f = w == 0 ? f0 : f1;
      dma4(rsrc(f + r0, (uint32_t)(nr * 4)), (uint32_t)(l * 4), stage + STAGEB + w * KT * 4);
    }
  }
  // wait until tile t has landed (tile t+1 may still be in flight), then the workgroup barrier
  AVSR_DEV void arrive(int t, int nt, int w) const {
    const bool more = t + 1 < nt;
    if (f0 != nullptr && w < 2) { if (more) vmwait<DMAS + 1>(); else vmwait<0>(); }
    else { if (more) vmwait<DMAS>(); else vmwait<0>(); }
    __builtin_amdgcn_s_barrier();          // tile t visible; every wave is done with tile t-1
    asm volatile("" ::: "memory");
  }
};

AVSR_DEV int next_stage(int s) { return s + 1 == NS ? 0 : s + 1; }
AVSR_DEV int prev_stage(int s) { return s == 0 ? NS - 1 : s - 1; }

// ----------------------------------------------------------------------------- forward
template <bool MASK>
__global__ __launch_bounds__(256, 3) void attn_fwd_kernel(AttnArgs a, int nqb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int id = xcd_id(blockIdx.x, gridDim.x);
  const int bh = id / nqb, qb = id - bh * nqb, b = bh / a.H, h = bh % a.H;
  const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63, c = l & 31, hh = l >> 5;
  const int q0 = qb * 128 + w * 32, qi = q0 + c;
  Ring ring;
  ring.init((const bf16*)a.k + (int64_t)b * a.Lk * a.ldk + h * DH, a.ldk,
            (const bf16*)a.v + (int64_t)b * a.Lk * a.ldv + h * DH, a.ldv, a.Lk, nullptr, nullptr, w, l);
  const int klen = a.klen ? min(a.klen[b], a.Lk) : a.Lk;
  const int nt = (klen + KT - 1) / KT;
  // tile 0's DMA, then the Q fragments; the empty asm reading them makes the compiler's own wait
  // for these loads (vmcnt(0), covering tile 0 too) happen here once instead of at their first
  // use inside the tile loop, where it would drain the ring's prefetch every tile
  if (nt > 0) ring.issue(smem, 0, w, l);
  const bf16* Q = (const bf16*)a.q + (int64_t)b * a.Lq * a.ldq + h * DH;
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = ldrow_sel(Q, a.ldq, qi, a.Lq, s * 16 + 8 * hh);
#pragma unroll
  for (int s = 0; s < 4; ++s) asm volatile("" ::"v"(qf[s]));
  if (nt > 1) ring.issue(smem + STAGEB, 1, w, l);
  FragOff fo;
  fo.init(l);
  const float sl2 = a.scale * LOG2E;
  const AttnDrop drop(a.drop_p, a.seed, a.B, a.H, a.Lq, a.Lk);
  const uint32_t rowG = MASK ? 0u : ((uint32_t)bh * (uint32_t)a.Lq + (uint32_t)min(qi, a.Lq - 1)) * drop.npair * GOLD;
  const int64_t mrow = MASK ? ((int64_t)bh * a.mnqb + (q0 >> 5)) * a.mnkb : 0;
  f32x16 o0, o1;
  zacc(o0); zacc(o1);
  float lsum = 0.f, mb = -INFINITY;          // lazy reference max, as res::attn_fwd_kernel
  int cs = 0;                                // stage of tile t
  for (int t = 0; t < nt; ++t) {
    ring.arrive(t, nt, w);
    if (t + 2 < nt) ring.issue(smem + prev_stage(cs) * STAGEB, t + 2, w, l);
    const char* Ks = smem + cs * STAGEB;
    const char* Vs = Ks + IMGB;
    uint64_t mw[32];
    if (MASK && a.drop_p > 0.f) {
      const smask_t mt = mask_tile(a.mq, mrow + 2 * t);
#pragma unroll
      for (int r = 0; r < 32; ++r) mw[r] = mt[r];
    }
    f32x16 s0, s1;
    zacc(s0); zacc(s1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      s0 = mfma32(ldA(Ks, fo.row[s]), qf[s], s0);
      s1 = mfma32(ldA(Ks + 4096, fo.row[s]), qf[s], s1);
    }
    const int k0 = t * KT;
    if (k0 + KT > klen) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s0[r] = k0 + qrow(r, hh) < klen ? s0[r] : -INFINITY;
        s1[r] = k0 + 32 + qrow(r, hh) < klen ? s1[r] : -INFINITY;
      }
    }
    // balanced trees (the 16-deep max / add chains were on the tile's dependent path)
    float mx[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) mx[r] = fmaxf(s0[r], s1[r]);
#pragma unroll
    for (int w2 = 8; w2 > 0; w2 >>= 1)
#pragma unroll
      for (int r = 0; r < w2; ++r) mx[r] = fmaxf(mx[r], mx[r + w2]);
    float mt = xor32_max(mx[0]) * sl2;
    const bool grow = mt > mb + 8.f;
    if (__any(grow)) {
      const float alpha = grow ? (mb == -INFINITY ? 0.f : fexp2(mb - mt)) : 1.f;
      mb = grow ? mt : mb;
      lsum *= alpha;
#pragma unroll
      for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
    }
    const float mbu = mb == -INFINITY ? 0.f : mb;
    float ts[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s0[r] = fexp2(fmaf(s0[r], sl2, -mbu));
      s1[r] = fexp2(fmaf(s1[r], sl2, -mbu));
      ts[r] = s0[r] + s1[r];
    }
#pragma unroll
    for (int w2 = 8; w2 > 0; w2 >>= 1)
#pragma unroll
      for (int r = 0; r < w2; ++r) ts[r] += ts[r + w2];
    lsum += ts[0];
    if (a.drop_p > 0.f) {
      if (MASK) {                            // the stored keep masks of key blocks 2t, 2t + 1
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          s0[r] = msel(s0[r], mw[r]);
          s1[r] = msel(s1[r], mw[16 + r]);
        }
      } else {
        drop_tile_sel(s0, rowG + (uint32_t)(k0 >> 1) * GOLD, drop, hh);
        drop_tile_sel(s1, rowG + (uint32_t)((k0 + 32) >> 1) * GOLD, drop, hh);
      }
    }
    const bf16x8 p0a = accb(s0, 0), p0b = accb(s0, 1), p1a = accb(s1, 0), p1b = accb(s1, 1);
    o0 = mfma32(ldT(Vs, 0, fo, 0), p0a, o0);
    o1 = mfma32(ldT(Vs, 0, fo, 1), p0a, o1);
    o0 = mfma32(ldT(Vs, 16, fo, 0), p0b, o0);
    o1 = mfma32(ldT(Vs, 16, fo, 1), p0b, o1);
    o0 = mfma32(ldT(Vs, 32, fo, 0), p1a, o0);
    o1 = mfma32(ldT(Vs, 32, fo, 1), p1a, o1);
    o0 = mfma32(ldT(Vs, 48, fo, 0), p1b, o0);
    o1 = mfma32(ldT(Vs, 48, fo, 1), p1b, o1);
    cs = next_stage(cs);
  }
  lsum = xor32_sum(lsum);
  if (hh == 0 && qi < a.Lq) a.lse[(int64_t)bh * a.Lq + qi] = lsum > 0.f ? (mb + log2f(lsum)) * LN2 : -INFINITY;
  __syncthreads();                           // the ring is free: reuse it as the store slabs
  const float inv = lsum > 0.f ? (a.drop_p > 0.f ? drop.scale : 1.f) / lsum : 0.f;
  bf16* O = (bf16*)a.o + ((int64_t)b * a.Lq + q0) * a.ldo + h * DH;
  store_t<bf16>(o0, o1, inv, (float*)smem + w * 32 * 65, O, a.ldo, a.Lq - q0);
}

}  // namespace sq

// =====================================================================================
// Encoder backward (bf16, non-causal, 128 <= Lq, Lk <= 384): one 12-wave workgroup per (b, h),
// the streamed operands of the head DMA'd (buffer_load ... lds, no staging registers) into
// unpadded XOR-swizzled [384][64] LDS images in four rounds of 96 rows that are all issued up
// front; the waves start on the first 32-row tiles while the later rounds are in flight. Every
// fragment address is a per-lane FragOff offset plus a tile base (swz(32t + x) = swz(x)).
//   dQ kernel (runs first): K, V images; per wave 32 queries (Q, dO rows in registers), delta =
//     rowsum(dO * O) from this lane's dO / O half-rows, published for the dK / dV kernel.
//   dK / dV kernel: Q, dO images, lse and delta rows, and each wave's own 32-row K image
//     (K fragments re-read per tile instead of held: the register file then holds dK, dV,
//     V and the tile without spilling at 3 waves per SIMD).
// DM: 0 no dropout, 1 hashed per element (AttnDrop), 2 stored keep masks (a.mq).
namespace rb {
using namespace sq;
constexpr int NTH = 768;                 // 12 waves
constexpr int IMG384 = MAXR * 128;       // one swizzled [384][64] bf16 image

// wave w's 8-row piece `piece` of a [n][64] operand (row stride ld) into a swizzled image; rows
// past n lie outside the buffer extent and land as zeros
AVSR_DEV void dma_piece(const bf16* base, int64_t ld, int n, char* img, int piece, int l) {
  const int row = 8 * piece + (l >> 3), ch = (l & 7) ^ swz(row);
  dma16(rsrc(base, (uint32_t)(((n - 1) * ld + DH) * 2)), (uint32_t)((row * ld + ch * 8) * 2), img + piece * 1024);
}
AVSR_DEV void round_barrier() {                    // LDS writes done, no vmcnt drain
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <typename OutT, int DM>
__global__ __launch_bounds__(NTH) void attn_bwd_dq_kernel(AttnArgs a, OutT* dq, int64_t lddq) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ks = smem;
  char* Vs = smem + IMG384;
  stamp_part(0, 0);
  const int bh = xcd_id(blockIdx.x, gridDim.x), b = bh / a.H, h = bh % a.H;
  const int tid = threadIdx.x, l = tid & 63, c = l & 31, hh = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q0 = w * 32, qi = q0 + c;
  const bool qok = qi < a.Lq;
  const bf16* Kg = (const bf16*)a.k + (int64_t)b * a.Lk * a.ldk + h * DH;
  const bf16* Vg = (const bf16*)a.v + (int64_t)b * a.Lk * a.ldv + h * DH;
  dma_piece(Kg, a.ldk, a.Lk, Ks, w, l);                    // round 0
  dma_piece(Vg, a.ldv, a.Lk, Vs, w, l);
  const bf16* Q = (const bf16*)a.q + (int64_t)b * a.Lq * a.ldq + h * DH;
  const bf16* dO = (const bf16*)a.dout + (int64_t)b * a.Lq * a.lddo + h * DH;
  const bf16* Og = (const bf16*)a.o + (int64_t)b * a.Lq * a.ldo + h * DH;
  bf16x8 qf[4], of[4], ov[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = ldrow_sel(Q, a.ldq, qi, a.Lq, s * 16 + 8 * hh);
    of[s] = ldrow_sel(dO, a.lddo, qi, a.Lq, s * 16 + 8 * hh);
    ov[s] = ldrow_sel(Og, a.ldo, qi, a.Lq, s * 16 + 8 * hh);
  }
  const int64_t bhq = (int64_t)bh * a.Lq + min(qi, a.Lq - 1);
  const float lq0 = a.lse[bhq];
  // the compiler's wait for these loads (vmcnt(0), covering round 0) happens here, once
#pragma unroll
  for (int s = 0; s < 4; ++s) asm volatile("" ::"v"(qf[s]), "v"(of[s]), "v"(ov[s]));
  asm volatile("" ::"v"(lq0));
  float dsum = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) dsum = fmaf((float)of[s][j], (float)ov[s][j], dsum);
  dsum = xor32_sum(dsum);
  if (hh == 0 && qok) a.delta[bhq] = dsum;
#pragma unroll
  for (int r = 1; r < 4; ++r) {                           // rounds 1..3 in flight from here on
    dma_piece(Kg, a.ldk, a.Lk, Ks, 12 * r + w, l);
    dma_piece(Vg, a.ldv, a.Lk, Vs, 12 * r + w, l);
  }
  const float lq = qok ? lq0 * LOG2E : 0.f;
  const float dl = qok ? dsum : 0.f;
  const int klen = a.klen ? min(a.klen[b], a.Lk) : a.Lk;
  const int nt = (klen + 31) >> 5;
  const float sl2 = a.scale * LOG2E;
  const AttnDrop drop(a.drop_p, a.seed, a.B, a.H, a.Lq, a.Lk);
  const float dscale = DM ? drop.scale : 1.f;
  const uint32_t rowG = DM == 1 ? ((uint32_t)bh * (uint32_t)a.Lq + (uint32_t)min(qi, a.Lq - 1)) * drop.npair * GOLD : 0u;
  const int64_t mrow = DM == 2 ? ((int64_t)bh * a.mnqb + w) * a.mnkb : 0;
  FragOff fo;
  fo.init(l);
  f32x16 dq0, dq1;
  zacc(dq0); zacc(dq1);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (r == 1) vmwait<4>();
    if (r == 2) vmwait<2>();
    if (r == 3) vmwait<0>();
    round_barrier();                                       // round r of every wave has landed
    if (r == 0) stamp_part(1, 0);
    if (q0 < a.Lq) {
#pragma unroll
      for (int u = 0; u < 3; ++u) {                        // unrolled: tile offsets become immediates
        const int t = 3 * r + u;
        if (t >= nt) break;
        uint64_t mw[16];
        if (DM == 2) {
          const smask_t mt = mask_tile(a.mq, mrow + t);
#pragma unroll
          for (int e = 0; e < 16; ++e) mw[e] = mt[e];
        }
        const char* Kt = Ks + t * 4096;
        const char* Vt = Vs + t * 4096;
        f32x16 st, dpt;
        zacc(st); zacc(dpt);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          st = mfma32(ldA(Kt, fo.row[s]), qf[s], st);
          dpt = mfma32(ldA(Vt, fo.row[s]), of[s], dpt);
        }
        if (t * 32 + 32 > klen) {                          // wave-uniform: keys past klen
#pragma unroll
          for (int e = 0; e < 16; ++e) st[e] = t * 32 + qrow(e, hh) < klen ? st[e] : -INFINITY;
        }
        // dP' = dropout(dP) (kept x 1/(1-p), dropped 0); the softmax scale of dS goes on dQ at the store
        if (DM == 1) {
#pragma unroll
          for (int e = 0; e < 16; ++e) dpt[e] *= dscale;
          drop_tile_sel(dpt, rowG + (uint32_t)(t * 16) * GOLD, drop, hh);
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float p = fexp2(fmaf(st[e], sl2, -lq));
          const float d = DM == 2 ? msel(dpt[e] * dscale, mw[e]) : dpt[e];   // rounding as DM 1
          dpt[e] = p * (d - dl);
        }
        const bf16x8 sa = accb(dpt, 0), sb = accb(dpt, 1);
        dq0 = mfma32(ldT(Ks, 32 * t, fo, 0), sa, dq0);
        dq0 = mfma32(ldT(Ks, 32 * t + 16, fo, 0), sb, dq0);
        dq1 = mfma32(ldT(Ks, 32 * t, fo, 1), sa, dq1);
        dq1 = mfma32(ldT(Ks, 32 * t + 16, fo, 1), sb, dq1);
      }
    }
  }
  stamp_part(2, 0);
  __syncthreads();                                         // images no longer read: store slabs
  if (q0 < a.Lq) {
    OutT* DQ = dq + ((int64_t)b * a.Lq + q0) * lddq + h * DH;
    store_t<OutT>(dq0, dq1, a.scale, (float*)smem + w * 32 * 65, DQ, lddq, a.Lq - q0);
  }
  if (g_stamps != nullptr) {
    __syncthreads();
    stamp_part(3, 0);
  }
}

template <int DM>
__global__ __launch_bounds__(NTH) void attn_bwd_dkdv_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Qs = smem;
  char* dOs = smem + IMG384;
  float* lss = (float*)(smem + 2 * IMG384);                // lse, then lse * log2(e) (0 past Lq)
  float* dls = lss + MAXR;                                 // delta (0 past Lq)
  char* Kw = smem + 2 * IMG384 + 2 * MAXR * 4;             // this wave's [32][64] K image
  stamp_part(0, 1);
  const int bh = xcd_id(blockIdx.x, gridDim.x), b = bh / a.H, h = bh % a.H;
  const int tid = threadIdx.x, l = tid & 63, c = l & 31, hh = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  Kw += w * 4096;
  const int kb0 = w * 32, key = kb0 + c;
  const bf16* Qg = (const bf16*)a.q + (int64_t)b * a.Lq * a.ldq + h * DH;
  const bf16* dOg = (const bf16*)a.dout + (int64_t)b * a.Lq * a.lddo + h * DH;
  const bf16* Kg = (const bf16*)a.k + ((int64_t)b * a.Lk + kb0) * a.ldk + h * DH;
  const bf16* V = (const bf16*)a.v + (int64_t)b * a.Lk * a.ldv + h * DH;
  // this wave's K rows (4 pieces; rows past Lk zero), round 0 of Q / dO, the lse / delta rows
  if (kb0 < a.Lk) {
#pragma unroll
    for (int i = 0; i < 4; ++i) dma_piece(Kg, a.ldk, min(32, a.Lk - kb0), Kw, i, l);
  }
  dma_piece(Qg, a.ldq, a.Lq, Qs, w, l);
  dma_piece(dOg, a.lddo, a.Lq, dOs, w, l);
  {                                                        // 6 x 64 floats of each array
    const float* f = (w < 6 ? a.lse : a.delta) + (int64_t)bh * a.Lq;
    dma4(rsrc(f, (uint32_t)(a.Lq * 4)), (uint32_t)((64 * (w % 6) + l) * 4), (char*)((w < 6 ? lss : dls) + 64 * (w % 6)));
  }
  bf16x8 vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) vf[s] = ldrow_sel(V, a.ldv, key, a.Lk, s * 16 + 8 * hh);
#pragma unroll
  for (int s = 0; s < 4; ++s) asm volatile("" ::"v"(vf[s]));    // vmcnt(0) here, covering round 0
#pragma unroll
  for (int r = 1; r < 4; ++r) {
    dma_piece(Qg, a.ldq, a.Lq, Qs, 12 * r + w, l);
    dma_piece(dOg, a.lddo, a.Lq, dOs, 12 * r + w, l);
  }
  round_barrier();
  if (tid < MAXR) lss[tid] *= LOG2E;
  const int klen = a.klen ? min(a.klen[b], a.Lk) : a.Lk;
  const bool active = kb0 < klen, kok = key < klen;
  const float sl2 = a.scale * LOG2E;
  const AttnDrop drop(a.drop_p, a.seed, a.B, a.H, a.Lq, a.Lk);
  const float dscale = DM ? drop.scale : 1.f;
  const uint32_t nG = DM == 1 ? drop.npair * GOLD : 0u;
  const uint32_t keyG = DM == 1 ? ((uint32_t)bh * (uint32_t)a.Lq * drop.npair + (uint32_t)(min(key, a.Lk - 1) >> 1)) * GOLD : 0u;
  const bool odd = c & 1;
  // DM 2: key c of this wave is bit (q & 31) + 32 hh' of lane mask r' of each (query block t, key
  // block w) tile of the query-on-the-lane masks, r' = (c & 3) + 4 (c >> 3), hh' = (c >> 2) & 1:
  // one 8-byte load per lane per tile, the half for this key, shifted to this lane's 4 hh rows
  const uint64_t* mp = DM == 2 ? a.mq + ((int64_t)bh * a.mnqb * a.mnkb + w) * 16 + ((c & 3) + 4 * (c >> 3)) : nullptr;
  const int mstride = a.mnkb * 16;
  const bool mhi = (c >> 2) & 1;
  const int nt = (a.Lq + 31) >> 5;
  FragOff fo;
  fo.init(l);
  f32x16 dv0, dv1, dk0, dk1;
  zacc(dv0); zacc(dv1); zacc(dk0); zacc(dk1);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (r == 1) vmwait<4>();
    if (r == 2) vmwait<2>();
    if (r == 3) vmwait<0>();
    round_barrier();                       // round r landed (r = 0: the lse scaling is visible)
    if (r == 0) stamp_part(1, 1);
    if (active) {
      // the round's 3 query tiles unrolled: tile offsets into the Q / dO images and the lse /
      // delta rows become instruction offsets (no per-fragment address add)
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int t = 3 * r + u;
        if (t >= nt) break;
        const int qt0 = t * 32;
        uint32_t mbits = 0;
        if (DM == 2) {
          const uint64_t m64 = mp[(int64_t)t * mstride];
          mbits = (mhi ? (uint32_t)(m64 >> 32) : (uint32_t)m64) >> (4 * hh);
        }
        const char* Qt = Qs + t * 4096;
        const char* dOt = dOs + t * 4096;
        f32x16 sc, dp;
        zacc(sc); zacc(dp);
        // K fragments re-read every tile: an opaque offset keeps the compiler from hoisting them
        // out of the loop into 16 more live registers (an integer, so the pointer stays LDS)
        uint32_t kz = 0;
        asm volatile("" : "+v"(kz));
        const char* Kt = Kw + kz;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          sc = mfma32(ldA(Qt, fo.row[s]), ldA(Kt, fo.row[s]), sc);
          dp = mfma32(ldA(dOt, fo.row[s]), vf[s], dp);
        }
        if (!(kb0 + 32 <= klen && qt0 + 32 <= a.Lq)) {     // wave-uniform: invalid keys / queries
#pragma unroll
          for (int e = 0; e < 16; ++e) sc[e] = kok & (qt0 + qrow(e, hh) < a.Lq) ? sc[e] : -INFINITY;
        }
        const uint32_t tG = keyG + (uint32_t)(qt0 + 4 * hh) * nG;
#pragma unroll
        for (int i = 0; i < 4; ++i) {                      // registers 4i..4i+3 = queries qt0 + 8i + 4hh + 0..3
          const f32x4 ls = *(const f32x4*)&lss[qt0 + 8 * i + 4 * hh];
          const f32x4 ds = *(const f32x4*)&dls[qt0 + 8 * i + 4 * hh];
          bool kb[4] = {true, true, true, true};
          if (DM == 1) {     // the key pair (2j, 2j+1) on lanes c, c^1 splits the 4 queries' hashes
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              const uint32_t mine = hashG(tG + (uint32_t)(8 * i + (odd ? 2 : 0) + u) * nG, drop.pre);
              const uint32_t other = __shfl_xor(mine, 1, 64);
              const uint32_t h0 = odd ? other : mine, h1 = odd ? mine : other;
              kb[u] = (odd ? (h0 >> 16) : (h0 & 0xFFFFu)) >= drop.thr;
              kb[u + 2] = (odd ? (h1 >> 16) : (h1 & 0xFFFFu)) >= drop.thr;
            }
          }
          // P' = dropout(P) unscaled (1/(1-p) goes on dV at the store), dS = P (dP' - delta)
          // with dP' = dropout(dP) / (1-p); the softmax scale goes on dK at the store
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r4 = 4 * i + e;
            const float p = fexp2(fmaf(sc[r4], sl2, -ls[e]));
            if (DM == 2) {
              const bool kp = (mbits >> ((r4 & 3) + 8 * (r4 >> 2))) & 1u;
              sc[r4] = kp ? p : 0.f;
              dp[r4] = p * fmaf(kp ? dp[r4] : 0.f, dscale, -ds[e]);
            } else {
              sc[r4] = kb[e] ? p : 0.f;
              dp[r4] = p * fmaf(kb[e] ? dp[r4] : 0.f, dscale, -ds[e]);
            }
          }
        }
        const bf16x8 pa = accb(sc, 0), pb = accb(sc, 1), sa = accb(dp, 0), sb = accb(dp, 1);
        dv0 = mfma32(ldT(dOs, qt0, fo, 0), pa, dv0);
        dv0 = mfma32(ldT(dOs, qt0 + 16, fo, 0), pb, dv0);
        dv1 = mfma32(ldT(dOs, qt0, fo, 1), pa, dv1);
        dv1 = mfma32(ldT(dOs, qt0 + 16, fo, 1), pb, dv1);
        dk0 = mfma32(ldT(Qs, qt0, fo, 0), sa, dk0);
        dk0 = mfma32(ldT(Qs, qt0 + 16, fo, 0), sb, dk0);
        dk1 = mfma32(ldT(Qs, qt0, fo, 1), sa, dk1);
        dk1 = mfma32(ldT(Qs, qt0 + 16, fo, 1), sb, dk1);
      }
    }
  }
  stamp_part(2, 1);
  __syncthreads();
  if (kb0 < a.Lk) {
    float* scr = (float*)smem + w * 32 * 65;
    bf16* DK = (bf16*)a.dk + ((int64_t)b * a.Lk + kb0) * a.lddk + h * DH;
    store_t<bf16>(dk0, dk1, a.scale, scr, DK, a.lddk, a.Lk - kb0);
    bf16* DV = (bf16*)a.dv + ((int64_t)b * a.Lk + kb0) * a.lddv + h * DH;
    store_t<bf16>(dv0, dv1, dscale, scr, DV, a.lddv, a.Lk - kb0);
  }
  if (g_stamps != nullptr) {
    __syncthreads();
    stamp_part(3, 1);
  }
}

constexpr size_t DQ_LDS = 2 * IMG384 > NTH / 64 * 32 * 65 * 4 ? 2 * IMG384 : NTH / 64 * 32 * 65 * 4;
constexpr size_t DKDV_LDS = 3 * IMG384 + 2 * MAXR * 4;
static_assert(DKDV_LDS <= 160 * 1024 && NTH / 64 * 32 * 65 * 4 <= DKDV_LDS, "dK/dV LDS");
}  // namespace rb

AttnArgs args(const avsr_attn_params* p) {
  AttnArgs a;
  a.B = p->B; a.H = p->H; a.Lq = p->Lq; a.Lk = p->Lk; a.scale = p->scale;
  a.q = p->q; a.ldq = p->ldq; a.k = p->k; a.ldk = p->ldk; a.v = p->v; a.ldv = p->ldv;
  a.o = p->o; a.ldo = p->ldo; a.lse = p->lse; a.klen = p->klen; a.causal = p->causal;
  a.drop_p = p->drop_p; a.seed = p->seed; a.dout = p->dout; a.lddo = p->lddo; a.delta = p->delta;
  a.dq = p->dq; a.lddq = p->lddq; a.dk = p->dk; a.lddk = p->lddk; a.dv = p->dv; a.lddv = p->lddv;
  a.mnqb = (p->Lq + 31) / 32;
  a.mnkb = 2 * ((p->Lk + 63) / 64);
  const bool m = p->drop_mask != nullptr && p->drop_p > 0.f && !p->causal && p->dtype == AVSR_BF16;
  a.mq = m ? p->drop_mask : nullptr;
  return a;
}

int check(const avsr_attn_params* p) {
  if (!p) return AVSR_E_ARG;
  const int ve = p->dtype == AVSR_BF16 ? 8 : 4;
  if (p->ldq % ve || p->ldk % ve || p->ldv % ve || p->ldo % ve) return AVSR_E_ALIGN;
  if (p->dtype != AVSR_BF16 && p->dtype != AVSR_F32) return AVSR_E_DTYPE;
  return 0;
}

}  // namespace

// diagnostic: device buffer of 6 x uint64 per workgroup for the resident forward kernel
// (nullptr: off). Not part of the product path.
extern "C" int avsr_debug_attn_stamps(unsigned long long* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(res::g_stamps), &buf, sizeof(buf));
}

// query-tiled streamed kernels for the encoder's self-attention (AVSR_OPT_ATTN_SQ_FWD = 0: the
// resident kernels, A/B runs)
static bool sq_enabled() { return avsr_opt(AVSR_OPT_ATTN_SQ_FWD) != 0; }

extern "C" int avsr_attn_fwd(const avsr_attn_params* p, void* stream) {
  int rc = check(p);
  if (rc) return rc;
  if (p->B * p->H == 0 || p->Lq == 0) return 0;
  AttnArgs a = args(p);
  if (p->dtype == AVSR_BF16 && !p->causal && p->Lq >= 128 && res::small_index(p) && sq_enabled() &&
      (p->ldk % 8) == 0 && (p->ldv % 8) == 0) {
    const int nqb = (p->Lq + 127) / 128;
    const long nwg = (long)p->B * p->H * nqb;
    if (nwg > 0x7fffffffL) return AVSR_E_SHAPE;
    if (a.mq)
      hipLaunchKernelGGL(sq::attn_fwd_kernel<true>, dim3((unsigned)nwg), dim3(256), sq::NS * sq::STAGEB, (hipStream_t)stream,
                         a, nqb);
    else
      hipLaunchKernelGGL(sq::attn_fwd_kernel<false>, dim3((unsigned)nwg), dim3(256), sq::NS * sq::STAGEB, (hipStream_t)stream,
                         a, nqb);
    AVSR_CHECK_LAUNCH();
    return 0;
  }
  if (p->dtype == AVSR_BF16 && p->Lk <= res::MAXR && res::small_index(p)) {
    const int nw = res::nwaves(p->Lq);
    const size_t lds = std::max(res::img_lds(p->Lk), res::slab_lds(nw));
    res::allow_lds(res::attn_fwd_kernel);
    dim3 g(p->B * p->H, (p->Lq + 32 * nw - 1) / (32 * nw));
    hipLaunchKernelGGL(res::attn_fwd_kernel, g, dim3(64 * nw), lds, (hipStream_t)stream, a);
    AVSR_CHECK_LAUNCH();
    return 0;
  }
  dim3 grid((p->Lq + 127) / 128, p->B * p->H);
  if (p->dtype == AVSR_BF16) hipLaunchKernelGGL(v2::attn_fwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(attn_fwd_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, a);
  AVSR_CHECK_LAUNCH();
  return 0;
}

extern "C" int avsr_attn_dropmask(const avsr_attn_params* p, void* stream) {
  if (!p || !p->drop_mask) return AVSR_E_ARG;
  if (!(p->drop_p > 0.f) || !res::small_index(p)) return AVSR_E_ARG;
  if (p->B * p->H == 0 || p->Lq == 0 || p->Lk == 0) return 0;
  avsr_attn_params q = *p;
  q.dtype = AVSR_BF16; q.causal = 0;                    // the layout args() fills for the mask readers
  AttnArgs a = args(&q);
  if ((int64_t)p->B * p->H > 65535) return AVSR_E_SHAPE;
  hipLaunchKernelGGL(res::attn_mask_kernel, dim3(a.mnqb, p->B * p->H), dim3(256), 0, (hipStream_t)stream, a,
                     const_cast<uint64_t*>(a.mq));
  AVSR_CHECK_LAUNCH();
  return 0;
}

// the encoder backward (rb::, bf16 non-causal 128..384 rows) computes delta in its dQ kernel,
// the resident bf16 backward (decoder shapes, Lq, Lk <= 384) inside its dK/dV kernel (Q / dO
// already in LDS); longer sequences take the tiled v2 kernels after avsr_attn_bwd_prep
static bool enc_bwd(const avsr_attn_params* p) {
  return p->dtype == AVSR_BF16 && !p->causal && p->Lq >= 128 && p->Lk >= 128 && p->Lq <= res::MAXR &&
         p->Lk <= res::MAXR && res::small_index(p) && (p->lddo % 8) == 0;
}
static bool resident_bwd(const avsr_attn_params* p) {
  return p->dtype == AVSR_BF16 && p->Lq <= res::MAXR && p->Lk <= res::MAXR && res::small_index(p);
}

extern "C" int avsr_attn_bwd_prep(const avsr_attn_params* p, void* stream) {
  int rc = check(p);
  if (rc) return rc;
  if (enc_bwd(p) || resident_bwd(p)) return 0;
  AttnArgs a = args(p);
  const int g = avsr_grid((int64_t)p->B * p->Lq * p->H);
  if (p->dtype == AVSR_BF16) hipLaunchKernelGGL(attn_prep_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(attn_prep_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, a);
  AVSR_CHECK_LAUNCH();
  return 0;
}

template <int DM>
static void launch_enc_bwd(const avsr_attn_params* p, const AttnArgs& a, hipStream_t st) {
  const dim3 g(p->B * p->H);
  if (p->dq_out) {
    res::allow_lds(rb::attn_bwd_dq_kernel<bf16, DM>);
    hipLaunchKernelGGL((rb::attn_bwd_dq_kernel<bf16, DM>), g, dim3(rb::NTH), rb::DQ_LDS, st, a, (bf16*)p->dq_out,
                       p->lddq_out);
  } else {
    res::allow_lds(rb::attn_bwd_dq_kernel<float, DM>);
    hipLaunchKernelGGL((rb::attn_bwd_dq_kernel<float, DM>), g, dim3(rb::NTH), rb::DQ_LDS, st, a, p->dq, p->lddq);
  }
  res::allow_lds(rb::attn_bwd_dkdv_kernel<DM>);
  hipLaunchKernelGGL(rb::attn_bwd_dkdv_kernel<DM>, g, dim3(rb::NTH), rb::DKDV_LDS, st, a);
}

static int attn_bwd_kernels(const avsr_attn_params* p, hipStream_t st) {
  AttnArgs a = args(p);
  dim3 grid((p->Lk + 127) / 128, p->B * p->H);
  if (p->dtype == AVSR_BF16) {
    if (p->dq_out && (p->lddq_out % 8 || !avsr_aligned16(p->dq_out))) return AVSR_E_ALIGN;
    if (!p->dq_out && (p->lddq % 4 || !avsr_aligned16(p->dq))) return AVSR_E_ALIGN;
    if (enc_bwd(p)) {
      if (!(p->drop_p > 0.f)) launch_enc_bwd<0>(p, a, st);
      else if (a.mq) launch_enc_bwd<2>(p, a, st);
      else launch_enc_bwd<1>(p, a, st);
      AVSR_CHECK_LAUNCH();
      return 0;
    }
    if (resident_bwd(p)) {
      // dK/dV: one workgroup per (b, h) of up to 12 waves (3 per SIMD), grid.y = 1 for L <= 384
      const int nwk = res::nwaves(p->Lk), nwq = res::nwaves(p->Lq);
      const size_t ldk = std::max(res::img_lds(p->Lq) + (size_t)2 * ((p->Lq + 31) & ~31) * sizeof(float), res::slab_lds(nwk));
      const dim3 gk(p->B * p->H, (p->Lk + 32 * nwk - 1) / (32 * nwk));
      res::allow_lds(res::attn_bwd_dkdv_kernel);
      hipLaunchKernelGGL(res::attn_bwd_dkdv_kernel, gk, dim3(64 * nwk), ldk, st, a);
      AVSR_CHECK_LAUNCH();
      const size_t ldq = std::max(res::img_lds(p->Lk), res::slab_lds(nwq));
      const dim3 gq(p->B * p->H, (p->Lq + 32 * nwq - 1) / (32 * nwq));
      if (p->dq_out) {
        res::allow_lds(res::attn_bwd_dq_kernel<bf16>);
        hipLaunchKernelGGL(res::attn_bwd_dq_kernel<bf16>, gq, dim3(64 * nwq), ldq, st, a, (bf16*)p->dq_out, p->lddq_out);
      } else {
        res::allow_lds(res::attn_bwd_dq_kernel<float>);
        hipLaunchKernelGGL(res::attn_bwd_dq_kernel<float>, gq, dim3(64 * nwq), ldq, st, a, p->dq, p->lddq);
      }
      AVSR_CHECK_LAUNCH();
      return 0;
    }
    hipLaunchKernelGGL(v2::attn_bwd_dkdv_kernel, grid, dim3(256), 0, st, a);
    AVSR_CHECK_LAUNCH();
    dim3 gq((p->Lq + 127) / 128, p->B * p->H);
    if (p->dq_out) hipLaunchKernelGGL(v2::attn_bwd_dq_kernel<bf16>, gq, dim3(256), 0, st, a, (bf16*)p->dq_out, p->lddq_out);
    else hipLaunchKernelGGL(v2::attn_bwd_dq_kernel<float>, gq, dim3(256), 0, st, a, p->dq, p->lddq);
  } else {
    hipLaunchKernelGGL(attn_bwd_kernel<float>, grid, dim3(256), 0, st, a);
  }
  AVSR_CHECK_LAUNCH();
  return 0;
}

// column sums per utterance of the stored dQ / dK / dV (the paths whose kernels do not write the
// bias partials themselves): ws[b][s][c], thread = one of the 3 * HD columns, rows in order
template <typename TQ, typename T>
__global__ __launch_bounds__(256) void attn_db_kernel(const TQ* dq, int64_t lddq, const T* dk, int64_t lddk, const T* dv,
                                                      int64_t lddv, int Lq, int Lk, int HD, float* ws) {
  const int b = blockIdx.y, col = blockIdx.x * 256 + threadIdx.x;
  if (col >= 3 * HD) return;
  const int s = col / HD, c = col % HD;
  float acc = 0.f;
  if (s == 0) {
    for (int i = 0; i < Lq; ++i) acc += (float)dq[((int64_t)b * Lq + i) * lddq + c];
  } else {
    const T* x = s == 1 ? dk : dv;
    const int64_t ld = s == 1 ? lddk : lddv;
    for (int i = 0; i < Lk; ++i) acc += (float)x[((int64_t)b * Lk + i) * ld + c];
  }
  ws[(int64_t)b * 3 * HD + col] = acc;
}

extern "C" int avsr_attn_bwd(const avsr_attn_params* p, void* stream) {
  int rc = check(p);
  if (rc) return rc;
  if (p->db && !p->db_ws) return AVSR_E_ARG;
  if (p->B * p->H == 0 || p->Lk == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  rc = attn_bwd_kernels(p, st);
  if (rc || !p->db) return rc;
  const int HD = p->H * DH;
  {
    const dim3 g((3 * HD + 255) / 256, p->B);
    if (p->dtype == AVSR_BF16 && p->dq_out)
      hipLaunchKernelGGL((attn_db_kernel<bf16, bf16>), g, dim3(256), 0, st, (const bf16*)p->dq_out, p->lddq_out,
                         (const bf16*)p->dk, p->lddk, (const bf16*)p->dv, p->lddv, p->Lq, p->Lk, HD, p->db_ws);
    else if (p->dtype == AVSR_BF16)
      hipLaunchKernelGGL((attn_db_kernel<float, bf16>), g, dim3(256), 0, st, (const float*)p->dq, p->lddq,
                         (const bf16*)p->dk, p->lddk, (const bf16*)p->dv, p->lddv, p->Lq, p->Lk, HD, p->db_ws);
    else
      hipLaunchKernelGGL((attn_db_kernel<float, float>), g, dim3(256), 0, st, (const float*)p->dq, p->lddq,
                         (const float*)p->dk, p->lddk, (const float*)p->dv, p->lddv, p->Lq, p->Lk, HD, p->db_ws);
    AVSR_CHECK_LAUNCH();
  }
  return colsum_launch(p->db_ws, p->B, (int64_t)3 * HD, 3 * HD, p->db, 0, nullptr, st);
}
