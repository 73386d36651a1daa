// K13: fused sampling. One workgroup per row of logits (vocab up to ~152k):
//   temperature <= 0        -> argmax (lowest index on ties)
//   otherwise               -> Gumbel-max over softmax(z / T) restricted to the top-k / top-p set:
//                              argmax_v (z_v / T + g_v), g_v = -log(-log u_v),
//                              u_v = hash(seed, step, v)  (counter-based: reproducible per request,
//                              graph-capturable, no RNG state).  No sort: the top-k and top-p
//                              thresholds are found by bisection over value with block reductions.
// The hash matches mxserve/ops/reference.py::_hash_u32 bit for bit.
#include <cstdlib>

#include "common.h"

namespace mxs {

__device__ __forceinline__ uint32_t hash_u32(uint32_t x) {
  x = (x ^ (x >> 16)) * 0x7FEB352Du;
  x = (x ^ (x >> 15)) * 0x846CA68Bu;
  return x ^ (x >> 16);
}

struct ArgMax {
  float v;
  int i;
};

__device__ __forceinline__ ArgMax better(ArgMax a, ArgMax b) {
  if (b.v > a.v || (b.v == a.v && b.i < a.i)) return b;
  return a;
}

__device__ ArgMax block_argmax(ArgMax a, float* sv, int* si) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax b{__shfl_xor(a.v, o, 64), __shfl_xor(a.i, o, 64)};
    a = better(a, b);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) {
    sv[wid] = a.v;
    si[wid] = a.i;
  }
  __syncthreads();
  ArgMax r{sv[0], si[0]};
  for (int w = 1; w < nw; ++w) r = better(r, ArgMax{sv[w], si[w]});
  return r;
}

__device__ __forceinline__ float ld(const float* p, int v) { return p[v]; }
__device__ __forceinline__ float ld(const bf16_t* p, int v) { return bf2f(p[v]); }

// 8 consecutive logits starting at v (v % 8 == 0, row 16-byte aligned)
__device__ __forceinline__ void ld8(const bf16_t* p, int v, float (&o)[8]) {
  const uint4 w = *reinterpret_cast<const uint4*>(p + v);
  const uint32_t u[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    o[2 * k] = bf2f_lo(u[k]);
    o[2 * k + 1] = bf2f_hi(u[k]);
  }
}
__device__ __forceinline__ void ld8(const float* p, int v, float (&o)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p + v), b = *reinterpret_cast<const float4*>(p + v + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

// Gumbel noise in base-2 units: argmax_v (z_v / T + G_v) with G = -ln(-ln u) is argmax_v of
// (z_v / T + G_v) log2(e) = z_v log2(e) / T - log2(-log2 u) + const, so the scores are taken as
// x * (log2(e) / T) + gumbel2(u) with two native v_log_f32 (log2) per logit instead of two
// full-precision logf (u is in [2^-25, 1 - 2^-25]: both logarithms see normal inputs).  The final
// Gumbel-max pass over a 128k-vocab row is the sampling kernel's dominant cost (79 us per 448-row
// decode step with logf, profiles/r5/headline).
__device__ __forceinline__ float gumbel2(uint32_t key, int v) {
  const uint32_t h = hash_u32(key ^ hash_u32(static_cast<uint32_t>(v) + 0x632BE5ABu));
  const float u = (static_cast<float>(h >> 8) + 0.5f) * (1.f / 16777216.f);
  return -__builtin_amdgcn_logf(-__builtin_amdgcn_logf(u));
}
constexpr float kSLog2e = 1.4426950408889634f;

template <typename T>
__global__ void __launch_bounds__(1024) sample_kernel(int64_t* __restrict__ out, const T* __restrict__ logits,
                                                      int V, long row_stride, const float* __restrict__ temperature,
                                                      const float* __restrict__ top_p, const int* __restrict__ top_k,
                                                      const int64_t* __restrict__ seeds,
                                                      const int64_t* __restrict__ steps) {
  __shared__ float sv[16];
  __shared__ int si[16];
  const int row = blockIdx.x;
  const T* z = logits + row * row_stride;
  const float t = temperature[row];
  // vectorised single pass when rows are 16-byte aligned (every vocab in the registry)
  const bool vec = (V % 8 == 0) && (row_stride % 8 == 0) && ((reinterpret_cast<uintptr_t>(logits) & 15) == 0);
  if (!(t > 0.f)) {
    ArgMax a{-INFINITY, 0x7FFFFFFF};
    if (vec) {
      for (int v = 8 * threadIdx.x; v < V; v += 8 * blockDim.x) {
        float x[8];
        ld8(z, v, x);
#pragma unroll
        for (int u = 0; u < 8; ++u) a = better(a, ArgMax{x[u], v + u});
      }
    } else {
      for (int v = threadIdx.x; v < V; v += blockDim.x) a = better(a, ArgMax{ld(z, v), v});
    }
    ArgMax r = block_argmax(a, sv, si);
    if (threadIdx.x == 0) out[row] = r.i;
    return;
  }
  const float invt = 1.f / t;
  const int k = top_k[row];
  const float p = top_p[row];
  float thr = -INFINITY;
  if ((k > 0 && k < V) || p < 1.f) {
    float mx = -INFINITY, mn = INFINITY;
    for (int v = threadIdx.x; v < V; v += blockDim.x) {
      mx = fmaxf(mx, ld(z, v));
      mn = fminf(mn, ld(z, v));
    }
    mx = block_max(mx, sv);
    mn = -block_max(-mn, sv);
    if (k > 0 && k < V) {  // largest tau with count(z >= tau) >= k
      float lo = mn, hi = mx;
      for (int it = 0; it < 32; ++it) {
        const float mid = 0.5f * (lo + hi);
        float cnt = 0.f;
        for (int v = threadIdx.x; v < V; v += blockDim.x) cnt += ld(z, v) >= mid ? 1.f : 0.f;
        cnt = block_sum(cnt, sv);
        if (cnt >= static_cast<float>(k)) lo = mid; else hi = mid;
      }
      thr = lo;
    }
    if (p < 1.f) {  // largest tau with mass(z >= tau) >= p * total, mass in softmax(z / T)
      float tot = 0.f;
      for (int v = threadIdx.x; v < V; v += blockDim.x) tot += __expf((ld(z, v) - mx) * invt);
      tot = block_sum(tot, sv);
      float lo = fmaxf(mn, mx - 88.f * t), hi = mx;
      for (int it = 0; it < 32; ++it) {
        const float mid = 0.5f * (lo + hi);
        float mass = 0.f;
        for (int v = threadIdx.x; v < V; v += blockDim.x) {
          const float zv = ld(z, v);
          mass += zv >= mid ? __expf((zv - mx) * invt) : 0.f;
        }
        mass = block_sum(mass, sv);
        if (mass >= p * tot) lo = mid; else hi = mid;
      }
      thr = fmaxf(thr, lo);
    }
  }
  const uint32_t key = hash_u32(static_cast<uint32_t>(static_cast<uint64_t>(seeds[row]) * 0x9E3779B1ull +
                                                      static_cast<uint64_t>(steps[row])));
  const float invt2 = invt * kSLog2e;
  ArgMax a{-INFINITY, 0x7FFFFFFF};
  if (vec) {
    for (int v = 8 * threadIdx.x; v < V; v += 8 * blockDim.x) {
      float x[8];
      ld8(z, v, x);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (x[u] >= thr) a = better(a, ArgMax{x[u] * invt2 + gumbel2(key, v + u), v + u});
    }
  } else {
    for (int v = threadIdx.x; v < V; v += blockDim.x) {
      const float zv = ld(z, v);
      if (zv >= thr) a = better(a, ArgMax{zv * invt2 + gumbel2(key, v), v});
    }
  }
  ArgMax r = block_argmax(a, sv, si);
  if (threadIdx.x == 0) out[row] = r.i;
}

// Register-resident form (bf16 rows up to 2048 * NV logits, 16-byte aligned): the workgroup loads
// its row ONCE into registers (NV packed bf16 pairs per thread, 8 consecutive logits per 16-byte
// load), and every bisection pass of the top-k / top-p thresholds, the max / min and the final
// Gumbel-max run on those registers.  The memory form above re-reads the row (256 KB at a 128k
// vocab) for each of up to 64 bisection passes.  Element e of a thread is logit
// 8 (tid + 1024 (e / 8)) + e % 8; slots past V hold -inf and are skipped.
template <int NV>
__global__ void __launch_bounds__(1024) sample_reg_kernel(int64_t* __restrict__ out, const bf16_t* __restrict__ logits,
                                                          int V, long row_stride, const float* __restrict__ temperature,
                                                          const float* __restrict__ top_p, const int* __restrict__ top_k,
                                                          const int64_t* __restrict__ seeds,
                                                          const int64_t* __restrict__ steps) {
  constexpr int NQ = NV / 4;  // 16-byte loads per thread
  constexpr int NE = 2 * NV;  // logits per thread
  __shared__ float sv[16];
  __shared__ int si[16];
  const int row = blockIdx.x, tid = threadIdx.x;
  const bf16_t* z = logits + row * row_stride;
  uint32_t r[NV];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int v0 = 8 * (tid + 1024 * q);
    uint4 w = make_uint4(0xFF80FF80u, 0xFF80FF80u, 0xFF80FF80u, 0xFF80FF80u);  // -inf pairs
    if (v0 < V) w = *reinterpret_cast<const uint4*>(z + v0);
    r[4 * q] = w.x;
    r[4 * q + 1] = w.y;
    r[4 * q + 2] = w.z;
    r[4 * q + 3] = w.w;
  }
  auto val = [&](int e) -> float { return (e & 1) ? bf2f_hi(r[e >> 1]) : bf2f_lo(r[e >> 1]); };
  // an empty asm "modifying" the packed row at the top of each pass: keeps hipcc from hoisting all
  // 2 NV unpacked floats out of the bisection loops (loop-invariant), which would spill
  auto opaque = [&] {
#pragma unroll
    for (int i = 0; i < NV; ++i) asm volatile("" : "+v"(r[i]));
  };
  auto idx = [&](int e) -> int { return 8 * (tid + 1024 * (e >> 3)) + (e & 7); };
  const float t = temperature[row];
  if (!(t > 0.f)) {
    ArgMax a{-INFINITY, 0x7FFFFFFF};
#pragma unroll
    for (int e = 0; e < NE; ++e)
      if (idx(e) < V) a = better(a, ArgMax{val(e), idx(e)});
    ArgMax res = block_argmax(a, sv, si);
    if (tid == 0) out[row] = res.i;
    return;
  }
  const float invt = 1.f / t;
  const int k = top_k[row];
  const float p = top_p[row];
  float thr = -INFINITY;
  if ((k > 0 && k < V) || p < 1.f) {
    float mx = -INFINITY, mn = INFINITY;
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const float x = val(e);
      mx = fmaxf(mx, x);
      if (x != -INFINITY) mn = fminf(mn, x);
    }
    mx = block_max(mx, sv);
    mn = -block_max(-mn, sv);
    if (k > 0 && k < V) {  // largest tau with count(z >= tau) >= k
      float lo = mn, hi = mx;
      for (int it = 0; it < 32; ++it) {
        const float mid = 0.5f * (lo + hi);
        float cnt = 0.f;
        opaque();
#pragma unroll
        for (int e = 0; e < NE; ++e) cnt += val(e) >= mid ? 1.f : 0.f;
        cnt = block_sum(cnt, sv);
        if (cnt >= static_cast<float>(k)) lo = mid; else hi = mid;
      }
      thr = lo;
    }
    if (p < 1.f) {  // largest tau with mass(z >= tau) >= p * total, mass in softmax(z / T)
      float tot = 0.f;
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        tot += __expf((val(e) - mx) * invt);
        __builtin_amdgcn_sched_barrier(0);  // one element at a time: keeps the row in registers
      }
      tot = block_sum(tot, sv);
      float lo = fmaxf(mn, mx - 88.f * t), hi = mx;
      for (int it = 0; it < 32; ++it) {
        const float mid = 0.5f * (lo + hi);
        float mass = 0.f;
        opaque();
#pragma unroll
        for (int e = 0; e < NE; ++e) {
          const float x = val(e);
          mass += x >= mid ? __expf((x - mx) * invt) : 0.f;
          __builtin_amdgcn_sched_barrier(0);
        }
        mass = block_sum(mass, sv);
        if (mass >= p * tot) lo = mid; else hi = mid;
      }
      thr = fmaxf(thr, lo);
    }
  }
  const uint32_t key = hash_u32(static_cast<uint32_t>(static_cast<uint64_t>(seeds[row]) * 0x9E3779B1ull +
                                                      static_cast<uint64_t>(steps[row])));
  const float invt2 = invt * kSLog2e;
  ArgMax a{-INFINITY, 0x7FFFFFFF};
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const float x = val(e);
    const int v = idx(e);
    if (v < V && x >= thr) a = better(a, ArgMax{x * invt2 + gumbel2(key, v), v});
    if ((e & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // 4 independent hash/log chains in flight
  }
  ArgMax res = block_argmax(a, sv, si);
  if (tid == 0) out[row] = res.i;
}

void launch_sample(int64_t* out, const void* logits, bool bf16, int B, int V, long row_stride,
                   const float* temperature, const float* top_p, const int* top_k, const int64_t* seeds,
                   const int64_t* steps, hipStream_t s) {
  if (B == 0) return;
  const bool vec = V % 8 == 0 && row_stride % 8 == 0 && (reinterpret_cast<uintptr_t>(logits) & 15) == 0;
  static const bool reg_ok = [] {  // MXS_SAMPLE_REG=0: the memory form (A/B measurements)
    const char* e = std::getenv("MXS_SAMPLE_REG");
    return e == nullptr || e[0] != '0';
  }();
  if (reg_ok && bf16 && vec && V <= 2048 * 64) {
    if (V <= 2048 * 16)
      hipLaunchKernelGGL(sample_reg_kernel<16>, dim3(B), dim3(1024), 0, s, out, static_cast<const bf16_t*>(logits), V,
                         row_stride, temperature, top_p, top_k, seeds, steps);
    else
      hipLaunchKernelGGL(sample_reg_kernel<64>, dim3(B), dim3(1024), 0, s, out, static_cast<const bf16_t*>(logits), V,
                         row_stride, temperature, top_p, top_k, seeds, steps);
    MXS_CHECK_LAUNCH();
    return;
  }
  if (bf16)
    hipLaunchKernelGGL(sample_kernel<bf16_t>, dim3(B), dim3(1024), 0, s, out, static_cast<const bf16_t*>(logits), V,
                       row_stride, temperature, top_p, top_k, seeds, steps);
  else
    hipLaunchKernelGGL(sample_kernel<float>, dim3(B), dim3(1024), 0, s, out, static_cast<const float*>(logits), V,
                       row_stride, temperature, top_p, top_k, seeds, steps);
  MXS_CHECK_LAUNCH();
}

// Log-probabilities for the rows that asked for them (OpenAI `logprobs` / `top_logprobs`).
// One workgroup per selected row: one pass for the row's log-sum-exp (online max / rescaled sum,
// merged across lanes and waves), then the sampled token's log-prob and the K best tokens by K
// block-argmax passes, each excluding everything at or above the previous pick in (value desc,
// index asc) order.  K <= 20, and only requesting rows are touched, so the extra reads are a few
// hundred KB of L2-resident logits per row.  Log-probs are of the raw model distribution (before
// temperature / top-k / top-p), as vLLM reports them.
template <typename T>
__global__ void __launch_bounds__(1024) logprobs_kernel(float* __restrict__ tok_lp, int64_t* __restrict__ top_ids,
                                                        float* __restrict__ top_lp, const T* __restrict__ logits,
                                                        int V, long row_stride, const int64_t* __restrict__ rows,
                                                        const int64_t* __restrict__ tokens, int K) {
  __shared__ float sv[16];
  __shared__ int si[16];
  __shared__ float sm[16], ss[16];
  const int b = blockIdx.x;
  const T* z = logits + rows[b] * row_stride;
  float m = -INFINITY, s = 0.f;
  for (int v = threadIdx.x; v < V; v += blockDim.x) {
    const float x = ld(z, v);
    if (x > m) {
      s = s * __expf(m - x) + 1.f;
      m = x;
    } else {
      s += __expf(x - m);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    const float M = fmaxf(m, m2);
    s = (M == -INFINITY) ? 0.f : s * __expf(m - M) + s2 * __expf(m2 - M);
    m = M;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane == 0) {
    sm[wid] = m;
    ss[wid] = s;
  }
  __syncthreads();
  float M = sm[0];
  for (int w = 1; w < nw; ++w) M = fmaxf(M, sm[w]);
  float S = 0.f;
  for (int w = 0; w < nw; ++w) S += sm[w] == -INFINITY ? 0.f : ss[w] * __expf(sm[w] - M);
  const float lse = M + logf(S);
  if (threadIdx.x == 0) tok_lp[b] = ld(z, static_cast<int>(tokens[b])) - lse;
  ArgMax prev{INFINITY, -1};
  for (int j = 0; j < K; ++j) {
    ArgMax a{-INFINITY, 0x7FFFFFFF};
    for (int v = threadIdx.x; v < V; v += blockDim.x) {
      const float x = ld(z, v);
      if (x < prev.v || (x == prev.v && v > prev.i)) a = better(a, ArgMax{x, v});
    }
    const ArgMax r = block_argmax(a, sv, si);
    if (threadIdx.x == 0) {
      top_ids[b * K + j] = r.i < V ? r.i : 0;
      top_lp[b * K + j] = r.v - lse;
    }
    prev = r;
  }
}

void launch_logprobs(float* tok_lp, int64_t* top_ids, float* top_lp, const void* logits, bool bf16, int n, int V,
                     long row_stride, const int64_t* rows, const int64_t* tokens, int K, hipStream_t s) {
  if (n == 0) return;
  if (bf16)
    hipLaunchKernelGGL(logprobs_kernel<bf16_t>, dim3(n), dim3(1024), 0, s, tok_lp, top_ids, top_lp,
                       static_cast<const bf16_t*>(logits), V, row_stride, rows, tokens, K);
  else
    hipLaunchKernelGGL(logprobs_kernel<float>, dim3(n), dim3(1024), 0, s, tok_lp, top_ids, top_lp,
                       static_cast<const float*>(logits), V, row_stride, rows, tokens, K);
  MXS_CHECK_LAUNCH();
}

// Sampling penalties (OpenAI frequency_penalty / presence_penalty, vLLM repetition_penalty),
// applied in place to the logits rows before sampling.  One workgroup per sampled row; rows with
// neutral penalties exit at once (the kernel sits in every decode graph).  The row's token history
// (prompt then generated tokens, written on the device every step) is hist[row, 0:hlen):
//   prompt tokens    -> LDS presence bitmap (V <= 163840 bits = 20 KiB)
//   generated tokens -> per-token counts in a global int32 scratch row (V x 4 B; LDS cannot hold
//                       counts for a 128k-152k vocab), zeroed first, atomics at L2, read back with
//                       atomic loads so no stale L1 line is used
// then for every v:  seen = in prompt or count > 0
//   repetition: z = seen ? (z > 0 ? z / rep : z * rep) : z;   z -= count * freq + (count > 0) * pres
constexpr int kPenMaxVocab = 163840;

template <typename T>
__device__ __forceinline__ void st(T* p, float v);
template <>
__device__ __forceinline__ void st<float>(float* p, float v) { *p = v; }
template <>
__device__ __forceinline__ void st<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }

template <typename T>
__global__ void __launch_bounds__(1024) penalties_kernel(T* __restrict__ logits, int V, long row_stride,
                                                         const int* __restrict__ hist, long hist_stride,
                                                         const int64_t* __restrict__ srows,
                                                         const int* __restrict__ hlen, const int* __restrict__ plen,
                                                         const float* __restrict__ rep,
                                                         const float* __restrict__ freq,
                                                         const float* __restrict__ pres, int* __restrict__ counts) {
  __shared__ unsigned bits[kPenMaxVocab / 32];
  const int b = blockIdx.x;
  const float rp = rep[b], fp = freq[b], pp = pres[b];
  if (rp == 1.f && fp == 0.f && pp == 0.f) return;
  T* z = logits + b * row_stride;
  int* cnt = counts + static_cast<long>(b) * V;
  const int* h = hist + srows[b] * hist_stride;
  const int n = hlen[b], np = min(plen[b], n);
  for (int w = threadIdx.x; w < (V + 31) / 32; w += blockDim.x) bits[w] = 0u;
  for (int v = threadIdx.x; v < V; v += blockDim.x) cnt[v] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int t = h[i];
    if (t < 0 || t >= V) continue;
    if (i < np)
      atomicOr(&bits[t >> 5], 1u << (t & 31));
    else
      atomicAdd(&cnt[t], 1);
  }
  __syncthreads();
  for (int v = threadIdx.x; v < V; v += blockDim.x) {
    const int c = __hip_atomic_load(&cnt[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool seen = c > 0 || ((bits[v >> 5] >> (v & 31)) & 1u);
    if (!seen) continue;
    float x = ld(z, v);
    if (rp != 1.f) x = x > 0.f ? x / rp : x * rp;
    if (c > 0) x -= static_cast<float>(c) * fp + pp;
    st(z + v, x);
  }
}

void launch_penalties(void* logits, bool bf16, int B, int V, long row_stride, const int* hist, long hist_stride,
                      const int64_t* srows, const int* hlen, const int* plen, const float* rep, const float* freq,
                      const float* pres, int* counts, hipStream_t s) {
  if (B == 0) return;
  if (bf16)
    hipLaunchKernelGGL(penalties_kernel<bf16_t>, dim3(B), dim3(1024), 0, s, static_cast<bf16_t*>(logits), V,
                       row_stride, hist, hist_stride, srows, hlen, plen, rep, freq, pres, counts);
  else
    hipLaunchKernelGGL(penalties_kernel<float>, dim3(B), dim3(1024), 0, s, static_cast<float*>(logits), V, row_stride,
                       hist, hist_stride, srows, hlen, plen, rep, freq, pres, counts);
  MXS_CHECK_LAUNCH();
}

}  // namespace mxs
