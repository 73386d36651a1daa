// K03+K04: (optional Qwen3 per-head q/k RMSNorm) -> rotate-half RoPE on q and k -> scatter k, v into
// the paged KV cache, all in one pass over the fused QKV projection output.
// Cache layout per layer (see mxserve/ops/reference.py): block b at kv + b*block_stride,
//   K: [Hkv][BS][D] (token-major)   V: [Hkv][D][BS] (dim-major, so attention's P*V operand is a
//   contiguous 16-byte load per lane).
// cos/sin come from a host-precomputed fp32 table (cdna_hip_programming.md App. B: no device trig).
// KT = bf16_t, or fp8_t for an fp8 (e4m3fn) cache: K and V stored as x / k_scale, x / v_scale.
#include <algorithm>

#include "common.h"

namespace mxs {

// Source of the fused QKV row: the projection's bf16 output, or (SLABS) the S fp32 split-K slabs
// [S][T][row_stride] a decode GEMM left unreduced, summed here and rounded to bf16 as the GEMM's own
// output would be -- the reduce kernel and the bf16 round trip of the qkv row disappear.
template <bool SLABS>
struct QkvRow {
  const bf16_t* row;
  const float* prow;
  int S;
  size_t slab;
  __device__ __forceinline__ float operator[](int j) const {
    if constexpr (SLABS) {
      // the slabs' loads issued 8 at a time, summed in slab order (a serial load -> add chain costs
      // one L2 round trip per slab: ~8 us for a TP-8 qkv shard's 8 slabs at batch 1)
      float a = prow[j];
      for (int s0 = 1; s0 < S; s0 += 8) {
        float b[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) b[u] = s0 + u < S ? prow[(s0 + u) * slab + j] : 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (s0 + u < S) a += b[u];
      }
      return bf2f(f2bf(a));
    } else {
      return bf2f(row[j]);
    }
  }
};

template <int D, bool QKNORM, typename KT, bool SLABS = false>
__global__ void __launch_bounds__(256) rope_cache_kernel(
    bf16_t* __restrict__ q_out, const bf16_t* __restrict__ qkv, const int64_t* __restrict__ positions,
    const float* __restrict__ cos_sin, KT* __restrict__ kv, long block_stride,
    const int64_t* __restrict__ slot_mapping, const bf16_t* __restrict__ qn, const bf16_t* __restrict__ kn,
    int Hq, int Hkv, int BS, float eps, float k_inv_scale, float v_inv_scale, const float* __restrict__ part = nullptr,
    int S = 1, int T = 0) {
  constexpr int HALF = D / 2;
  const int t = blockIdx.x;
  const int row_stride = (Hq + 2 * Hkv) * D;
  QkvRow<SLABS> src{qkv + static_cast<size_t>(t) * row_stride,
                    SLABS ? part + static_cast<size_t>(t) * row_stride : nullptr, S,
                    static_cast<size_t>(T) * row_stride};
  const long pos = positions[t];
  const long slot = slot_mapping[t];
  const float* cs = cos_sin + pos * D;
  KT* kblk = nullptr;
  int off = 0;
  if (slot >= 0) {
    kblk = kv + (slot / BS) * block_stride;
    off = static_cast<int>(slot % BS);
  }
  // rotary part: (Hq + Hkv) heads x HALF pairs; a head's pairs are HALF consecutive lanes.  q_out ==
  // nullptr: K / V only (the attention kernels read q from the qkv rows and rotate it themselves)
  const int hbeg = q_out != nullptr ? 0 : Hq;
  const int n_items = (Hq + Hkv - hbeg) * HALF;
  // blockIdx.y splits a token's items over gridDim.y workgroups (small decode batches: a token per
  // workgroup alone leaves the chip idle); bases stay multiples of blockDim.x, so a head's pairs
  // stay in one wave for the q/k-norm shuffles
  const int ystep = gridDim.y * blockDim.x;
  for (int base = blockIdx.y * blockDim.x; base < n_items; base += ystep) {
    const int i = base + threadIdx.x;
    const bool active = i < n_items;
    const int head = hbeg + (active ? i / HALF : 0);
    const int p = i % HALF;
    float x1 = 0.f, x2 = 0.f;
    if (active) {
      x1 = src[head * D + p];
      x2 = src[head * D + p + HALF];
    }
    if (QKNORM) {
      float ss = x1 * x1 + x2 * x2;
#pragma unroll
      for (int o = HALF / 2; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
      const float inv = rsqrtf(ss / D + eps);
      const bf16_t* nw = head < Hq ? qn : kn;
      if (active) {
        x1 = bf2f(f2bf(x1 * inv * bf2f(nw[p])));
        x2 = bf2f(f2bf(x2 * inv * bf2f(nw[p + HALF])));
      }
    }
    if (!active) continue;
    const float c = cs[p], s = cs[HALF + p];
    const float o1 = x1 * c - x2 * s;
    const float o2 = x2 * c + x1 * s;
    if (head < Hq) {
      bf16_t* qo = q_out + (static_cast<size_t>(t) * Hq + head) * D;
      qo[p] = f2bf(o1);
      qo[p + HALF] = f2bf(o2);
    } else if (kblk) {
      KT* kd = kblk + (static_cast<size_t>(head - Hq) * BS + off) * D;
      kv_store(kd + p, o1, k_inv_scale);
      kv_store(kd + p + HALF, o2, k_inv_scale);
    }
  }
  if (!kblk) return;
  // V: copy into the dim-major half of the block
  const int v0 = (Hq + Hkv) * D;
  KT* vblk = kblk + static_cast<size_t>(Hkv) * BS * D;
  for (int j = blockIdx.y * blockDim.x + threadIdx.x; j < Hkv * D; j += ystep) {
    const int h = j / D, d = j % D;
    KT* dst = vblk + (static_cast<size_t>(h) * D + d) * BS + off;
    if constexpr (sizeof(KT) == 2 && !SLABS)
      *dst = src.row[v0 + j];  // bf16 -> bf16: bit copy
    else
      kv_store(dst, src[v0 + j], v_inv_scale);
  }
}

// Prefill form (no q/k norm): 16 consecutive tokens per workgroup.  The rotation moves 4 pairs per
// lane (8-byte loads and stores instead of 2-byte ones), and when the 16 tokens fill one run of a
// block's slots (a prefill chunk's tokens are consecutive slots of their sequence) their V rows are
// staged in LDS and written as 32-byte runs of the dim-major V block instead of one 2-byte store
// per (token, dim).  Any other slot pattern falls back to per-element V stores.
__device__ __forceinline__ void kv_store4(bf16_t* p, const float* x, float) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack2(x[0], x[1]), pack2(x[2], x[3]));
}
__device__ __forceinline__ void kv_store4(fp8_t* p, const float* x, float inv) {
#pragma unroll
  for (int e = 0; e < 4; ++e) p[e] = f2fp8(x[e] * inv);
}

template <int D, typename KT>
__global__ void __launch_bounds__(256) rope_cache_t16_kernel(
    bf16_t* __restrict__ q_out, const bf16_t* __restrict__ qkv, const int64_t* __restrict__ positions,
    const float* __restrict__ cos_sin, KT* __restrict__ kv, long block_stride, const int64_t* __restrict__ slot_mapping,
    int Hq, int Hkv, int BS, int T, float k_inv_scale, float v_inv_scale) {
  constexpr int HALF = D / 2, V4 = HALF / 4, TPB = 16;
  extern __shared__ __attribute__((aligned(16))) bf16_t vstage[];  // [TPB][Hkv * D]
  __shared__ int64_t s_slot0;
  __shared__ int s_fast;
  const int t0 = blockIdx.x * TPB, nt = min(TPB, T - t0);
  const int row_stride = (Hq + 2 * Hkv) * D, hkd = Hkv * D;
  const int hbeg = q_out != nullptr ? 0 : Hq;  // nullptr: K / V only (see rope_cache_kernel)
  const int per_tok = (Hq + Hkv - hbeg) * V4;
  if (threadIdx.x < 64) {  // wave 0: the nt slots in parallel (one load per lane, not a serial chain)
    const int k = threadIdx.x;
    const int64_t sk = k < nt ? slot_mapping[t0 + k] : 0;
    const int64_t s0 = __shfl(sk, 0, 64);
    const bool ok = k >= nt || sk == s0 + k;
    const bool all_ok = __all(ok);
    if (k == 0) {
      s_slot0 = s0;
      s_fast = all_ok && s0 >= 0 && (s0 % BS) + nt <= BS;
    }
  }
  for (int i = threadIdx.x; i < nt * per_tok; i += blockDim.x) {
    const int tt = i / per_tok, rem = i - tt * per_tok, hh = rem / V4, p = (rem - hh * V4) * 4, head = hbeg + hh;
    const int t = t0 + tt;
    const bf16_t* src = qkv + static_cast<size_t>(t) * row_stride + head * D;
    const uint2 a = *reinterpret_cast<const uint2*>(src + p), b = *reinterpret_cast<const uint2*>(src + p + HALF);
    const float* cs = cos_sin + positions[t] * D;
    const float4 c = *reinterpret_cast<const float4*>(cs + p), sn = *reinterpret_cast<const float4*>(cs + HALF + p);
    const float x1[4] = {bf2f_lo(a.x), bf2f_hi(a.x), bf2f_lo(a.y), bf2f_hi(a.y)};
    const float x2[4] = {bf2f_lo(b.x), bf2f_hi(b.x), bf2f_lo(b.y), bf2f_hi(b.y)};
    const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {sn.x, sn.y, sn.z, sn.w};
    float o1[4], o2[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o1[e] = x1[e] * cc[e] - x2[e] * ss[e];
      o2[e] = x2[e] * cc[e] + x1[e] * ss[e];
    }
    if (head < Hq) {
      bf16_t* qo = q_out + (static_cast<size_t>(t) * Hq + head) * D;
      *reinterpret_cast<uint2*>(qo + p) = make_uint2(pack2(o1[0], o1[1]), pack2(o1[2], o1[3]));
      *reinterpret_cast<uint2*>(qo + p + HALF) = make_uint2(pack2(o2[0], o2[1]), pack2(o2[2], o2[3]));
    } else {
      const int64_t slot = slot_mapping[t];
      if (slot >= 0) {
        KT* kd = kv + (slot / BS) * block_stride + (static_cast<size_t>(head - Hq) * BS + slot % BS) * D;
        kv_store4(kd + p, o1, k_inv_scale);
        kv_store4(kd + p + HALF, o2, k_inv_scale);
      }
    }
  }
  __syncthreads();
  const bf16_t* vbase = qkv + static_cast<size_t>(t0) * row_stride + (Hq + Hkv) * D;
  if (!s_fast) {  // tokens of different blocks (or unmapped): one store per (token, dim)
    for (int i = threadIdx.x; i < nt * hkd; i += blockDim.x) {
      const int tt = i / hkd, j = i - tt * hkd;
      const int64_t slot = slot_mapping[t0 + tt];
      if (slot < 0) continue;
      KT* dst = kv + (slot / BS) * block_stride + static_cast<size_t>(Hkv) * BS * D + static_cast<size_t>(j) * BS +
                slot % BS;
      const bf16_t v = vbase[static_cast<size_t>(tt) * row_stride + j];
      if constexpr (sizeof(KT) == 2) *dst = v;
      else kv_store(dst, bf2f(v), v_inv_scale);
    }
    return;
  }
  // stage the nt V rows (16-byte loads), then write each (head, dim) row's run of nt slots
  for (int i = threadIdx.x; i < nt * (hkd / 8); i += blockDim.x) {
    const int tt = i / (hkd / 8), j = (i - tt * (hkd / 8)) * 8;
    *reinterpret_cast<uint4*>(vstage + tt * hkd + j) =
        *reinterpret_cast<const uint4*>(vbase + static_cast<size_t>(tt) * row_stride + j);
  }
  __syncthreads();
  const int64_t s0 = s_slot0;
  const int off0 = static_cast<int>(s0 % BS);
  KT* vblk = kv + (s0 / BS) * block_stride + static_cast<size_t>(Hkv) * BS * D;
  for (int j = threadIdx.x; j < hkd; j += blockDim.x) {
    KT* dst = vblk + static_cast<size_t>(j) * BS + off0;
    if constexpr (sizeof(KT) == 2) {
      if (nt == TPB && off0 == 0 && BS == TPB) {  // a whole 32-byte row of the block
        uint32_t w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
          w[k] = static_cast<uint32_t>(vstage[(2 * k) * hkd + j]) | (static_cast<uint32_t>(vstage[(2 * k + 1) * hkd + j]) << 16);
        *reinterpret_cast<uint4*>(dst) = make_uint4(w[0], w[1], w[2], w[3]);
        *reinterpret_cast<uint4*>(dst + 8) = make_uint4(w[4], w[5], w[6], w[7]);
        continue;
      }
    }
    for (int tt = 0; tt < nt; ++tt) {
      if constexpr (sizeof(KT) == 2) dst[tt] = vstage[tt * hkd + j];
      else kv_store(dst + tt, bf2f(vstage[tt * hkd + j]), v_inv_scale);
    }
  }
}

// Prefill K / V-only form (q is rotated inside the attention kernels, llama.py _fused_q_rope): 16
// tokens per workgroup, and every global load of the tile is in flight before the first is used.
// rope_cache_t16_kernel walks 8-byte items in a loop whose every trip chains a positions load, a
// cos/sin load and the stores (37.6 us per 6144-token call in the headline run, ~10x its HBM time:
// profiles/r4/bench_q48_kernel_stats.csv).  Here a thread owns NI 8-pair chunks of K (16-byte
// loads of both halves, 2 x 32-byte cos/sin) and NV 16-byte pieces of the V rows, all issued up
// front; the slot / position loads are the only dependent round trip.  Loads index with clamped
// (always valid) addresses instead of predicates, so no load is branched around
// (cdna_hip_programming.md §5 trap (c)); only the stores are predicated.
__device__ __forceinline__ void kv_store8(bf16_t* p, const float* x, float) {
  *reinterpret_cast<uint4*>(p) = make_uint4(pack2(x[0], x[1]), pack2(x[2], x[3]), pack2(x[4], x[5]), pack2(x[6], x[7]));
}
__device__ __forceinline__ void kv_store8(fp8_t* p, const float* x, float inv) {
  uint32_t w[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint32_t v = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) v |= static_cast<uint32_t>(static_cast<uint8_t>(f2fp8(x[4 * h + e] * inv))) << (8 * e);
    w[h] = v;
  }
  *reinterpret_cast<uint2*>(p) = make_uint2(w[0], w[1]);
}

// MXS_KV_T16_LEGACY=1: the older rope_cache_t16_kernel for this case (A/B probes)
static bool kv_t16_legacy() {
  static const bool v = [] {
    const char* e = getenv("MXS_KV_T16_LEGACY");
    return e != nullptr && e[0] == '1';
  }();
  return v;
}

// V rows of the dim-major cache block ([Hkv][D][BS]) take a tile's tokens as RUNS: consecutive
// tokens with consecutive slots inside one block (a prefill chunk: one run, or two when the chunk
// starts mid-block -- every continuation chunk does; a decode row: a run of one).  A run of n values
// at element offset o of a row is written in aligned pieces of 8 / 4 / 2 / 1 elements (a whole
// 16-token row: two 16-byte stores for bf16), not one 2-byte store per element.
// src: the run's first value in the LDS stage, consecutive tokens `stride` elements apart (values are
// read per piece from LDS: a dynamically indexed register array would live in scratch)
template <typename KT>
__device__ __forceinline__ void kv_put(KT* row, int o, int n, const bf16_t* src, int stride, float inv) {
  int i = 0;
  while (i < n) {
    const int a = o + i, left = n - i;
    const bf16_t* p = src + i * stride;
    if ((a & 7) == 0 && left >= 8) {
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = bf2f(p[e * stride]);
      kv_store8(row + a, x, inv);
      i += 8;
    } else if ((a & 3) == 0 && left >= 4) {
      float x[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = bf2f(p[e * stride]);
      if constexpr (sizeof(KT) == 2) {
        *reinterpret_cast<uint2*>(row + a) = make_uint2(pack2(x[0], x[1]), pack2(x[2], x[3]));
      } else {
        uint32_t v = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) v |= static_cast<uint32_t>(static_cast<uint8_t>(f2fp8(x[e] * inv))) << (8 * e);
        *reinterpret_cast<uint32_t*>(row + a) = v;
      }
      i += 4;
    } else if ((a & 1) == 0 && left >= 2) {
      const float x0 = bf2f(p[0]), x1 = bf2f(p[stride]);
      if constexpr (sizeof(KT) == 2) {
        *reinterpret_cast<uint32_t*>(row + a) = pack2(x0, x1);
      } else {
        const uint32_t lo = static_cast<uint8_t>(f2fp8(x0 * inv)), hi = static_cast<uint8_t>(f2fp8(x1 * inv));
        *reinterpret_cast<unsigned short*>(row + a) = static_cast<unsigned short>(lo | (hi << 8));
      }
      i += 2;
    } else {
      kv_store(row + a, bf2f(p[0]), inv);
      i += 1;
    }
  }
}

template <int D, typename KT, int NI, int NV>
__global__ void __launch_bounds__(256) kv_rope_t16_kernel(
    const bf16_t* __restrict__ qkv, const int64_t* __restrict__ positions, const float* __restrict__ cos_sin,
    KT* __restrict__ kv, long block_stride, const int64_t* __restrict__ slot_mapping, int Hq, int Hkv, int BS, int T,
    float k_inv_scale, float v_inv_scale) {
  constexpr int HALF = D / 2, CH = HALF / 8, TPB = 16;
  extern __shared__ __attribute__((aligned(16))) bf16_t vstage[];  // [TPB][hpw * D]
  __shared__ unsigned s_runs;       // bit k: token k starts a run
  __shared__ int64_t s_slot[TPB];
  // blockIdx.y: a group of hpw kv heads (gridDim.y groups), so short chunks still fill the chip
  const int hpw = Hkv / gridDim.y, h0 = blockIdx.y * hpw;
  const int t0 = blockIdx.x * TPB, nt = min(TPB, T - t0), tid = threadIdx.x;
  const int row_stride = (Hq + 2 * Hkv) * D, hkd = hpw * D;
  const int n_k = nt * hpw * CH, n_v = nt * (hkd / 8);
  const bf16_t* tile = qkv + static_cast<size_t>(t0) * row_stride;
  // V rows into registers (independent of everything else)
  uint4 vr[NV];
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int i = min(tid + 256 * u, n_v - 1), tt = i / (hkd / 8), j = (i - tt * (hkd / 8)) * 8;
    vr[u] = *reinterpret_cast<const uint4*>(tile + static_cast<size_t>(tt) * row_stride + (Hq + Hkv + h0) * D + j);
  }
  // K chunks: both halves of 8 pairs, and the token's position / slot
  uint4 ka[NI], kb[NI];
  int64_t pos[NI], slot[NI];
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int i = min(tid + 256 * u, n_k - 1), tt = i / (hpw * CH), r = i - tt * (hpw * CH), h = h0 + r / CH,
              c = r % CH;
    const bf16_t* src = tile + static_cast<size_t>(tt) * row_stride + (Hq + h) * D + 8 * c;
    ka[u] = *reinterpret_cast<const uint4*>(src);
    kb[u] = *reinterpret_cast<const uint4*>(src + HALF);
    pos[u] = positions[t0 + tt];
    slot[u] = slot_mapping[t0 + tt];
  }
  if (tid < 64) {  // wave 0: the tile's runs (unmapped tokens, slot -1, start a run and are skipped)
    const int64_t sk = tid < nt ? slot_mapping[t0 + tid] : -1;
    const int64_t sp = __shfl_up(sk, 1, 64);
    const bool start = tid < nt && (tid == 0 || sk < 0 || sp < 0 || sk != sp + 1 || sk % BS == 0);
    const unsigned long long m = __ballot(start);
    if (tid < nt) s_slot[tid] = sk;
    if (tid == 0) s_runs = static_cast<unsigned>(m & 0xFFFFu);
  }
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int i = tid + 256 * u;
    if (i < n_v) {
      const int tt = i / (hkd / 8), j = (i - tt * (hkd / 8)) * 8;
      *reinterpret_cast<uint4*>(vstage + tt * hkd + j) = vr[u];
    }
  }
  // rotate and store K
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int i = tid + 256 * u, r = i % (hpw * CH), h = h0 + r / CH, c = r % CH;
    const float* cs = cos_sin + pos[u] * D + 8 * c;
    const float4 c0 = *reinterpret_cast<const float4*>(cs), c1 = *reinterpret_cast<const float4*>(cs + 4);
    const float4 s0 = *reinterpret_cast<const float4*>(cs + HALF), s1 = *reinterpret_cast<const float4*>(cs + HALF + 4);
    const float cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const uint32_t xa[4] = {ka[u].x, ka[u].y, ka[u].z, ka[u].w}, xb[4] = {kb[u].x, kb[u].y, kb[u].z, kb[u].w};
    float o1[8], o2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x1 = (e & 1) ? bf2f_hi(xa[e >> 1]) : bf2f_lo(xa[e >> 1]);
      const float x2 = (e & 1) ? bf2f_hi(xb[e >> 1]) : bf2f_lo(xb[e >> 1]);
      o1[e] = x1 * cc[e] - x2 * sn[e];
      o2[e] = x2 * cc[e] + x1 * sn[e];
    }
    if (i < n_k && slot[u] >= 0) {
      KT* kd = kv + (slot[u] / BS) * block_stride + (static_cast<size_t>(h) * BS + slot[u] % BS) * D + 8 * c;
      kv_store8(kd, o1, k_inv_scale);
      kv_store8(kd + HALF, o2, k_inv_scale);
    }
  }
  __syncthreads();
  // V: each thread owns rows j (one (head, dim) of the block's dim-major image); the run loop is
  // wave-uniform (the runs belong to the tile)
  const unsigned runs = s_runs;
  for (int j = tid; j < hkd; j += blockDim.x) {
    unsigned rest = runs;
    while (rest) {
      const int a = __builtin_ctz(rest);
      rest &= rest - 1;
      const int b = rest ? __builtin_ctz(rest) : nt;  // run = tokens [a, b)
      const int64_t sl = s_slot[a];
      if (sl < 0) continue;
      KT* row = kv + (sl / BS) * block_stride + static_cast<size_t>(Hkv) * BS * D + static_cast<size_t>(h0 * D + j) * BS;
      kv_put(row, static_cast<int>(sl % BS), b - a, vstage + a * hkd + j, hkd, v_inv_scale);
    }
  }
}

// workgroups per token of rope_cache_kernel: up to one per 256 items at small decode batches
static int rope_grid_y(int T, int Hq, int Hkv, int D) {
  if (T > 64) return 1;
  const int items = std::max((Hq + Hkv) * (D / 2), Hkv * D);
  return std::min(8, (items + 255) / 256);
}

template <typename KT>
static void launch_rope_typed(bf16_t* q_out, const bf16_t* qkv, const int64_t* positions, const float* cos_sin,
                              KT* kv, long block_stride, const int64_t* slot_mapping, const bf16_t* qn,
                              const bf16_t* kn, int T, int Hq, int Hkv, int D, int BS, float eps, float kis, float vis,
                              hipStream_t s) {
  const bool norm = qn != nullptr;
  if (!norm && q_out == nullptr && T >= 512 && (D == 64 || D == 128) && Hkv * D <= 1024 && !kv_t16_legacy()) {
    // kv-head groups per 16-token tile: about 2 workgroups per CU for short chunks (a 2,400-token
    // chunk is only 150 tiles), whole-head groups that divide Hkv
    const int tiles = (T + 15) / 16;
    int hgroups = 1;
    while (hgroups * 2 <= Hkv && Hkv % (hgroups * 2) == 0 && tiles * hgroups < 512) hgroups *= 2;
    const dim3 g16(tiles, hgroups), b16(256);
    const size_t lds = static_cast<size_t>(16) * (Hkv / hgroups) * D * sizeof(bf16_t);
    const bool small = Hkv * D <= 512;
#define MXS_KV16(DD, NI, NV)                                                                                    \
  hipLaunchKernelGGL((kv_rope_t16_kernel<DD, KT, NI, NV>), g16, b16, lds, s, qkv, positions, cos_sin, kv,       \
                     block_stride, slot_mapping, Hq, Hkv, BS, T, kis, vis)
    if (D == 64) {
      if (small) MXS_KV16(64, 2, 4); else MXS_KV16(64, 4, 8);
    } else {
      if (small) MXS_KV16(128, 2, 4); else MXS_KV16(128, 4, 8);
    }
#undef MXS_KV16
    MXS_CHECK_LAUNCH();
    return;
  }
  if (!norm && T >= 512 && D % 8 == 0 && (D == 64 || D == 128) && Hkv * D * 16 * 2 <= 64 * 1024) {
    const dim3 g16((T + 15) / 16), b16(256);
    const size_t lds = static_cast<size_t>(16) * Hkv * D * sizeof(bf16_t);
    if (D == 64)
      hipLaunchKernelGGL((rope_cache_t16_kernel<64, KT>), g16, b16, lds, s, q_out, qkv, positions, cos_sin, kv,
                         block_stride, slot_mapping, Hq, Hkv, BS, T, kis, vis);
    else
      hipLaunchKernelGGL((rope_cache_t16_kernel<128, KT>), g16, b16, lds, s, q_out, qkv, positions, cos_sin, kv,
                         block_stride, slot_mapping, Hq, Hkv, BS, T, kis, vis);
    MXS_CHECK_LAUNCH();
    return;
  }
  dim3 g(T, rope_grid_y(T, Hq, Hkv, D)), b(256);
#define MXS_ROPE_CASE(DD)                                                                                   \
  if (D == DD) {                                                                                            \
    if (norm)                                                                                               \
      hipLaunchKernelGGL((rope_cache_kernel<DD, true, KT>), g, b, 0, s, q_out, qkv, positions, cos_sin, kv, \
                         block_stride, slot_mapping, qn, kn, Hq, Hkv, BS, eps, kis, vis);                   \
    else                                                                                                    \
      hipLaunchKernelGGL((rope_cache_kernel<DD, false, KT>), g, b, 0, s, q_out, qkv, positions, cos_sin,    \
                         kv, block_stride, slot_mapping, qn, kn, Hq, Hkv, BS, eps, kis, vis);               \
    MXS_CHECK_LAUNCH();                                                                                     \
    return;                                                                                                 \
  }
  MXS_ROPE_CASE(64)
  MXS_ROPE_CASE(128)
  MXS_ROPE_CASE(32)
#undef MXS_ROPE_CASE
}

template <typename KT>
static void launch_rope_slabs_typed(bf16_t* q_out, const float* part, int S, const int64_t* positions,
                                    const float* cos_sin, KT* kv, long block_stride, const int64_t* slot_mapping,
                                    const bf16_t* qn, const bf16_t* kn, int T, int Hq, int Hkv, int D, int BS, float eps,
                                    float kis, float vis, hipStream_t s) {
  dim3 g(T, rope_grid_y(T, Hq, Hkv, D)), b(256);
#define MXS_ROPE_SLAB(DD)                                                                                      \
  if (D == DD) {                                                                                               \
    if (qn != nullptr)                                                                                         \
      hipLaunchKernelGGL((rope_cache_kernel<DD, true, KT, true>), g, b, 0, s, q_out, nullptr, positions, cos_sin, \
                         kv, block_stride, slot_mapping, qn, kn, Hq, Hkv, BS, eps, kis, vis, part, S, T);        \
    else                                                                                                       \
      hipLaunchKernelGGL((rope_cache_kernel<DD, false, KT, true>), g, b, 0, s, q_out, nullptr, positions,       \
                         cos_sin, kv, block_stride, slot_mapping, qn, kn, Hq, Hkv, BS, eps, kis, vis, part, S, T); \
    MXS_CHECK_LAUNCH();                                                                                        \
    return;                                                                                                    \
  }
  MXS_ROPE_SLAB(64)
  MXS_ROPE_SLAB(128)
#undef MXS_ROPE_SLAB
}

// rope_and_cache from the unreduced split-K slabs of the qkv projection (decode batches)
bool launch_splitk_rope_and_cache(bf16_t* q_out, const float* part, int S, const int64_t* positions,
                                  const float* cos_sin, void* kv, bool kv_fp8, long block_stride,
                                  const int64_t* slot_mapping, const bf16_t* qn, const bf16_t* kn, int T, int Hq,
                                  int Hkv, int D, int BS, float eps, float k_scale, float v_scale, hipStream_t s) {
  if (T == 0) return true;
  if (D != 64 && D != 128) return false;
  if (kv_fp8)
    launch_rope_slabs_typed(q_out, part, S, positions, cos_sin, static_cast<fp8_t*>(kv), block_stride, slot_mapping,
                            qn, kn, T, Hq, Hkv, D, BS, eps, 1.f / k_scale, 1.f / v_scale, s);
  else
    launch_rope_slabs_typed(q_out, part, S, positions, cos_sin, static_cast<bf16_t*>(kv), block_stride,
                            slot_mapping, qn, kn, T, Hq, Hkv, D, BS, eps, 1.f, 1.f, s);
  return true;
}

// kv_fp8: the cache holds e4m3fn bytes (block_stride in elements = bytes); k/v_scale: stored = x / scale
void launch_rope_and_cache(bf16_t* q_out, const bf16_t* qkv, const int64_t* positions, const float* cos_sin,
                           void* kv, bool kv_fp8, long block_stride, const int64_t* slot_mapping, const bf16_t* qn,
                           const bf16_t* kn, int T, int Hq, int Hkv, int D, int BS, float eps, float k_scale,
                           float v_scale, hipStream_t s) {
  if (T == 0) return;
  if (kv_fp8)
    launch_rope_typed(q_out, qkv, positions, cos_sin, static_cast<fp8_t*>(kv), block_stride, slot_mapping, qn, kn, T,
                      Hq, Hkv, D, BS, eps, 1.f / k_scale, 1.f / v_scale, s);
  else
    launch_rope_typed(q_out, qkv, positions, cos_sin, static_cast<bf16_t*>(kv), block_stride, slot_mapping, qn, kn,
                      T, Hq, Hkv, D, BS, eps, 1.f, 1.f, s);
}

}  // namespace mxs
