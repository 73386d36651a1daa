// K03+K04: (optional Qwen3 per-head q/k RMSNorm) -> rotate-half RoPE on q and k -> scatter k, v into
// the paged KV cache, all in one pass over the fused QKV projection output.
// Cache layout per layer (see mxserve/ops/reference.py): block b at kv + b*block_stride,
//   K: [Hkv][BS][D] (token-major)   V: [Hkv][D][BS] (dim-major, so attention's P*V operand is a
//   contiguous 16-byte load per lane).
// cos/sin come from a host-precomputed fp32 table (cdna_hip_programming.md App. B: no device trig).
// KT = bf16_t, or fp8_t for an fp8 (e4m3fn) cache: K and V stored as x / k_scale, x / v_scale.
#include "common.h"

namespace mxs {

template <int D, bool QKNORM, typename KT>
__global__ void __launch_bounds__(256) rope_cache_kernel(
    bf16_t* __restrict__ q_out, const bf16_t* __restrict__ qkv, const int64_t* __restrict__ positions,
    const float* __restrict__ cos_sin, KT* __restrict__ kv, long block_stride,
    const int64_t* __restrict__ slot_mapping, const bf16_t* __restrict__ qn, const bf16_t* __restrict__ kn,
    int Hq, int Hkv, int BS, float eps, float k_inv_scale, float v_inv_scale) {
  constexpr int HALF = D / 2;
  const int t = blockIdx.x;
  const int row_stride = (Hq + 2 * Hkv) * D;
  const bf16_t* src = qkv + static_cast<size_t>(t) * row_stride;
  const long pos = positions[t];
  const long slot = slot_mapping[t];
  const float* cs = cos_sin + pos * D;
  KT* kblk = nullptr;
  int off = 0;
  if (slot >= 0) {
    kblk = kv + (slot / BS) * block_stride;
    off = static_cast<int>(slot % BS);
  }
  // rotary part: (Hq + Hkv) heads x HALF pairs; a head's pairs are HALF consecutive lanes
  const int n_items = (Hq + Hkv) * HALF;
  for (int base = 0; base < n_items; base += blockDim.x) {
    const int i = base + threadIdx.x;
    const bool active = i < n_items;
    const int head = active ? i / HALF : 0;
    const int p = i % HALF;
    float x1 = 0.f, x2 = 0.f;
    if (active) {
      x1 = bf2f(src[head * D + p]);
      x2 = bf2f(src[head * D + p + HALF]);
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
  const bf16_t* vsrc = src + (Hq + Hkv) * D;
  KT* vblk = kblk + static_cast<size_t>(Hkv) * BS * D;
  for (int j = threadIdx.x; j < Hkv * D; j += blockDim.x) {
    const int h = j / D, d = j % D;
    KT* dst = vblk + (static_cast<size_t>(h) * D + d) * BS + off;
    if constexpr (sizeof(KT) == 2)
      *dst = vsrc[j];  // bf16 -> bf16: bit copy
    else
      kv_store(dst, bf2f(vsrc[j]), v_inv_scale);
  }
}

template <typename KT>
static void launch_rope_typed(bf16_t* q_out, const bf16_t* qkv, const int64_t* positions, const float* cos_sin,
                              KT* kv, long block_stride, const int64_t* slot_mapping, const bf16_t* qn,
                              const bf16_t* kn, int T, int Hq, int Hkv, int D, int BS, float eps, float kis, float vis,
                              hipStream_t s) {
  dim3 g(T), b(256);
  const bool norm = qn != nullptr;
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
