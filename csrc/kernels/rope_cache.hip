// K03+K04: (optional Qwen3 per-head q/k RMSNorm) -> rotate-half RoPE on q and k -> scatter k, v into
// the paged KV cache, all in one pass over the fused QKV projection output.
// Cache layout per layer (see mxserve/ops/reference.py): block b at kv + b*block_stride,
//   K: [Hkv][BS][D] (token-major)   V: [Hkv][D][BS] (dim-major, so attention's P*V operand is a
//   contiguous 16-byte load per lane).
// cos/sin come from a host-precomputed fp32 table (cdna_hip_programming.md App. B: no device trig).
#include "common.h"

namespace mxs {

template <int D, bool QKNORM>
__global__ void __launch_bounds__(256) rope_cache_kernel(
    bf16_t* __restrict__ q_out, const bf16_t* __restrict__ qkv, const int64_t* __restrict__ positions,
    const float* __restrict__ cos_sin, bf16_t* __restrict__ kv, long block_stride,
    const int64_t* __restrict__ slot_mapping, const bf16_t* __restrict__ qn, const bf16_t* __restrict__ kn,
    int Hq, int Hkv, int BS, float eps) {
  constexpr int HALF = D / 2;
  const int t = blockIdx.x;
  const int row_stride = (Hq + 2 * Hkv) * D;
  const bf16_t* src = qkv + static_cast<size_t>(t) * row_stride;
  const long pos = positions[t];
  const long slot = slot_mapping[t];
  const float* cs = cos_sin + pos * D;
  bf16_t* kblk = nullptr;
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
      bf16_t* kd = kblk + (static_cast<size_t>(head - Hq) * BS + off) * D;
      kd[p] = f2bf(o1);
      kd[p + HALF] = f2bf(o2);
    }
  }
  if (!kblk) return;
  // V: copy into the dim-major half of the block
  const bf16_t* vsrc = src + (Hq + Hkv) * D;
  bf16_t* vblk = kblk + static_cast<size_t>(Hkv) * BS * D;
  for (int j = threadIdx.x; j < Hkv * D; j += blockDim.x) {
    const int h = j / D, d = j % D;
    vblk[(static_cast<size_t>(h) * D + d) * BS + off] = vsrc[j];
  }
}

void launch_rope_and_cache(bf16_t* q_out, const bf16_t* qkv, const int64_t* positions, const float* cos_sin,
                           bf16_t* kv, long block_stride, const int64_t* slot_mapping, const bf16_t* qn,
                           const bf16_t* kn, int T, int Hq, int Hkv, int D, int BS, float eps, hipStream_t s) {
  if (T == 0) return;
  dim3 g(T), b(256);
  const bool norm = qn != nullptr;
#define MXS_ROPE_CASE(DD)                                                                                   \
  if (D == DD) {                                                                                            \
    if (norm)                                                                                               \
      hipLaunchKernelGGL((rope_cache_kernel<DD, true>), g, b, 0, s, q_out, qkv, positions, cos_sin, kv,     \
                         block_stride, slot_mapping, qn, kn, Hq, Hkv, BS, eps);                             \
    else                                                                                                    \
      hipLaunchKernelGGL((rope_cache_kernel<DD, false>), g, b, 0, s, q_out, qkv, positions, cos_sin, kv,    \
                         block_stride, slot_mapping, qn, kn, Hq, Hkv, BS, eps);                             \
    MXS_CHECK_LAUNCH();                                                                                     \
    return;                                                                                                 \
  }
  MXS_ROPE_CASE(64)
  MXS_ROPE_CASE(128)
  MXS_ROPE_CASE(32)
#undef MXS_ROPE_CASE
}

}  // namespace mxs
