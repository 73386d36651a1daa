// Shared device helpers for the gfx950 (CDNA4, wave64) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MXS_CHECK_LAUNCH() (void)hipGetLastError()

// Kernel bounds checks.  `MXS_DEBUG_KERNELS=1 python setup_ext.py` compiles every
// kernel with -DMXS_DEBUG_KERNELS into build/obj-debug: a failing MXS_KCHECK prints the condition,
// file, line and block, then traps (the launch fails instead of reading or writing out of bounds).
// Release builds compile the checks away.
#ifdef MXS_DEBUG_KERNELS
#include <stdio.h>
#define MXS_KCHECK(cond)                                                                                   \
  do {                                                                                                     \
    if (!(cond)) {                                                                                         \
      printf("MXS_KCHECK failed %s:%d block %d thread %d: %s\n", __FILE__, __LINE__, (int)blockIdx.x,       \
             (int)threadIdx.x, #cond);                                                                      \
      __builtin_trap();                                                                                    \
    }                                                                                                      \
  } while (0)
#else
#define MXS_KCHECK(cond) ((void)0)
#endif

namespace mxs {

constexpr int kWave = 64;

typedef unsigned short bf16_t;  // raw bf16 bits
typedef short short8 __attribute__((ext_vector_type(8)));
typedef short short4 __attribute__((ext_vector_type(4)));
typedef float float4_ __attribute__((ext_vector_type(4)));
typedef float float16_ __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(static_cast<uint32_t>(v) << 16); }
__device__ __forceinline__ float bf2f_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf2f_hi(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }

// round-to-nearest-even f32 -> bf16 (NaN-preserving: a quiet-NaN pattern stays NaN)
__device__ __forceinline__ bf16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x7FFFFFu)) return static_cast<bf16_t>((u >> 16) | 0x40);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return static_cast<bf16_t>(u >> 16);
}
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return static_cast<uint32_t>(f2bf(lo)) | (static_cast<uint32_t>(f2bf(hi)) << 16);
}

// ---- fp8 KV cache (OCP e4m3fn, the gfx950 format; torch.float8_e4m3fn).  Every e4m3 value is exact
// in bf16 (3 mantissa bits, exponents well inside bf16's), so fp8 -> bf16 is v_cvt_pk_f32_fp8 and a
// truncation of the f32 bits; attention then runs its bf16 math unchanged on the converted words.
typedef unsigned char fp8_t;
typedef float f32x2_t __attribute__((ext_vector_type(2)));
constexpr float kFp8Max = 448.f;

// 4 fp8 (one dword) -> 4 bf16 (two dwords: {b0 | b1 << 16, b2 | b3 << 16})
__device__ __forceinline__ uint2 fp8x4_to_bf16x4(uint32_t w) {
  const f32x2_t a = __builtin_amdgcn_cvt_pk_f32_fp8(static_cast<int>(w), false);
  const f32x2_t b = __builtin_amdgcn_cvt_pk_f32_fp8(static_cast<int>(w), true);
  return make_uint2((__float_as_uint(a.x) >> 16) | (__float_as_uint(a.y) & 0xFFFF0000u),
                    (__float_as_uint(b.x) >> 16) | (__float_as_uint(b.y) & 0xFFFF0000u));
}
// 8 fp8 (two dwords) -> 8 bf16 (one 16-byte vector, same element order)
__device__ __forceinline__ uint4 fp8x8_to_bf16x8(uint2 w) {
  const uint2 lo = fp8x4_to_bf16x4(w.x), hi = fp8x4_to_bf16x4(w.y);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}
// f32 -> fp8 byte, saturating to +-448 (round to nearest even; NaN stays NaN)
__device__ __forceinline__ fp8_t f2fp8(float f) {
  const float c = fminf(fmaxf(f, -kFp8Max), kFp8Max);
  return static_cast<fp8_t>(__builtin_amdgcn_cvt_pk_fp8_f32(f != f ? f : c, 0.f, 0, false) & 0xFF);
}

// element store for a KV cache of bf16 or fp8 (scaled: stored = x * inv_scale)
__device__ __forceinline__ void kv_store(bf16_t* p, float x, float) { *p = f2bf(x); }
__device__ __forceinline__ void kv_store(fp8_t* p, float x, float inv_scale) { *p = f2fp8(x * inv_scale); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum with a caller-provided LDS scratch of >= (blockDim/64) floats.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += scratch[i];
  return t;
}
__device__ __forceinline__ float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, scratch[i]);
  return t;
}

}  // namespace mxs
