// K02 RMSNorm (+ fused residual add), K01 embedding gather fused into the first RMSNorm, and K10
// SiLU*mul for gfx950.
// Memory-bound: every access is a 16-byte bf16x8 vector (cdna_hip_programming.md Guideline 13),
// the row stays in registers between the reduction and the scaled write (one HBM pass).
#include "common.h"
#include <cstdlib>

namespace mxs {

// One workgroup per row. NV = number of bf16x8 vectors each thread keeps in registers.
// EMBED: row r of x is the embedding row ids[r] (x = the table); the gathered row is also written to
// `residual` (the residual stream starts as the embedding), so the first layer's input norm reads
// the table once instead of an embedding kernel writing x and the norm reading it back.
template <int NV, bool ADD, bool EMBED = false>
__global__ void __launch_bounds__(1024) rmsnorm_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ x,
                                                       bf16_t* __restrict__ residual, const bf16_t* __restrict__ w,
                                                       int H, int x_stride, float eps,
                                                       const int64_t* __restrict__ ids = nullptr) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const bf16_t* xr = x + (EMBED ? ids[row] : static_cast<int64_t>(row)) * x_stride;
  bf16_t* rr = (ADD || EMBED) ? residual + static_cast<size_t>(row) * H : nullptr;
  const int nvec = H >> 3;
  uint4 v[NV];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      uint4 a = *reinterpret_cast<const uint4*>(xr + c * 8);
      if (ADD) {
        const uint4 b = *reinterpret_cast<const uint4*>(rr + c * 8);
        uint32_t* pa = reinterpret_cast<uint32_t*>(&a);
        const uint32_t* pb = reinterpret_cast<const uint32_t*>(&b);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          pa[k] = pack2(bf2f_lo(pa[k]) + bf2f_lo(pb[k]), bf2f_hi(pa[k]) + bf2f_hi(pb[k]));
        *reinterpret_cast<uint4*>(rr + c * 8) = a;
      }
      if (EMBED) *reinterpret_cast<uint4*>(rr + c * 8) = a;
      v[i] = a;
      const uint32_t* p = reinterpret_cast<const uint32_t*>(&a);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float lo = bf2f_lo(p[k]), hi = bf2f_hi(p[k]);
        ss += lo * lo + hi * hi;
      }
    }
  }
  const float inv = rsqrtf(block_sum(ss, scratch) / static_cast<float>(H) + eps);
  bf16_t* orow = out + static_cast<size_t>(row) * H;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      const uint4 wv = *reinterpret_cast<const uint4*>(w + c * 8);
      const uint32_t* p = reinterpret_cast<const uint32_t*>(&v[i]);
      const uint32_t* pw = reinterpret_cast<const uint32_t*>(&wv);
      uint4 o;
      uint32_t* po = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        po[k] = pack2(bf2f_lo(p[k]) * inv * bf2f_lo(pw[k]), bf2f_hi(p[k]) * inv * bf2f_hi(pw[k]));
      *reinterpret_cast<uint4*>(orow + c * 8) = o;
    }
  }
}

// One WAVE per row (4 rows per 256-thread workgroup) for H = 512 NVW: lane l holds vectors l + 64 i,
// so every load / store instruction of a wave moves 1 KiB contiguous, and the sum of squares is a
// wave reduction (no LDS, no barrier).  The workgroup-per-row form above spends a block reduction and
// a barrier on each 4 KiB row at H = 2048; at prefill row counts it reads and writes at ~4.5 TB/s.
template <int NVW, bool ADD>
__global__ void __launch_bounds__(256) rmsnorm_rows_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ x,
                                                          bf16_t* __restrict__ residual, const bf16_t* __restrict__ w,
                                                          int rows, int H, int x_stride, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;  // wave-uniform: no barrier below
  const bf16_t* xr = x + static_cast<int64_t>(row) * x_stride;
  bf16_t* rr = ADD ? residual + static_cast<size_t>(row) * H : nullptr;
  // every load of the row (x, the residual, the weight) issued before the first use: one latency
  uint4 v[NVW], rv[ADD ? NVW : 1], wv[NVW];
#pragma unroll
  for (int i = 0; i < NVW; ++i) {
    v[i] = *reinterpret_cast<const uint4*>(xr + (lane + 64 * i) * 8);
    if constexpr (ADD) rv[i] = *reinterpret_cast<const uint4*>(rr + (lane + 64 * i) * 8);
  }
#pragma unroll
  for (int i = 0; i < NVW; ++i) wv[i] = *reinterpret_cast<const uint4*>(w + (lane + 64 * i) * 8);
  if constexpr (ADD) {
#pragma unroll
    for (int i = 0; i < NVW; ++i) {
      uint32_t* pa = reinterpret_cast<uint32_t*>(&v[i]);
      const uint32_t* pb = reinterpret_cast<const uint32_t*>(&rv[i]);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        pa[k] = pack2(bf2f_lo(pa[k]) + bf2f_lo(pb[k]), bf2f_hi(pa[k]) + bf2f_hi(pb[k]));
      *reinterpret_cast<uint4*>(rr + (lane + 64 * i) * 8) = v[i];
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NVW; ++i) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(&v[i]);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float lo = bf2f_lo(p[k]), hi = bf2f_hi(p[k]);
      ss += lo * lo + hi * hi;
    }
  }
  const float inv = rsqrtf(wave_sum(ss) / static_cast<float>(H) + eps);
  bf16_t* orow = out + static_cast<size_t>(row) * H;
#pragma unroll
  for (int i = 0; i < NVW; ++i) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(&v[i]);
    const uint32_t* pw = reinterpret_cast<const uint32_t*>(&wv[i]);
    uint4 o;
    uint32_t* po = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      po[k] = pack2(bf2f_lo(p[k]) * inv * bf2f_lo(pw[k]), bf2f_hi(p[k]) * inv * bf2f_hi(pw[k]));
    *reinterpret_cast<uint4*>(orow + (lane + 64 * i) * 8) = o;
  }
}

template <bool ADD, bool EMBED = false>
static void launch_rmsnorm_t(bf16_t* out, const bf16_t* x, bf16_t* res, const bf16_t* w, int rows, int H,
                             int x_stride, float eps, hipStream_t s, const int64_t* ids = nullptr) {
  if (rows == 0) return;
  if constexpr (!EMBED) {
    const int nvw = H % 512 == 0 ? H / 512 : 0;  // vectors per lane of the wave-per-row form
    static const bool block_only = [] {  // MXS_RMS_BLOCK=1: the workgroup-per-row form (A/B only)
      const char* e = std::getenv("MXS_RMS_BLOCK");
      return e != nullptr && e[0] == '1';
    }();
    // the workgroup-per-row form has the lower latency for decode-sized row counts; the wave form
    // moves more bytes per second from ~2k rows (4k with the residual add): 6,144 x 2,048 plain
    // 11.2 -> 9.6 us, 8,192 14.1 -> 11.4 us (scripts/probes/rmsnorm_probe.py)
    const bool wave_form = !block_only && rows >= (ADD ? 4096 : 2048) &&
                           ((nvw >= 1 && nvw <= 8) || nvw == 10 || nvw == 12 || nvw == 14 || nvw == 16);
    if (wave_form && (reinterpret_cast<uintptr_t>(x) & 15) == 0 && x_stride % 8 == 0) {
      dim3 g((rows + 3) / 4), b(256);
#define MXS_RMSW(NV) \
  case NV:           \
    hipLaunchKernelGGL((rmsnorm_rows_kernel<NV, ADD>), g, b, 0, s, out, x, res, w, rows, H, x_stride, eps); break;
      switch (nvw) {
        MXS_RMSW(1) MXS_RMSW(2) MXS_RMSW(3) MXS_RMSW(4) MXS_RMSW(5) MXS_RMSW(6) MXS_RMSW(7) MXS_RMSW(8)
        MXS_RMSW(10) MXS_RMSW(12) MXS_RMSW(14) MXS_RMSW(16)
        default: break;
      }
#undef MXS_RMSW
      MXS_CHECK_LAUNCH();
      return;
    }
  }
  const int nvec = H / 8;
  // one bf16x8 per thread up to H = 8192 (1024 threads); wider rows keep NV vectors per thread
  const int threads = nvec <= 1024 ? ((nvec + 63) / 64) * 64 : 1024;
  const int nv = (nvec + threads - 1) / threads;
  dim3 g(rows), b(threads);
#define MXS_RMS(NVV) \
  hipLaunchKernelGGL((rmsnorm_kernel<NVV, ADD, EMBED>), g, b, 0, s, out, x, res, w, H, x_stride, eps, ids)
  switch (nv) {
    case 1: MXS_RMS(1); break;
    case 2: MXS_RMS(2); break;
    case 3: MXS_RMS(3); break;
    case 4: MXS_RMS(4); break;
    default: MXS_RMS(8); break;
  }
#undef MXS_RMS
  MXS_CHECK_LAUNCH();
}

// h = rmsnorm(table[ids]) * w, residual = table[ids]
void launch_embed_rms_norm(bf16_t* out, bf16_t* residual, const int64_t* ids, const bf16_t* table, const bf16_t* w,
                           int rows, int H, float eps, hipStream_t s) {
  launch_rmsnorm_t<false, true>(out, table, residual, w, rows, H, H, eps, s, ids);
}

void launch_rms_norm(bf16_t* out, const bf16_t* x, const bf16_t* w, int rows, int H, int x_stride, float eps,
                     hipStream_t s) {
  launch_rmsnorm_t<false>(out, x, nullptr, w, rows, H, x_stride, eps, s);
}

void launch_fused_add_rms_norm(bf16_t* out, const bf16_t* x, bf16_t* residual, const bf16_t* w, int rows, int H,
                               float eps, hipStream_t s) {
  launch_rmsnorm_t<true>(out, x, residual, w, rows, H, H, eps, s);
}

// Split-K epilogue of a projection that feeds the residual stream (o_proj, down_proj at TP = 1):
// y = sum of the S fp32 slabs [S][M][N] the GEMM left (gemm_decode.hip, reduce skipped), rounded to
// bf16 as the GEMM's own output would be; residual += y (in place); out = RMSNorm(residual) * w.
// One launch instead of the split-K reduce kernel plus the fused add + RMSNorm kernel, and the
// projection output never makes a bf16 round trip through memory.  One workgroup per row, the row
// in registers between the reduction and the scaled write.
template <int NV>
__global__ void __launch_bounds__(1024) splitk_add_rmsnorm_kernel(bf16_t* __restrict__ out, bf16_t* __restrict__ residual,
                                                                  const float* __restrict__ part, int S, int M,
                                                                  int H, const bf16_t* __restrict__ w, float eps) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  bf16_t* rr = residual + static_cast<size_t>(row) * H;
  const int nvec = H >> 3;
  const size_t slab = static_cast<size_t>(M) * H;
  uint4 v[NV];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      const float* p = part + static_cast<size_t>(row) * H + c * 8;
      float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
      // 4 slabs' loads in flight at a time, summed in slab order (a load -> add chain costs one L2
      // round trip per slab, the whole latency of a batch-1 row)
      for (int s0 = 1; s0 < S; s0 += 4) {
        float4 a2[4], b2[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const size_t o = static_cast<size_t>(s0 + j < S ? s0 + j : 0) * slab;
          a2[j] = *reinterpret_cast<const float4*>(p + o);
          b2[j] = *reinterpret_cast<const float4*>(p + o + 4);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (s0 + j < S) {
            a.x += a2[j].x; a.y += a2[j].y; a.z += a2[j].z; a.w += a2[j].w;
            b.x += b2[j].x; b.y += b2[j].y; b.z += b2[j].z; b.w += b2[j].w;
          }
      }
      const float y[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      const uint4 rv = *reinterpret_cast<const uint4*>(rr + c * 8);
      const uint32_t* pr = reinterpret_cast<const uint32_t*>(&rv);
      uint4 o;
      uint32_t* po = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
      for (int k = 0; k < 4; ++k)  // bf16(y) + residual, rounded as the unfused path rounds it
        po[k] = pack2(bf2f(f2bf(y[2 * k])) + bf2f_lo(pr[k]), bf2f(f2bf(y[2 * k + 1])) + bf2f_hi(pr[k]));
      *reinterpret_cast<uint4*>(rr + c * 8) = o;
      v[i] = o;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float lo = bf2f_lo(po[k]), hi = bf2f_hi(po[k]);
        ss += lo * lo + hi * hi;
      }
    }
  }
  const float inv = rsqrtf(block_sum(ss, scratch) / static_cast<float>(H) + eps);
  bf16_t* orow = out + static_cast<size_t>(row) * H;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      const uint4 wv = *reinterpret_cast<const uint4*>(w + c * 8);
      const uint32_t* p = reinterpret_cast<const uint32_t*>(&v[i]);
      const uint32_t* pw = reinterpret_cast<const uint32_t*>(&wv);
      uint4 o;
      uint32_t* po = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        po[k] = pack2(bf2f_lo(p[k]) * inv * bf2f_lo(pw[k]), bf2f_hi(p[k]) * inv * bf2f_hi(pw[k]));
      *reinterpret_cast<uint4*>(orow + c * 8) = o;
    }
  }
}

void launch_splitk_add_rms_norm(bf16_t* out, bf16_t* residual, const float* part, int S, int M, int H, const bf16_t* w,
                                float eps, hipStream_t s) {
  if (M == 0) return;
  const int nvec = H / 8;
  const int threads = nvec <= 1024 ? ((nvec + 63) / 64) * 64 : 1024;
  const int nv = (nvec + threads - 1) / threads;
#define MXS_SKR(NVV)                                                                                        \
  hipLaunchKernelGGL((splitk_add_rmsnorm_kernel<NVV>), dim3(M), dim3(threads), 0, s, out, residual, part, S, M, \
                     H, w, eps)
  switch (nv) {
    case 1: MXS_SKR(1); break;
    case 2: MXS_SKR(2); break;
    case 3: MXS_SKR(3); break;
    case 4: MXS_SKR(4); break;
    default: MXS_SKR(8); break;
  }
#undef MXS_SKR
  MXS_CHECK_LAUNCH();
}

// out[t, i] = silu(gu[t, i]) * gu[t, I + i]; 8 elements per thread, grid-stride.
__global__ void silu_mul_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ gu, int rows, int I) {
  const int vec_per_row = I >> 3;
  const long total = static_cast<long>(rows) * vec_per_row;
  for (long idx = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; idx < total;
       idx += static_cast<long>(gridDim.x) * blockDim.x) {
    const long r = idx / vec_per_row;
    const int c = static_cast<int>(idx - r * vec_per_row) * 8;
    const bf16_t* g = gu + r * 2 * I + c;
    const uint4 gv = *reinterpret_cast<const uint4*>(g);
    const uint4 uv = *reinterpret_cast<const uint4*>(g + I);
    const uint32_t* pg = reinterpret_cast<const uint32_t*>(&gv);
    const uint32_t* pu = reinterpret_cast<const uint32_t*>(&uv);
    uint4 o;
    uint32_t* po = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float g0 = bf2f_lo(pg[k]), g1 = bf2f_hi(pg[k]);
      const float s0 = g0 / (1.f + __expf(-g0)), s1 = g1 / (1.f + __expf(-g1));
      po[k] = pack2(s0 * bf2f_lo(pu[k]), s1 * bf2f_hi(pu[k]));
    }
    *reinterpret_cast<uint4*>(out + r * I + c) = o;
  }
}

void launch_silu_mul(bf16_t* out, const bf16_t* gu, int rows, int I, hipStream_t s) {
  const long total = static_cast<long>(rows) * (I / 8);
  long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(silu_mul_kernel, dim3(blocks), dim3(256), 0, s, out, gu, rows, I);
  MXS_CHECK_LAUNCH();
}

}  // namespace mxs
