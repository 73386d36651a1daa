// K14 (MoE router): softmax over experts -> top-k -> renormalise, one wave per token (lane = expert).
// K15 (MoE align): tokens bucketed by expert with a counting sort so each expert's rows are
// contiguous for the grouped GEMM; K17 (MoE combine): each token gathers its top-k expert rows
// through the inverse permutation and sums them with the routing weights (no scatter atomics).
#include "common.h"

namespace mxs {

__global__ void moe_topk_softmax_kernel(float* __restrict__ topk_w, int* __restrict__ topk_ids,
                                        const bf16_t* __restrict__ logits, int T, int E, int K) {
  const int t = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= T) return;
  float x = lane < E ? bf2f(logits[static_cast<size_t>(t) * E + lane]) : -INFINITY;
  const float mx = wave_max(x);
  const float e = lane < E ? __expf(x - mx) : 0.f;
  const float sum = wave_sum(e);
  float p = e / sum;
  float picked = 0.f, myw = 0.f;
  int myid = 0;
  for (int k = 0; k < K; ++k) {
    float bv = lane < E ? p : -1.f;
    int bi = lane;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if (lane == k) {
      myw = bv;
      myid = bi;
    }
    picked += bv;
    if (lane == bi) p = -2.f;  // remove from further rounds
  }
  if (lane < K) {
    topk_w[static_cast<size_t>(t) * K + lane] = myw / picked;
    topk_ids[static_cast<size_t>(t) * K + lane] = myid;
  }
}

void launch_moe_topk_softmax(float* w, int* ids, const bf16_t* logits, int T, int E, int K, hipStream_t s) {
  if (T == 0) return;
  const int waves = 4;
  hipLaunchKernelGGL(moe_topk_softmax_kernel, dim3((T + waves - 1) / waves), dim3(64 * waves), 0, s, w, ids,
                     logits, T, E, K);
  MXS_CHECK_LAUNCH();
}

// Counting sort of the T*K (token, slot) assignments by expert, stable in assignment order.
// Outputs: expert_offsets[E_local+1] (row ranges in the permuted order), perm[] = flat (t*K + k)
// index of each permuted row.  Only experts in [e_lo, e_lo + E_local) are kept (expert parallel).
// inv (optional): inv[i] = permuted row of assignment i, -1 when its expert is not local.
// One 1024-thread workgroup (a prefill chunk of 8192 tokens x top-2 is 16 passes, not 256):
//   counts   LDS atomics, then an exclusive scan by thread 0 (E_local <= 256);
//   ranks    per 1024-assignment pass, one ballot per local expert gives each lane its rank among
//            equal experts in its wave; a wave's offset is the sum of the earlier waves' counts
//            (kept per wave in LDS), so the order stays the assignment order with no atomics.
constexpr int kAlignMaxE = 256;
constexpr int kAlignWaves = 16;

__global__ void __launch_bounds__(1024) moe_align_kernel(int* __restrict__ expert_offsets, int* __restrict__ perm,
                                                         const int* __restrict__ topk_ids, int TK, int e_lo,
                                                         int E_local, int* __restrict__ inv) {
  __shared__ int base[kAlignMaxE + 1];
  __shared__ int wave_tot[kAlignWaves][kAlignMaxE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (int e = tid; e <= E_local; e += blockDim.x) base[e] = 0;
  __syncthreads();
  for (int i = tid; i < TK; i += blockDim.x) {
    const int e = topk_ids[i] - e_lo;
    if (e >= 0 && e < E_local) atomicAdd(&base[e + 1], 1);
  }
  __syncthreads();
  if (tid == 0) {
    for (int e = 0; e < E_local; ++e) base[e + 1] += base[e];
    for (int e = 0; e <= E_local; ++e) expert_offsets[e] = base[e];
  }
  __syncthreads();
  for (int p0 = 0; p0 < TK; p0 += blockDim.x) {
    const int i = p0 + tid;
    int e = i < TK ? topk_ids[i] - e_lo : -1;
    if (e >= E_local) e = -1;
    int rank = 0;
    for (int x = 0; x < E_local; ++x) {
      const unsigned long long m = __ballot(e == x);
      if (e == x) rank = __popcll(m & lt);
      if (lane == 0) wave_tot[wid][x] = __popcll(m);
    }
    __syncthreads();
    int dst = -1;
    if (e >= 0) {
      dst = base[e] + rank;
      for (int w = 0; w < wid; ++w) dst += wave_tot[w][e];
      perm[dst] = i;
    }
    if (inv != nullptr && i < TK) inv[i] = dst;
    __syncthreads();
    const int nw = blockDim.x >> 6;
    for (int x = tid; x < E_local; x += blockDim.x) {
      int t = 0;
      for (int w = 0; w < nw; ++w) t += wave_tot[w][x];
      base[x] += t;
    }
    __syncthreads();
  }
}

void launch_moe_align(int* expert_offsets, int* perm, const int* topk_ids, int TK, int e_lo, int E_local,
                      int* inv, hipStream_t s) {
  if (E_local < 1 || E_local > kAlignMaxE) return;
  hipLaunchKernelGGL(moe_align_kernel, dim3(1), dim3(1024), 0, s, expert_offsets, perm, topk_ids, TK, e_lo,
                     E_local, inv);
  MXS_CHECK_LAUNCH();
}

// out[t] = sum_k w[t, k] * ys[inv[t K + k]] (rows with inv < 0 belong to other ranks' experts).
// One workgroup per token; 16-byte vectors, fp32 accumulation, one bf16 write per element.
__global__ void __launch_bounds__(256) moe_combine_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ ys,
                                                          const float* __restrict__ topk_w,
                                                          const int* __restrict__ inv, int K, int H) {
  const int t = blockIdx.x;
  int rows[8];
  float ws[8];
  for (int k = 0; k < K; ++k) {
    rows[k] = inv[t * K + k];
    ws[k] = topk_w[t * K + k];
  }
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; ++k) {
      if (rows[k] < 0) continue;
      const uint4 v = *reinterpret_cast<const uint4*>(ys + static_cast<size_t>(rows[k]) * H + c * 8);
      const uint32_t* p = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[2 * j] += ws[k] * bf2f_lo(p[j]);
        acc[2 * j + 1] += ws[k] * bf2f_hi(p[j]);
      }
    }
    uint4 o;
    o.x = pack2(acc[0], acc[1]);
    o.y = pack2(acc[2], acc[3]);
    o.z = pack2(acc[4], acc[5]);
    o.w = pack2(acc[6], acc[7]);
    *reinterpret_cast<uint4*>(out + static_cast<size_t>(t) * H + c * 8) = o;
  }
}

void launch_moe_combine(bf16_t* out, const bf16_t* ys, const float* topk_w, const int* inv, int T, int K, int H,
                        hipStream_t s) {
  if (T == 0) return;
  hipLaunchKernelGGL(moe_combine_kernel, dim3(T), dim3(256), 0, s, out, ys, topk_w, inv, K, H);
  MXS_CHECK_LAUNCH();
}

// Split-K variant: the expert rows are S fp32 partial slices [S][rows][H] (moe_grouped_gemm split).
// One thread per (token, 4 columns): grid (T, H / 1024), every K x S slab load of the thread issued
// back to back (the loops are unrolled to their bounds, K <= 8 and S <= 8, with guards), so a decode
// batch of ~100 tokens is 400 workgroups of independent loads instead of 100 workgroups walking
// their rows with one dependent load at a time.
__global__ void __launch_bounds__(256) moe_combine_partials_kernel(bf16_t* __restrict__ out,
                                                                   const float* __restrict__ part,
                                                                   const float* __restrict__ topk_w,
                                                                   const int* __restrict__ inv, int K, int H, int S,
                                                                   long slice) {
  const int t = blockIdx.x;
  const int c = blockIdx.y * blockDim.x + threadIdx.x;
  if (c >= H / 4) return;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (k >= K) break;
    const int row = inv[t * K + k];
    if (row < 0) continue;
    const float w = topk_w[t * K + k];
    const float* p = part + static_cast<size_t>(row) * H + c * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int z = 0; z < 8; ++z) {
      if (z >= S) break;
      const float4 u = *reinterpret_cast<const float4*>(p + z * slice);
      v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    acc.x += w * v.x; acc.y += w * v.y; acc.z += w * v.z; acc.w += w * v.w;
  }
  *reinterpret_cast<uint2*>(out + static_cast<size_t>(t) * H + c * 4) = make_uint2(pack2(acc.x, acc.y),
                                                                                   pack2(acc.z, acc.w));
}

// Split-K gate_up: h[r, j] = silu(sum_z P[z][r][j]) * sum_z P[z][r][I + j]  (P: [S][rows][2I] fp32)
__global__ void silu_mul_partials_kernel(bf16_t* __restrict__ h, const float* __restrict__ part, int rows, int I,
                                         int S, long slice) {
  const long total = static_cast<long>(rows) * (I / 4);
  for (long idx = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; idx < total;
       idx += static_cast<long>(gridDim.x) * blockDim.x) {
    const long r = idx / (I / 4);
    const int j = static_cast<int>(idx - r * (I / 4)) * 4;
    const float* pg = part + r * 2 * I + j;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f), u = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int z = 0; z < 8; ++z) {  // S <= 8: unrolled so the slab loads are in flight together
      if (z >= S) break;
      const float4 a = *reinterpret_cast<const float4*>(pg + z * slice);
      const float4 b = *reinterpret_cast<const float4*>(pg + z * slice + I);
      g.x += a.x; g.y += a.y; g.z += a.z; g.w += a.w;
      u.x += b.x; u.y += b.y; u.z += b.z; u.w += b.w;
    }
    const float o0 = g.x / (1.f + __expf(-g.x)) * u.x, o1 = g.y / (1.f + __expf(-g.y)) * u.y;
    const float o2 = g.z / (1.f + __expf(-g.z)) * u.z, o3 = g.w / (1.f + __expf(-g.w)) * u.w;
    *reinterpret_cast<uint2*>(h + r * I + j) = make_uint2(pack2(o0, o1), pack2(o2, o3));
  }
}

void launch_silu_mul_partials(bf16_t* h, const float* part, int rows, int I, int S, long slice, hipStream_t s) {
  const long total = static_cast<long>(rows) * (I / 4);
  if (total == 0) return;
  long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(silu_mul_partials_kernel, dim3(blocks), dim3(256), 0, s, h, part, rows, I, S, slice);
  MXS_CHECK_LAUNCH();
}

void launch_moe_combine_partials(bf16_t* out, const float* part, const float* topk_w, const int* inv, int T, int K,
                                 int H, int S, long slice, hipStream_t s) {
  if (T == 0) return;
  if (K > 8 || S > 8) return;  // callers: top-k <= 8, split-K <= 8 (checked in the bindings)
  hipLaunchKernelGGL(moe_combine_partials_kernel, dim3(T, (H / 4 + 255) / 256), dim3(256), 0, s, out, part, topk_w,
                     inv, K, H, S, slice);
  MXS_CHECK_LAUNCH();
}

}  // namespace mxs
