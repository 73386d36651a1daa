// K14 (MoE router): softmax over experts -> top-k -> renormalise, one wave per token (lane = expert).
// K15 (MoE align): tokens bucketed by expert with a counting sort so each expert's rows are
// contiguous for the grouped GEMM; K17 combine is a weighted scatter-add back to token order.
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
// One workgroup: per 64-assignment chunk every wave-lane learns its rank among equal experts from
// one ballot per local expert (E_local <= 64 on every config here).
__global__ void __launch_bounds__(64) moe_align_kernel(int* __restrict__ expert_offsets, int* __restrict__ perm,
                                                       const int* __restrict__ topk_ids, int TK, int e_lo,
                                                       int E_local) {
  __shared__ int cnt[257];
  const int lane = threadIdx.x;
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (int e = lane; e <= E_local; e += 64) cnt[e] = 0;
  __syncthreads();
  for (int i = lane; i < TK; i += 64) {
    const int e = topk_ids[i] - e_lo;
    if (e >= 0 && e < E_local) atomicAdd(&cnt[e + 1], 1);
  }
  __syncthreads();
  if (lane == 0) {
    for (int e = 0; e < E_local; ++e) cnt[e + 1] += cnt[e];
    for (int e = 0; e <= E_local; ++e) expert_offsets[e] = cnt[e];
  }
  __syncthreads();
  for (int base = 0; base < TK; base += 64) {
    const int i = base + lane;
    const int e = i < TK ? topk_ids[i] - e_lo : -1;
    int dst = -1;
    for (int x = 0; x < E_local; ++x) {
      const unsigned long long m = __ballot(e == x);
      if (m == 0ull) continue;
      if (e == x) dst = cnt[x] + __popcll(m & lt);
      __syncthreads();
      if (lane == 0) cnt[x] += __popcll(m);
      __syncthreads();
    }
    if (dst >= 0) perm[dst] = i;
  }
}

void launch_moe_align(int* expert_offsets, int* perm, const int* topk_ids, int TK, int e_lo, int E_local,
                      hipStream_t s) {
  hipLaunchKernelGGL(moe_align_kernel, dim3(1), dim3(64), 0, s, expert_offsets, perm, topk_ids, TK, e_lo,
                     E_local);
  MXS_CHECK_LAUNCH();
}

}  // namespace mxs
