// Expert-parallel token dispatch on the device (Mixtral EP=8).
//
// Each rank routes its slice of S tokens (top-k experts each, P = S*k pairs) and sends every pair's
// hidden row to the rank owning the expert.  Destination d's rows go to a segment of C rows of a
// send buffer (C = capacity); the IPC all-to-all then pushes only the first counts[d] rows of each
// segment over xGMI, so the wire carries the real rows, not the worst-case capacity.
//
//   ep_route        one workgroup: dest / local expert of every pair, a STABLE position inside its
//                   destination (wave ballots + a cross-wave prefix in LDS, pairs in order), the
//                   pair's slot = d*C + pos (-1 for padding rows), the segment's expert ids (-1
//                   past the count) and the per-destination counts.  Deterministic, no atomics.
//   ep_gather_rows  send_x[slot[p]] = hs[p / k] (16-byte vectors, one workgroup per pair).
//   ep_segment_rows counts[s] = valid expert ids in segment s of a received id buffer (the rows to
//                   push back on the return trip).
// The weighted combine back into token order is the K17 kernel (moe_combine) with inv = slot.
#include "common.h"

namespace mxs {

constexpr int kEpMaxRanks = 8;

__global__ void __launch_bounds__(1024) ep_route_kernel(int* __restrict__ slot, int* __restrict__ send_e,
                                                        int* __restrict__ counts, const int* __restrict__ topk_ids,
                                                        int P, int k, int valid_rows, int e_local, int nranks,
                                                        int C) {
  __shared__ int wave_tot[16][kEpMaxRanks];
  __shared__ int base[kEpMaxRanks];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nw = blockDim.x >> 6;
  if (tid < kEpMaxRanks) base[tid] = 0;
  // every expert-id entry starts invalid (graph replays reuse the buffer)
  for (int i = tid; i < nranks * C; i += blockDim.x) send_e[i] = -1;
  __syncthreads();
  for (int p0 = 0; p0 < P; p0 += blockDim.x) {
    const int p = p0 + tid;
    int d = -1, le = -1;
    if (p < P && p / k < valid_rows) {
      const int e = topk_ids[p];
      d = e / e_local;
      le = e - d * e_local;
      if (d < 0 || d >= nranks) d = -1;
    }
    int my_pos = 0;
    for (int r = 0; r < nranks; ++r) {
      const unsigned long long m = __ballot(d == r);
      if (d == r) my_pos = __popcll(m & ((1ull << lane) - 1ull));
      if (lane == 0) wave_tot[wid][r] = __popcll(m);
    }
    __syncthreads();
    if (d >= 0) {
      int pre = base[d];
      for (int w = 0; w < wid; ++w) pre += wave_tot[w][d];
      const int pos = pre + my_pos;
      MXS_KCHECK(pos < C);
      slot[p] = d * C + pos;
      send_e[d * C + pos] = le;
    } else if (p < P) {
      slot[p] = -1;
    }
    __syncthreads();
    if (tid < nranks) {
      int t = 0;
      for (int w = 0; w < nw; ++w) t += wave_tot[w][tid];
      base[tid] += t;
    }
    __syncthreads();
  }
  if (tid < nranks) counts[tid] = base[tid];
}

__global__ void __launch_bounds__(256) ep_gather_rows_kernel(bf16_t* __restrict__ send_x, const bf16_t* __restrict__ hs,
                                                             const int* __restrict__ slot, int k, int H, int nrows) {
  const int p = blockIdx.x;
  const int s = slot[p];
  if (s < 0) return;
  MXS_KCHECK(s < nrows);
  const uint4* src = reinterpret_cast<const uint4*>(hs + static_cast<size_t>(p / k) * H);
  uint4* dst = reinterpret_cast<uint4*>(send_x + static_cast<size_t>(s) * H);
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) dst[c] = src[c];
}

__global__ void __launch_bounds__(256) ep_segment_rows_kernel(int* __restrict__ counts, const int* __restrict__ ids,
                                                              int C) {
  const int s = blockIdx.x;
  int n = 0;
  for (int i = threadIdx.x; i < C; i += blockDim.x) n += ids[s * C + i] >= 0;
  __shared__ int part[4];
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) counts[s] = part[0] + part[1] + part[2] + part[3];
}

void launch_ep_route(int* slot, int* send_e, int* counts, const int* topk_ids, int P, int k, int valid_rows,
                     int e_local, int nranks, int C, hipStream_t s) {
  hipLaunchKernelGGL(ep_route_kernel, dim3(1), dim3(1024), 0, s, slot, send_e, counts, topk_ids, P, k, valid_rows,
                     e_local, nranks, C);
  MXS_CHECK_LAUNCH();
}

void launch_ep_gather_rows(bf16_t* send_x, const bf16_t* hs, const int* slot, int P, int k, int H, int nrows,
                           hipStream_t s) {
  if (P == 0) return;
  hipLaunchKernelGGL(ep_gather_rows_kernel, dim3(P), dim3(256), 0, s, send_x, hs, slot, k, H, nrows);
  MXS_CHECK_LAUNCH();
}

void launch_ep_segment_rows(int* counts, const int* ids, int nseg, int C, hipStream_t s) {
  hipLaunchKernelGGL(ep_segment_rows_kernel, dim3(nseg), dim3(256), 0, s, counts, ids, C);
  MXS_CHECK_LAUNCH();
}

}  // namespace mxs
