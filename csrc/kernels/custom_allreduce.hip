// K18: one-shot IPC all-reduce for TP decode.
//
// xGMI on an MI355X node is a full mesh: every GPU has a direct link to each of its 7 peers, so a
// ring (RCCL's algorithm for small messages) walks one link per hop and pays 2(N-1) latencies.
// Here every rank PUSHES its input straight into a receive slot of every peer (N-1 links carry
// stores at once, posted writes: no round trip), raises one flag per (block, peer), waits for the
// N-1 flags addressed to it, and sums the N slots from its OWN memory.
//
// Buffers (allocated once per rank with hipDeviceMallocUncached, exported with hipIpc, mapped by
// every peer; each well under 2 GiB, see mxserve/disagg/kv_transfer.py for the size rule):
//   recv[2][N][max_elems]  two parities: call k writes parity k & 1, so a peer can run one call
//                          ahead without overwriting slots this rank is still summing (it cannot
//                          run two ahead: call k+1 waits for this rank's flags of call k+1, which
//                          are only raised after this rank has finished call k) - no exit barrier
//   flags[max_blocks][N]   flag[b][r] = last epoch rank r published for block b
//   epoch[max_blocks]      per-block call counter kept on the device (hipGraph-safe: no host
//                          epoch argument that a captured graph would freeze)
// Memory model: payload stores + __threadfence_system() (release at system scope) before a flag is
// stored with a system-scope atomic; the waiter polls with system-scope atomic loads and then
// fences acquire at system scope.  The uncached allocation keeps stale lines out of every L2.
// Spins are bounded: a peer that never arrives sets err[0] and the call returns (the host then
// falls back to RCCL for good), so a broken link cannot hang the GPU.
#include "common.h"

namespace mxs {

constexpr int kArMaxRanks = 8;
constexpr int kArMaxBlocks = 64;

struct ArPeers {
  char* recv[kArMaxRanks];    // each rank's recv base, mapped into this process
  unsigned* flags[kArMaxRanks];
};

__device__ __forceinline__ void st_flag(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned ld_flag(unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// x: this rank's input (bf16, n elements, n % 8 == 0); out: result (may alias x)
__global__ void __launch_bounds__(512) custom_allreduce_kernel(bf16_t* out, const bf16_t* __restrict__ x, long n,
                                                               ArPeers peers, int rank, int nranks,
                                                               long slot_elems, unsigned* epochs, unsigned* err) {
  const int b = blockIdx.x;
  const long nv = n / 8;  // 16-byte vectors
  const long per = (nv + gridDim.x - 1) / gridDim.x;
  const long v0 = b * per, v1 = min(nv, v0 + per);
  __shared__ unsigned s_epoch;
  if (threadIdx.x == 0) s_epoch = epochs[b] + 1;
  __syncthreads();
  const unsigned e = s_epoch;
  const int par = e & 1;
  // 1. push this block's chunk into slot [par][rank] of every rank (self included)
  const uint4* xs = reinterpret_cast<const uint4*>(x);
  for (int r = 0; r < nranks; ++r) {
    uint4* dst = reinterpret_cast<uint4*>(peers.recv[r] + ((static_cast<long>(par) * nranks + rank) * slot_elems) * 2);
    for (long v = v0 + threadIdx.x; v < v1; v += blockDim.x) dst[v] = xs[v];
  }
  // 2. release + one flag per peer
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < nranks) st_flag(peers.flags[threadIdx.x] + b * kArMaxRanks + rank, e);
  // 3. wait for every rank's flag of this epoch (bounded spin)
  if (threadIdx.x < nranks) {
    unsigned* f = peers.flags[rank] + b * kArMaxRanks + threadIdx.x;
    long spins = 0;
    while (static_cast<int>(ld_flag(f) - e) < 0) {
      if (++spins > (1L << 26) || ld_flag(err) != 0) {
        atomicExch(err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  // 4. sum the N slots (local memory) in fp32, rank order (every rank gets identical bits)
  const char* mine = peers.recv[rank] + (static_cast<long>(par) * nranks * slot_elems) * 2;
  uint4* o = reinterpret_cast<uint4*>(out);
  for (long v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < nranks; ++r) {
      const uint4 w = reinterpret_cast<const uint4*>(mine + r * slot_elems * 2)[v];
      const uint32_t u[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[2 * k] += bf2f_lo(u[k]);
        acc[2 * k + 1] += bf2f_hi(u[k]);
      }
    }
    uint4 rr;
    rr.x = pack2(acc[0], acc[1]);
    rr.y = pack2(acc[2], acc[3]);
    rr.z = pack2(acc[4], acc[5]);
    rr.w = pack2(acc[6], acc[7]);
    o[v] = rr;
  }
  if (threadIdx.x == 0) epochs[b] = e;
}

void launch_custom_allreduce(bf16_t* out, const bf16_t* x, long n, const ArPeers& peers, int rank, int nranks,
                             long slot_elems, unsigned* epochs, unsigned* err, hipStream_t s) {
  // ALWAYS kArMaxBlocks blocks: every block then counts the same calls, so the parity of a call is
  // the same in every block and chunk ranges may differ between calls of different sizes without a
  // peer that runs one call ahead ever writing into the parity this rank is still summing
  hipLaunchKernelGGL(custom_allreduce_kernel, dim3(kArMaxBlocks), dim3(512), 0, s, out, x, n, peers, rank, nranks,
                     slot_elems, epochs, err);
  MXS_CHECK_LAUNCH();
}

// Two-shot variant for larger messages (N > 2): reduce-scatter by push, then all-gather by push.
// Rank q owns slice q (1/N of the vectors).  Phase 1 pushes slice r of the input into rank r's slot
// [par][rank]; phase 2 sums the N contributions to the owned slice and pushes the result into every
// rank's slot [par][rank] at the same positions (the phase-1 data there sits at the receiver's own
// slice: disjoint); phase 3 reads every slice from its owner's slot.  Each xGMI link carries 2/N of
// the message instead of the one-shot's whole message, for one more flag round trip.  Same
// buffers, epochs and parity argument as the one-shot kernel (a peer can only get one call ahead:
// call k+1's phase 2 needs this rank's phase-1 flag of k+1); phase-2 flags live in the second half
// of the flag page.
constexpr int kArFlags2 = kArMaxBlocks * kArMaxRanks;

__device__ __forceinline__ void ar_wait(unsigned* f, unsigned e, unsigned* err) {
  long spins = 0;
  while (static_cast<int>(ld_flag(f) - e) < 0) {
    if (++spins > (1L << 26) || ld_flag(err) != 0) {
      atomicExch(err, 1u);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

__global__ void __launch_bounds__(512) custom_allreduce_2shot_kernel(bf16_t* out, const bf16_t* __restrict__ x,
                                                                     long n, ArPeers peers, int rank, int nranks,
                                                                     long slot_elems, unsigned* epochs,
                                                                     unsigned* err) {
  const int b = blockIdx.x;
  const long nv = n / 8;
  const long sl = (nv + nranks - 1) / nranks;
  const long per = (sl + gridDim.x - 1) / gridDim.x;
  const long o0 = b * per, o1 = min(sl, o0 + per);
  __shared__ unsigned s_epoch;
  if (threadIdx.x == 0) s_epoch = epochs[b] + 1;
  __syncthreads();
  const unsigned e = s_epoch;
  const int par = e & 1;
  const long my_slot = (static_cast<long>(par) * nranks + rank) * slot_elems * 2;  // bytes
  // 1. reduce-scatter push: slice r -> rank r
  const uint4* xs = reinterpret_cast<const uint4*>(x);
  for (int r = 0; r < nranks; ++r) {
    uint4* dst = reinterpret_cast<uint4*>(peers.recv[r] + my_slot);
    const long base = r * sl;
    for (long o = o0 + threadIdx.x; o < o1; o += blockDim.x) {
      const long v = base + o;
      if (v < nv) dst[v] = xs[v];
    }
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < nranks) st_flag(peers.flags[threadIdx.x] + b * kArMaxRanks + rank, e);
  if (threadIdx.x < nranks) ar_wait(peers.flags[rank] + b * kArMaxRanks + threadIdx.x, e, err);
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  // 2. sum the owned slice (fp32, rank order) and push it to every rank
  const char* mine = peers.recv[rank] + (static_cast<long>(par) * nranks * slot_elems) * 2;
  {
    const long base = rank * sl;
    for (long o = o0 + threadIdx.x; o < o1; o += blockDim.x) {
      const long v = base + o;
      if (v >= nv) break;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int r = 0; r < nranks; ++r) {
        const uint4 w = reinterpret_cast<const uint4*>(mine + r * slot_elems * 2)[v];
        const uint32_t u[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          acc[2 * k] += bf2f_lo(u[k]);
          acc[2 * k + 1] += bf2f_hi(u[k]);
        }
      }
      uint4 rr;
      rr.x = pack2(acc[0], acc[1]);
      rr.y = pack2(acc[2], acc[3]);
      rr.z = pack2(acc[4], acc[5]);
      rr.w = pack2(acc[6], acc[7]);
      for (int r = 0; r < nranks; ++r) reinterpret_cast<uint4*>(peers.recv[r] + my_slot)[v] = rr;
    }
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < nranks) st_flag(peers.flags[threadIdx.x] + kArFlags2 + b * kArMaxRanks + rank, e);
  if (threadIdx.x < nranks) ar_wait(peers.flags[rank] + kArFlags2 + b * kArMaxRanks + threadIdx.x, e, err);
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  // 3. gather: slice q from slot [par][q] (local memory)
  uint4* o = reinterpret_cast<uint4*>(out);
  for (int q = 0; q < nranks; ++q) {
    const uint4* src = reinterpret_cast<const uint4*>(mine + q * slot_elems * 2);
    const long base = q * sl;
    for (long oo = o0 + threadIdx.x; oo < o1; oo += blockDim.x) {
      const long v = base + oo;
      if (v < nv) o[v] = src[v];
    }
  }
  if (threadIdx.x == 0) epochs[b] = e;
}

void launch_custom_allreduce_2shot(bf16_t* out, const bf16_t* x, long n, const ArPeers& peers, int rank,
                                   int nranks, long slot_elems, unsigned* epochs, unsigned* err, hipStream_t s) {
  hipLaunchKernelGGL(custom_allreduce_2shot_kernel, dim3(kArMaxBlocks), dim3(512), 0, s, out, x, n, peers, rank,
                     nranks, slot_elems, epochs, err);
  MXS_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------------------------
// Fused TP epilogue of a projection that feeds the residual stream (o_proj / down_proj at TP > 1):
//   y = AllReduce(x) rounded to bf16, residual += y (in place), h = RMSNorm(residual) * w
// -- one launch instead of the all-reduce plus the fused add + RMSNorm kernel, and the reduced
// projection output never makes a bf16 round trip through memory.  The input is this rank's partial
// projection, either bf16 [M, H] or S fp32 split-K slabs [S][M][H] left by the decode GEMM with its
// reduce skipped (summed and rounded to bf16 here, as the GEMM's own output would be), so the split-K
// reduce kernel disappears too.  Rounding follows the unfused path: bf16 partials, an fp32 sum in
// rank order rounded to bf16, bf16 residual add (the residual matches bit for bit), the norm over
// the rounded residual (its sum of squares reduced over this kernel's thread layout).
//
// The pushes spread over all blocks (a decode batch of a few rows still uses every block's links);
// the norm needs whole rows, so after the exchange a block waits for EVERY (block, rank) flag of the
// call (64 x N flags, one per thread) and then owns rows blockIdx.x, + gridDim.x, ...  Epochs, parity
// and the one-call-ahead argument are the one-shot kernel's (a peer's call k + 2 needs this rank's
// flags of call k + 1, raised only by this rank's next launch, which the stream starts after every
// block of this one has finished reading).  TWO: the two-shot exchange (reduce-scatter by push, owner
// sums, all-gather by push) for large messages; its row phase reads each slice from its owner's slot.
template <int NV, bool TWO>
__global__ void __launch_bounds__(512) car_add_rmsnorm_kernel(
    bf16_t* __restrict__ h, bf16_t* __restrict__ residual, const bf16_t* __restrict__ x,
    const float* __restrict__ part, int S, int M, int H, const bf16_t* __restrict__ w, float eps, ArPeers peers,
    int rank, int nranks, long slot_elems, unsigned* epochs, unsigned* err) {
  __shared__ float scratch[16];
  __shared__ unsigned s_epoch;
  const int b = blockIdx.x, tid = threadIdx.x;
  const long nv = static_cast<long>(M) * H / 8;
  const long sl = TWO ? (nv + nranks - 1) / nranks : nv;  // vectors per owner slice
  const long per = (sl + gridDim.x - 1) / gridDim.x;
  const long o0 = b * per, o1 = min(sl, o0 + per);
  if (tid == 0) s_epoch = epochs[b] + 1;
  __syncthreads();
  const unsigned e = s_epoch;
  const int par = e & 1;
  const long my_slot = (static_cast<long>(par) * nranks + rank) * slot_elems * 2;  // bytes
  const size_t slab = static_cast<size_t>(M) * H;
  // this rank's partial of vector v, rounded to bf16
  auto partial = [&](long v) -> uint4 {
    if (part == nullptr) return reinterpret_cast<const uint4*>(x)[v];
    const float* p = part + v * 8;
    float4 a = *reinterpret_cast<const float4*>(p), c = *reinterpret_cast<const float4*>(p + 4);
    // 4 slabs' loads in flight at a time, summed in slab order (no load -> add round trip per slab)
    for (int s0 = 1; s0 < S; s0 += 4) {
      float4 a2[4], c2[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const size_t o = static_cast<size_t>(s0 + j < S ? s0 + j : 0) * slab;
        a2[j] = *reinterpret_cast<const float4*>(p + o);
        c2[j] = *reinterpret_cast<const float4*>(p + o + 4);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (s0 + j < S) {
          a.x += a2[j].x; a.y += a2[j].y; a.z += a2[j].z; a.w += a2[j].w;
          c.x += c2[j].x; c.y += c2[j].y; c.z += c2[j].z; c.w += c2[j].w;
        }
    }
    return make_uint4(pack2(a.x, a.y), pack2(a.z, a.w), pack2(c.x, c.y), pack2(c.z, c.w));
  };
  auto sum_slots = [&](const char* base, long v) -> uint4 {  // fp32 sum over ranks, rank order
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    uint4 q[kArMaxRanks];  // every rank's slot loaded before the first add (one round trip, not nranks)
#pragma unroll
    for (int r = 0; r < kArMaxRanks; ++r)
      if (r < nranks) q[r] = reinterpret_cast<const uint4*>(base + r * slot_elems * 2)[v];
#pragma unroll
    for (int r = 0; r < kArMaxRanks; ++r) {
      if (r >= nranks) break;
      const uint32_t u[4] = {q[r].x, q[r].y, q[r].z, q[r].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[2 * k] += bf2f_lo(u[k]);
        acc[2 * k + 1] += bf2f_hi(u[k]);
      }
    }
    return make_uint4(pack2(acc[0], acc[1]), pack2(acc[2], acc[3]), pack2(acc[4], acc[5]), pack2(acc[6], acc[7]));
  };
  auto wait_all = [&](int flag_base) {  // every (block, rank) flag of this epoch: one per thread
    if (tid < static_cast<int>(gridDim.x) * nranks) {
      const int bb = tid / nranks, r = tid - bb * nranks;
      ar_wait(peers.flags[rank] + flag_base + bb * kArMaxRanks + r, e, err);
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  };
  const char* mine = peers.recv[rank] + (static_cast<long>(par) * nranks * slot_elems) * 2;
  if constexpr (!TWO) {
    // 1. push this block's vectors into slot [par][rank] of every rank (self included)
    for (long v = o0 + tid; v < o1; v += blockDim.x) {
      const uint4 val = partial(v);
      for (int r = 0; r < nranks; ++r) reinterpret_cast<uint4*>(peers.recv[r] + my_slot)[v] = val;
    }
    __threadfence_system();
    __syncthreads();
    if (tid < nranks) st_flag(peers.flags[tid] + b * kArMaxRanks + rank, e);
    wait_all(0);
  } else {
    // 1. reduce-scatter push: slice r of the partial -> rank r
    for (int r = 0; r < nranks; ++r) {
      uint4* dst = reinterpret_cast<uint4*>(peers.recv[r] + my_slot);
      for (long o = o0 + tid; o < o1; o += blockDim.x) {
        const long v = r * sl + o;
        if (v < nv) dst[v] = partial(v);
      }
    }
    __threadfence_system();
    __syncthreads();
    if (tid < nranks) st_flag(peers.flags[tid] + b * kArMaxRanks + rank, e);
    if (tid < nranks) ar_wait(peers.flags[rank] + b * kArMaxRanks + tid, e, err);
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    // 2. sum the owned slice and push it to every rank's slot [par][rank]
    for (long o = o0 + tid; o < o1; o += blockDim.x) {
      const long v = rank * sl + o;
      if (v >= nv) break;
      const uint4 rr = sum_slots(mine, v);
      for (int r = 0; r < nranks; ++r) reinterpret_cast<uint4*>(peers.recv[r] + my_slot)[v] = rr;
    }
    __threadfence_system();
    __syncthreads();
    if (tid < nranks) st_flag(peers.flags[tid] + kArFlags2 + b * kArMaxRanks + rank, e);
    wait_all(kArFlags2);
  }
  // 3. rows: reduced y (+ residual) -> residual, RMSNorm -> h
  const int hv = H / 8;
  for (int row = b; row < M; row += gridDim.x) {
    bf16_t* rr = residual + static_cast<size_t>(row) * H;
    uint4 vals[NV];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = tid + i * blockDim.x;
      if (c < hv) {
        const long v = static_cast<long>(row) * hv + c;
        uint4 y;
        if constexpr (TWO) {
          const int q = static_cast<int>(v / sl);
          y = reinterpret_cast<const uint4*>(mine + q * slot_elems * 2)[v];
        } else {
          y = sum_slots(mine, v);
        }
        const uint4 rv = *reinterpret_cast<const uint4*>(rr + c * 8);
        const uint32_t py[4] = {y.x, y.y, y.z, y.w}, pr[4] = {rv.x, rv.y, rv.z, rv.w};
        uint32_t po[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          po[k] = pack2(bf2f_lo(py[k]) + bf2f_lo(pr[k]), bf2f_hi(py[k]) + bf2f_hi(pr[k]));
          const float lo = bf2f_lo(po[k]), hi = bf2f_hi(po[k]);
          ss += lo * lo + hi * hi;
        }
        vals[i] = make_uint4(po[0], po[1], po[2], po[3]);
        *reinterpret_cast<uint4*>(rr + c * 8) = vals[i];
      }
    }
    const float inv = rsqrtf(block_sum(ss, scratch) / static_cast<float>(H) + eps);
    bf16_t* hr = h + static_cast<size_t>(row) * H;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = tid + i * blockDim.x;
      if (c < hv) {
        const uint4 wv = *reinterpret_cast<const uint4*>(w + c * 8);
        const uint32_t p[4] = {vals[i].x, vals[i].y, vals[i].z, vals[i].w}, pw[4] = {wv.x, wv.y, wv.z, wv.w};
        uint32_t po[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          po[k] = pack2(bf2f_lo(p[k]) * inv * bf2f_lo(pw[k]), bf2f_hi(p[k]) * inv * bf2f_hi(pw[k]));
        *reinterpret_cast<uint4*>(hr + c * 8) = make_uint4(po[0], po[1], po[2], po[3]);
      }
    }
    __syncthreads();  // scratch reuse by the next row's block_sum
  }
  if (tid == 0) epochs[b] = e;
}

void launch_car_add_rmsnorm(bf16_t* h, bf16_t* residual, const bf16_t* x, const float* part, int S, int M, int H,
                            const bf16_t* w, float eps, const ArPeers& peers, int rank, int nranks, long slot_elems,
                            unsigned* epochs, unsigned* err, bool two_shot, hipStream_t s) {
  const int nv = (H / 8 + 511) / 512;
#define MXS_CARN(NVV, TW)                                                                                     \
  hipLaunchKernelGGL((car_add_rmsnorm_kernel<NVV, TW>), dim3(kArMaxBlocks), dim3(512), 0, s, h, residual, x, \
                     part, S, M, H, w, eps, peers, rank, nranks, slot_elems, epochs, err)
  if (two_shot) {
    switch (nv) {
      case 1: MXS_CARN(1, true); break;
      case 2: MXS_CARN(2, true); break;
      default: MXS_CARN(4, true); break;
    }
  } else {
    switch (nv) {
      case 1: MXS_CARN(1, false); break;
      case 2: MXS_CARN(2, false); break;
      default: MXS_CARN(4, false); break;
    }
  }
#undef MXS_CARN
  MXS_CHECK_LAUNCH();
}

// Equal-split all-to-all over the same IPC slots (EP dispatch / combine of fixed-capacity MoE
// layouts, SURVEY.md §5.8 "direct peer writes into pre-registered IPC receive buffers"): segment d
// of the input is pushed into rank d's slot [par][rank], one flag per (block, peer), then segment r
// of the output is read from this rank's slot [par][r].  Every rank pushes on all N-1 links at
// once.  Same epochs / flags / parity rule as the all-reduce kernels (calls of both kinds may
// interleave: every rank issues the same sequence).  V = uint4 when segments are 16-byte multiples.
// push_rows (optional, device): segment d carries only its first push_rows[d] rows of row_v vectors
// over the link (variable-size EP dispatch: the rest of the segment is capacity, not payload).
template <typename V>
__global__ void __launch_bounds__(512) ipc_all_to_all_kernel(V* __restrict__ out, const V* __restrict__ in,
                                                             long seg_v, ArPeers peers, int rank, int nranks,
                                                             long slot_bytes, unsigned* epochs, unsigned* err,
                                                             const int* __restrict__ push_rows, long row_v) {
  const int b = blockIdx.x;
  const long per = (seg_v + gridDim.x - 1) / gridDim.x;
  const long v0 = b * per, v1 = min(seg_v, v0 + per);
  __shared__ unsigned s_epoch;
  if (threadIdx.x == 0) s_epoch = epochs[b] + 1;
  __syncthreads();
  const unsigned e = s_epoch;
  const int par = e & 1;
  for (int d = 0; d < nranks; ++d) {
    V* dst = reinterpret_cast<V*>(peers.recv[d] + (static_cast<long>(par) * nranks + rank) * slot_bytes);
    const V* src = in + d * seg_v;
    const long lim = push_rows == nullptr ? v1 : min(v1, static_cast<long>(push_rows[d]) * row_v);
    for (long v = v0 + threadIdx.x; v < lim; v += blockDim.x) dst[v] = src[v];
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < nranks) st_flag(peers.flags[threadIdx.x] + b * kArMaxRanks + rank, e);
  if (threadIdx.x < nranks) ar_wait(peers.flags[rank] + b * kArMaxRanks + threadIdx.x, e, err);
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  for (int r = 0; r < nranks; ++r) {
    const V* src = reinterpret_cast<const V*>(peers.recv[rank] + (static_cast<long>(par) * nranks + r) * slot_bytes);
    V* dst = out + r * seg_v;
    for (long v = v0 + threadIdx.x; v < v1; v += blockDim.x) dst[v] = src[v];
  }
  if (threadIdx.x == 0) epochs[b] = e;
}

void launch_ipc_all_to_all(void* out, const void* in, long seg_bytes, const ArPeers& peers, int rank, int nranks,
                           long slot_bytes, unsigned* epochs, unsigned* err, hipStream_t s, const int* push_rows,
                           long row_bytes) {
  if (seg_bytes % 16 == 0 && (push_rows == nullptr || row_bytes % 16 == 0))
    hipLaunchKernelGGL(ipc_all_to_all_kernel<uint4>, dim3(kArMaxBlocks), dim3(512), 0, s, static_cast<uint4*>(out),
                       static_cast<const uint4*>(in), seg_bytes / 16, peers, rank, nranks, slot_bytes, epochs, err,
                       push_rows, row_bytes / 16);
  else
    hipLaunchKernelGGL(ipc_all_to_all_kernel<uint32_t>, dim3(kArMaxBlocks), dim3(512), 0, s,
                       static_cast<uint32_t*>(out), static_cast<const uint32_t*>(in), seg_bytes / 4, peers, rank,
                       nranks, slot_bytes, epochs, err, push_rows, row_bytes / 4);
  MXS_CHECK_LAUNCH();
}

}  // namespace mxs
