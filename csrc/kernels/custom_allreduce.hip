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
//   signal page (64 KiB, uint32 words):
//     [0, 1024)     flags[phase][max_blocks][N]: last epoch rank r published for block b
//     [1024, 1088)  epoch[max_blocks]: per-block call counter kept on the device (hipGraph-safe: no
//                   host epoch argument that a captured graph would freeze)
//     [2048]        error word: 0 healthy, else 1 + the rank that gave up first
//     [3072, 3088)  give-up record of this rank (kDiag* fields below), written once per fault
//     [3104, 3106)  wall clock at this rank's first collective since the last reset
//
// EVERY wait pairs block b of this rank with block b of each peer only: no kernel here needs more
// than one block per rank resident at a time, so ranks that time-share one GPU (the functional
// tests) or a grid that is only partly resident cannot deadlock each other.
// Memory model: payload stores + __threadfence_system() (release at system scope) before a flag is
// stored with a system-scope atomic; the waiter polls with system-scope atomic loads and then
// fences acquire at system scope.  The uncached allocation keeps stale lines out of every L2.
// Waits are bounded by WALL-CLOCK time (the 100 MHz constant counter, ArPeers::timeout_ticks) and
// end early once this rank's error word is set.  A rank that gives up first records what it was
// waiting for, then raises the error word of EVERY rank (before any of its later, stale-based output
// can reach a peer), so every wait in flight anywhere ends at once and the driver rank's per-step
// poll (car_poll_err_kernel) sees the fault for the step that contains it: the engine discards and
// recomputes that step (mxserve/engine/engine.py _recover_collective_fault).
#include "common.h"

namespace mxs {

constexpr int kArMaxRanks = 8;
constexpr int kArMaxBlocks = 64;
// signal-page word offsets (mirrored in mxserve/parallel/custom_allreduce.py)
constexpr int kSigEpochs = 1024;
constexpr int kSigErr = 2048;
constexpr int kSigDiag = 3072;
constexpr int kSigFirst = 3104;
// give-up record fields
enum : int {
  kDiagValid = 0, kDiagKind, kDiagEpoch, kDiagSeen, kDiagBlock, kDiagPeer, kDiagRank, kDiagRanks,
  kDiagT0Lo, kDiagT0Hi, kDiagT1Lo, kDiagT1Hi, kDiagWords = 16
};
// kernel / phase ids in the record
enum : int { kKindOneShot = 1, kKindTwoShot1, kKindTwoShot2, kKindNorm1, kKindNorm2Shot1, kKindNorm2Shot2, kKindA2A };

struct ArPeers {
  char* recv[kArMaxRanks];    // each rank's recv base, mapped into this process
  unsigned* flags[kArMaxRanks];  // each rank's signal page
  long long timeout_ticks;    // wait budget in wall-clock ticks
};

__device__ __forceinline__ void st_flag(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned ld_flag(unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Wait until *f reaches epoch e.  False when this rank's error word is (or becomes) set: another
// block or rank gave up, or this wait ran out of time -- then it claims the error word, fills in the
// give-up record and raises every peer's error word.
__device__ __forceinline__ bool ar_wait(const ArPeers& P, unsigned* f, unsigned e, int rank, int nranks, int kind,
                                     int peer) {
  unsigned* sig = P.flags[rank];
  unsigned* err = sig + kSigErr;
  if (static_cast<int>(ld_flag(f) - e) >= 0) return true;
  const long long t0 = wall_clock64();
  unsigned it = 0;
  while (true) {
    const unsigned seen = ld_flag(f);
    if (static_cast<int>(seen - e) >= 0) return true;
    if ((++it & 31u) == 0) {
      if (ld_flag(err) != 0) return false;
      const long long t1 = wall_clock64();
      if (t1 - t0 > P.timeout_ticks) {
        if (atomicCAS(err, 0u, 1u + rank) == 0u) {  // first to give up on this rank: record it
          unsigned* d = sig + kSigDiag;
          d[kDiagKind] = kind;
          d[kDiagEpoch] = e;
          d[kDiagSeen] = seen;
          d[kDiagBlock] = blockIdx.x;
          d[kDiagPeer] = peer;
          d[kDiagRank] = rank;
          d[kDiagRanks] = nranks;
          d[kDiagT0Lo] = static_cast<unsigned>(t0);
          d[kDiagT0Hi] = static_cast<unsigned>(static_cast<unsigned long long>(t0) >> 32);
          d[kDiagT1Lo] = static_cast<unsigned>(t1);
          d[kDiagT1Hi] = static_cast<unsigned>(static_cast<unsigned long long>(t1) >> 32);
          __threadfence_system();
          st_flag(d + kDiagValid, 1u);
          for (int r = 0; r < nranks; ++r)
            if (r != rank) st_flag(P.flags[r] + kSigErr, 1u + rank);
          __threadfence_system();
        }
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Block prologue shared by every kernel: this block's next epoch (and, on the first call since a
// reset, this rank's arrival time on the device clock).
__device__ __forceinline__ unsigned ar_enter(const ArPeers& P, int rank, unsigned* epochs, unsigned* s_epoch) {
  if (threadIdx.x == 0) {
    const unsigned e = epochs[blockIdx.x] + 1;
    *s_epoch = e;
    if (e == 1 && blockIdx.x == 0) {
      const unsigned long long t = static_cast<unsigned long long>(wall_clock64());
      unsigned* w = P.flags[rank] + kSigFirst;
      w[0] = static_cast<unsigned>(t);
      w[1] = static_cast<unsigned>(t >> 32);
    }
  }
  __syncthreads();
  return *s_epoch;
}

// Raise this block's flag (flag page `base`) at every rank, then wait for every rank's flag of this
// block and epoch.  Payload stores before it are released at system scope.
__device__ __forceinline__ void ar_exchange(const ArPeers& P, int base, unsigned e, int rank, int nranks, int kind) {
  const int b = blockIdx.x;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < nranks) {
    st_flag(P.flags[threadIdx.x] + base + b * kArMaxRanks + rank, e);
    ar_wait(P, P.flags[rank] + base + b * kArMaxRanks + threadIdx.x, e, rank, nranks, kind, threadIdx.x);
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

__device__ __forceinline__ uint4 sum_bf16x8(const char* base, long slot_bytes, long v, int nranks) {
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  uint4 q[kArMaxRanks];  // every rank's slot loaded before the first add (one round trip, not nranks)
#pragma unroll
  for (int r = 0; r < kArMaxRanks; ++r)
    if (r < nranks) q[r] = reinterpret_cast<const uint4*>(base + r * slot_bytes)[v];
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
}

// x: this rank's input (bf16, n elements, n % 8 == 0); out: result (may alias x)
__global__ void __launch_bounds__(512) custom_allreduce_kernel(bf16_t* out, const bf16_t* __restrict__ x, long n,
                                                               ArPeers peers, int rank, int nranks,
                                                               long slot_elems, unsigned* epochs) {
  const int b = blockIdx.x;
  const long nv = n / 8;  // 16-byte vectors
  const long per = (nv + gridDim.x - 1) / gridDim.x;
  const long v0 = b * per, v1 = min(nv, v0 + per);
  __shared__ unsigned s_epoch;
  const unsigned e = ar_enter(peers, rank, epochs, &s_epoch);
  const int par = e & 1;
  const long slot_bytes = slot_elems * 2;
  // 1. push this block's chunk into slot [par][rank] of every rank (self included)
  const uint4* xs = reinterpret_cast<const uint4*>(x);
  for (int r = 0; r < nranks; ++r) {
    uint4* dst = reinterpret_cast<uint4*>(peers.recv[r] + (static_cast<long>(par) * nranks + rank) * slot_bytes);
    for (long v = v0 + threadIdx.x; v < v1; v += blockDim.x) dst[v] = xs[v];
  }
  // 2. flags out, wait for every rank's flag of this block
  ar_exchange(peers, 0, e, rank, nranks, kKindOneShot);
  // 3. sum the N slots (local memory) in fp32, rank order (every rank gets identical bits)
  const char* mine = peers.recv[rank] + static_cast<long>(par) * nranks * slot_bytes;
  uint4* o = reinterpret_cast<uint4*>(out);
  for (long v = v0 + threadIdx.x; v < v1; v += blockDim.x) o[v] = sum_bf16x8(mine, slot_bytes, v, nranks);
  if (threadIdx.x == 0) epochs[b] = e;
}

void launch_custom_allreduce(bf16_t* out, const bf16_t* x, long n, const ArPeers& peers, int rank, int nranks,
                             long slot_elems, unsigned* epochs, hipStream_t s) {
  // ALWAYS kArMaxBlocks blocks: every block then counts the same calls, so the parity of a call is
  // the same in every block and chunk ranges may differ between calls of different sizes without a
  // peer that runs one call ahead ever writing into the parity this rank is still summing
  hipLaunchKernelGGL(custom_allreduce_kernel, dim3(kArMaxBlocks), dim3(512), 0, s, out, x, n, peers, rank, nranks,
                     slot_elems, epochs);
  MXS_CHECK_LAUNCH();
}

// Two-shot variant for larger messages (N > 2): reduce-scatter by push, then all-gather by push.
// Rank q owns slice q (1/N of the vectors).  Phase 1 pushes slice r of the input into rank r's slot
// [par][rank]; phase 2 sums the N contributions to the owned slice and pushes the result into every
// rank's slot [par][rank] at the same positions (the phase-1 data there sits at the receiver's own
// slice: disjoint); phase 3 reads every slice from its owner's slot.  Block b of a rank only ever
// exchanges with block b of its peers (its sub-range of every slice).  Each xGMI link carries 2/N
// of the message instead of the one-shot's whole message, for one more flag round trip.  Phase-2
// flags live in the second half of the flag page.
constexpr int kArFlags2 = kArMaxBlocks * kArMaxRanks;

__global__ void __launch_bounds__(512) custom_allreduce_2shot_kernel(bf16_t* out, const bf16_t* __restrict__ x,
                                                                     long n, ArPeers peers, int rank, int nranks,
                                                                     long slot_elems, unsigned* epochs) {
  const int b = blockIdx.x;
  const long nv = n / 8;
  const long sl = (nv + nranks - 1) / nranks;
  const long per = (sl + gridDim.x - 1) / gridDim.x;
  const long o0 = b * per, o1 = min(sl, o0 + per);
  __shared__ unsigned s_epoch;
  const unsigned e = ar_enter(peers, rank, epochs, &s_epoch);
  const int par = e & 1;
  const long slot_bytes = slot_elems * 2;
  const long my_slot = (static_cast<long>(par) * nranks + rank) * slot_bytes;
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
  ar_exchange(peers, 0, e, rank, nranks, kKindTwoShot1);
  // 2. sum the owned slice (fp32, rank order) and push it to every rank
  const char* mine = peers.recv[rank] + static_cast<long>(par) * nranks * slot_bytes;
  {
    const long base = rank * sl;
    for (long o = o0 + threadIdx.x; o < o1; o += blockDim.x) {
      const long v = base + o;
      if (v >= nv) break;
      const uint4 rr = sum_bf16x8(mine, slot_bytes, v, nranks);
      for (int r = 0; r < nranks; ++r) reinterpret_cast<uint4*>(peers.recv[r] + my_slot)[v] = rr;
    }
  }
  ar_exchange(peers, kArFlags2, e, rank, nranks, kKindTwoShot2);
  // 3. gather: slice q from slot [par][q] (local memory)
  uint4* o = reinterpret_cast<uint4*>(out);
  for (int q = 0; q < nranks; ++q) {
    const uint4* src = reinterpret_cast<const uint4*>(mine + q * slot_bytes);
    const long base = q * sl;
    for (long oo = o0 + threadIdx.x; oo < o1; oo += blockDim.x) {
      const long v = base + oo;
      if (v < nv) o[v] = src[v];
    }
  }
  if (threadIdx.x == 0) epochs[b] = e;
}

void launch_custom_allreduce_2shot(bf16_t* out, const bf16_t* x, long n, const ArPeers& peers, int rank,
                                   int nranks, long slot_elems, unsigned* epochs, hipStream_t s) {
  hipLaunchKernelGGL(custom_allreduce_2shot_kernel, dim3(kArMaxBlocks), dim3(512), 0, s, out, x, n, peers, rank,
                     nranks, slot_elems, epochs);
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
// Block b owns WHOLE ROWS: rows j with j % gridDim.x == b, in every phase and on every rank, so the
// norm never needs data another block of this rank produced and block b only waits for block b of
// its peers (no whole-grid co-residency).  One-shot: block b pushes its rows into slot [par][rank]
// of every rank, exchanges flags with block b of every peer, sums its rows over the N slots and
// finishes them (add + norm).  TWO (two-shot, large messages): rows are owned by ranks in contiguous
// runs of ceil(M / N); phase 1 pushes each of block b's rows only to its owner rank, phase 2 has the
// owner's block b sum its owned rows and push the reduced rows to every rank (slot [par][owner] at
// the row's position: disjoint from the phase-1 rows any rank receives, which are the receiver's
// own), phase 3 finishes block b's rows from slot [par][owner].  Epochs, parity and the
// one-call-ahead argument are the one-shot all-reduce's, per block.
template <int NV, bool TWO>
__global__ void __launch_bounds__(512) car_add_rmsnorm_kernel(
    bf16_t* __restrict__ h, bf16_t* __restrict__ residual, const bf16_t* __restrict__ x,
    const float* __restrict__ part, int S, int M, int H, const bf16_t* __restrict__ w, float eps, ArPeers peers,
    int rank, int nranks, long slot_elems, unsigned* epochs) {
  __shared__ float scratch[16];
  __shared__ unsigned s_epoch;
  const int b = blockIdx.x, tid = threadIdx.x, G = gridDim.x;
  const int hv = H / 8;
  const unsigned e = ar_enter(peers, rank, epochs, &s_epoch);
  const int par = e & 1;
  const long slot_bytes = slot_elems * 2;
  const long my_slot = (static_cast<long>(par) * nranks + rank) * slot_bytes;  // bytes
  const size_t slab = static_cast<size_t>(M) * H;
  const int rpo = (M + nranks - 1) / nranks;  // rows per owner rank (two-shot)
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
  // fn(row, vector index) over every vector of this block's rows in [lo, hi)
  auto block_rows = [&](int lo, int hi, auto&& fn) {
    const int j0 = lo + ((b - lo % G) % G + G) % G;
    if (j0 >= hi) return;
    const long tot = static_cast<long>((hi - j0 + G - 1) / G) * hv;
    for (long k = tid; k < tot; k += blockDim.x) {
      const int i = static_cast<int>(k / hv);
      const int j = j0 + i * G;
      fn(j, static_cast<long>(j) * hv + (k - static_cast<long>(i) * hv));
    }
  };
  const char* mine = peers.recv[rank] + static_cast<long>(par) * nranks * slot_bytes;
  if constexpr (!TWO) {
    // 1. push this block's rows into slot [par][rank] of every rank (self included)
    block_rows(0, M, [&](int, long v) {
      const uint4 val = partial(v);
      for (int r = 0; r < nranks; ++r) reinterpret_cast<uint4*>(peers.recv[r] + my_slot)[v] = val;
    });
    ar_exchange(peers, 0, e, rank, nranks, kKindNorm1);
  } else {
    // 1. reduce-scatter push: each of this block's rows -> its owner rank
    block_rows(0, M, [&](int j, long v) {
      reinterpret_cast<uint4*>(peers.recv[j / rpo] + my_slot)[v] = partial(v);
    });
    ar_exchange(peers, 0, e, rank, nranks, kKindNorm2Shot1);
    // 2. sum this block's owned rows and push them to every rank's slot [par][rank]
    block_rows(rank * rpo, min(M, rank * rpo + rpo), [&](int, long v) {
      const uint4 rr = sum_bf16x8(mine, slot_bytes, v, nranks);
      for (int r = 0; r < nranks; ++r) reinterpret_cast<uint4*>(peers.recv[r] + my_slot)[v] = rr;
    });
    ar_exchange(peers, kArFlags2, e, rank, nranks, kKindNorm2Shot2);
  }
  // 3. rows: reduced y (+ residual) -> residual, RMSNorm -> h
  for (int row = b; row < M; row += G) {
    bf16_t* rr = residual + static_cast<size_t>(row) * H;
    const char* ysrc = TWO ? mine + static_cast<long>(row / rpo) * slot_bytes : mine;
    uint4 vals[NV];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = tid + i * blockDim.x;
      if (c < hv) {
        const long v = static_cast<long>(row) * hv + c;
        uint4 y;
        if constexpr (TWO) {
          y = reinterpret_cast<const uint4*>(ysrc)[v];
        } else {
          y = sum_bf16x8(mine, slot_bytes, v, nranks);
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
                            unsigned* epochs, bool two_shot, hipStream_t s) {
  const int nv = (H / 8 + 511) / 512;
#define MXS_CARN(NVV, TW)                                                                                     \
  hipLaunchKernelGGL((car_add_rmsnorm_kernel<NVV, TW>), dim3(kArMaxBlocks), dim3(512), 0, s, h, residual, x, \
                     part, S, M, H, w, eps, peers, rank, nranks, slot_elems, epochs)
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
                                                             long slot_bytes, unsigned* epochs,
                                                             const int* __restrict__ push_rows, long row_v) {
  const int b = blockIdx.x;
  const long per = (seg_v + gridDim.x - 1) / gridDim.x;
  const long v0 = b * per, v1 = min(seg_v, v0 + per);
  __shared__ unsigned s_epoch;
  const unsigned e = ar_enter(peers, rank, epochs, &s_epoch);
  const int par = e & 1;
  for (int d = 0; d < nranks; ++d) {
    V* dst = reinterpret_cast<V*>(peers.recv[d] + (static_cast<long>(par) * nranks + rank) * slot_bytes);
    const V* src = in + d * seg_v;
    const long lim = push_rows == nullptr ? v1 : min(v1, static_cast<long>(push_rows[d]) * row_v);
    for (long v = v0 + threadIdx.x; v < lim; v += blockDim.x) dst[v] = src[v];
  }
  ar_exchange(peers, 0, e, rank, nranks, kKindA2A);
  for (int r = 0; r < nranks; ++r) {
    const V* src = reinterpret_cast<const V*>(peers.recv[rank] + (static_cast<long>(par) * nranks + r) * slot_bytes);
    V* dst = out + r * seg_v;
    for (long v = v0 + threadIdx.x; v < v1; v += blockDim.x) dst[v] = src[v];
  }
  if (threadIdx.x == 0) epochs[b] = e;
}

void launch_ipc_all_to_all(void* out, const void* in, long seg_bytes, const ArPeers& peers, int rank, int nranks,
                           long slot_bytes, unsigned* epochs, hipStream_t s, const int* push_rows, long row_bytes) {
  if (seg_bytes % 16 == 0 && (push_rows == nullptr || row_bytes % 16 == 0))
    hipLaunchKernelGGL(ipc_all_to_all_kernel<uint4>, dim3(kArMaxBlocks), dim3(512), 0, s, static_cast<uint4*>(out),
                       static_cast<const uint4*>(in), seg_bytes / 16, peers, rank, nranks, slot_bytes, epochs,
                       push_rows, row_bytes / 16);
  else
    hipLaunchKernelGGL(ipc_all_to_all_kernel<uint32_t>, dim3(kArMaxBlocks), dim3(512), 0, s,
                       static_cast<uint32_t*>(out), static_cast<const uint32_t*>(in), seg_bytes / 4, peers, rank,
                       nranks, slot_bytes, epochs, push_rows, row_bytes / 4);
  MXS_CHECK_LAUNCH();
}

// Per-step health poll (driver rank, end of every TP step): copy every rank's error word into a
// host-pinned array on the step's own stream, so the host reads it after the step's completion
// event -- no synchronous device read on the step loop.
__global__ void car_poll_err_kernel(unsigned* __restrict__ out, ArPeers peers, int nranks) {
  if (threadIdx.x < nranks) out[threadIdx.x] = ld_flag(peers.flags[threadIdx.x] + kSigErr);
}

void launch_car_poll_err(unsigned* out, const ArPeers& peers, int nranks, hipStream_t s) {
  hipLaunchKernelGGL(car_poll_err_kernel, dim3(1), dim3(64), 0, s, out, peers, nranks);
  MXS_CHECK_LAUNCH();
}

}  // namespace mxs
