// K05-K08 at full prefill chunks (M = 1k-8k tokens): Y[M, N] = X[M, K] . W[N, K]^T with the
// projection's elementwise tail fused into the epilogue, on MFMA.
//
// At an 8192-token chunk the four projections of a Llama-3.2-1B layer are ~1 PF/s GEMMs, and the
// SiLU*mul pass after gate_up moved 402 MB per layer on its own (67 us, 6 % of a prefill chunk;
// profiles/r3/prefill_chunk8192_kernel_stats.csv).  This kernel computes gate_up and applies
// SiLU(gate) * up in registers, so only the [M, I] activation is written.
//
//   * 256 (weight rows n) x 256 (tokens m) x 64 (k) tile per 512-thread workgroup, one workgroup per
//     CU; 8 waves as 4 (n) x 2 (m), each 64 x 128 outputs = 4 x 8 fragments of
//     v_mfma_f32_16x16x32_bf16 with A = W (output columns on the accumulator rows) and B = X^T
//     (tokens on the lanes): a lane's accumulator is Y[token][4 consecutive columns];
//   * both operands go HBM/L2 -> LDS by global_load_lds_dwordx4 (1 KB per wave instruction = 8
//     rows x 128 B, no VGPRs, no ds_write pass) into two 64 KB stages; the 16-byte chunks of a row
//     are XOR-swizzled by (row >> 1) & 7 on the SOURCE address and un-swizzled on the ds_read_b128,
//     so the 16 rows of a read group hit 16 distinct bank slots (cdna_hip_programming.md T2, rule 21);
//   * one raw s_barrier per k-group; the next group's DMA is issued right after it and has the
//     whole group's 64 MFMAs per wave (2048 cycles per SIMD) to land; fragment reads of sub-step
//     q + 1 fly under the MFMAs of sub-step q;
//   * workgroups are remapped XCD-contiguous (bijective for any count), then grouped 8 row tiles per
//     column sweep, so the tiles an XCD runs together share their W and X panels in its L2;
//   * EPI_SWIGLU: the W image of a tile interleaves 16 gate rows and the 16 matching up rows (the
//     DMA source addresses do the gather; the weights keep their [gate; up] layout), so fragments
//     2p and 2p+1 of a wave hold gate and up of the same features in the same lanes.
#include <algorithm>

#include "common.h"

namespace mxs {

typedef __bf16 gb_bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int gb_u32x4 __attribute__((ext_vector_type(4)));

constexpr int GB_EPI_NONE = 0;
constexpr int GB_EPI_SWIGLU = 1;

__device__ __forceinline__ int gb_slot(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
__device__ __forceinline__ gb_bf16x8 gb_frag(const gb_u32x4& v) { return __builtin_bit_cast(gb_bf16x8, v); }
__device__ __forceinline__ float gb_silu(float g) { return g / (1.f + __expf(-g)); }

template <int EPI, int TW = 0>  // TW (tweaks): bit 0 static s_setprio 1 for waves 4-7, bit 1 16 row tiles per sweep
__global__ void __launch_bounds__(512) gemm_big_kernel(bf16_t* __restrict__ Y, const bf16_t* __restrict__ X,
                                                       const bf16_t* __restrict__ W, int M, int K, int ldx, int ldy,
                                                       int inter, int ntm, int ntn) {
  constexpr int BM = 256, BN = 256, STAGE = (BM + BN) * 128, NI = 8;  // NI: DMA instructions per wave per stage
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  // ---- workgroup -> tile: XCD-contiguous ranges (blocks b and b + 8 share an XCD), then GM row
  // tiles per column sweep inside each range
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  constexpr int GM = (TW & 2) ? 16 : 8;
  const int per_group = GM * ntn, grp = wg / per_group, first_m = grp * GM;
  const int gsz = min(ntm - first_m, GM), in_grp = wg - grp * per_group;
  const int tm = first_m + in_grp % gsz, tn = in_grp / gsz;
  const int m0 = tm * BM;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid & 3, wmi = wid >> 2;  // wave: image W rows [64 wn, +64), X rows [128 wmi, +128)
  if constexpr (TW & 1) {  // the second-dispatched half loses VALU arbitration otherwise (MI355X_MICROARCH item 4)
    if (__builtin_amdgcn_readfirstlane(tid) >= 256) __builtin_amdgcn_s_setprio(1);
  }

  // ---- DMA sources: instruction j of this wave fills image rows 8 (wid + 8 j) .. +7; lane -> row
  // + (lane >> 3), LDS chunk (lane & 7) <- global chunk (lane & 7) ^ swizzle(row)
  const bf16_t* src[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int row = 8 * (wid + 8 * j) + (lane >> 3);
    const int gch = (lane & 7) ^ ((row >> 1) & 7);
    const bf16_t* base;
    if (row < BN) {
      int wrow;
      if constexpr (EPI == GB_EPI_SWIGLU) {  // image row 64 w + 16 f + i, f = 2 p + (0 gate | 1 up)
        const int f = (row >> 4) & 3, feat = tn * 128 + 32 * (row >> 6) + 16 * (f >> 1) + (row & 15);
        wrow = (f & 1) ? inter + feat : feat;
      } else {
        wrow = tn * BN + row;
      }
      base = W + static_cast<size_t>(wrow) * K;
    } else {  // token rows past M re-read row M-1: loaded, never stored
      base = X + static_cast<size_t>(min(m0 + row - BN, M - 1)) * ldx;
    }
    src[j] = base + 8 * gch;
  }
  auto stage = [&](int g, int buf) {
    char* dst = smem + buf * STAGE;
#pragma unroll
    for (int j = 0; j < NI; ++j)
      __builtin_amdgcn_global_load_lds(static_cast<const void*>(src[j] + 64 * g),
                                       (__attribute__((address_space(3))) void*)(dst + (wid + 8 * j) * 1024), 16, 0, 0);
  };

  float4_ acc[4][8];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[f][t] = float4_{0.f, 0.f, 0.f, 0.f};

  const int r16 = lane & 15, kq = lane >> 4;
  int arow[4], brow[8];  // image rows of this lane's fragments
#pragma unroll
  for (int f = 0; f < 4; ++f) arow[f] = 64 * wn + 16 * f + r16;
#pragma unroll
  for (int t = 0; t < 8; ++t) brow[t] = BN + 128 * wmi + 16 * t + r16;

  const int ng = K / 64;
  stage(0, 0);
  for (int g = 0; g < ng; ++g) {
    // this wave's DMA of group g has landed; the barrier publishes every wave's and retires every
    // wave's reads of the other buffer (group g - 1), which group g + 1's DMA overwrites
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (g + 1 < ng) stage(g + 1, (g + 1) & 1);
    const char* b = smem + (g & 1) * STAGE;
    gb_u32x4 fa[2][4], fb[2][4];
    auto rd_a = [&](int kk, gb_u32x4(&a)[4]) {
#pragma unroll
      for (int f = 0; f < 4; ++f) a[f] = *reinterpret_cast<const gb_u32x4*>(b + gb_slot(arow[f], 4 * kk + kq));
    };
    auto rd_b = [&](int kk, int hm, gb_u32x4(&bb)[4]) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
        bb[t] = *reinterpret_cast<const gb_u32x4*>(b + gb_slot(brow[4 * hm + t], 4 * kk + kq));
    };
    auto mma = [&](const gb_u32x4(&a)[4], const gb_u32x4(&bb)[4], int hm) {
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int t = 0; t < 4; ++t)
          acc[f][4 * hm + t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gb_frag(a[f]), gb_frag(bb[t]),
                                                                        acc[f][4 * hm + t], 0, 0, 0);
    };
    // sub-steps (kk, token half): each issues the next one's fragment reads, then its 16 MFMAs
    rd_a(0, fa[0]);
    rd_b(0, 0, fb[0]);
    rd_b(0, 1, fb[1]);
    __builtin_amdgcn_sched_barrier(0);
    mma(fa[0], fb[0], 0);
    __builtin_amdgcn_sched_barrier(0);
    rd_a(1, fa[1]);
    rd_b(1, 0, fb[0]);
    __builtin_amdgcn_sched_barrier(0);
    mma(fa[0], fb[1], 1);
    __builtin_amdgcn_sched_barrier(0);
    rd_b(1, 1, fb[1]);
    __builtin_amdgcn_sched_barrier(0);
    mma(fa[1], fb[0], 0);
    __builtin_amdgcn_sched_barrier(0);
    mma(fa[1], fb[1], 1);
    __builtin_amdgcn_sched_barrier(0);
  }

  // ---- epilogue: lane (r16, kq), fragment (f, t): token m0 + 128 wmi + 16 t + r16, image columns
  // 64 wn + 16 f + 4 kq + e (e = register)
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int m = m0 + 128 * wmi + 16 * t + r16;
    if (m >= M) continue;
    bf16_t* yr = Y + static_cast<size_t>(m) * ldy;
    if constexpr (EPI == GB_EPI_SWIGLU) {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const float4_& g = acc[2 * p][t];
        const float4_& u = acc[2 * p + 1][t];
        const int n = tn * 128 + 32 * wn + 16 * p + 4 * kq;
        uint2 o;
        o.x = pack2(gb_silu(g[0]) * u[0], gb_silu(g[1]) * u[1]);
        o.y = pack2(gb_silu(g[2]) * u[2], gb_silu(g[3]) * u[3]);
        *reinterpret_cast<uint2*>(yr + n) = o;
      }
    } else {
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const float4_& a = acc[f][t];
        const int n = tn * BN + 64 * wn + 16 * f + 4 * kq;
        uint2 o;
        o.x = pack2(a[0], a[1]);
        o.y = pack2(a[2], a[3]);
        *reinterpret_cast<uint2*>(yr + n) = o;
      }
    }
  }
}

// Variant with a 4-deep ring of 32-k half stages (4 x 32 KB): the DMA of half stage h + 3 is issued
// right after the barrier of h, so two half stages are always in flight under the MFMAs of the
// current one (counted vmcnt, never 0 in the loop) instead of one full stage landing at the next
// barrier.  Rows are 64 B (4 chunks), swizzled by (row >> 1) & 3 on the source address: conflict-free
// for the ds_read_b128 lane groups ({0-3, 12-15, 20-27}, ...: 16 rows, two chunks per group).
__device__ __forceinline__ int gb_slot64(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 1) & 3)) << 4); }

template <int EPI, bool PRIO>
__global__ void __launch_bounds__(512) gemm_big_ring_kernel(bf16_t* __restrict__ Y, const bf16_t* __restrict__ X,
                                                            const bf16_t* __restrict__ W, int M, int K, int ldx,
                                                            int ldy, int inter, int ntm, int ntn) {
  constexpr int BM = 256, BN = 256, HS = (BM + BN) * 64, NR = 4, NI = 4;  // NI: DMA instrs per wave per half stage
  __shared__ __attribute__((aligned(16))) char smem[NR * HS];

  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  constexpr int GM = 8;
  const int per_group = GM * ntn, grp = wg / per_group, first_m = grp * GM;
  const int gsz = min(ntm - first_m, GM), in_grp = wg - grp * per_group;
  const int tm = first_m + in_grp % gsz, tn = in_grp / gsz;
  const int m0 = tm * BM;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid & 3, wmi = wid >> 2;

  // DMA: instruction j of this wave fills image rows 16 (wid + 8 j) .. +15 (64 B each); lane -> row
  // + (lane >> 2), LDS chunk (lane & 3) <- global chunk (lane & 3) ^ swizzle(row)
  const bf16_t* src[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int row = 16 * (wid + 8 * j) + (lane >> 2);
    const int gch = (lane & 3) ^ ((row >> 1) & 3);
    const bf16_t* base;
    if (row < BN) {
      int wrow;
      if constexpr (EPI == GB_EPI_SWIGLU) {
        const int f = (row >> 4) & 3, feat = tn * 128 + 32 * (row >> 6) + 16 * (f >> 1) + (row & 15);
        wrow = (f & 1) ? inter + feat : feat;
      } else {
        wrow = tn * BN + row;
      }
      base = W + static_cast<size_t>(wrow) * K;
    } else {
      base = X + static_cast<size_t>(min(m0 + row - BN, M - 1)) * ldx;
    }
    src[j] = base + 8 * gch;
  }
  auto stage = [&](int h, int buf) {
    char* dst = smem + buf * HS;
#pragma unroll
    for (int j = 0; j < NI; ++j)
      __builtin_amdgcn_global_load_lds(static_cast<const void*>(src[j] + 32 * h),
                                       (__attribute__((address_space(3))) void*)(dst + (wid + 8 * j) * 1024), 16, 0, 0);
  };

  float4_ acc[4][8];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[f][t] = float4_{0.f, 0.f, 0.f, 0.f};
  const int r16 = lane & 15, kq = lane >> 4;
  int aslot[4], bslot[8];  // byte offsets of this lane's fragments inside a half stage
#pragma unroll
  for (int f = 0; f < 4; ++f) aslot[f] = gb_slot64(64 * wn + 16 * f + r16, kq);
#pragma unroll
  for (int t = 0; t < 8; ++t) bslot[t] = gb_slot64(BN + 128 * wmi + 16 * t + r16, kq);

  const int nh = K / 32;
#pragma unroll
  for (int p = 0; p < NR - 1; ++p)
    if (p < nh) stage(p, p);
  for (int h = 0; h < nh; ++h) {
    // half stage h has landed for this wave (the newer ones may still fly); the barrier publishes it
    // for every wave and retires every wave's reads of the buffer read at h - 1 (refilled below)
    const int ahead = min(NR - 2, nh - 1 - h);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NI) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (h + NR - 1 < nh) stage(h + NR - 1, (h + NR - 1) % NR);
    const char* b = smem + (h % NR) * HS;
    gb_u32x4 fa[4], fb[8];
#pragma unroll
    for (int f = 0; f < 4; ++f) fa[f] = *reinterpret_cast<const gb_u32x4*>(b + aslot[f]);
#pragma unroll
    for (int t = 0; t < 8; ++t) fb[t] = *reinterpret_cast<const gb_u32x4*>(b + bslot[t]);
#pragma unroll
    for (int hm = 0; hm < 2; ++hm) {
      __builtin_amdgcn_sched_barrier(0);
      if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int t = 0; t < 4; ++t)
          acc[f][4 * hm + t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gb_frag(fa[f]), gb_frag(fb[4 * hm + t]),
                                                                        acc[f][4 * hm + t], 0, 0, 0);
      if (PRIO) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int m = m0 + 128 * wmi + 16 * t + r16;
    if (m >= M) continue;
    bf16_t* yr = Y + static_cast<size_t>(m) * ldy;
    if constexpr (EPI == GB_EPI_SWIGLU) {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const float4_& g = acc[2 * p][t];
        const float4_& u = acc[2 * p + 1][t];
        const int n = tn * 128 + 32 * wn + 16 * p + 4 * kq;
        uint2 o;
        o.x = pack2(gb_silu(g[0]) * u[0], gb_silu(g[1]) * u[1]);
        o.y = pack2(gb_silu(g[2]) * u[2], gb_silu(g[3]) * u[3]);
        *reinterpret_cast<uint2*>(yr + n) = o;
      }
    } else {
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const float4_& a = acc[f][t];
        const int n = tn * BN + 64 * wn + 16 * f + 4 * kq;
        uint2 o;
        o.x = pack2(a[0], a[1]);
        o.y = pack2(a[2], a[3]);
        *reinterpret_cast<uint2*>(yr + n) = o;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------------
// Ping-pong variant (variant 6): the same 256 x 256 x 64 tile, but the 8 waves run as two groups of 4
// that are one barrier apart (waves w and w + 4 share a SIMD), so on every SIMD one wave's 16-MFMA
// segment runs beside its partner's LDS-read / DMA-issue segment (cdna_hip_programming.md §5 "256²
// 8-phase template", MI355X_MICROARCH.md "Two waves per SIMD").
//
//   * a wave owns 128 tokens x 64 weight rows (acc[4 w-frags][8 token-frags]); a k-tile is 4 phases,
//     one output quadrant (2 w-frags x 4 token-frags x 2 k-steps = 16 MFMAs) each, visited in the
//     order (w0,t0) (w1,t0) (w1,t1) (w0,t1): fragment reads per phase 12 / 4 / 8 / 0 ds_read_b128,
//     each operand read once per k-tile;
//   * LDS = 2 k-tile buffers x 4 half-tiles (X rows 0-127, X rows 128-255, W rows 0-127, W rows
//     128-255) of 16 KB; half-tiles of k-tile u + 1 are DMA'd at phases 3 (of u - 1), 0 and 1 (of u),
//     each thread issuing 2 global_load_lds_dwordx4 per half-tile, and the only vmcnt wait is at phase
//     3 (vmcnt(0), before that phase's DMA issue) -- the youngest half-tile then has had two phases to
//     land.  Buffer u & 1 is last read at phase 2 of u, and refilled from phase 3 of u on;
//   * every load segment ends with lgkmcnt(0) before its barrier, so a barrier retires all reads
//     issued before it (the DMA that reuses a buffer is issued behind such a barrier).
template <int EPI>
__global__ void __launch_bounds__(512, 1) gemm_pp_kernel(bf16_t* __restrict__ Y, const bf16_t* __restrict__ X,
                                                         const bf16_t* __restrict__ W, int M, int K, int ldx, int ldy,
                                                         int inter, int ntm, int ntn) {
  constexpr int HT = 16384, KT = 4 * HT;
  __shared__ __attribute__((aligned(16))) char smem[2 * KT];

  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  constexpr int GM = 8;
  const int per_group = GM * ntn, grp = wg / per_group, first_m = grp * GM;
  const int gsz = min(ntm - first_m, GM), in_grp = wg - grp * per_group;
  const int tm = first_m + in_grp % gsz, tn = in_grp / gsz;
  const int m0 = tm * 256;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;  // token half, 64-row weight block

  // DMA sources: half-tile h, instruction j (0, 1) of this wave fills half-tile rows 8 (2 wid + j) .. +7
  const bf16_t* src[4][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 8 * (2 * wid + j) + (lane >> 3);  // row inside the half-tile
    const int gch = (lane & 7) ^ ((row >> 1) & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      src[h][j] = X + static_cast<size_t>(min(m0 + 128 * h + row, M - 1)) * ldx + 8 * gch;
      const int r = 128 * h + row;  // weight image row
      int wrow;
      if constexpr (EPI == GB_EPI_SWIGLU) {
        const int fr = (r >> 4) & 3, feat = tn * 128 + 32 * (r >> 6) + 16 * (fr & 1) + (r & 15);
        wrow = fr < 2 ? feat : inter + feat;
      } else {
        wrow = tn * 256 + r;
      }
      src[2 + h][j] = W + static_cast<size_t>(wrow) * K + 8 * gch;
    }
  }
  auto stage = [&](int h, int u) {  // half-tile h of k-tile u
    char* dst = smem + (u & 1) * KT + h * HT;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds(static_cast<const void*>(src[h][j] + 64 * u),
                                       (__attribute__((address_space(3))) void*)(dst + (2 * wid + j) * 1024), 16, 0,
                                       0);
  };

  float4_ acc[4][8];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[f][t] = float4_{0.f, 0.f, 0.f, 0.f};

  const int r16 = lane & 15, kq = lane >> 4;
  // byte offsets (inside a k-tile buffer) of this lane's fragment rows, k-chunk 0
  int woff[4], xoff[8];
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const int row = 64 * (wc & 1) + 16 * f + r16;
    woff[f] = (2 + (wc >> 1)) * HT + row * 128;
  }
#pragma unroll
  for (int t = 0; t < 8; ++t) xoff[t] = wr * HT + (16 * t + r16) * 128;
  // chunk c of row r sits at slot c ^ ((r >> 1) & 7); r16 fixes (r >> 1) & 7 for every fragment row
  const int swz = (r16 >> 1) & 7;
  const int sl0 = ((kq) ^ swz) << 4, sl1 = ((4 + kq) ^ swz) << 4;

  gb_u32x4 wa[2][2][2], xb[4][2];  // [w half][frag][k-step], [token frag][k-step]
  auto rd_w = [&](const char* b, int a) {
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      wa[a][f][0] = *reinterpret_cast<const gb_u32x4*>(b + woff[2 * a + f] + sl0);
      wa[a][f][1] = *reinterpret_cast<const gb_u32x4*>(b + woff[2 * a + f] + sl1);
    }
  };
  auto rd_x = [&](const char* b, int hb) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      xb[t][0] = *reinterpret_cast<const gb_u32x4*>(b + xoff[4 * hb + t] + sl0);
      xb[t][1] = *reinterpret_cast<const gb_u32x4*>(b + xoff[4 * hb + t] + sl1);
    }
  };
  auto quad = [&](int a, int hb) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int t = 0; t < 4; ++t)
          acc[2 * a + f][4 * hb + t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              gb_frag(wa[a][f][kk]), gb_frag(xb[t][kk]), acc[2 * a + f][4 * hb + t], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
#define PP_BAR()                           \
  do {                                     \
    __builtin_amdgcn_sched_barrier(0);     \
    __builtin_amdgcn_s_barrier();          \
    __builtin_amdgcn_sched_barrier(0);     \
  } while (0)
#define PP_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

  const int nk = K / 64;
  // prologue: all of k-tile 0, half-tiles 0 and 1 of k-tile 1
#pragma unroll
  for (int h = 0; h < 4; ++h) stage(h, 0);
  if (nk > 1) {
    stage(0, 1);
    stage(1, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  PP_BAR();
  if (wr == 1) PP_BAR();  // the stagger: waves 4-7 run one barrier behind waves 0-3

  for (int u = 0; u < nk; ++u) {
    const char* b = smem + (u & 1) * KT;
    const bool nxt = u + 1 < nk;
    // phase 0: quadrant (w0, t0)
    if (nxt) stage(2, u + 1);
    rd_w(b, 0);
    rd_x(b, 0);
    PP_LGKM0();
    PP_BAR();
    quad(0, 0);
    PP_BAR();
    // phase 1: (w1, t0)
    if (nxt) stage(3, u + 1);
    rd_w(b, 1);
    PP_LGKM0();
    PP_BAR();
    quad(1, 0);
    PP_BAR();
    // phase 2: (w1, t1) -- the last reads of buffer u & 1
    rd_x(b, 1);
    PP_LGKM0();
    PP_BAR();
    quad(1, 1);
    PP_BAR();
    // phase 3: (w0, t1); k-tile u + 1 complete; start k-tile u + 2 in buffer u & 1
    if (nxt) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (u + 2 < nk) {
        stage(0, u + 2);
        stage(1, u + 2);
      }
    }
    PP_BAR();
    quad(0, 1);
    PP_BAR();
  }
  if (wr == 0) PP_BAR();  // balance the stagger barrier
#undef PP_BAR
#undef PP_LGKM0

  // epilogue: lane (r16, kq), acc[f][t]: token m0 + 128 wr + 16 t + r16, image rows 64 wc + 16 f + 4 kq + e
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int m = m0 + 128 * wr + 16 * t + r16;
    if (m >= M) continue;
    bf16_t* yr = Y + static_cast<size_t>(m) * ldy;
    if constexpr (EPI == GB_EPI_SWIGLU) {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const float4_& g = acc[p][t];
        const float4_& v = acc[p + 2][t];
        const int n = tn * 128 + 32 * wc + 16 * p + 4 * kq;
        uint2 o;
        o.x = pack2(gb_silu(g[0]) * v[0], gb_silu(g[1]) * v[1]);
        o.y = pack2(gb_silu(g[2]) * v[2], gb_silu(g[3]) * v[3]);
        *reinterpret_cast<uint2*>(yr + n) = o;
      }
    } else {
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const float4_& a = acc[f][t];
        const int n = tn * 256 + 64 * wc + 16 * f + 4 * kq;
        uint2 o;
        o.x = pack2(a[0], a[1]);
        o.y = pack2(a[2], a[3]);
        *reinterpret_cast<uint2*>(yr + n) = o;
      }
    }
  }
}

// Two-phase ping-pong (variant 7): as variant 6, but a k-tile is 2 phases of 32 MFMAs (all 4 weight
// fragments x one token half), so each load segment (16 / 8 ds_read_b128 + DMA issue) is shorter
// than the partner's MFMA segment.  DMA granules: W half-tiles (16 KB) and X quarter-tiles (64
// tokens, 8 KB); k-tile u + 1's W and X(., 0) are issued at phase 1 of u - 1 (their regions were last
// read at phase 0 of u - 1), its X(., 1) at phase 0 of u; the only vmcnt wait is at phase 1 of u.
template <int EPI>
__global__ void __launch_bounds__(512, 1) gemm_pp2_kernel(bf16_t* __restrict__ Y, const bf16_t* __restrict__ X,
                                                          const bf16_t* __restrict__ W, int M, int K, int ldx,
                                                          int ldy, int inter, int ntm, int ntn) {
  constexpr int HT = 16384, QT = 8192, KT = 4 * HT, XB = 2 * HT;  // X region starts at XB
  __shared__ __attribute__((aligned(16))) char smem[2 * KT];

  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  constexpr int GM = 8;
  const int per_group = GM * ntn, grp = wg / per_group, first_m = grp * GM;
  const int gsz = min(ntm - first_m, GM), in_grp = wg - grp * per_group;
  const int tm = first_m + in_grp % gsz, tn = in_grp / gsz;
  const int m0 = tm * 256;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;

  // DMA sources: W half h, instruction j: half-tile rows 8 (2 wid + j) .. +7; X quarter (h, t):
  // quarter rows 8 wid .. +7
  const bf16_t* wsrc[2][2];
  const bf16_t* xsrc[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 8 * (2 * wid + j) + (lane >> 3);
    const int gch = (lane & 7) ^ ((row >> 1) & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = 128 * h + row;
      int wrow;
      if constexpr (EPI == GB_EPI_SWIGLU) {
        const int fr = (r >> 4) & 3, feat = tn * 128 + 32 * (r >> 6) + 16 * (fr & 1) + (r & 15);
        wrow = fr < 2 ? feat : inter + feat;
      } else {
        wrow = tn * 256 + r;
      }
      wsrc[h][j] = W + static_cast<size_t>(wrow) * K + 8 * gch;
    }
  }
  {
    const int rq = 8 * wid + (lane >> 3);
    const int gch = (lane & 7) ^ ((rq >> 1) & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        xsrc[h][t] = X + static_cast<size_t>(min(m0 + 128 * h + 64 * t + rq, M - 1)) * ldx + 8 * gch;
  }
  typedef __attribute__((address_space(3))) void lds_t;
  auto dma_w = [&](int u) {  // both W half-tiles of k-tile u
    char* dst = smem + (u & 1) * KT;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        __builtin_amdgcn_global_load_lds(static_cast<const void*>(wsrc[h][j] + 64 * u),
                                         (lds_t*)(dst + h * HT + (2 * wid + j) * 1024), 16, 0, 0);
  };
  auto dma_x = [&](int u, int t) {  // X quarters (0, t) and (1, t) of k-tile u
    char* dst = smem + (u & 1) * KT + XB + t * QT;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      __builtin_amdgcn_global_load_lds(static_cast<const void*>(xsrc[h][t] + 64 * u),
                                       (lds_t*)(dst + h * HT + wid * 1024), 16, 0, 0);
  };

  float4_ acc[4][8];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[f][t] = float4_{0.f, 0.f, 0.f, 0.f};

  const int r16 = lane & 15, kq = lane >> 4;
  int woff[4], xoff[8];
#pragma unroll
  for (int f = 0; f < 4; ++f) woff[f] = (wc >> 1) * HT + (64 * (wc & 1) + 16 * f + r16) * 128;
#pragma unroll
  for (int t = 0; t < 8; ++t) xoff[t] = XB + wr * HT + (16 * t + r16) * 128;
  const int swz = (r16 >> 1) & 7;
  const int sl0 = (kq ^ swz) << 4, sl1 = ((4 + kq) ^ swz) << 4;

  gb_u32x4 wa[4][2], xb[4][2];  // [w frag][k-step], [token frag][k-step]
  auto rd_w = [&](const char* b) {
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      wa[f][0] = *reinterpret_cast<const gb_u32x4*>(b + woff[f] + sl0);
      wa[f][1] = *reinterpret_cast<const gb_u32x4*>(b + woff[f] + sl1);
    }
  };
  auto rd_x = [&](const char* b, int hb) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      xb[t][0] = *reinterpret_cast<const gb_u32x4*>(b + xoff[4 * hb + t] + sl0);
      xb[t][1] = *reinterpret_cast<const gb_u32x4*>(b + xoff[4 * hb + t] + sl1);
    }
  };
  auto mma = [&](int hb) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int t = 0; t < 4; ++t)
          acc[f][4 * hb + t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gb_frag(wa[f][kk]), gb_frag(xb[t][kk]),
                                                                        acc[f][4 * hb + t], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
#define PP_BAR()                           \
  do {                                     \
    __builtin_amdgcn_sched_barrier(0);     \
    __builtin_amdgcn_s_barrier();          \
    __builtin_amdgcn_sched_barrier(0);     \
  } while (0)
#define PP_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

  const int nk = K / 64;
  dma_w(0);
  dma_x(0, 0);
  dma_x(0, 1);
  if (nk > 1) {
    dma_w(1);
    dma_x(1, 0);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  PP_BAR();
  if (wr == 1) PP_BAR();

  for (int u = 0; u < nk; ++u) {
    const char* b = smem + (u & 1) * KT;
    // phase 0: token half 0; X(., 1) of k-tile u + 1 (its region was last read at phase 1 of u - 1)
    if (u + 1 < nk) dma_x(u + 1, 1);
    rd_w(b);
    rd_x(b, 0);
    PP_LGKM0();
    PP_BAR();
    mma(0);
    PP_BAR();
    // phase 1: token half 1; k-tile u + 1 complete; W and X(., 0) of k-tile u + 2 into buffer u & 1
    // (last read at phase 0, retired by the lgkmcnt + barrier above)
    if (u + 1 < nk) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (u + 2 < nk) {
        dma_w(u + 2);
        dma_x(u + 2, 0);
      }
    }
    rd_x(b, 1);
    PP_LGKM0();
    PP_BAR();
    mma(1);
    PP_BAR();
  }
  if (wr == 0) PP_BAR();
#undef PP_BAR
#undef PP_LGKM0

#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int m = m0 + 128 * wr + 16 * t + r16;
    if (m >= M) continue;
    bf16_t* yr = Y + static_cast<size_t>(m) * ldy;
    if constexpr (EPI == GB_EPI_SWIGLU) {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const float4_& g = acc[p][t];
        const float4_& v = acc[p + 2][t];
        const int n = tn * 128 + 32 * wc + 16 * p + 4 * kq;
        uint2 o;
        o.x = pack2(gb_silu(g[0]) * v[0], gb_silu(g[1]) * v[1]);
        o.y = pack2(gb_silu(g[2]) * v[2], gb_silu(g[3]) * v[3]);
        *reinterpret_cast<uint2*>(yr + n) = o;
      }
    } else {
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const float4_& a = acc[f][t];
        const int n = tn * 256 + 64 * wc + 16 * f + 4 * kq;
        uint2 o;
        o.x = pack2(a[0], a[1]);
        o.y = pack2(a[2], a[3]);
        *reinterpret_cast<uint2*>(yr + n) = o;
      }
    }
  }
}

// epi 0: Y [M, N] = X W^T (N % 256 == 0).  epi 1 (SwiGLU): W = [gate; up] rows [2 I, K], Y [M, I] =
// SiLU(X gate^T) * (X up^T) (I % 128 == 0).  K % 64 == 0, 16-byte aligned rows.  False when the
// shape is not supported (the caller keeps its other path).
// variant: 0 = two 64-k stages, 1 = 4-deep ring of 32-k half stages, 2 = ring + s_setprio around
// the MFMA clusters
bool launch_gemm_big(bf16_t* Y, const bf16_t* X, const bf16_t* W, int M, int N, int K, int ldx, int ldy, int epi,
                     int variant, hipStream_t s) {
  if (M <= 0 || K % 64 != 0 || ldx % 8 != 0 || ldy % 4 != 0 || variant < 0 || variant > 7) return false;
  if ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W)) & 15) return false;
  if (reinterpret_cast<uintptr_t>(Y) & 7) return false;
  if (N % 256 != 0 || (epi != GB_EPI_NONE && epi != GB_EPI_SWIGLU)) return false;  // SwiGLU: N = 2 I, I % 128 == 0
  const int ntm = (M + 255) / 256;
  const int inter = epi == GB_EPI_SWIGLU ? N / 2 : 0, ntn = epi == GB_EPI_SWIGLU ? inter / 128 : N / 256;
  const dim3 g(ntm * ntn), b(512);
#define MXS_GB(KERN) hipLaunchKernelGGL(KERN, g, b, 0, s, Y, X, W, M, K, ldx, ldy, inter, ntm, ntn)
  if (epi == GB_EPI_SWIGLU) {
    if (variant == 0) MXS_GB(gemm_big_kernel<GB_EPI_SWIGLU>);
    else if (variant == 1) MXS_GB((gemm_big_ring_kernel<GB_EPI_SWIGLU, false>));
    else if (variant == 2) MXS_GB((gemm_big_ring_kernel<GB_EPI_SWIGLU, true>));
    else if (variant == 3) MXS_GB((gemm_big_kernel<GB_EPI_SWIGLU, 1>));
    else if (variant == 4) MXS_GB((gemm_big_kernel<GB_EPI_SWIGLU, 2>));
    else if (variant == 5) MXS_GB((gemm_big_kernel<GB_EPI_SWIGLU, 3>));
    else if (variant == 6) MXS_GB(gemm_pp_kernel<GB_EPI_SWIGLU>);
    else MXS_GB(gemm_pp2_kernel<GB_EPI_SWIGLU>);
  } else {
    if (variant == 0) MXS_GB(gemm_big_kernel<GB_EPI_NONE>);
    else if (variant == 1) MXS_GB((gemm_big_ring_kernel<GB_EPI_NONE, false>));
    else if (variant == 2) MXS_GB((gemm_big_ring_kernel<GB_EPI_NONE, true>));
    else if (variant == 3) MXS_GB((gemm_big_kernel<GB_EPI_NONE, 1>));
    else if (variant == 4) MXS_GB((gemm_big_kernel<GB_EPI_NONE, 2>));
    else if (variant == 5) MXS_GB((gemm_big_kernel<GB_EPI_NONE, 3>));
    else if (variant == 6) MXS_GB(gemm_pp_kernel<GB_EPI_NONE>);
    else MXS_GB(gemm_pp2_kernel<GB_EPI_NONE>);
  }
#undef MXS_GB
  MXS_CHECK_LAUNCH();
  return true;
}

}  // namespace mxs
