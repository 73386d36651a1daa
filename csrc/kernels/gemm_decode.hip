// K05-K09 decode projections: Y[M, N] = X[M, K] . W[N, K]^T for M <= 256 (the decode batch), on MFMA.
//
// Decode steps (batch B = M rows) stream every weight byte once; at B = 64-256 the library GEMMs tile
// for large M and leave the narrow projections (Llama-3.2-1B qkv 3072, o 2048, down 2048 columns)
// with a dozen workgroups on a 256-CU chip.  This kernel is shaped for the decode regime:
//
//   * v_mfma_f32_16x16x32_bf16 with A = a 16-row slice of W (16 output columns x 32 k) and B = X^T
//     (32 k x 16 tokens): a lane's accumulator holds Y[token][4 consecutive columns], so the store
//     is one 8-byte write and no transpose is needed;
//   * a wave owns MF x NF fragments (up to 64 tokens x 64 columns): 16 MFMAs per k-step against
//     MF + NF 16-byte fragment loads, both operands straight from global memory into registers
//     (W streamed once, non-temporal; X, ~1 MB, stays in L2), the next k-step's fragments in flight
//     while the current ones are multiplied;
//   * a workgroup is WM x WN waves; split-K over gridDim.z fills the chip when there are few column
//     tiles (o / down at N = 2048), fp32 partial slabs summed by a reduce kernel that also applies
//     the epilogue;
//   * EPI_SILU (gate_up): each wave holds the gate columns n and the matching up columns I + n in
//     the same lane positions, so SiLU(gate) * up is applied in registers and only the [M, I]
//     activation is written (no [M, 2I] round trip, no separate SiLU*mul kernel).
// The Python side (mxserve/ops/decode_gemm.py) times these configurations against hipBLASLt per
// (graph bucket, projection) when the decode graphs are captured and keeps the faster one.
//
// Grouped form (G = true, K16 at decode batches): W is [E, N, K] per-expert weights and X holds the
// routed rows sorted by expert (moe_align offsets `offs`); blockIdx.y = expert * rt + row tile, so
// every expert with routed rows streams its weights once and an expert nobody picked costs nothing.
// Mixtral decode routes ~2T/8 rows per expert: the wave tile is sized to those rows, not to the
// 128-row tiles of the prefill grouped GEMM (moe_gemm.hip), which streams weights through LDS with
// 2 workgroups per CU and leaves the HBM pipe half empty at that size.
#include <algorithm>

#include "common.h"

namespace mxs {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2_gv_t __attribute__((ext_vector_type(2)));

constexpr int EPI_NONE = 0;
constexpr int EPI_SILU = 1;

__device__ __forceinline__ bf16x8_t as_bf16x8(const u32x4& v) { return __builtin_bit_cast(bf16x8_t, v); }
__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }

// k-steps per load group: ~8-12 fragments of 16 B per lane in flight per group (x2 with the next one)
__host__ __device__ constexpr int decode_gemm_unroll(int mf, int nf) { return mf + nf <= 3 ? 8 : (mf + nf <= 6 ? 4 : 2); }

template <int MF, int NF, int WM, int WN, int EPI, bool G>
__global__ void __launch_bounds__(256) decode_gemm_kernel(bf16_t* __restrict__ Y, float* __restrict__ part,
                                                          const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                          int M, int N, int K, int ldx, int ldy, int kslice,
                                                          int inter, const int* __restrict__ offs, int rt) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int i = lane & 15, kq = lane >> 4;
  constexpr int NH = EPI == EPI_SILU ? NF / 2 : NF;  // output fragments per wave
  int m0 = (blockIdx.y * WM + wm) * MF * 16;
  int mlim = M;  // rows [.., mlim) are this wave's to store; M stays the split-K slab row count
  if constexpr (G) {
    const int e = blockIdx.y / rt, r = blockIdx.y - e * rt;
    const int lo = offs[e], hi = offs[e + 1];
    m0 = lo + (r * WM + wm) * MF * 16;
    if (m0 >= hi) return;  // no barriers in this kernel: a wave without rows just leaves
    mlim = hi;
    W += static_cast<size_t>(e) * N * K;
  }
  const int c0 = (blockIdx.x * WN + wn) * NH * 16;  // first OUTPUT column of the wave
  const int kbeg = blockIdx.z * kslice;

  // weight rows (output columns) of each fragment; gate_up: fragment j < NH is gate column
  // c0 + 16 j, fragment NH + j the matching up column inter + c0 + 16 j
  const bf16_t* wp[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int col = (EPI == EPI_SILU && j >= NH) ? inter + c0 + 16 * (j - NH) : c0 + 16 * (j % NH);
    wp[j] = W + static_cast<size_t>(col + i) * K + kbeg + 8 * kq;
  }
  // rows past M read row M-1 (never stored: an output element depends only on its own token row);
  // unconditional loads keep hipcc from branching around each one and draining vmcnt per load
  const bf16_t* xp[MF];
  bool xv[MF];
#pragma unroll
  for (int t = 0; t < MF; ++t) {
    const int m = m0 + 16 * t + i;
    xv[t] = m < mlim;
    xp[t] = X + static_cast<size_t>(min(m, mlim - 1)) * ldx + kbeg + 8 * kq;
  }
  float4_ acc[MF][NF];
#pragma unroll
  for (int t = 0; t < MF; ++t)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[t][j] = float4_{0.f, 0.f, 0.f, 0.f};

  // U k-steps per group, all their loads issued back to back (enough bytes in flight per CU to
  // stream HBM); the next group's loads are in flight while this group's MFMAs run
  constexpr int U = decode_gemm_unroll(MF, NF);
  u32x4 a[U][NF], b[U][MF];
  auto load = [&](int k, u32x4 (&ad)[U][NF], u32x4 (&bd)[U][MF]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int j = 0; j < NF; ++j)
        ad[u][j] = *reinterpret_cast<const u32x4*>(wp[j] + k + 32 * u);
#pragma unroll
      for (int t = 0; t < MF; ++t)
        bd[u][t] = *reinterpret_cast<const u32x4*>(xp[t] + k + 32 * u);
    }
  };
  load(0, a, b);
  for (int k = 0; k < kslice; k += 32 * U) {
    u32x4 an[U][NF], bn[U][MF];
    const bool more = k + 32 * U < kslice;
    if (more) load(k + 32 * U, an, bn);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < MF; ++t)
#pragma unroll
        for (int j = 0; j < NF; ++j)
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a[u][j]), as_bf16x8(b[u][t]), acc[t][j], 0,
                                                              0, 0);
    if (more) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int j = 0; j < NF; ++j) a[u][j] = an[u][j];
#pragma unroll
        for (int t = 0; t < MF; ++t) b[u][t] = bn[u][t];
      }
    }
  }

  // lane (i, kq) holds Y[m0 + 16 t + i][col_j + 4 kq + r], r = 0..3
#pragma unroll
  for (int t = 0; t < MF; ++t) {
    if (!xv[t]) continue;
    const int m = m0 + 16 * t + i;
#pragma unroll
    for (int j = 0; j < NH; ++j) {
      const int n = c0 + 16 * j + 4 * kq;
      if (part != nullptr) {  // split-K: fp32 slab, raw (pre-epilogue) columns
        const size_t row = (static_cast<size_t>(blockIdx.z) * M + m) * static_cast<size_t>(N);
        *reinterpret_cast<float4_*>(part + row + n) = acc[t][j];
        if constexpr (EPI == EPI_SILU) *reinterpret_cast<float4_*>(part + row + inter + n) = acc[t][j + NH];
        continue;
      }
      float v[4];
      if constexpr (EPI == EPI_SILU) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = silu(acc[t][j][r]) * acc[t][j + NH][r];
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[t][j][r];
      }
      uint2 o;
      o.x = pack2(v[0], v[1]);
      o.y = pack2(v[2], v[3]);
      *reinterpret_cast<uint2*>(Y + static_cast<size_t>(m) * ldy + n) = o;
    }
  }
}

// LDS form: the same wave tiles (4 waves side by side over N, all on the workgroup's MF x 16 rows),
// but the X tile of each U-step group is loaded ONCE per workgroup (each thread a few 16-byte
// chunks, coalesced row segments) and written to LDS in MFMA-fragment order, where every wave reads
// its B fragments with conflict-free ds_read_b128 (lane l reads 16 bytes at 16 l).  The register
// kernel above has every wave load the X fragments itself: 4x the X traffic from L2, which at
// 32-64 rows per tile (MoE experts at decode, M >= 64 dense) is as many bytes as the weights.
// One barrier per group: the group's X chunks and W fragments for the NEXT group are issued before
// this group's MFMAs (X first, so the wait before the LDS write leaves the W loads in flight).
template <int MF, int NF, int U, int EPI, bool G>
__global__ void __launch_bounds__(256) decode_gemm_lds_kernel(bf16_t* __restrict__ Y, float* __restrict__ part,
                                                              const bf16_t* __restrict__ X,
                                                              const bf16_t* __restrict__ W, int M, int N, int K,
                                                              int ldx, int ldy, int kslice, int inter,
                                                              const int* __restrict__ offs, int rt) {
  constexpr int KG = 32 * U;                 // k per group
  constexpr int BM = MF * 16;                // rows of the workgroup
  constexpr int XCH = BM * KG / 8;           // 16-byte chunks of one X tile
  constexpr int XPT = (XCH + 255) / 256;     // chunks per thread
  constexpr int NH = EPI == EPI_SILU ? NF / 2 : NF;
  __shared__ __attribute__((aligned(16))) u32x4 xs[2][XCH];
  const int tid = threadIdx.x, lane = tid & 63, wn = tid >> 6;
  const int i = lane & 15, kq = lane >> 4;
  int m0 = blockIdx.y * BM;
  int mlim = M;
  if constexpr (G) {
    const int e = blockIdx.y / rt, r = blockIdx.y - e * rt;
    const int lo = offs[e], hi = offs[e + 1];
    m0 = lo + r * BM;
    if (m0 >= hi) return;  // uniform over the workgroup
    mlim = hi;
    W += static_cast<size_t>(e) * N * K;
  }
  const int c0 = (blockIdx.x * 4 + wn) * NH * 16;
  const int kbeg = blockIdx.z * kslice;
  const bf16_t* wp[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int col = (EPI == EPI_SILU && j >= NH) ? inter + c0 + 16 * (j - NH) : c0 + 16 * (j % NH);
    wp[j] = W + static_cast<size_t>(col + i) * K + kbeg + 8 * kq;
  }
  // X chunk q of the tile <-> LDS slot q = ((t * U + u) * 64 + kq' * 16 + i'): row m0 + 16 t + i',
  // k offset 32 u + 8 kq' (rows past the limit re-read row mlim - 1: loaded, never stored)
  const bf16_t* xsrc[XPT];
#pragma unroll
  for (int s2 = 0; s2 < XPT; ++s2) {
    const int q = tid + 256 * s2;
    const int ii = q & 15, kk = (q >> 4) & 3, tu = q >> 6;
    const int t = tu / U, u = tu - t * U;
    const int row = min(m0 + 16 * t + ii, mlim - 1);
    xsrc[s2] = X + static_cast<size_t>(row) * ldx + kbeg + 32 * u + 8 * kk;
  }
  auto load_x = [&](int k, u32x4 (&xr)[XPT]) {
#pragma unroll
    for (int s2 = 0; s2 < XPT; ++s2)
      if (XCH % 256 == 0 || tid + 256 * s2 < XCH) xr[s2] = *reinterpret_cast<const u32x4*>(xsrc[s2] + k);
  };
  auto store_x = [&](int buf, const u32x4 (&xr)[XPT]) {
#pragma unroll
    for (int s2 = 0; s2 < XPT; ++s2)
      if (XCH % 256 == 0 || tid + 256 * s2 < XCH) xs[buf][tid + 256 * s2] = xr[s2];
  };
  auto load_w = [&](int k, u32x4 (&ad)[U][NF]) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < NF; ++j) ad[u][j] = *reinterpret_cast<const u32x4*>(wp[j] + k + 32 * u);
  };
  float4_ acc[MF][NF];
#pragma unroll
  for (int t = 0; t < MF; ++t)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[t][j] = float4_{0.f, 0.f, 0.f, 0.f};

  u32x4 a[U][NF], xr[XPT];
  load_x(0, xr);
  load_w(0, a);
  store_x(0, xr);
  __syncthreads();
  int cur = 0;
  for (int k = 0; k < kslice; k += KG) {
    const bool more = k + KG < kslice;
    u32x4 an[U][NF];
    if (more) {
      load_x(k + KG, xr);
      load_w(k + KG, an);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < MF; ++t) {
        const u32x4 b = xs[cur][(t * U + u) * 64 + lane];
#pragma unroll
        for (int j = 0; j < NF; ++j)
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a[u][j]), as_bf16x8(b), acc[t][j], 0, 0, 0);
      }
    if (more) {
      store_x(cur ^ 1, xr);
      __syncthreads();
      cur ^= 1;
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < NF; ++j) a[u][j] = an[u][j];
    }
  }

#pragma unroll
  for (int t = 0; t < MF; ++t) {
    const int m = m0 + 16 * t + i;
    if (m >= mlim) continue;
#pragma unroll
    for (int j = 0; j < NH; ++j) {
      const int n = c0 + 16 * j + 4 * kq;
      if (part != nullptr) {
        const size_t row = (static_cast<size_t>(blockIdx.z) * M + m) * static_cast<size_t>(N);
        *reinterpret_cast<float4_*>(part + row + n) = acc[t][j];
        if constexpr (EPI == EPI_SILU) *reinterpret_cast<float4_*>(part + row + inter + n) = acc[t][j + NH];
        continue;
      }
      float v[4];
      if constexpr (EPI == EPI_SILU) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = silu(acc[t][j][r]) * acc[t][j + NH][r];
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[t][j][r];
      }
      uint2 o;
      o.x = pack2(v[0], v[1]);
      o.y = pack2(v[2], v[3]);
      *reinterpret_cast<uint2*>(Y + static_cast<size_t>(m) * ldy + n) = o;
    }
  }
}

// Sum S fp32 slabs [S][M][N] and apply the epilogue: Y[m][n] (EPI_NONE, N columns) or
// Y[m][n] = SiLU(sum gate[n]) * sum up[inter + n] (EPI_SILU, inter columns).
template <int EPI>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(bf16_t* __restrict__ Y, const float* __restrict__ part,
                                                            int M, int N, int S, int ldy, int inter) {
  const int ncols = EPI == EPI_SILU ? inter : N;
  const long total4 = static_cast<long>(M) * ncols / 4;
  for (long q = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; q < total4;
       q += static_cast<long>(gridDim.x) * blockDim.x) {
    const int m = static_cast<int>((q * 4) / ncols), n = static_cast<int>((q * 4) % ncols);
    float4_ g = {0.f, 0.f, 0.f, 0.f}, u = {0.f, 0.f, 0.f, 0.f};
    const size_t sstride = static_cast<size_t>(M) * N;
    const float* row0 = part + static_cast<size_t>(m) * N + n;
    // 4 slabs' loads in flight at a time, summed in slab order (a load -> add chain pays one L2 round
    // trip per slab)
    for (int s0 = 0; s0 < S; s0 += 4) {
      float4_ bg[4], bu[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float* row = row0 + (s0 + j < S ? s0 + j : 0) * sstride;
        bg[j] = *reinterpret_cast<const float4_*>(row);
        if (EPI == EPI_SILU) bu[j] = *reinterpret_cast<const float4_*>(row + inter);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (s0 + j < S) {
          g += bg[j];
          if (EPI == EPI_SILU) u += bu[j];
        }
    }
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = EPI == EPI_SILU ? silu(g[r]) * u[r] : g[r];
    uint2 o;
    o.x = pack2(v[0], v[1]);
    o.y = pack2(v[2], v[3]);
    *reinterpret_cast<uint2*>(Y + static_cast<size_t>(m) * ldy + n) = o;
  }
}

// ---------------------------------------------------------------------------------------------------
// Skinny form ("sk"): M <= 16 rows (small-batch decode) against a weight whose columns alone cannot
// fill 256 CUs with long enough streams -- the tensor-parallel shards of a large model (Llama-3-70B
// at TP 8: qkv 1280 x 8192, o 8192 x 1024, down 8192 x 3584).  Pure weight streaming: every W byte is
// read once, so the whole game is bytes in flight per CU.
//   * a workgroup = 4 waves on ONE 16-row slice of W and 4 consecutive k-ranges of KR; a wave issues
//     all its KR / 32 W fragment loads (16 B per lane, non-temporal) and the matching X loads up front,
//     then runs v_mfma_f32_16x16x32_bf16 (A = W slice, B = X^T, padded rows of X read as zeros):
//     at KR = 256 a wave keeps 8 KiB of W in flight, ~10 waves per CU on the TP-8 qkv shard;
//   * the 4 partial 16 x 16 tiles meet in LDS; blockIdx.y is a k-group of 4 KR: one group writes
//     bf16 Y, several write fp32 slabs [group][M][N] that the consumer sums (the split-K reduce, the
//     fused rope / all-reduce + RMSNorm epilogues read slabs directly).
// MF token fragments of 16 (M <= 16 MF): every W fragment feeds MF MFMAs against the matching X
// fragments (tokens 16 f + r), so the weight is still read once while M grows to 64 (the TP-8 shard
// shapes at decode batches 17-64, where hipBLASLt streams the narrow qkv at 0.6-0.8 TB/s); the KR
// choices shrink with MF to hold the X fragments in registers.
template <int KR, int MF>
__global__ void __launch_bounds__(256) skinny_gemm_kernel(bf16_t* __restrict__ Y, float* __restrict__ part,
                                                          const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                          int M, int N, int K, int ldx, int ldy) {
  constexpr int STEPS = KR / 32;
  __shared__ float red[4][16][16 * MF + 1];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int k0 = (blockIdx.y * 4 + wid) * KR + 8 * q;
  const bf16_t* wp = W + static_cast<size_t>(n0 + r) * K + k0;
  u32x4 wf[STEPS], xf[MF][STEPS];
#pragma unroll
  for (int s = 0; s < STEPS; ++s) wf[s] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wp + 32 * s));
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int m = 16 * f + r;
    const bf16_t* xp = X + static_cast<size_t>(m) * ldx + k0;
    // lanes of padded rows issue no X loads (at M = 1, 60 of 64 lanes): only W occupies the memory pipe
    if (m < M) {
#pragma unroll
      for (int s = 0; s < STEPS; ++s) xf[f][s] = *reinterpret_cast<const u32x4*>(xp + 32 * s);
    } else {
#pragma unroll
      for (int s = 0; s < STEPS; ++s) xf[f][s] = u32x4{0u, 0u, 0u, 0u};
    }
  }
  float4_ acc[MF];
#pragma unroll
  for (int f = 0; f < MF; ++f) acc[f] = float4_{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < STEPS; ++s)
#pragma unroll
    for (int f = 0; f < MF; ++f)
      acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wf[s]), as_bf16x8(xf[f][s]), acc[f], 0, 0, 0);
  // acc[f][i] = C[n = 4 q + i][m = 16 f + r]
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wid][4 * q + i][16 * f + r] = acc[f][i];
  __syncthreads();
  if (wid != 0) return;
  // wave 0: 16 x 16 MF outputs, 4 per lane and fragment: n = 4 q + i, m = 16 f + r
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int m = 16 * f + r;
    if (m >= M) continue;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = 4 * q + i;
      v[i] = red[0][n][m] + red[1][n][m] + red[2][n][m] + red[3][n][m];
    }
    if (part != nullptr) {
      float* pr = part + (static_cast<size_t>(blockIdx.y) * M + m) * N + n0 + 4 * q;
      *reinterpret_cast<float4_*>(pr) = float4_{v[0], v[1], v[2], v[3]};
    } else {
      bf16_t* yr = Y + static_cast<size_t>(m) * ldy + n0 + 4 * q;
      *reinterpret_cast<uint2*>(yr) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
    }
  }
}

// epi = EPI_SILU: W = [gate; up] (N = 2 inter rows), Y [M, inter] = SiLU(gate) * up -- the two halves
// of an output column live in different workgroups, so every group writes its slab (even a single
// one) and the reduce kernel applies SiLU*mul as it sums them.
bool launch_skinny_gemm(bf16_t* Y, float* part, const bf16_t* X, const bf16_t* W, int M, int N, int K, int ldx,
                        int ldy, int KR, bool reduce, int epi, hipStream_t s) {
  // M <= 16: KR 128 / 256; M <= 32 (two token fragments): 64 / 128; M <= 64 (four): 64 / 128
  if (M <= 0 || M > 64 || N % 16 != 0 || ldx % 8 != 0 || ldy % 4 != 0) return false;
  if (epi != EPI_NONE && (epi != EPI_SILU || N % 32 != 0 || !reduce || part == nullptr)) return false;
  const int MF = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  if (MF == 1 ? (KR != 128 && KR != 256) : (KR != 64 && KR != 128)) return false;
  if (K % (4 * KR) != 0) return false;
  const int groups = K / (4 * KR);
  if (groups > 1 && part == nullptr) return false;
  dim3 grid(N / 16, groups), blk(256);
  float* p = groups > 1 || epi == EPI_SILU ? part : nullptr;
  if (MF == 1) {
    if (KR == 128) hipLaunchKernelGGL((skinny_gemm_kernel<128, 1>), grid, blk, 0, s, Y, p, X, W, M, N, K, ldx, ldy);
    else hipLaunchKernelGGL((skinny_gemm_kernel<256, 1>), grid, blk, 0, s, Y, p, X, W, M, N, K, ldx, ldy);
  } else if (MF == 2) {
    if (KR == 64) hipLaunchKernelGGL((skinny_gemm_kernel<64, 2>), grid, blk, 0, s, Y, p, X, W, M, N, K, ldx, ldy);
    else hipLaunchKernelGGL((skinny_gemm_kernel<128, 2>), grid, blk, 0, s, Y, p, X, W, M, N, K, ldx, ldy);
  } else {
    if (KR == 64) hipLaunchKernelGGL((skinny_gemm_kernel<64, 4>), grid, blk, 0, s, Y, p, X, W, M, N, K, ldx, ldy);
    else hipLaunchKernelGGL((skinny_gemm_kernel<128, 4>), grid, blk, 0, s, Y, p, X, W, M, N, K, ldx, ldy);
  }
  MXS_CHECK_LAUNCH();
  if (epi == EPI_SILU) {
    const long total4 = static_cast<long>(M) * (N / 2) / 4;
    const int blocks = static_cast<int>(std::min<long>((total4 + 255) / 256, 1024));
    hipLaunchKernelGGL(splitk_reduce_kernel<EPI_SILU>, dim3(blocks), dim3(256), 0, s, Y, part, M, N, groups, ldy,
                       N / 2);
    MXS_CHECK_LAUNCH();
  } else if (groups > 1 && reduce) {
    const long total4 = static_cast<long>(M) * N / 4;
    const int blocks = static_cast<int>(std::min<long>((total4 + 255) / 256, 1024));
    hipLaunchKernelGGL(splitk_reduce_kernel<EPI_NONE>, dim3(blocks), dim3(256), 0, s, Y, part, M, N, groups, ldy, 0);
    MXS_CHECK_LAUNCH();
  }
  return true;
}

// ---------------------------------------------------------------------------------------------------
// Row-stream form ("gv"): M <= 4 decode rows (small-batch decode of the TP shards, batch-1 decode of any
// model) against a weight read exactly once.  The skinny form above reads 16 W rows x 64 B per load
// instruction (16 partial lines per instruction) and goes through MFMA fragments sized for 16 tokens;
// this one walks WHOLE rows: lane l of a wave holds the 16-byte chunks l, l + 64, ... of the wave's
// k-range, so every load instruction is one contiguous 1 KiB of a row, the NR rows x CH chunks of a wave
// are all issued before the first use (non-temporal), and the dot products are v_dot2_f32_bf16 against
// x chunks the workgroup staged in LDS once.
//   * a workgroup is 4 waves; KW of them split one row group's K (partial sums meet in LDS), so narrow
//     shards (TP-8 qkv: 1280 rows x 8192) still put ~2.5 workgroups on every CU, and 4 / KW row groups
//     of NR rows run side by side when K is short (o at TP 8: K = 1024);
//   * EPI_SILU: a wave's NR rows are NR / 2 gate rows and the matching up rows (inter + n), so the
//     workgroup writes SiLU(gate) * up directly -- no fp32 slabs, no reduce kernel;
//   * the output is bf16 Y, or with `part` an fp32 [M][N] row-parallel partial (the TP all-reduce +
//     RMSNorm epilogue reads it as a one-slab split-K result).
template <int MR, int NR, int KW, int EPI>
__global__ void __launch_bounds__(256) gemv_stream_kernel(bf16_t* __restrict__ Y, float* __restrict__ part,
                                                          const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                          int M, int N, int K, int ldx, int ldy, int inter,
                                                          int kslice) {
  extern __shared__ __attribute__((aligned(16))) char gv_smem[];
  constexpr int RG = 4 / KW;                           // row groups per workgroup
  constexpr int OUT = EPI == EPI_SILU ? NR / 2 : NR;  // output columns per row group
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int rg = wid / KW, kq = wid % KW;
  const int z = blockIdx.y, kg = gridDim.y;       // k-group of this workgroup (split-K over the grid)
  const int ch = kslice / (512 * KW);             // 16-byte chunks per lane of this wave's k-range
  const int kw0 = kq * (kslice / KW);             // the wave's k-range, relative to the workgroup's slice
  const int kbase = z * kslice + kw0;
  // stage the workgroup's k-slice of the M x rows into LDS: [MR][kslice] bf16, 16-byte chunks
  const int nchunk = kslice / 8;
  for (int i = tid; i < MR * nchunk; i += 256) {
    const int m = i / nchunk, c = i % nchunk;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (m < M) v = *reinterpret_cast<const u32x4*>(X + static_cast<size_t>(m) * ldx + z * kslice + 8 * c);
    *reinterpret_cast<u32x4*>(gv_smem + (static_cast<size_t>(m) * nchunk + c) * 16) = v;
  }
  __syncthreads();
  const int col0 = (blockIdx.x * RG + rg) * OUT;  // first output column of this row group
  const bf16_t* wrow[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int n = EPI == EPI_SILU ? (r < OUT ? col0 + r : inter + col0 + r - OUT) : col0 + r;
    wrow[r] = W + static_cast<size_t>(n) * K + kbase + 8 * lane;
  }
  float acc[MR][NR];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[m][r] = 0.f;
  constexpr int JC = 16 / NR;  // chunks per row per batch: 16 loads (64 VGPRs) in flight per wave
  for (int j0 = 0; j0 < ch; j0 += JC) {
    u32x4 wv[NR][JC];
#pragma unroll
    for (int j = 0; j < JC; ++j)
#pragma unroll
      for (int r = 0; r < NR; ++r)
        if (j0 + j < ch) wv[r][j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wrow[r] + 512 * (j0 + j)));
#pragma unroll
    for (int j = 0; j < JC; ++j) {
      if (j0 + j >= ch) break;
      const int c = (kw0 >> 3) + lane + 64 * (j0 + j);
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        const u32x4 xv = *reinterpret_cast<const u32x4*>(gv_smem + (static_cast<size_t>(m) * nchunk + c) * 16);
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            // copy the vector elements out first: hipcc (ROCm 7.2) bit-casts an ext_vector element
            // subscript as element 0 whatever the index (every dot2 would read the chunk's first pair)
            const uint32_t we = wv[r][j][e], xe = xv[e];
            acc[m][r] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_gv_t, we),
                                                        __builtin_bit_cast(bf16x2_gv_t, xe), acc[m][r], false);
          }
      }
    }
  }
  // 64-lane sums, then the KW partial sums of a row group through LDS
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      float v = acc[m][r];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      acc[m][r] = v;
    }
  __syncthreads();  // the x tiles are no longer read: the LDS is reused for the partials
  float* red = reinterpret_cast<float*>(gv_smem);  // [4 waves][MR][NR]
  if (lane == 0) {
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
      for (int r = 0; r < NR; ++r) red[(wid * MR + m) * NR + r] = acc[m][r];
  }
  __syncthreads();
  if (kq != 0) return;
  for (int idx = lane; idx < MR * OUT; idx += 64) {
    const int m = idx / OUT, o = idx % OUT;
    if (m >= M) break;
    auto sum = [&](int r) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < KW; ++q) s += red[((rg * KW + q) * MR + m) * NR + r];
      return s;
    };
    if (kg > 1) {  // split-K slab [z][M][N] of raw sums (SwiGLU: gate and up columns; the reduce applies it)
      float* pr = part + (static_cast<size_t>(z) * M + m) * N;
      pr[col0 + o] = sum(o);
      if constexpr (EPI == EPI_SILU) pr[inter + col0 + o] = sum(o + OUT);
      continue;
    }
    const float v = EPI == EPI_SILU ? silu(sum(o)) * sum(o + OUT) : sum(o);
    if (part != nullptr)
      part[static_cast<size_t>(m) * N + col0 + o] = v;
    else
      Y[static_cast<size_t>(m) * ldy + col0 + o] = f2bf(v);
  }
}

// kg > 1: split-K over gridDim.y, fp32 slabs [kg][M][N] in `part` (summed with the epilogue by
// splitk_reduce_kernel when reduce, else left for the caller's fused epilogue).
bool launch_gemv_stream(bf16_t* Y, float* part, const bf16_t* X, const bf16_t* W, int M, int N, int K, int ldx,
                        int ldy, int nr, int kw, int epi, int kg, bool reduce, hipStream_t s) {
  if (M <= 0 || M > 16 || kg < 1 || K % (512 * kw * kg) != 0 || ldx % 8 != 0) return false;
  if (!(nr == 2 || nr == 4) || !(kw == 1 || kw == 2 || kw == 4)) return false;
  if (epi != EPI_NONE && (epi != EPI_SILU || N % 2 != 0)) return false;
  if (kg == 1 && epi == EPI_SILU && part != nullptr) return false;  // the fp32 result form is epi 0 only
  if (kg > 1 && part == nullptr) return false;
  const int out_cols = epi == EPI_SILU ? N / 2 : N;
  if (kg > 1 && (out_cols % 4 != 0 || ldy % 4 != 0)) return false;  // the reduce writes 4 columns at a time
  const int per_wg = (4 / kw) * (epi == EPI_SILU ? nr / 2 : nr);
  if (out_cols % per_wg != 0) return false;
  const int mr = M <= 1 ? 1 : (M <= 2 ? 2 : (M <= 4 ? 4 : (M <= 8 ? 8 : 16)));
  const int kslice = K / kg;
  const size_t lds = std::max<size_t>(static_cast<size_t>(mr) * kslice * 2, 4 * 16 * 4 * sizeof(float));
  if (lds > 64 * 1024) return false;
  const dim3 grid(out_cols / per_wg, kg), blk(256);
  const int inter = epi == EPI_SILU ? N / 2 : 0;
  bool launched = false;
#define MXS_GV(MRR, NRR, KWW, EE)                                                                           \
  if (!launched && mr == MRR && nr == NRR && kw == KWW && epi == EE) {                                      \
    hipLaunchKernelGGL((gemv_stream_kernel<MRR, NRR, KWW, EE>), grid, blk, lds, s, Y, part, X, W, M, N, K, ldx, \
                       ldy, inter, kslice);                                                                 \
    MXS_CHECK_LAUNCH();                                                                                     \
    launched = true;                                                                                        \
  }
#define MXS_GV_K(MRR, NRR, EE) MXS_GV(MRR, NRR, 1, EE) MXS_GV(MRR, NRR, 2, EE) MXS_GV(MRR, NRR, 4, EE)
#define MXS_GV_M(MRR, EE) MXS_GV_K(MRR, 2, EE) MXS_GV_K(MRR, 4, EE)
  MXS_GV_M(1, EPI_NONE) MXS_GV_M(2, EPI_NONE) MXS_GV_M(4, EPI_NONE) MXS_GV_M(8, EPI_NONE) MXS_GV_M(16, EPI_NONE)
  MXS_GV_M(1, EPI_SILU) MXS_GV_M(2, EPI_SILU) MXS_GV_M(4, EPI_SILU) MXS_GV_M(8, EPI_SILU) MXS_GV_M(16, EPI_SILU)
#undef MXS_GV_M
#undef MXS_GV_K
#undef MXS_GV
  if (!launched) return false;
  if (kg > 1 && reduce) {
    const long total4 = static_cast<long>(M) * out_cols / 4;
    const int blocks = static_cast<int>(std::min<long>((total4 + 255) / 256, 1024));
    if (epi == EPI_SILU)
      hipLaunchKernelGGL(splitk_reduce_kernel<EPI_SILU>, dim3(blocks), dim3(256), 0, s, Y, part, M, N, kg, ldy, N / 2);
    else
      hipLaunchKernelGGL(splitk_reduce_kernel<EPI_NONE>, dim3(blocks), dim3(256), 0, s, Y, part, M, N, kg, ldy, 0);
    MXS_CHECK_LAUNCH();
  }
  return true;
}

// ---------------------------------------------------------------------------------------------------
// Medium-M form ("mt"): decode batches of 64-256 rows (and short prefill chunks), where the weight
// bytes no longer dominate the on-chip traffic: at M = 256 every weight element feeds 512 FLOP, so
// the MFMA pipe, the LDS read port and the L2 re-reads of X all matter (cdna_hip_programming.md §5,
// "Projection GEMM at M = 256").  The kernel above re-streams W once per 64-row tile and reads
// fragment-shaped pieces (16 rows x 64 B per instruction) straight into registers; this one:
//
//   * covers up to all 256 rows in ONE workgroup (WM x WN waves, each 32 MR rows x 32 WNF weight
//     rows = output columns), so each W element is read from HBM once per row tile and shared by the
//     WM waves through LDS;
//   * v_mfma_f32_32x32x16_bf16 (A = 32 W rows, B = X^T with 32 tokens), MR x WNF accumulator tiles
//     per wave: MR + WNF fragment reads feed MR x WNF MFMAs, which keeps the LDS read port (256 B/clk
//     per CU: 2 KB of fresh operands per 32-cycle MFMA would saturate it) below the MFMA pipe;
//   * the fragment reads of k-step s + 1 are issued before the MFMAs of step s (counted lgkmcnt);
//   * stages both operands with global_load_lds_dwordx4 in full 128-byte lines (8 rows x 128 B per
//     wave instruction, no VGPRs, no ds_write pass) into a ring of as many 64-k stages as the LDS
//     holds (3-6), one raw s_barrier per k-group, counted vmcnt waits;
//   * the 16-byte chunks of a row are XOR-swizzled by (row >> 1) & 7 on the SOURCE address (the
//     LDS image stays lane-linear, as the DMA writes it) and un-swizzled on the ds_read_b128, so the
//     16 lanes of a read group (16 rows, one chunk) hit 16 distinct bank slots;
//   * split-K over the grid (fp32 slabs, summed with the epilogue by splitk_reduce_kernel) and an
//     XCD-aware block order (consecutive blocks of one XCD share their X slice in its L2);
//   * EPI_SILU: a wave's fragments are gate columns and the matching up columns, so gate_up writes
//     SiLU(gate) * up directly.
__device__ __forceinline__ int mt_slot(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

template <int WM, int WN, int MR, int WNF, int EPI>
__global__ void __launch_bounds__(WM* WN * 64) mt_gemm_kernel(bf16_t* __restrict__ Y, float* __restrict__ part,
                                                              const bf16_t* __restrict__ X,
                                                              const bf16_t* __restrict__ W, int M, int N, int K,
                                                              int ldx, int ldy, int kslice, int inter, int ntm,
                                                              int ntn, int* __restrict__ cnt, int order) {
  constexpr int NW = WM * WN;
  constexpr int BM = 32 * MR * WM, BN = 32 * WNF * WN;  // X rows / W rows of a stage image
  constexpr int ROWS = BN + BM, STAGE = ROWS * 128;
  constexpr int NS = (160 * 1024 / STAGE) < 6 ? (160 * 1024 / STAGE) : 6;  // ring depth: the LDS it fits
  constexpr int NI = ROWS / 8 / NW;  // DMA instructions per wave per k-group
  constexpr int HF = EPI == EPI_SILU ? WNF / 2 : WNF;  // output fragments per wave
  constexpr int OUTB = 32 * HF * WN;                    // output columns of the workgroup
  static_assert(ROWS % (8 * NW) == 0 && (EPI != EPI_SILU || WNF % 2 == 0), "mt tile");
  static_assert(NS >= 3 && NI * 4 <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];

  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  // order 0: column tiles fastest; 1: row tiles fastest, so the row tiles sharing a weight slice run
  // back to back on one XCD and the slice is read from HBM once (its second read hits that L2)
  const int tn = order ? (wg / ntm) % ntn : wg % ntn, tm = order ? wg % ntm : (wg / ntn) % ntm;
  const int z = wg / (ntn * ntm);
  const int m0 = tm * BM, c0 = tn * OUTB, kbeg = z * kslice;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;

  // DMA sources: instruction j of this wave fills image rows 8 (wid + NW j) .. +7; lane -> row
  // + (lane >> 3), LDS chunk (lane & 7) <- global chunk (lane & 7) ^ swizzle(row).  W image row
  // 32 (wn' WNF + f) + i is output column c0 + 32 (wn' HF + f % HF) + i (+ inter for up fragments).
  const bf16_t* src[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int row = 8 * (wid + NW * j) + (lane >> 3);
    const int gch = (lane & 7) ^ ((row >> 1) & 7);
    const bf16_t* base;
    if (row < BN) {
      const int wv = row / (32 * WNF), f = (row / 32) % WNF, i = row & 31;
      const int col = c0 + 32 * (wv * HF + f % HF) + i;
      base = W + static_cast<size_t>((EPI == EPI_SILU && f >= HF) ? inter + col : col) * K;
    } else {  // rows past M re-read row M-1: loaded, never stored
      base = X + static_cast<size_t>(min(m0 + row - BN, M - 1)) * ldx;
    }
    src[j] = base + kbeg + 8 * gch;
  }
  auto stage = [&](int g, int buf) {
    char* dst = smem + buf * STAGE;
#pragma unroll
    for (int j = 0; j < NI; ++j)
      __builtin_amdgcn_global_load_lds(static_cast<const void*>(src[j] + 64 * g),
                                       (__attribute__((address_space(3))) void*)(dst + (wid + NW * j) * 1024), 16, 0,
                                       0);
  };

  float16_ acc[MR][WNF];
#pragma unroll
  for (int t = 0; t < MR; ++t)
#pragma unroll
    for (int f = 0; f < WNF; ++f)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[t][f][e] = 0.f;

  const int r32 = lane & 31, h = lane >> 5;
  const bool rows = m0 + wm * 32 * MR < M;  // wave-uniform: a wave past M only stages
  int aoff[WNF], boff[MR];                   // image rows of this lane's fragments
#pragma unroll
  for (int f = 0; f < WNF; ++f) aoff[f] = 32 * (wn * WNF + f) + r32;
#pragma unroll
  for (int t = 0; t < MR; ++t) boff[t] = BN + 32 * (wm * MR + t) + r32;

  const int ng = kslice / 64;
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < ng) stage(p, p);
  for (int g = 0; g < ng; ++g) {
    // this wave's DMA of k-group g has landed (the next min(NS-2, ng-1-g) groups may still fly); the
    // barrier publishes every wave's, and retires every wave's reads of the buffer read at g - 1,
    // which the group g + NS - 1 DMA then overwrites
    const int ahead = min(NS - 2, ng - 1 - g);
    if (ahead >= 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI * 4) : "memory");
    else if (ahead == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI * 3) : "memory");
    else if (ahead == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI * 2) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (g + NS - 1 < ng) stage(g + NS - 1, (g + NS - 1) % NS);
    const char* b = smem + (g % NS) * STAGE;
    if (rows) {
      u32x4 fa[2][WNF], fb[2][MR];
      auto rd = [&](int s, u32x4 (&a)[WNF], u32x4 (&bb)[MR]) {
#pragma unroll
        for (int t = 0; t < MR; ++t) bb[t] = *reinterpret_cast<const u32x4*>(b + mt_slot(boff[t], 2 * s + h));
#pragma unroll
        for (int f = 0; f < WNF; ++f) a[f] = *reinterpret_cast<const u32x4*>(b + mt_slot(aoff[f], 2 * s + h));
      };
      rd(0, fa[0], fb[0]);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (s < 3) rd(s + 1, fa[(s + 1) & 1], fb[(s + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);  // step s + 1's reads fly under step s's MFMAs
#pragma unroll
        for (int t = 0; t < MR; ++t)
#pragma unroll
          for (int f = 0; f < WNF; ++f)
            acc[t][f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(fa[s & 1][f]), as_bf16x8(fb[s & 1][t]),
                                                                acc[t][f], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }

  // lane (r32, h), register e of tile (t, f): token m0 + 32 (wm MR + t) + r32, column 32 f' + 8 (e >> 2)
  // + 4 h + (e & 3) of the wave's output columns
  if (rows) {
#pragma unroll
    for (int t = 0; t < MR; ++t) {
      const int m = m0 + 32 * (wm * MR + t) + r32;
      if (m >= M) continue;
#pragma unroll
      for (int f = 0; f < HF; ++f)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int n = c0 + 32 * (wn * HF + f) + 8 * gq + 4 * h;
          const float16_& a = acc[t][f];
          if (part != nullptr) {  // split-K: this slice's raw fp32 slab
            const size_t row = (static_cast<size_t>(z) * M + m) * static_cast<size_t>(N);
            *reinterpret_cast<float4_*>(part + row + n) =
                float4_{a[4 * gq], a[4 * gq + 1], a[4 * gq + 2], a[4 * gq + 3]};
            if constexpr (EPI == EPI_SILU) {
              const float16_& u = acc[t][f + HF];
              *reinterpret_cast<float4_*>(part + row + inter + n) =
                  float4_{u[4 * gq], u[4 * gq + 1], u[4 * gq + 2], u[4 * gq + 3]};
            }
            continue;
          }
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[e] = EPI == EPI_SILU ? silu(a[4 * gq + e]) * acc[t][f + HF][4 * gq + e] : a[4 * gq + e];
          uint2 o;
          o.x = pack2(v[0], v[1]);
          o.y = pack2(v[2], v[3]);
          *reinterpret_cast<uint2*>(Y + static_cast<size_t>(m) * ldy + n) = o;
        }
    }
  }
  if (part == nullptr || cnt == nullptr) return;  // unsplit, or slabs summed by splitk_reduce_kernel

  // In-launch split-K reduction (cdna_hip_programming.md §5 "Projection GEMM at M = 256" item 2):
  // every slice publishes its slab with one agent-scope release before drawing a ticket; the slice
  // that draws S - 1 acquires, sums the S slabs of the tile in slice order (deterministic) and
  // writes the epilogue, then re-arms the tile's counter for the next launch.  Correct for any
  // placement of the slices over XCDs.
  const int S = gridDim.x / (ntm * ntn);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave's slab stores are complete; the staging ring is no longer read
  int* flag = reinterpret_cast<int*>(smem);
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int ticket = __hip_atomic_fetch_add(cnt + tm * ntn + tn, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = ticket == S - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      cnt[tm * ntn + tn] = 0;
    }
    flag[0] = last;
  }
  __syncthreads();
  if (!flag[0]) return;
  const int nr = min(BM, M - m0);
  constexpr int Q4 = OUTB / 4;
  for (int idx = tid; idx < nr * Q4; idx += NW * 64) {
    const int m = m0 + idx / Q4, n = c0 + 4 * (idx % Q4);
    float4_ g = {0.f, 0.f, 0.f, 0.f}, u = {0.f, 0.f, 0.f, 0.f};
    for (int zz = 0; zz < S; ++zz) {
      const float* row = part + (static_cast<size_t>(zz) * M + m) * static_cast<size_t>(N);
      g += *reinterpret_cast<const float4_*>(row + n);
      if constexpr (EPI == EPI_SILU) u += *reinterpret_cast<const float4_*>(row + inter + n);
    }
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = EPI == EPI_SILU ? silu(g[e]) * u[e] : g[e];
    uint2 o;
    o.x = pack2(v[0], v[1]);
    o.y = pack2(v[2], v[3]);
    *reinterpret_cast<uint2*>(Y + static_cast<size_t>(m) * ldy + n) = o;
  }
}

// (wm, wn, mr, wnf): WM x WN waves of 32 MR rows x 32 WNF W rows; false when the shape is not tiled
// or the layout is not built.
// With a tile-counter array `cnt` (>= tiles ints, zero on first use; every launch leaves it zero) the
// split-K slabs are summed inside the launch, else by splitk_reduce_kernel.
bool launch_mt_gemm(bf16_t* Y, float* part, const bf16_t* X, const bf16_t* W, int M, int N, int K, int ldx, int ldy,
                    int wm, int wn, int mr, int wnf, int splitk, int epi, hipStream_t s, int* cnt, int cnt_len,
                    int order, int reduce) {
  if (M <= 0 || splitk < 1 || K % (64 * splitk) != 0 || ldx % 8 != 0 || ldy % 4 != 0) return false;
  if (epi == EPI_SILU && (N % 2 != 0 || wnf % 2 != 0)) return false;
  if (splitk > 1 && part == nullptr) return false;
  const int outN = epi == EPI_SILU ? N / 2 : N;
  const int outb = 32 * (epi == EPI_SILU ? wnf / 2 : wnf) * wn;
  if (outN % outb != 0) return false;
  const int bm = 32 * mr * wm;
  const int ntm = (M + bm - 1) / bm, ntn = outN / outb;
  const long nwg = static_cast<long>(ntm) * ntn * splitk;
  if (nwg > (1L << 30)) return false;
  float* p = splitk > 1 ? part : nullptr;
  int* cnt_ = splitk > 1 && reduce && cnt != nullptr && cnt_len >= ntm * ntn ? cnt : nullptr;
  const int kslice = K / splitk;
  bool launched = false;
#define MXS_MT(a, b, c, d, e)                                                                                  \
  if (!launched && wm == a && wn == b && mr == c && wnf == d && epi == e) {                                   \
    hipLaunchKernelGGL((mt_gemm_kernel<a, b, c, d, e>), dim3(nwg), dim3(a * b * 64), 0, s, Y, p, X, W, M, N, K, \
                       ldx, ldy, kslice, N / 2, ntm, ntn, cnt_, order);                                       \
    launched = true;                                                                                          \
  }
#define MXS_MT_E(a, b, c, d) MXS_MT(a, b, c, d, EPI_NONE) MXS_MT(a, b, c, d, EPI_SILU)
  MXS_MT_E(4, 1, 2, 2) MXS_MT_E(4, 2, 2, 2) MXS_MT_E(4, 1, 2, 4) MXS_MT_E(2, 2, 2, 2) MXS_MT_E(2, 2, 2, 4)
  MXS_MT_E(2, 4, 2, 2) MXS_MT_E(1, 4, 2, 2) MXS_MT_E(1, 2, 2, 2) MXS_MT_E(2, 1, 2, 2) MXS_MT_E(8, 1, 1, 4)
  MXS_MT_E(4, 2, 1, 2) MXS_MT_E(2, 4, 1, 2)
#undef MXS_MT_E
#undef MXS_MT
  if (!launched) return false;
  MXS_CHECK_LAUNCH();
  if (splitk > 1 && cnt_ == nullptr && reduce) {  // !reduce: the caller's epilogue kernel sums the slabs
    const long total4 = static_cast<long>(M) * outN / 4;
    const int blocks = static_cast<int>(std::min<long>((total4 + 255) / 256, 1024));
    if (epi == EPI_SILU)
      hipLaunchKernelGGL(splitk_reduce_kernel<EPI_SILU>, dim3(blocks), dim3(256), 0, s, Y, part, M, N, splitk, ldy,
                         N / 2);
    else
      hipLaunchKernelGGL(splitk_reduce_kernel<EPI_NONE>, dim3(blocks), dim3(256), 0, s, Y, part, M, N, splitk, ldy,
                         0);
    MXS_CHECK_LAUNCH();
  }
  return true;
}

// config id = ((MF-1) * 2 + (NF/2-1)) * 3 + wave layout {0: 1x4, 1: 2x2, 2: 4x1}; MF in {1, 2, 4}
// returns false when the configuration does not tile the shape (the caller keeps hipBLASLt).
// Grouped form: offs != nullptr, E experts (W [E, N, K]), M = routed rows (slab rows), rows_max = the
// most rows one expert can get (T tokens: an expert appears at most once in a token's top-k).
bool launch_decode_gemm(bf16_t* Y, float* part, const bf16_t* X, const bf16_t* W, int M, int N, int K, int ldx,
                        int ldy, int MF, int NF, int WM, int splitk, int epi, hipStream_t s, const int* offs,
                        int E, int rows_max, int LU, int reduce) {
  if (LU > 0) WM = 1;  // LDS form: 4 waves side by side over N
  const int WN = 4 / WM;
  if (M <= 0 || splitk < 1 || ldx % 8 != 0 || ldy % 4 != 0) return false;
  if (offs == nullptr ? M > 256 : (E < 1 || rows_max < 1 || rows_max > 256 || WM > 2)) return false;
  if (LU != 0 && LU != 2 && LU != 4) return false;
  if (K % (32 * (LU > 0 ? LU : decode_gemm_unroll(MF, NF)) * splitk) != 0) return false;
  const int outN = epi == EPI_SILU ? N / 2 : N;
  const int NH = epi == EPI_SILU ? NF / 2 : NF;
  const int BM = WM * MF * 16, BN = WN * NH * 16;
  if (outN % BN != 0 || (epi == EPI_SILU && N % 2 != 0)) return false;
  if (splitk > 1 && part == nullptr) return false;
  const int kslice = K / splitk;
  const int rt = offs == nullptr ? 1 : (rows_max + BM - 1) / BM;
  dim3 grid(outN / BN, offs == nullptr ? (M + BM - 1) / BM : E * rt, splitk), blk(256);
  float* p = splitk > 1 ? part : nullptr;
  const bool g = offs != nullptr;
#define MXS_DG(mf, nf, wm, e, gr)                                                                                   \
  if (MF == mf && NF == nf && WM == wm && epi == e && g == gr) {                                                  \
    hipLaunchKernelGGL((decode_gemm_kernel<mf, nf, wm, 4 / wm, e, gr>), grid, blk, 0, s, Y, p, X, W, M, N, K, ldx, \
                       ldy, kslice, N / 2, offs, rt);                                                             \
    launched = true;                                                                                              \
  }
  bool launched = false;
#define MXS_DGL(mf, nf, lu, e, gr)                                                                                 \
  if (LU == lu && MF == mf && NF == nf && epi == e && g == gr) {                                                  \
    hipLaunchKernelGGL((decode_gemm_lds_kernel<mf, nf, lu, e, gr>), grid, blk, 0, s, Y, p, X, W, M, N, K, ldx, ldy, \
                       kslice, N / 2, offs, rt);                                                                  \
    launched = true;                                                                                              \
  }
#define MXS_DGL_ALL(mf, nf, e) \
  MXS_DGL(mf, nf, 2, e, false) MXS_DGL(mf, nf, 4, e, false) MXS_DGL(mf, nf, 2, e, true) MXS_DGL(mf, nf, 4, e, true)
  if (LU > 0) {
    MXS_DGL_ALL(1, 2, 0) MXS_DGL_ALL(1, 4, 0) MXS_DGL_ALL(2, 2, 0) MXS_DGL_ALL(2, 4, 0) MXS_DGL_ALL(4, 2, 0)
    MXS_DGL_ALL(4, 4, 0) MXS_DGL_ALL(1, 2, 1) MXS_DGL_ALL(1, 4, 1) MXS_DGL_ALL(2, 2, 1) MXS_DGL_ALL(2, 4, 1)
    MXS_DGL_ALL(4, 2, 1) MXS_DGL_ALL(4, 4, 1)
  }
#undef MXS_DGL_ALL
#undef MXS_DGL
#define MXS_DG_WM(mf, nf, e) \
  MXS_DG(mf, nf, 1, e, false) MXS_DG(mf, nf, 2, e, false) MXS_DG(mf, nf, 4, e, false) MXS_DG(mf, nf, 1, e, true) MXS_DG(mf, nf, 2, e, true)
  if (LU == 0) {
    MXS_DG_WM(1, 2, 0) MXS_DG_WM(1, 4, 0) MXS_DG_WM(2, 2, 0) MXS_DG_WM(2, 4, 0) MXS_DG_WM(4, 2, 0) MXS_DG_WM(4, 4, 0)
    MXS_DG_WM(1, 2, 1) MXS_DG_WM(1, 4, 1) MXS_DG_WM(2, 2, 1) MXS_DG_WM(2, 4, 1) MXS_DG_WM(4, 2, 1) MXS_DG_WM(4, 4, 1)
  }
#undef MXS_DG_WM
#undef MXS_DG
  if (!launched) return false;
  MXS_CHECK_LAUNCH();
  if (splitk > 1 && offs == nullptr && reduce) {  // grouped: the MoE combine / silu_mul_partials kernels sum the slabs
    const long total4 = static_cast<long>(M) * outN / 4;
    const int blocks = static_cast<int>(std::min<long>((total4 + 255) / 256, 1024));
    if (epi == EPI_SILU)
      hipLaunchKernelGGL(splitk_reduce_kernel<EPI_SILU>, dim3(blocks), dim3(256), 0, s, Y, part, M, N, splitk, ldy,
                         N / 2);
    else
      hipLaunchKernelGGL(splitk_reduce_kernel<EPI_NONE>, dim3(blocks), dim3(256), 0, s, Y, part, M, N, splitk, ldy,
                         0);
    MXS_CHECK_LAUNCH();
  }
  return true;
}

}  // namespace mxs
