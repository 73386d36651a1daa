// K05-K08 at prefill sizes: Y[T, N] = X[T, K] . W[N, K]^T for the narrow projections (Llama-3.2-1B
// qkv N 3072, o / down N 2048) at T = 512-4096 tokens, where the library's 256 x 256 tiles leave most
// of the 256 CUs idle (hipBLASLt 0.2-0.9 PF/s there, profiles/r2_prefill_gemm_hipblaslt.jsonl).
//
// Tile BM x BN x 64 (BM 64 / 128, BN 128) per 256-thread workgroup, 4 waves in 2 x 2, each wave
// (BM/2) x (BN/2) outputs as 16 x 16 fragments of v_mfma_f32_16x16x32_bf16 with A = W (output
// columns on the accumulator rows) and B = X^T (tokens on the lanes), so a lane's accumulator is
// Y[token][4 consecutive columns] and the store is one 8-byte write.
// Both operand tiles go global -> registers -> LDS (two buffers; the next k-tile's loads are in
// flight under this k-tile's MFMAs, one barrier per k-tile), rows of 128 B with the 16-byte chunks
// XOR-swizzled by (row & 7) so the fragment reads (16 rows, one chunk) spread over the banks.
// Split-K (gridDim.z > 1) writes fp32 slabs that prefill_splitk_reduce_kernel sums.  The workgroup
// id is remapped so that consecutive tiles of one XCD share their X rows in that XCD's L2.
#include <algorithm>

#include "common.h"

namespace mxs {

typedef __bf16 pg_bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned int pg_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int pg_swz(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

template <int BM, int BN>
__global__ void __launch_bounds__(256) prefill_gemm_kernel(bf16_t* __restrict__ Y, float* __restrict__ part,
                                                           const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                           int M, int N, int K, int ldx, int ldy, int kslice, int ntm,
                                                           int ntn) {
  constexpr int BK = 64;
  constexpr int WTM = BM / 2, WTN = BN / 2;   // wave tile
  constexpr int FM = WTM / 16, FN = WTN / 16;  // fragments
  constexpr int XCHK = BM * BK / 8 / 256;      // 16-byte chunks per thread per stage
  constexpr int WCHK = BN * BK / 8 / 256;
  constexpr int STAGE = (BM + BN) * 128;       // bytes of one stage (X tile, then W tile)
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  // ---- workgroup -> (z, tile_m, tile_n), XCD-aware: the 8 XCDs take workgroups round-robin, so
  // give XCD x a contiguous range of the tile order (bijective for any count)
  const int nwg = gridDim.x;
  const int bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tn = wg % ntn, tm = (wg / ntn) % ntm, z = wg / (ntn * ntm);
  const int m0 = tm * BM, n0 = tn * BN, kbeg = z * kslice;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int i16 = lane & 15, kq = lane >> 4;

  // global sources of this thread's chunks (rows past M re-read row M-1: loaded, never stored)
  const bf16_t* xsrc[XCHK];
  int xoff[XCHK];
#pragma unroll
  for (int s = 0; s < XCHK; ++s) {
    const int c = tid + 256 * s, row = c >> 3, ch = c & 7;
    xsrc[s] = X + static_cast<size_t>(min(m0 + row, M - 1)) * ldx + kbeg + ch * 8;
    xoff[s] = pg_swz(row, ch);
  }
  const bf16_t* wsrc[WCHK];
  int woff[WCHK];
#pragma unroll
  for (int s = 0; s < WCHK; ++s) {
    const int c = tid + 256 * s, row = c >> 3, ch = c & 7;
    wsrc[s] = W + static_cast<size_t>(n0 + row) * K + kbeg + ch * 8;
    woff[s] = BM * 128 + pg_swz(row, ch);
  }
  pg_u32x4 gx[XCHK], gw[WCHK];
  auto gload = [&](int k) {
#pragma unroll
    for (int s = 0; s < XCHK; ++s) gx[s] = *reinterpret_cast<const pg_u32x4*>(xsrc[s] + k);
#pragma unroll
    for (int s = 0; s < WCHK; ++s) gw[s] = *reinterpret_cast<const pg_u32x4*>(wsrc[s] + k);
  };
  auto sstore = [&](int st) {
    char* base = smem + st * STAGE;
#pragma unroll
    for (int s = 0; s < XCHK; ++s) *reinterpret_cast<pg_u32x4*>(base + xoff[s]) = gx[s];
#pragma unroll
    for (int s = 0; s < WCHK; ++s) *reinterpret_cast<pg_u32x4*>(base + woff[s]) = gw[s];
  };

  float4_ acc[FN][FM];
#pragma unroll
  for (int a = 0; a < FN; ++a)
#pragma unroll
    for (int b = 0; b < FM; ++b) acc[a][b] = float4_{0.f, 0.f, 0.f, 0.f};

  const int nk = kslice / BK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) gload((kt + 1) * BK);
    const char* base = smem + st * STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {  // two 32-k MFMA steps per 64-k tile
      pg_u32x4 af[FN], bfr[FM];
#pragma unroll
      for (int a = 0; a < FN; ++a)
        af[a] = *reinterpret_cast<const pg_u32x4*>(base + BM * 128 + pg_swz(wc * WTN + a * 16 + i16, kk * 4 + kq));
#pragma unroll
      for (int b = 0; b < FM; ++b)
        bfr[b] = *reinterpret_cast<const pg_u32x4*>(base + pg_swz(wr * WTM + b * 16 + i16, kk * 4 + kq));
#pragma unroll
      for (int a = 0; a < FN; ++a)
#pragma unroll
        for (int b = 0; b < FM; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(pg_bf16x8_t, af[a]),
                                                              __builtin_bit_cast(pg_bf16x8_t, bfr[b]), acc[a][b],
                                                              0, 0, 0);
    }
    if (more) {
      sstore(st ^ 1);
      __syncthreads();
    }
  }

  // ---- epilogue: acc[a][b][reg] = Y[m0 + wr WTM + 16 b + i16][n0 + wc WTN + 16 a + 4 kq + reg]
#pragma unroll
  for (int b = 0; b < FM; ++b) {
    const int m = m0 + wr * WTM + 16 * b + i16;
    if (m >= M) continue;
#pragma unroll
    for (int a = 0; a < FN; ++a) {
      const int n = n0 + wc * WTN + 16 * a + 4 * kq;
      if (part != nullptr) {
        *reinterpret_cast<float4_*>(part + (static_cast<size_t>(z) * M + m) * N + n) = acc[a][b];
      } else {
        uint2 o;
        o.x = pack2(acc[a][b][0], acc[a][b][1]);
        o.y = pack2(acc[a][b][2], acc[a][b][3]);
        *reinterpret_cast<uint2*>(Y + static_cast<size_t>(m) * ldy + n) = o;
      }
    }
  }
}

__global__ void __launch_bounds__(256) prefill_splitk_reduce_kernel(bf16_t* __restrict__ Y, const float* __restrict__ part,
                                                                    int M, int N, int S, int ldy) {
  const long total4 = static_cast<long>(M) * N / 4;
  for (long q = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; q < total4;
       q += static_cast<long>(gridDim.x) * blockDim.x) {
    const int m = static_cast<int>((q * 4) / N), n = static_cast<int>((q * 4) % N);
    float4_ g = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < S; ++s) g += *reinterpret_cast<const float4_*>(part + (static_cast<size_t>(s) * M + m) * N + n);
    uint2 o;
    o.x = pack2(g[0], g[1]);
    o.y = pack2(g[2], g[3]);
    *reinterpret_cast<uint2*>(Y + static_cast<size_t>(m) * ldy + n) = o;
  }
}

// bm in {64, 128}, BN 128; false when the configuration does not tile the shape.
bool launch_prefill_gemm(bf16_t* Y, float* part, const bf16_t* X, const bf16_t* W, int M, int N, int K, int ldx,
                         int ldy, int bm, int splitk, hipStream_t s) {
  constexpr int BN = 128;
  if (M <= 0 || N % BN != 0 || splitk < 1 || K % (64 * splitk) != 0 || ldx % 8 != 0 || ldy % 4 != 0) return false;
  if (bm != 64 && bm != 128) return false;
  if (splitk > 1 && part == nullptr) return false;
  const int ntm = (M + bm - 1) / bm, ntn = N / BN;
  const long nwg = static_cast<long>(ntm) * ntn * splitk;
  if (nwg > (1L << 30)) return false;
  float* p = splitk > 1 ? part : nullptr;
  if (bm == 128)
    hipLaunchKernelGGL((prefill_gemm_kernel<128, BN>), dim3(nwg), dim3(256), 0, s, Y, p, X, W, M, N, K, ldx, ldy,
                       K / splitk, ntm, ntn);
  else
    hipLaunchKernelGGL((prefill_gemm_kernel<64, BN>), dim3(nwg), dim3(256), 0, s, Y, p, X, W, M, N, K, ldx, ldy,
                       K / splitk, ntm, ntn);
  MXS_CHECK_LAUNCH();
  if (splitk > 1) {
    const long total4 = static_cast<long>(M) * N / 4;
    const int blocks = static_cast<int>(std::min<long>((total4 + 255) / 256, 2048));
    hipLaunchKernelGGL(prefill_splitk_reduce_kernel, dim3(blocks), dim3(256), 0, s, Y, part, M, N, splitk, ldy);
    MXS_CHECK_LAUNCH();
  }
  return true;
}

}  // namespace mxs
