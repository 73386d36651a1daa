// K05-K09 (decode): weight-streaming skinny GEMM  Y[M,N] = X[M,K] . W[N,K]^T,  M <= 256.
//
// Decode projections are weight-bandwidth bound (Llama-3.2-1B: 121 MB of weights per layer against
// ~1 MB of activations), but library GEMMs tile them with 256-wide macro tiles: N=3072 becomes a
// dozen workgroups and each projection costs 11-28 us instead of the ~2-11 us its weight bytes need
// at HBM speed.  This kernel is shaped for the weights instead:
//
//   * a wave owns 16 weight rows and MT tokens: v_mfma_f32_16x16x32_bf16 with A = W (16 x 32 k),
//     B = X^T (32 k x 16 tokens), MT/16 accumulators of 4 fp32;
//   * a workgroup is 4 waves arranged WN (along N) x WK (along K): WK > 1 splits each weight row's
//     K range across waves (combined through LDS), so narrow projections still launch >= 128-256
//     workgroups and every weight byte is read exactly once per token tile;
//   * operands go straight from global memory to registers (the guide's "GEMV / M <= 16" row): every
//     lane loads 16 B (8 k) per MFMA, 4 lanes cover 64 contiguous bytes of a row, and the next 128-k
//     block is in flight while the current one is multiplied;
//   * M > MT launches one workgroup per token tile; blockIdx is remapped so the token tiles of one
//     weight tile run on the same XCD and share its L2 copy of the weights.
#include "common.h"

namespace mxs {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8_t u4_as_bf16x8(const u32x4& v) { return __builtin_bit_cast(bf16x8_t, v); }

template <int MT, int WN, int WK>
__global__ void __launch_bounds__(256) skinny_gemm_kernel(bf16_t* __restrict__ Y, const bf16_t* __restrict__ X,
                                                          const bf16_t* __restrict__ W, int M, int N, int K,
                                                          int ldx, int ldy, int mtiles) {
  constexpr int TT = MT / 16;
  constexpr int NT = 16 * WN;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wn = wid % WN, wk = wid / WN;
  // XCD-aware tile order: hardware deals workgroups round-robin over 8 XCDs; make consecutive
  // virtual ids land on one XCD so the token tiles of a weight tile hit the same L2
  const int G = gridDim.x, g = blockIdx.x;
  const int v = (G % 8 == 0) ? (g % 8) * (G / 8) + g / 8 : g;
  const int ntile = v / mtiles, mtile = v - ntile * mtiles;
  const int n0 = ntile * NT + wn * 16;
  const int m0 = mtile * MT;
  const int i = lane & 15, kq = lane >> 4;
  const int kper = K / WK;
  const int kbeg = wk * kper;

  const bf16_t* wp = W + static_cast<size_t>(n0 + i) * K + kbeg + 8 * kq;
  const bf16_t* xp[TT];
  bool xv[TT];
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    const int m = m0 + 16 * t + i;
    xv[t] = m < M;
    xp[t] = X + static_cast<size_t>(xv[t] ? m : 0) * ldx + kbeg + 8 * kq;
  }

  float4_ acc[TT];
#pragma unroll
  for (int t = 0; t < TT; ++t) acc[t] = float4_{0.f, 0.f, 0.f, 0.f};

  // one 128-k block = 4 MFMA k-steps; lane (i, kq) of k-step j holds k = 32 j + 8 kq .. + 7
  u32x4 a[4], b[TT][4];
  auto load = [&](int kb, u32x4 (&ad)[4], u32x4 (&bd)[TT][4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) ad[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wp + kb + 32 * j));
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bd[t][j] = xv[t] ? *reinterpret_cast<const u32x4*>(xp[t] + kb + 32 * j) : u32x4{0u, 0u, 0u, 0u};
  };
  load(0, a, b);
  for (int kb = 0; kb < kper; kb += 128) {
    u32x4 an[4], bn[TT][4];
    const bool more = kb + 128 < kper;
    if (more) load(kb + 128, an, bn);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < TT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(u4_as_bf16x8(a[j]), u4_as_bf16x8(b[t][j]), acc[t], 0, 0, 0);
    if (more) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] = an[j];
#pragma unroll
        for (int t = 0; t < TT; ++t) b[t][j] = bn[t][j];
      }
    }
  }

  if constexpr (WK > 1) {
    __shared__ float red[WK - 1][WN][TT][4][64];
    if (wk > 0) {
#pragma unroll
      for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wk - 1][wn][t][r][lane] = acc[t][r];
    }
    __syncthreads();
    if (wk > 0) return;
#pragma unroll
    for (int s = 0; s < WK - 1; ++s)
#pragma unroll
      for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[t][r] += red[s][wn][t][r][lane];
  }
  // C^T fragment: lane (i, kq) holds Y[m0 + 16 t + i][n0 + 4 kq + r], r = 0..3
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    if (!xv[t]) continue;
    uint2 o;
    o.x = pack2(acc[t][0], acc[t][1]);
    o.y = pack2(acc[t][2], acc[t][3]);
    *reinterpret_cast<uint2*>(Y + static_cast<size_t>(m0 + 16 * t + i) * ldy + n0 + 4 * kq) = o;
  }
}

// Returns false when the shape is outside what the kernel supports (caller falls back).
bool launch_skinny_gemm(bf16_t* Y, const bf16_t* X, const bf16_t* W, int M, int N, int K, int ldx, int ldy,
                        hipStream_t s) {
  if (M <= 0 || M > 256 || N % 16 != 0 || K % 128 != 0 || ldx % 8 != 0 || ldy % 4 != 0) return false;
  const int MT = M <= 16 ? 16 : (M <= 32 ? 32 : 64);
  const int mtiles = (M + MT - 1) / MT;
  // widen along N while that still leaves >= 256 workgroups, otherwise split K inside the workgroup
  int WN = 4;
  while (WN > 1 && (N % (16 * WN) != 0 || (N / (16 * WN)) * mtiles < 256)) WN >>= 1;
  int WK = 4 / WN;
  while (WK > 1 && K % (128 * WK) != 0) WK >>= 1;
  if (WN * WK != 4) {  // K too short to split 4 ways: fall back to full-N tiles
    WN = 4;
    WK = 1;
    if (N % 64 != 0) return false;
  }
  const int ntiles = N / (16 * WN);
  dim3 grid(ntiles * mtiles), blk(256);
#define MXS_SG(MM, A, B)                                                                               \
  if (MT == MM && WN == A && WK == B) {                                                                \
    hipLaunchKernelGGL((skinny_gemm_kernel<MM, A, B>), grid, blk, 0, s, Y, X, W, M, N, K, ldx, ldy, mtiles); \
    MXS_CHECK_LAUNCH();                                                                                \
    return true;                                                                                       \
  }
  MXS_SG(16, 4, 1) MXS_SG(16, 2, 2) MXS_SG(16, 1, 4)
  MXS_SG(32, 4, 1) MXS_SG(32, 2, 2) MXS_SG(32, 1, 4)
  MXS_SG(64, 4, 1) MXS_SG(64, 2, 2) MXS_SG(64, 1, 4)
#undef MXS_SG
  return false;
}

}  // namespace mxs
