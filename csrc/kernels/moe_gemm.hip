// K16: MoE grouped GEMM over expert-sorted rows, MFMA bf16, LDS double-buffered.
//
//   Y[r, :] = X[r, :] . W[e(r)]^T       W: [E_local, N, K] (nn.Linear layout), rows sorted by expert
//   SILU variant (gate_up): W rows are [gate (N/2); up (N/2)] and the epilogue writes
//   silu(gate) * up, width N/2 -- the activation never round-trips HBM.
//
// Tiling: a workgroup owns a 128-column x 128-row tile of C^T = W . X^T (4 waves, 2 x 2, each wave
// 64 x 64 = 2 x 2 v_mfma_f32_32x32x16_bf16 tiles); K in steps of 64 through two LDS buffers (the
// next step's global loads are in flight while the current one is multiplied).  LDS rows are 128 B
// with the 16-byte chunks XOR-swizzled by (row & 7) so the ds_read_b128 fragment reads of 32
// consecutive rows spread over the banks.  C^T puts the TOKEN on the lane: each lane stores 4
// consecutive output columns with one 8-byte store.
// Expert scheduling is on the device: a workgroup derives (expert, row block) from the
// moe_align offsets itself (prefix over ceil(count_e / 128)), so the launch needs no host sync and is
// hipGraph-capturable; the grid is sized for the worst case and surplus workgroups exit.
// Split-K (plain variant, gridDim.z > 1): decode routes a few rows per expert, so the down
// projection (N 4,096, K 14,336) has only N/128 x experts workgroups, each streaming a 3.7 MB weight
// slice through 224 K-steps -- one workgroup per CU, latency-bound.  With split-K each z-slice
// streams K/z and writes fp32 partials [z][row][n]; the combine kernel sums the slices.
#include "common.h"

namespace mxs {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kGBM = 128;  // token rows per tile
constexpr int kGBN = 128;  // weight rows per tile
constexpr int kGBK = 64;   // k per stage

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

template <bool SILU>
__global__ void __launch_bounds__(256) moe_grouped_gemm_kernel(bf16_t* __restrict__ Y, const bf16_t* __restrict__ X,
                                                               const bf16_t* __restrict__ W,
                                                               const int* __restrict__ offs, int E, int N, int K,
                                                               int ldy, float* __restrict__ partial, int rows_cap) {
  __shared__ __attribute__((aligned(16))) char smem[2][2][kGBN * 128];  // [stage][W | X][rows x 128 B]
  // ---- which expert / row block is this workgroup's
  int tile = blockIdx.y, e = -1, r0 = 0, r1 = 0;
  {
    int acc = 0;
    for (int x = 0; x < E; ++x) {
      const int a = offs[x], b = offs[x + 1];
      const int nt = (b - a + kGBM - 1) / kGBM;
      if (tile < acc + nt) {
        e = x;
        r0 = a + (tile - acc) * kGBM;
        r1 = b;
        break;
      }
      acc += nt;
    }
  }
  if (e < 0) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nh = wid & 1, mh = wid >> 1;  // this wave: weight rows 64 nh.., token rows 64 mh..
  // weight rows of this tile: plain = [n0, n0 + 128); SILU = gate [j0, j0 + 64) + up [I + j0, ...)
  const int I = N / 2;
  const int n0 = blockIdx.x * (SILU ? kGBN / 2 : kGBN);
  const bf16_t* We = W + static_cast<size_t>(e) * N * K;

  // ---- global -> register staging: 4 x 16 B of W and of X per thread per stage
  u32x4 gw[4], gx[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int row = (tid >> 3) + 32 * it, chunk = tid & 7;
      const int wrow = SILU ? (row < 64 ? n0 + row : I + n0 + row - 64) : n0 + row;
      gw[it] = *reinterpret_cast<const u32x4*>(We + static_cast<size_t>(wrow) * K + k0 + chunk * 8);
      const int xr = r0 + row;
      gx[it] = xr < r1 ? *reinterpret_cast<const u32x4*>(X + static_cast<size_t>(xr) * K + k0 + chunk * 8)
                       : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto sstore = [&](int st) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int row = (tid >> 3) + 32 * it, chunk = tid & 7;
      *reinterpret_cast<u32x4*>(&smem[st][0][swz(row, chunk)]) = gw[it];
      *reinterpret_cast<u32x4*>(&smem[st][1][swz(row, chunk)]) = gx[it];
    }
  };

  float16_ acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

  const int i32 = lane & 31, h = lane >> 5;
  const int nk_all = K / kGBK, S = gridDim.z, z = blockIdx.z;
  const int ks_lo = nk_all * z / S, nk = nk_all * (z + 1) / S - ks_lo;
  const int k_lo = ks_lo * kGBK;
  gload(k_lo);
  sstore(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int st = ks & 1;
    if (ks + 1 < nk) gload(k_lo + (ks + 1) * kGBK);  // next stage in flight under this stage's MFMAs
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {  // 16-k MFMA steps; lane half h takes chunk 2 kk + h
      bf16x8_t af[2], bf[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int row = nh * 64 + a * 32 + i32;
        af[a] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u32x4*>(&smem[st][0][swz(row, 2 * kk + h)]));
      }
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int row = mh * 64 + b * 32 + i32;
        bf[b] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u32x4*>(&smem[st][1][swz(row, 2 * kk + h)]));
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bf[b], acc[a][b], 0, 0, 0);
    }
    if (ks + 1 < nk) {
      sstore(st ^ 1);
      __syncthreads();
    }
  }

  // ---- epilogue.  acc[a][b][reg]: weight row nh*64 + a*32 + (reg&3) + 8*(reg>>2) + 4h,
  //                                 token row  mh*64 + b*32 + lane%32
  if constexpr (!SILU) {
    if (S > 1) {  // fp32 partial slice z: [z][row][n], summed by the combine kernel
      float* pz = partial + static_cast<size_t>(z) * rows_cap * N;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int m = r0 + mh * 64 + b * 32 + i32;
        if (m >= r1) continue;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int n = n0 + nh * 64 + a * 32 + 8 * g + 4 * h;
            *reinterpret_cast<float4*>(pz + static_cast<size_t>(m) * N + n) =
                make_float4(acc[a][b][4 * g], acc[a][b][4 * g + 1], acc[a][b][4 * g + 2], acc[a][b][4 * g + 3]);
          }
      }
      return;
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int m = r0 + mh * 64 + b * 32 + i32;
      if (m >= r1) continue;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = n0 + nh * 64 + a * 32 + 8 * g + 4 * h;
          uint2 v;
          v.x = pack2(acc[a][b][4 * g], acc[a][b][4 * g + 1]);
          v.y = pack2(acc[a][b][4 * g + 2], acc[a][b][4 * g + 3]);
          *reinterpret_cast<uint2*>(Y + static_cast<size_t>(m) * ldy + n) = v;
        }
    }
  } else {
    // up waves (nh = 1) hand their accumulators to the gate waves (nh = 0) through LDS
    __syncthreads();
    float* up = reinterpret_cast<float*>(&smem[0][0][0]);  // [128 token rows][64 + 1] fp32 (padded)
    constexpr int LD = 65;
    if (nh == 1) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int j = a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            const int t = mh * 64 + b * 32 + i32;
            up[t * LD + j] = acc[a][b][r];
          }
    }
    __syncthreads();
    if (nh == 0) {
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int t = mh * 64 + b * 32 + i32;
        const int m = r0 + t;
        if (m >= r1) continue;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            float o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int j = a * 32 + 8 * g + 4 * h + q;
              const float gv = acc[a][b][4 * g + q];
              o[q] = gv / (1.f + __expf(-gv)) * up[t * LD + j];
            }
            uint2 v;
            v.x = pack2(o[0], o[1]);
            v.y = pack2(o[2], o[3]);
            *reinterpret_cast<uint2*>(Y + static_cast<size_t>(m) * ldy + n0 + a * 32 + 8 * g + 4 * h) = v;
          }
      }
    }
  }
}

// rows_upper: upper bound on the routed rows (T * top_k); the grid covers the worst case.
// split > 1 (plain variant only): fp32 partials into partial[split][rows_upper][N] instead of Y.
bool launch_moe_grouped_gemm(bf16_t* Y, const bf16_t* X, const bf16_t* W, const int* offs, int E, int rows_upper,
                             int N, int K, int ldy, bool silu, int split, float* partial, hipStream_t s) {
  if (K % kGBK != 0) return false;
  if (silu ? ((N / 2) % (kGBN / 2) != 0 || N % 2) : (N % kGBN != 0)) return false;
  if (split < 1 || split > K / kGBK || (split > 1 && (silu || partial == nullptr))) return false;
  const int max_tiles = (rows_upper + kGBM - 1) / kGBM + E;
  dim3 grid(silu ? (N / 2) / (kGBN / 2) : N / kGBN, max_tiles, split), blk(256);
  if (silu)
    hipLaunchKernelGGL(moe_grouped_gemm_kernel<true>, grid, blk, 0, s, Y, X, W, offs, E, N, K, ldy, partial,
                       rows_upper);
  else
    hipLaunchKernelGGL(moe_grouped_gemm_kernel<false>, grid, blk, 0, s, Y, X, W, offs, E, N, K, ldy, partial,
                       rows_upper);
  MXS_CHECK_LAUNCH();
  return true;
}

}  // namespace mxs
