// K05-K08 at prefill chunks, second form: Y[M, N] = X[M, K] . W[N, K]^T with FOUR waves per workgroup
// and a 128 x 128 output block per wave (gemm_pf: eight waves of 64 x 128).
//
// Why a second form.  At 256 x 256 x 64 per workgroup, the LDS bytes a wave reads per MFMA fall with
// the wave's output block: (Mw + Nw) / (Mw Nw) = 0.0156 B/FLOP at 128 x 128 against 0.0234 at 64 x 128
// -- a third fewer ds_read_b128 per k-tile (128 KB instead of 192 KB per CU) -- and fewer LDS read
// bytes per MFMA are what lets the chip hold a higher clock under an MFMA-dense loop (MI355X_MICROARCH.md
// "DVFS give-back", cdna_hip_programming.md §5.4 rule 28).  hipBLASLt's fastest kernels on these shapes
// are 256-thread MT256x256 tiles of this kind.
//
// Structure (one workgroup per CU, persistent over its tiles, data-parallel):
//   * 4 waves as 2 (token halves) x 2 (weight halves); v_mfma_f32_16x16x32_bf16 with A = W (output
//     columns on the accumulator rows) and B = X^T, so a lane holds Y[token][4 consecutive columns]
//     (the gemm_pf convention); acc[8 w-frags][8 token frags] = 256 VGPRs;
//   * operands HBM/L2 -> LDS by LDS-DMA (buffer_load ... lds, 16 B per lane, 1 KB per instruction),
//     two 64 KB stages (W 256 rows x 128 B, X 256 rows x 128 B); the 16-byte chunks of a 128-byte row
//     XOR-swizzled by (row >> 1) & 7 on the SOURCE address and un-swizzled on the read (conflict-free
//     for the ds_read_b128 lane groups, the gemm_pf image);
//   * fragments double-buffered in registers at k-step (32-deep) granularity: a k-tile is two phases,
//     A = MFMAs of k-step 0 beside the reads of k-step 1, B = MFMAs of k-step 1 beside the LDS-DMA of
//     the k-tile two ahead (into the stage just released) and the reads of the next k-tile's k-step 0.
//     ONE barrier per k-tile, between the phases: every wave has read the stage (its lgkmcnt(0)) and
//     every wave's DMA of the next k-tile has landed (its counted vmcnt);
//   * the k-tile stream runs on across a workgroup's tiles (the next tile's first k-tiles are in LDS
//     while the finished tile's epilogue stores); tiles visited in the host tile map's XCD-aware order.
// EPI_NONE / EPI_SWIGLU / EPI_RESID as gemm_pf (W = [gate; up] interleaved per 16 rows for SwiGLU).
#include <algorithm>

#include "common.h"

namespace mxs {

typedef __bf16 w4_bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int w4_u32x4 __attribute__((ext_vector_type(4)));

constexpr int W4_EPI_NONE = 0;
constexpr int W4_EPI_SWIGLU = 1;
constexpr int W4_EPI_RESID = 2;

struct W4Args {
  bf16_t* Y;
  const bf16_t* X;
  const bf16_t* W;
  const bf16_t* R;       // EPI_RESID: residual rows (ldr), may equal Y
  int M, K, ldx, ldy, ldr, nk, ntm, ntn, ntiles, inter, nrows_w;
};

__device__ __forceinline__ w4_bf16x8 w4_frag(const w4_u32x4& v) { return __builtin_bit_cast(w4_bf16x8, v); }
__device__ __forceinline__ float w4_silu(float g) { return g / (1.f + __expf(-g)); }
// two floats -> two bf16 in a dword by plain casts (hipcc: one v_cvt_pk_bf16_f32, NaN kept)
__device__ __forceinline__ uint32_t w4_pack(float lo, float hi) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, bf16x2_t{static_cast<__bf16>(lo), static_cast<__bf16>(hi)});
}
// logical tile L -> (token tile, weight tile): pf_tile_map's order (8 token tiles per weight-column
// sweep, so the 32 consecutive tiles an XCD runs together share W and X panels), computed on the
// scalar unit once per tile instead of a table load that would drain the DMA queue
__device__ __forceinline__ void w4_tile(int L, int ntm, int ntn, int& tm, int& tn) {
  const int per = 8 * ntn, grp = L / per, first = grp * 8;
  const int gsz = min(ntm - first, 8), ing = L - grp * per;
  tm = first + ing % gsz;
  tn = ing / gsz;
}

template <int EPI>
__global__ void __launch_bounds__(256, 1) gemm_w4_kernel(const W4Args a) {
  constexpr int STG = 32768, XO = 16384;  // stage bytes (a 32-deep k-block); X image offset in a stage
  __shared__ __attribute__((aligned(16))) char smem[4 * STG];

  const int G = gridDim.x, nk = a.nk;  // one workgroup per tile; nk: 32-deep k-blocks
  // blocks b and b + 8 share an XCD: give each XCD a contiguous range of the tile order, so the 32
  // workgroups an XCD runs at a time share W and X panels in its L2
  const int bid = blockIdx.x, xcd = bid & 7, q8 = G >> 3, r8 = G & 7;
  const int o = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ns = nk;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;

  // ---- LDS-DMA sources.  Image rows are 64 B (32 k); piece i (0..15) of an operand fills rows
  // 16 i + (lane >> 2), chunk p = lane & 3 of a row holding source chunk p ^ ((row >> 2) & 3) =
  // p ^ (lane >> 4) for every i.  Wave wid issues pieces 4 wid + j (j = 0..3) of W and of X.
  const int csrc = (lane & 3) ^ (lane >> 4);
  const int wvo = ((lane >> 2) * a.K + 8 * csrc) * 2;  // W: per lane; piece rows go to the soffset
  int wso[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = 4 * wid + j;
    int row;
    if constexpr (EPI == W4_EPI_SWIGLU) {  // image row r -> [gate | up] row (gemm_pf's interleave)
      row = ((i & 3) >= 2 ? a.inter : 0) + 32 * (i >> 2) + 16 * (i & 1);
    } else {
      row = 16 * i;
    }
    wso[j] = row * a.K * 2;
  }
  int xvo[4];  // X: the whole row offset per lane (rows past M fall outside the tile's descriptor -> 0)
#pragma unroll
  for (int j = 0; j < 4; ++j) xvo[j] = ((16 * (4 * wid + j) + (lane >> 2)) * a.ldx + 8 * csrc) * 2;

  constexpr int WSTEP = EPI == W4_EPI_SWIGLU ? 128 : 256;  // weight rows (from W's base) per tile step
  const long w_bytes = 2L * a.K * a.nrows_w;
  typedef __attribute__((address_space(3))) void lds_t;

  int tm, tn;
  w4_tile(o, a.ntm, a.ntn, tm, tn);
  // the 8 DMA pieces (4 W, 4 X) this wave issues for stream position c, into stage c & 3
  const long woff = 2L * tn * WSTEP * a.K;
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(a.W) + woff / 2, static_cast<short>(0),
      static_cast<int>(min(w_bytes - woff, 0x7FFFFFFFL)), 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(a.X) + static_cast<size_t>(tm) * 256 * a.ldx, static_cast<short>(0),
      (a.M - tm * 256) * a.ldx * 2, 0x00020000);
  auto dma = [&](int c) {
    const int k = c;
    char* st = smem + (c & 3) * STG;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_t*)(st + (4 * wid + j) * 1024), 16, wvo, wso[j] + 64 * k,
                                               0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_t*)(st + XO + (4 * wid + j) * 1024), 16, xvo[j], 64 * k,
                                               0, 0);
    }
  };

  // ---- fragments of v_mfma_f32_32x32x16_bf16: lane (r32, h) reads row r32 of a 32-row fragment,
  // logical chunk 2 ks + h of the 64-byte row, stored at chunk (2 ks + h) ^ ((r32 >> 2) & 3)
  const int r32 = lane & 31, h = lane >> 5, swz = (r32 >> 2) & 3;
  const int ch0 = (h ^ swz) << 4, ch1 = ((2 + h) ^ swz) << 4;
  const int wb = (128 * wn + r32) * 64, xb = XO + (128 * wm + r32) * 64;
  w4_u32x4 fa0[4], fb0[4], fa1[4], fb1[4];  // k-step 0 / 1: [w frag], [token frag]
  auto rd = [&](w4_u32x4 (&fa)[4], w4_u32x4 (&fb)[4], int stage, int ks) {
    const char* base = smem + stage * STG;
    const int ch = ks ? ch1 : ch0;
#pragma unroll
    for (int f = 0; f < 4; ++f) fa[f] = *reinterpret_cast<const w4_u32x4*>(base + wb + ch + f * 2048);
#pragma unroll
    for (int t = 0; t < 4; ++t) fb[t] = *reinterpret_cast<const w4_u32x4*>(base + xb + ch + t * 2048);
  };

  float16_ acc[4][4];  // [w frag][token frag]
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[f][t] = float16_{};
  auto mma = [&](const w4_u32x4 (&fa)[4], const w4_u32x4 (&fb)[4]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int t = 0; t < 4; ++t)
        acc[f][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w4_frag(fa[f]), w4_frag(fb[t]), acc[f][t], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // epilogue of a finished tile: lane (r32, h), acc[f][t][4 g + e] = Y[token m0 + 128 wm + 32 t + r32]
  // [image column 128 wn + 32 f + 8 g + 4 h + e]
  auto epilogue = [&](int tm, int tn) {
    const int m0 = tm * 256;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int m = m0 + 128 * wm + 32 * t + r32;
      if (m >= a.M) continue;
      bf16_t* yr = a.Y + static_cast<size_t>(m) * a.ldy;
      if constexpr (EPI == W4_EPI_SWIGLU) {
#pragma unroll
        for (int f = 0; f < 4; f += 2) {  // (gate, up) fragment pairs (f, f + 1)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const float16_& gv = acc[f][t];
            const float16_& uv = acc[f + 1][t];
            const int n = tn * 128 + 64 * wn + 32 * (f >> 1) + 8 * g + 4 * h;
            uint2 ov;
            ov.x = w4_pack(w4_silu(gv[4 * g]) * uv[4 * g], w4_silu(gv[4 * g + 1]) * uv[4 * g + 1]);
            ov.y = w4_pack(w4_silu(gv[4 * g + 2]) * uv[4 * g + 2], w4_silu(gv[4 * g + 3]) * uv[4 * g + 3]);
            *reinterpret_cast<uint2*>(yr + n) = ov;
            __builtin_amdgcn_sched_barrier(0);  // one group of accumulators at a time: no mass AGPR reads
          }
        }
      } else {
#pragma unroll
        for (int f = 0; f < 4; ++f) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const float16_& v = acc[f][t];
            const int n = tn * 256 + 128 * wn + 32 * f + 8 * g + 4 * h;
            float r0 = 0.f, r1 = 0.f, r2 = 0.f, r3 = 0.f;
            if constexpr (EPI == W4_EPI_RESID) {
              const uint2 rv = *reinterpret_cast<const uint2*>(a.R + static_cast<size_t>(m) * a.ldr + n);
              r0 = bf2f_lo(rv.x);
              r1 = bf2f_hi(rv.x);
              r2 = bf2f_lo(rv.y);
              r3 = bf2f_hi(rv.y);
            }
            uint2 ov;
            ov.x = w4_pack(v[4 * g] + r0, v[4 * g + 1] + r1);
            ov.y = w4_pack(v[4 * g + 2] + r2, v[4 * g + 3] + r3);
            *reinterpret_cast<uint2*>(yr + n) = ov;
            __builtin_amdgcn_sched_barrier(0);  // one group of accumulators at a time: no mass AGPR reads
          }
        }
      }
    }
  };

#define W4_BAR()                           \
  do {                                     \
    __builtin_amdgcn_sched_barrier(0);     \
    __builtin_amdgcn_s_barrier();          \
    __builtin_amdgcn_sched_barrier(0);     \
  } while (0)

  // prologue: positions 0..2 in flight, position 0 landed and visible, its k-step 0 in registers
  dma(0);
  if (ns > 1) dma(1);
  if (ns > 2) dma(2);
  if (ns > 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (ns > 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  W4_BAR();
  rd(fa0, fb0, 0, 0);

#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[f][t] = float16_{};
  for (int c = 0; c < ns; ++c) {
    const int s = c & 3;
    // half 1: DMA of k-block c + 3 into the stage read at c - 1 (every wave passed the barrier after
    // those reads), the reads of k-step 1, the MFMAs of k-step 0
    if (c + 3 < ns) dma(c + 3);
    rd(fa1, fb1, s, 1);
    mma(fa0, fb0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // one MFMA, one DMA piece, one fragment read, ...
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // k-block c + 1 landed: the pieces of c + 2 and c + 3 (8 each, issued at c - 1 and c) may stay in
    // flight; the count runs oldest-first
    if (c + 3 < ns) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (c + 2 < ns) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    W4_BAR();  // k-block c + 1 visible in its stage; every wave is done reading stage s
    // half 2: the reads of k-block c + 1's k-step 0 beside the MFMAs of k-step 1
    if (c + 1 < ns) rd(fa0, fb0, (c + 1) & 3, 0);
    mma(fa1, fb1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // two MFMAs, one fragment read, ...
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  epilogue(tm, tn);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef W4_BAR
}

// Grid = min(CUs, tiles) workgroups of 256 threads.  Returns false when the shape is not supported.
bool launch_gemm_w4(bf16_t* Y, const bf16_t* X, const bf16_t* W, int M, int N, int K, int ldx, int ldy, int epi,
                    int num_cu, hipStream_t s, const bf16_t* R, int ldr) {
  if (M <= 0 || K % 64 != 0 || N % 256 != 0 || ldx % 8 != 0 || ldy % 4 != 0) return false;
  if (epi != W4_EPI_NONE && epi != W4_EPI_SWIGLU && epi != W4_EPI_RESID) return false;
  if (epi == W4_EPI_RESID && (R == nullptr || ldr % 4 != 0 || (reinterpret_cast<uintptr_t>(R) & 7))) return false;
  if ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W)) & 15) return false;
  if (reinterpret_cast<uintptr_t>(Y) & 7) return false;
  if (static_cast<long>(M) * ldx * 2 > 0x7FFFFFFFL) return false;  // X rows addressed by 32-bit offsets
  if (static_cast<long>(N) * K * 2 > 0x7FFFFFFFL) return false;    // W rows by 32-bit soffsets
  const int ntm = (M + 255) / 256, ntn = N / 256, ntiles = ntm * ntn;
  W4Args a;
  a.Y = Y;
  a.X = X;
  a.W = W;
  a.R = R;
  a.ntm = ntm;
  a.ntn = ntn;
  a.M = M;
  a.K = K;
  a.ldx = ldx;
  a.ldy = ldy;
  a.ldr = ldr;
  a.nk = K / 32;
  a.ntiles = ntiles;
  a.inter = epi == W4_EPI_SWIGLU ? N / 2 : 0;
  a.nrows_w = N;
  (void)num_cu;  // one workgroup per tile; the LDS (128 KB) admits one per CU
  const dim3 g(ntiles), b(256);
  if (epi == W4_EPI_SWIGLU) hipLaunchKernelGGL(gemm_w4_kernel<W4_EPI_SWIGLU>, g, b, 0, s, a);
  else if (epi == W4_EPI_RESID) hipLaunchKernelGGL(gemm_w4_kernel<W4_EPI_RESID>, g, b, 0, s, a);
  else hipLaunchKernelGGL(gemm_w4_kernel<W4_EPI_NONE>, g, b, 0, s, a);
  MXS_CHECK_LAUNCH();
  return true;
}

}  // namespace mxs
