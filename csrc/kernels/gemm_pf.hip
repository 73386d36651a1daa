// K05-K08 at prefill chunks (M = 1k-16k tokens): Y[M, N] = X[M, K] . W[N, K]^T on MFMA, with the
// projection's elementwise tail fused into the epilogue.  Replaces hipBLASLt (+ the separate SiLU*mul
// pass) on the prefill path.
//
// Tile: 256 weight rows (n) x 256 tokens (m) x 64 (k) per 512-thread workgroup, one workgroup per CU.
//   * 8 waves as 2 (token halves) x 4 (64-row weight blocks); a wave owns acc[4 w-frags][8 token
//     frags] of v_mfma_f32_16x16x32_bf16 with A = W (output columns on the accumulator rows) and
//     B = X^T, so a lane holds Y[token][4 consecutive columns];
//   * ping-pong: waves 4-7 run one barrier behind waves 0-3 (waves w and w + 4 share a SIMD), so on
//     every SIMD one wave's 32-MFMA segment runs beside its partner's LDS-read / DMA-issue segment
//     (cdna_hip_programming.md §5 "256² 8-phase template", MI355X_MICROARCH.md "Two waves per
//     SIMD").  A k-tile is two phases (token half 0, token half 1) of 32 MFMAs; fragment reads per
//     phase: 8 W + 8 X / 8 X ds_read_b128;
//   * operands go HBM/L2 -> LDS by global_load_lds_dwordx4 (lane-linear 1 KB pieces, no VGPRs):
//     2 k-tile buffers of W half-tiles (128 rows, 16 KB) and X quarter-tiles (64 tokens, 8 KB); the
//     16-byte chunks of a 128-byte row are XOR-swizzled by (row >> 1) & 7 on the SOURCE address and
//     un-swizzled on the read, conflict-free for the ds_read_b128 lane groups (T2, rule 21);
//     k-tile s + 1's W and X(., 0) are issued at phase 1 of s - 1 (their regions were last read at
//     phase 0 of s - 1), its X(., 1) at phase 0 of s; the one vmcnt wait is at the end of phase 1's
//     load segment (counted: the pieces issued for s + 2 stay in flight);
//   * persistent stream-K (hybrid data-parallel + stream-K): the grid is at most one workgroup per
//     CU; full rounds of tiles run data-parallel, the last one-to-two rounds' k-iterations are split
//     evenly over the workgroups.  Every workgroup runs ONE continuous k-tile pipeline over its
//     positions (a new tile's first k-tiles are already in LDS when the previous tile's epilogue
//     runs).  A tile split over workgroups is finished by its HEAD (the owner of its first k-tiles,
//     whose segment ends that owner's range while the others open theirs): the other segments
//     publish fp32 slabs (write-through sc1 stores, then a count), the head adds them to the
//     accumulators it holds in segment order (deterministic: fp32 addition commutes) and runs the
//     epilogue (§5 "Projection GEMM at M = 256" item 2, sc1 form);
//   * tiles are visited XCD-aware: the 32 workgroups of an XCD take 32 consecutive tiles of a round
//     in the host-built tile map's order (8 token tiles per weight-column sweep), so they share W and
//     X panels in their L2.
//
// EPI_NONE: Y = acc.  EPI_SWIGLU: W = [gate; up] [2 I, K]; a tile's image interleaves 16 gate and the
// 16 matching up rows per fragment pair (the DMA addresses gather them), Y [M, I] = SiLU(g) * u.
// EPI_RESID: Y = R + acc (R may be Y: the residual stream updated in place by o_proj / down_proj).
//
// RS (row scale, the consumer half of a fused RMSNorm): X is the un-normalised residual stream and
// W's columns carry the norm weight (W' = W diag(g), folded at load), so RMSNorm(x) W^T = rstd(x) *
// (x W'^T) with rstd(x) = rsqrt(mean(x^2) + eps) over the K = hidden columns the tile streams
// anyway.  Every wave sums x^2 of its X fragments as they pass through its registers (v_dot2 of a
// bf16 pair with itself: 16 VALU per phase beside 32 MFMAs), the 4 k-quarter lanes of a row are
// combined in the epilogue and the accumulators scaled before the SwiGLU / store.  The separate
// normalisation pass over [M, hidden] (read + write) disappears; partial sums of stream-K segments
// travel in the slab with the accumulators.
#include <algorithm>
#include <type_traits>

#include "common.h"

namespace mxs {

typedef __bf16 pf_bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int pf_u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 pf_bf16x2 __attribute__((ext_vector_type(2)));

constexpr int PF_SC1 = 16;  // buffer cache-policy bits: sc1 (CPol::SC1 = SCC): write-through / L2-coherent
constexpr int PF_EPI_NONE = 0;
constexpr int PF_EPI_SWIGLU = 1;
constexpr int PF_EPI_RESID = 2;
constexpr int PF_SLAB_FRAGS = 34;  // 32 accumulator fragments + 2 float4 of RS row sums per thread

__device__ __forceinline__ pf_bf16x8 pf_frag(const pf_u32x4& v) { return __builtin_bit_cast(pf_bf16x8, v); }
__device__ __forceinline__ float pf_silu(float g) { return g / (1.f + __expf(-g)); }
// a dword as two bf16, by value: __builtin_bit_cast of a vector ELEMENT (q.y, q[d]) reads dword 0 of
// the vector (hipcc / ROCm 7.2: the element's "address" is the vector's), so copy it out first
__device__ __forceinline__ pf_bf16x2 pf_pair(unsigned v) { return __builtin_bit_cast(pf_bf16x2, v); }

struct PfArgs {
  bf16_t* Y;
  const bf16_t* X;
  const bf16_t* W;
  float* slab;  // stream-K partials: [grid][34 fragments][512 threads][4] fp32 (one per workgroup)
  int* cnt;     // per stream-K tile arrival counters (zero between launches)
  int* err;     // count of stream-K heads whose wait timed out (checked by the host; never reset here)
  const int* tile_map;  // logical tile -> token tile | weight tile << 16 (pf_tile_map)
  int M, K, ldx, ldy, inter, ntm, ntn, nk;
  int nrows_w;  // rows of W
  const bf16_t* R;  // EPI_RESID: residual rows (ldr), may equal Y
  int ldr;
  float inv_k, eps;  // RS: 1 / K, RMSNorm epsilon
  int dp_rounds;  // full data-parallel rounds of tiles
  int sk_tiles;   // tiles after them, split over the grid by k-iterations
};

// a segment of a workgroup's k-tile stream: k-tiles [k0, k1) of logical tile L (token tile tm,
// weight tile tn), starting at stream position c
struct PfSeg {
  int c, L, k0, k1, tm, tn;
};

template <int EPI, bool RS, int TMF>
__global__ void __launch_bounds__(512, 1) gemm_pf_kernel(const PfArgs a) {
  constexpr int HT = 16384, QT = 8192, KT = 4 * HT, XB = 2 * HT;  // W halves at 0 / HT, X halves at XB
  // token tile: TMF 16-row fragments per wave row-half, 32 TMF rows (256, 224, 192, 160, 128); a wave's
  // fragments split over the two phases of a k-tile as P0 + P1.  The X image keeps its four 64-row
  // quarters (h, t): quarter (wr, hb) holds the P_hb fragments wave row-half wr multiplies in phase
  // hb -- tile rows 16 TMF h + 16 P0 t + [0, 16 P_t) -- so a phase reads only its own quarters and the
  // phase-1 DMA of k-tile s + 2 into the (., 0) quarters never races a read (the 256-row layout's
  // invariant for any height).  Rows of a quarter past 16 P_t are not loaded (wave-uniform skip).
  constexpr int TROWS = 32 * TMF, P0 = (TMF + 1) / 2, P1 = TMF - P0;
  static_assert(TMF >= 4 && TMF <= 8, "token tile of 128..256 rows");
  __shared__ __attribute__((aligned(16))) char smem[2 * KT];

  const int G = gridDim.x, nk = a.nk;
  // order of this workgroup: blocks b and b + 8 share an XCD; give each XCD a contiguous range
  const int bid = blockIdx.x, xcd = bid & 7, q8 = G >> 3, r8 = G & 7;
  const int o = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int I = a.sk_tiles * nk;  // stream-K iterations (< 2 * grid * nk: fits 32 bits with o * I)
  const int sk_lo = o * I / G, sk_hi = (o + 1) * I / G;
  // data-parallel rounds of this workgroup (the last round may be partial: min_iters 0 = no stream-K)
  const int my_rounds = o < a.ntm * a.ntn ? min(a.dp_rounds, (a.ntm * a.ntn - 1 - o) / G + 1) : 0;
  const int dp_end = my_rounds * nk;
  const int ns = dp_end + sk_hi - sk_lo;  // positions of this workgroup's stream

  // the segment starting at stream position c (c < ns): a data-parallel round's whole tile, or a
  // stream-K piece; its tile coordinates come from the host-built map (one scalar load per segment)
  auto make_seg = [&](int c) -> PfSeg {
    PfSeg g;
    g.c = c;
    if (c < dp_end) {
      g.L = (c / nk) * G + o;
      g.k0 = 0;
      g.k1 = nk;
    } else {
      const int i = sk_lo + c - dp_end;
      g.L = a.dp_rounds * G + i / nk;
      g.k0 = i % nk;
      g.k1 = min(nk, g.k0 + sk_hi - i);
    }
    const int v = __builtin_amdgcn_readfirstlane(a.tile_map[g.L]);
    g.tm = v & 0xFFFF;
    g.tn = v >> 16;
    return g;
  };

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  // the wave index as a scalar: LDS-DMA destinations (M0) then need no VALU + readfirstlane per issue
  const int wid_s = __builtin_amdgcn_readfirstlane(wid);

  // DMA sources: buffer descriptors per tile (scalar), per-lane byte offsets (VGPR, fixed), the
  // k-tile in the scalar offset: no address arithmetic on the VALU in the loop.  X rows past M fall
  // outside the tile's descriptor and load as zeros (never stored).
  int wvo[2][2];  // W half h, instruction j
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 8 * (2 * wid + j) + (lane >> 3);
    const int ch = 8 * ((lane & 7) ^ ((row >> 1) & 7));
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = 128 * h + row;
      int wr_l;
      if constexpr (EPI == PF_EPI_SWIGLU) {
        const int fr = (r >> 4) & 3;
        wr_l = (fr < 2 ? 0 : a.inter) + 32 * (r >> 6) + 16 * (fr & 1) + (r & 15);
      } else {
        wr_l = r;
      }
      wvo[h][j] = (wr_l * a.K + ch) * 2;
    }
  }
  int xvo[2][2];  // X quarter (h, t)
  {
    const int rq = 8 * wid + (lane >> 3);
    const int ch = 8 * ((lane & 7) ^ ((rq >> 1) & 7));
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int t = 0; t < 2; ++t) xvo[h][t] = ((16 * TMF * h + 16 * P0 * t + rq) * a.ldx + ch) * 2;
  }
  constexpr int WSTEP = EPI == PF_EPI_SWIGLU ? 128 : 256;  // weight rows per tile step
  const long w_bytes = 2L * a.K * a.nrows_w;

  typedef __attribute__((address_space(3))) void lds_t;
  auto rsrc_w = [&](int tn) -> __amdgpu_buffer_rsrc_t {  // W rows of weight tile tn
    const long off = 2L * tn * WSTEP * a.K;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a.W) + off / 2, static_cast<short>(0),
                                             static_cast<int>(min(w_bytes - off, 0x7FFFFFFFL)), 0x00020000);
  };
  auto rsrc_x = [&](int tm) -> __amdgpu_buffer_rsrc_t {  // X rows of token tile tm (rows past M: out of range)
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a.X) + static_cast<size_t>(tm) * TROWS * a.ldx,
                                             static_cast<short>(0), (a.M - tm * TROWS) * a.ldx * 2, 0x00020000);
  };
  auto dma_w = [&](int pos, __amdgpu_buffer_rsrc_t rs, int k) {  // both W half-tiles of position pos
    char* dst = smem + (pos & 1) * KT;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_t*)(dst + h * HT + (2 * wid_s + j) * 1024), 16,
                                                 wvo[h][j], 128 * k, 0, 0);
  };
  auto dma_x = [&](int pos, __amdgpu_buffer_rsrc_t rs, int k, int t) {  // X quarters (0, t), (1, t) of pos
    char* dst = smem + (pos & 1) * KT + XB + t * QT;
    if (8 * wid_s < 16 * (t ? P1 : P0)) {  // this wave's 8 rows of the quarter are used
#pragma unroll
      for (int h = 0; h < 2; ++h)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_t*)(dst + h * HT + wid_s * 1024), 16, xvo[h][t], 128 * k,
                                                 0, 0);
    }
  };

  float4_ acc[4][TMF];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int t = 0; t < TMF; ++t) acc[f][t] = float4_{0.f, 0.f, 0.f, 0.f};
  float ssq[TMF];  // RS: sum of x^2 over this lane's k-quarter of token rows 16 TMF wr + 16 t + r16
#pragma unroll
  for (int t = 0; t < TMF; ++t) ssq[t] = 0.f;

  const int r16 = lane & 15, kq = lane >> 4;
  // fragment addresses: one VGPR base per (operand, k-step); fragments f / t of a wave sit 2048 bytes
  // apart (16 rows), folded into the ds_read immediate offsets
  const int swz = (r16 >> 1) & 7;
  const int sl0 = (kq ^ swz) << 4, sl1 = ((4 + kq) ^ swz) << 4;
  const int wbase = (wc >> 1) * HT + (64 * (wc & 1) + r16) * 128, xbase = XB + wr * HT + r16 * 128;
  const int wb0 = wbase + sl0, wb1 = wbase + sl1, xb0 = xbase + sl0, xb1 = xbase + sl1;

  pf_u32x4 wa[4][2], xb[4][2];  // [w frag][k-step], [token frag][k-step]
  auto rd_w = [&](const char* b) {
    const char* p0 = b + wb0;
    const char* p1 = b + wb1;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      wa[f][0] = *reinterpret_cast<const pf_u32x4*>(p0 + f * 2048);
      wa[f][1] = *reinterpret_cast<const pf_u32x4*>(p1 + f * 2048);
    }
  };
  auto rd_x = [&](const char* b, int hb) {  // phase hb's fragments, from quarter (wr, hb)
    const char* p0 = b + xb0 + hb * QT;
    const char* p1 = b + xb1 + hb * QT;
#pragma unroll
    for (int t = 0; t < P0; ++t) {
      if (hb && t >= P1) break;
      xb[t][0] = *reinterpret_cast<const pf_u32x4*>(p0 + t * 2048);
      xb[t][1] = *reinterpret_cast<const pf_u32x4*>(p1 + t * 2048);
    }
  };
  // RS: x^2 of this phase's X fragments, in the wave's LDS-read segment (after its reads landed, before
  // the barrier into its MFMA segment) while the partner wave on the SIMD runs its MFMAs
  auto rs_sum = [&](int hb) {
    if constexpr (RS) {
#pragma unroll
      for (int t = 0; t < P0; ++t) {
        if (hb && t >= P1) break;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            const pf_bf16x2 v = pf_pair(xb[t][kk][d]);
            ssq[hb * P0 + t] = __builtin_amdgcn_fdot2_f32_bf16(v, v, ssq[hb * P0 + t], false);
          }
      }
    }
  };
  auto mma = [&](int hb) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int t = 0; t < P0; ++t) {
          if (hb && t >= P1) break;
          acc[f][hb * P0 + t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf_frag(wa[f][kk]), pf_frag(xb[t][kk]),
                                                                         acc[f][hb * P0 + t], 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
  };

  // epilogue of a finished tile from acc: lane (r16, kq), acc[f][t] = Y[token m0 + 16 TMF wr + 16 t +
  // r16][image column 64 wc + 16 f + 4 kq + e]
  auto epilogue = [&](int tm, int tn) {
    const int m0 = tm * TROWS;
    if constexpr (RS) {  // the 4 k-quarter lanes of each row: full-row sums -> rstd, applied to acc
#pragma unroll
      for (int t = 0; t < TMF; ++t) {
        float v = ssq[t];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        const float r = rsqrtf(v * a.inv_k + a.eps);
#pragma unroll
        for (int f = 0; f < 4; ++f) acc[f][t] *= r;
      }
    }
#pragma unroll
    for (int t = 0; t < TMF; ++t) {
      const int m = m0 + 16 * TMF * wr + 16 * t + r16;
      if (m >= a.M) continue;
      bf16_t* yr = a.Y + static_cast<size_t>(m) * a.ldy;
      if constexpr (EPI == PF_EPI_RESID) {
        const bf16_t* rr = a.R + static_cast<size_t>(m) * a.ldr;
        uint2 rv[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) rv[f] = *reinterpret_cast<const uint2*>(rr + tn * 256 + 64 * wc + 16 * f + 4 * kq);
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const float4_& v = acc[f][t];
          const int n = tn * 256 + 64 * wc + 16 * f + 4 * kq;
          uint2 ov;
          ov.x = pack2(v[0] + bf2f_lo(rv[f].x), v[1] + bf2f_hi(rv[f].x));
          ov.y = pack2(v[2] + bf2f_lo(rv[f].y), v[3] + bf2f_hi(rv[f].y));
          *reinterpret_cast<uint2*>(yr + n) = ov;
        }
        continue;
      }
      if constexpr (EPI == PF_EPI_SWIGLU) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const float4_& g = acc[p][t];
          const float4_& v = acc[p + 2][t];
          const int n = tn * 128 + 32 * wc + 16 * p + 4 * kq;
          uint2 ov;
          ov.x = pack2(pf_silu(g[0]) * v[0], pf_silu(g[1]) * v[1]);
          ov.y = pack2(pf_silu(g[2]) * v[2], pf_silu(g[3]) * v[3]);
          *reinterpret_cast<uint2*>(yr + n) = ov;
        }
      } else {
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const float4_& v = acc[f][t];
          const int n = tn * 256 + 64 * wc + 16 * f + 4 * kq;
          uint2 ov;
          ov.x = pack2(v[0], v[1]);
          ov.y = pack2(v[2], v[3]);
          *reinterpret_cast<uint2*>(yr + n) = ov;
        }
      }
    }
  };
  auto zero_acc = [&]() {
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int t = 0; t < TMF; ++t) acc[f][t] = float4_{0.f, 0.f, 0.f, 0.f};
    if constexpr (RS) {
#pragma unroll
      for (int t = 0; t < TMF; ++t) ssq[t] = 0.f;
    }
  };
  // stream-K bookkeeping: owner of SK iteration i (order q owns [q I / G, (q + 1) I / G))
  auto sk_owner = [&](int i) -> int { return ((i + 1) * G + I - 1) / I - 1; };
  constexpr int SLAB = PF_SLAB_FRAGS * 512 * 4;  // floats per segment slab

#define PF_BAR()                           \
  do {                                     \
    __builtin_amdgcn_sched_barrier(0);     \
    __builtin_amdgcn_s_barrier();          \
    __builtin_amdgcn_sched_barrier(0);     \
  } while (0)
#define PF_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

  if (ns <= 0) return;  // every wave of the workgroup leaves together: no barrier is pending

  PfSeg seg = make_seg(0);
  PfSeg nseg = seg.k1 - seg.k0 < ns ? make_seg(seg.k1 - seg.k0) : seg;  // valid iff nseg.c > seg.c
  // k-tile of the position d ahead of k when it lies past the current segment: (tm, tn, k)
  auto ahead = [&](int k, int d, int& tm, int& tn, int& kk) {
    const int e = k + d - seg.k1, nl = nseg.k1 - nseg.k0;
    if (e < nl) {
      tm = nseg.tm;
      tn = nseg.tn;
      kk = nseg.k0 + e;
      return;
    }
    const PfSeg n2 = make_seg(nseg.c + nl);  // rare: a one-k-tile segment in between
    tm = n2.tm;
    tn = n2.tn;
    kk = n2.k0 + e - nl;
  };
  __amdgpu_buffer_rsrc_t rw = rsrc_w(seg.tn), rx = rsrc_x(seg.tm);  // the current segment's operands
  const bool x0_loads = 8 * wid_s < 16 * P0;  // wave-uniform: this wave issues dma_x(., t = 0) pieces

  dma_w(0, rw, seg.k0);
  dma_x(0, rx, seg.k0, 0);
  dma_x(0, rx, seg.k0, 1);
  if (ns > 1) {
    if (seg.k0 + 1 < seg.k1) {
      dma_w(1, rw, seg.k0 + 1);
      dma_x(1, rx, seg.k0 + 1, 0);
    } else {
      int tm1, tn1, k1;
      ahead(seg.k0, 1, tm1, tn1, k1);
      dma_w(1, rsrc_w(tn1), k1);
      dma_x(1, rsrc_x(tm1), k1, 0);
    }
    if (x0_loads) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // position 1's 4 W + 2 X pieces
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  PF_BAR();
  if (wr == 1) PF_BAR();  // the stagger

  // one stream position: the k-tile in buffer s & 1 (two phases), and the DMA of positions s + 1 and
  // s + 2.  FAST: both lie in the current segment (the common case: no segment arithmetic)
  auto position = [&](auto fast, int s, int k) {
    constexpr bool FAST = decltype(fast)::value;
    const char* b = smem + (s & 1) * KT;
    // phase 0: token half 0; X(., 1) of position s + 1 (its region was last read at phase 1 of s - 1)
    if (FAST) {
      dma_x(s + 1, rx, k + 1, 1);
    } else if (s + 1 < ns) {
      if (k + 1 < seg.k1) {
        dma_x(s + 1, rx, k + 1, 1);
      } else {
        int tm1, tn1, k1;
        ahead(k, 1, tm1, tn1, k1);
        dma_x(s + 1, rsrc_x(tm1), k1, 1);
      }
    }
    rd_w(b);
    rd_x(b, 0);
    PF_LGKM0();
    rs_sum(0);
    PF_BAR();
    mma(0);
    PF_BAR();
    // phase 1: token half 1; W and X(., 0) of position s + 2 into buffer s & 1 (last read at phase 0,
    // retired by the lgkmcnt + barrier above); position s + 1 complete
    rd_x(b, 1);
    if (FAST || s + 2 < ns) {
      if (FAST || k + 2 < seg.k1) {
        dma_w(s, rw, k + 2);
        dma_x(s, rx, k + 2, 0);
      } else {
        int tm2, tn2, k2;
        ahead(k, 2, tm2, tn2, k2);
        dma_w(s, rsrc_w(tn2), k2);
        dma_x(s, rsrc_x(tm2), k2, 0);
      }
      // the pieces just issued for s + 2 (4 W, and 2 X if this wave loads (., 0) rows) stay in flight:
      // waiting here, after this segment's issue work, gives the youngest piece of s + 1 (issued at
      // phase 0) the whole segment to land
      if (x0_loads) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    PF_LGKM0();
    rs_sum(1);
    PF_BAR();
    mma(1);
    PF_BAR();
  };

  int s = 0;  // stream position (k-tile buffer parity)
  for (;;) {
    int k = seg.k0;
    for (; k + 2 < seg.k1; ++k, ++s) position(std::integral_constant<bool, true>(), s, k);
    for (; k < seg.k1; ++k, ++s) position(std::integral_constant<bool, false>(), s, k);

    // end of a segment
    bool write = seg.k0 == 0 && seg.k1 == nk;  // the whole tile
#ifdef PF_PROBE_NO_FIXUP  // scripts/probes/gemm_pf_sk_probe.hip: the schedule without the hand-off (wrong sums)
    write = seg.k0 == 0;
    if (false) {
#else
    if (!write) {  // a stream-K segment of tile l
#endif
      if (wr == 0) PF_BAR();  // un-stagger: both halves meet here
      const int l = seg.L - a.dp_rounds * G;  // stream-K tile
      const int t0 = l * nk;
      const int o_lo = sk_owner(t0), o_hi = sk_owner(t0 + nk - 1);
      if (seg.k0 != 0) {
        // not the tile's head: publish the partial in this workgroup's slab (a workgroup has at most
        // one such segment: the first of its range) and count it in.  Hand-off without agent-scope
        // fences (MI355X_MICROARCH.md "Valid forms", first table row): write-through (sc1) 16-byte
        // slab stores, every storing wave drained before the barrier, one lane's agent-scope count.
        const __amdgpu_buffer_rsrc_t ms = __builtin_amdgcn_make_buffer_rsrc(
            a.slab + static_cast<size_t>(o) * SLAB, static_cast<short>(0), SLAB * 4, 0x00020000);
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
          for (int t = 0; t < TMF; ++t)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(pf_u32x4, acc[f][t]), ms, tid * 16,
                                                   (f * 8 + t) * 8192, PF_SC1);
        if constexpr (RS) {
#pragma unroll
          for (int h = 0; h < 2; ++h)
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(pf_u32x4, float4_{ssq[(4 * h) % TMF], ssq[(4 * h + 1) % TMF],
                                                     ssq[(4 * h + 2) % TMF], ssq[(4 * h + 3) % TMF]}),
                ms, tid * 16, (32 + h) * 8192, PF_SC1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PF_BAR();  // every wave's slab stores are complete
        if (tid == 0) __hip_atomic_fetch_add(a.cnt + l, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        // the tile's head (k-tiles from 0): its segment is the LAST of its range, while the tile's other
        // segments open their owners' ranges, so they are published by the time it gets here.  It waits
        // for their count, then adds their slabs to the accumulators it holds, in segment order:
        // ((s0 + s1) + s2) ... with s0 in registers -- fp32 addition commutes, so the bits do not depend
        // on which workgroup finishes when.  No own slab round trip, no arrival ticket.
        if (tid == 0) {
          // Deadlock-free only while every owner is resident: true for one grid (G <= CUs, one
          // workgroup per CU) but not guaranteed when another process's grid holds CUs.  The wait is
          // bounded by the 100 MHz wall clock (0.5 s); a timeout is counted in *err (the host reads it,
          // ops.gemm_pf_faults) instead of passing silently.  The counter is re-armed by subtracting
          // `want`, so segments arriving after a timeout bring it back to zero for the next launch.
          const int want = o_hi - o_lo;
          const long long t_end = wall_clock64() + 50000000LL;
          while (__hip_atomic_load(a.cnt + l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
            if (wall_clock64() > t_end) {
              __hip_atomic_fetch_add(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              break;
            }
            __builtin_amdgcn_s_sleep(2);
          }
          __hip_atomic_fetch_add(a.cnt + l, -want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        PF_BAR();
        for (int q = o_lo + 1; q <= o_hi; ++q) {
          const __amdgpu_buffer_rsrc_t ss = __builtin_amdgcn_make_buffer_rsrc(
              a.slab + static_cast<size_t>(q) * SLAB, static_cast<short>(0), SLAB * 4, 0x00020000);
#pragma unroll
          for (int f = 0; f < 4; f += 2) {  // 16 loads in flight (the k-loop's fragment registers are free)
            pf_u32x4 v[2][TMF];
#pragma unroll
            for (int ff = 0; ff < 2; ++ff)
#pragma unroll
              for (int t = 0; t < TMF; ++t)
                v[ff][t] = __builtin_amdgcn_raw_buffer_load_b128(ss, tid * 16, ((f + ff) * 8 + t) * 8192, PF_SC1);
#pragma unroll
            for (int ff = 0; ff < 2; ++ff)
#pragma unroll
              for (int t = 0; t < TMF; ++t) acc[f + ff][t] += __builtin_bit_cast(float4_, v[ff][t]);
            __builtin_amdgcn_sched_barrier(0);
          }
          if constexpr (RS) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const float4_ v = __builtin_bit_cast(
                  float4_, __builtin_amdgcn_raw_buffer_load_b128(ss, tid * 16, (32 + h) * 8192, PF_SC1));
#pragma unroll
              for (int e = 0; e < 4; ++e)
                if (4 * h + e < TMF) ssq[4 * h + e] += v[e];
            }
          }
        }
        write = true;
      }
      if (wr == 1) PF_BAR();  // re-stagger
    }
    if (write) epilogue(seg.tm, seg.tn);
    zero_acc();
    if (nseg.c <= seg.c) break;  // the stream ends
    seg = nseg;
    rw = rsrc_w(seg.tn);
    rx = rsrc_x(seg.tm);
    const int nc = seg.c + seg.k1 - seg.k0;
    if (nc < ns) nseg = make_seg(nc);
    else nseg.c = -1;  // no further segment
  }
  if (wr == 0) PF_BAR();  // balance the stagger barrier
#undef PF_BAR
#undef PF_LGKM0
}

// Launch geometry: grid = min(CUs, work / min_iters) workgroups; full rounds of tiles data-parallel,
// the rest stream-K.  trows: token-tile height (256, 224, 192, 160 or 128 rows).  Returns the grid (0 = not
// launched: shape unsupported).
int pf_plan(int M, int N, int K, int epi, int num_cu, int min_iters, int* dp_rounds, int* sk_tiles, int* grid,
            int trows) {
  if (M <= 0 || K % 64 != 0 || N % 256 != 0) return 0;
  if (trows != 256 && trows != 224 && trows != 192 && trows != 160 && trows != 128) return 0;
  const int ntm = (M + trows - 1) / trows, ntn = N / 256;
  const int T = ntm * ntn, nk = K / 64;
  const long work = static_cast<long>(T) * nk;
  if (min_iters <= 0) {  // data-parallel only: one workgroup per tile, the last round may be partial
    *grid = std::min(num_cu, T);
    *dp_rounds = (T + *grid - 1) / *grid;
    *sk_tiles = 0;
    return *grid;
  }
  int G = static_cast<int>(std::min<long>(num_cu, std::max<long>(1, work / std::max(1, min_iters))));
  if (T % G == 0) {  // whole rounds: no stream-K
    *dp_rounds = T / G;
    *sk_tiles = 0;
  } else {
    const int R = T / G;
    *dp_rounds = R > 0 ? R - 1 : 0;
    *sk_tiles = T - *dp_rounds * G;
  }
  *grid = G;
  return G;
}

// epi 0: Y [M, N] = X W^T (N % 256 == 0).  epi 1 (SwiGLU): W = [gate; up] rows [2 I, K], Y [M, I]
// (I % 128 == 0).  epi 2: Y = R + X W^T.  row_scale (epi 0 / 1): rows scaled by rsqrt(mean(x^2) + eps).  K % 64 == 0, 16-byte aligned rows.  slab: >= 2 * grid * 32 * 512 * 4 floats; cnt:
// > sk_tiles ints, zero (left zero by every launch; the last word counts stream-K wait timeouts).  False when the shape is not supported.
bool launch_gemm_pf(bf16_t* Y, const bf16_t* X, const bf16_t* W, int M, int N, int K, int ldx, int ldy, int epi,
                    float* slab, long slab_floats, int* cnt, int cnt_len, const int* tile_map, int map_len,
                    int num_cu, int min_iters, hipStream_t s, const bf16_t* R, int ldr, bool row_scale,
                    float eps, int trows) {
  if (M <= 0 || K % 64 != 0 || ldx % 8 != 0 || ldy % 4 != 0) return false;
  if (epi != PF_EPI_NONE && epi != PF_EPI_SWIGLU && epi != PF_EPI_RESID) return false;
  if (epi == PF_EPI_RESID && (R == nullptr || ldr % 4 != 0 || (reinterpret_cast<uintptr_t>(R) & 7) || row_scale))
    return false;
  if ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W)) & 15) return false;
  if (reinterpret_cast<uintptr_t>(Y) & 7) return false;
  if (N % 256 != 0) return false;  // SwiGLU: N = 2 I with I % 128 == 0
  int dp, sk, G;
  if (!pf_plan(M, N, K, epi, num_cu, min_iters, &dp, &sk, &G, trows)) return false;
  if (row_scale && trows != 256) return false;  // the fused-RMSNorm forms exist at 256 rows
  if (sk > 0 && (slab == nullptr || cnt == nullptr || cnt_len <= sk || slab_floats < 2L * G * PF_SLAB_FRAGS * 512 * 4))
    return false;
  if (tile_map == nullptr || map_len < ((M + trows - 1) / trows) * (N / 256)) return false;
  if (static_cast<long>(M) * ldx * 2 > 0x7FFFFFFFL) return false;  // X rows addressed by 32-bit buffer offsets
  PfArgs a;
  a.Y = Y;
  a.X = X;
  a.W = W;
  a.slab = slab;
  a.cnt = cnt;
  a.err = cnt + cnt_len - 1;  // the counters' last word (never a tile counter: cnt_len > sk_tiles)
  a.tile_map = tile_map;
  a.nrows_w = N;
  a.M = M;
  a.K = K;
  a.ldx = ldx;
  a.ldy = ldy;
  a.inter = epi == PF_EPI_SWIGLU ? N / 2 : 0;
  a.ntm = (M + trows - 1) / trows;
  a.ntn = N / 256;
  a.nk = K / 64;
  a.dp_rounds = dp;
  a.sk_tiles = sk;
  a.R = R;
  a.ldr = ldr;
  a.inv_k = 1.f / static_cast<float>(K);
  a.eps = eps;
  const dim3 g(G), b(512);
#define MXS_PF(E, RSV, T) hipLaunchKernelGGL((gemm_pf_kernel<E, RSV, T>), g, b, 0, s, a)
#define MXS_PF_ROWS(E)              \
  switch (trows) {                  \
    case 224: MXS_PF(E, false, 7); break; \
    case 192: MXS_PF(E, false, 6); break; \
    case 160: MXS_PF(E, false, 5); break; \
    case 128: MXS_PF(E, false, 4); break; \
    default: MXS_PF(E, false, 8); break;  \
  }
  if (epi == PF_EPI_SWIGLU) {
    if (row_scale) MXS_PF(PF_EPI_SWIGLU, true, 8);
    else MXS_PF_ROWS(PF_EPI_SWIGLU);
  } else if (epi == PF_EPI_RESID) {
    MXS_PF_ROWS(PF_EPI_RESID);
  } else {
    if (row_scale) MXS_PF(PF_EPI_NONE, true, 8);
    else MXS_PF_ROWS(PF_EPI_NONE);
  }
#undef MXS_PF_ROWS
#undef MXS_PF
  MXS_CHECK_LAUNCH();
  return true;
}

}  // namespace mxs
