// K12: paged attention, decode (one query token per sequence), GQA-packed, split-KV.
//
// Regime: HBM-bound on the KV read (bench shape: 256 seqs x 4k context x 32 KiB/token = 35 GB per
// step against 2.5 GB of weights).  v1 of this kernel put one TOKEN per lane for QK^T, so every
// 16-byte load instruction touched 64 different 128-byte K rows; it streamed at 2.2 TB/s.  v2 (this
// file) reads every K and V block as contiguous 1 KiB wave-instructions:
//   * grid (Hkv, B, P): one workgroup per (kv head, sequence, partition); the G = Hq/Hkv query heads
//     of a kv head are processed together so each K/V byte is read once.  P is chosen on the host so
//     the grid has >= ~2048 workgroups (8 per CU) and partitions are as long as possible (P = 1 at
//     large batch: no merge kernel at all).
//   * K (token-major [16][D] per block): lane l loads 16-byte vectors v = l + 64 i, i.e. token
//     v / (D/8), dims 8 (l % (D/8)) .. +7.  Each lane keeps its 8 dims of q (all G heads) in
//     registers, so QK^T is FMAs + an in-register DPP reduction over the D/8 lanes of a token
//     (quad_perm xor1/xor2, row_half_mirror, row_mirror): no LDS, no ds_bpermute.
//   * softmax: per-token max over heads via DPP row_ror + permlane16/32 swaps (VALU only); lane
//     (token, j) exponentiates head j, so exps are not duplicated; p goes to LDS once.
//   * V (dim-major [D][16] per block): lane l loads dim v / 2, tokens 8 (l % 2) .. +7 -> P*V is FMAs
//     with p read back from LDS as broadcast 16-byte reads; the two token halves of a dim are
//     merged once at the end.
//   * 2 blocks (32 tokens) per wave iteration with the next iteration's K/V loads issued before the
//     current iteration's math (software pipeline); block ids come from scalar loads.
//   * EB = 1: fp8 (e4m3fn) cache.  Same lane -> (token, dims) map with 8-byte loads (still whole
//     512-byte wave-instructions), converted to bf16 words in registers right before the math, so
//     the step reads half the bytes; k_scale folds into q, v_scale into the output.
#include <cstdlib>

#include "common.h"

namespace mxs {

constexpr int kBS = 16;  // tokens per KV block (SGLang --page-size 16, sglang/agg.yaml:38-39)
constexpr int kWaves = 4;
constexpr int kSweepBlocks = 8;  // host partition lengths are multiples of 8 blocks (128 tokens)
constexpr float kLog2e = 1.4426950408889634f;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// v_dot2c_f32_bf16: c + a.lo * b.lo + a.hi * b.hi (bf16 products are exact in fp32)
__device__ __forceinline__ float dot2(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b), c, false);
}
// round-to-nearest-even for finite values (softmax weights are in [0, 1])
__device__ __forceinline__ uint32_t f2bf_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

// DPP helpers (gfx9 encodings): quad_perm xor1 = 0xB1, xor2 = 0x4E, row_half_mirror = 0x141,
// row_mirror = 0x140, row_ror:8 = 0x128.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float perm16_max(float v) {
  // the swap returns {row 2k in both rows, row 2k+1 in both rows}: combine the pair
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  return fmaxf(__int_as_float(r[0]), __int_as_float(r[1]));
}
__device__ __forceinline__ float perm32_max(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return fmaxf(__int_as_float(r[0]), __int_as_float(r[1]));
}
__device__ __forceinline__ float perm16_sum(float v) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(r[0]) + __int_as_float(r[1]);
}
__device__ __forceinline__ float perm32_sum(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(r[0]) + __int_as_float(r[1]);
}

// sum over the LPT = D/8 lanes that hold one token (all of them receive the total)
template <int LPT>
__device__ __forceinline__ float token_sum(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  if constexpr (LPT == 16) v += dpp<0x140>(v);
  return v;
}

// max over all 64 lanes, in which each run of LPT lanes holds the same value
template <int LPT>
__device__ __forceinline__ float wave_max_tok(float v) {
  if constexpr (LPT == 8) v = fmaxf(v, dpp<0x128>(v));
  v = perm16_max(v);
  return perm32_max(v);
}

__device__ __forceinline__ int decode_part_len(int L, int P) {
  const int per = (L + P - 1) / P;
  return ((per + 127) / 128) * 128;
}

template <int EB>
struct KVVec;
template <>
struct KVVec<2> {  // 8 bf16
  using raw = u32x4;
  using reg = uint4;
  __device__ static uint4 bf16(const uint4& v) { return v; }
};
template <>
struct KVVec<1> {  // 8 fp8
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  using raw = u32x2;
  using reg = uint2;
  __device__ static uint4 bf16(const uint2& v) { return fp8x8_to_bf16x8(v); }
};

template <int D, int G, int EB>
__global__ void __launch_bounds__(256) paged_decode_kernel(
    bf16_t* __restrict__ out, float* __restrict__ tmp_out, float* __restrict__ tmp_ml,
    const bf16_t* __restrict__ q, const void* __restrict__ kv, long block_stride,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ seq_lens, int Hkv,
    float scale, int part_len, float v_scale) {
  using Vec = KVVec<EB>;
  using KR = typename Vec::reg;
  using KRaw = typename Vec::raw;
  // blocks per wave iteration: 2 at D = 64; 1 at D = 128, where a block is already 4 KiB per lane-set
  // and a second prefetched block would cost 64 more VGPRs
  constexpr int kBPI = D <= 64 ? 2 : 1;
  constexpr int LPT = D / 8;        // lanes per token in the K layout
  constexpr int TPI = 64 / LPT;     // tokens per K wave-instruction
  constexpr int KV = D / 32;        // 16-byte vectors per lane per block (K and V alike)
  constexpr int TOK = kBPI * kBS;   // tokens per wave iteration
  constexpr int KT = kBPI * KV;     // K tokens handled per lane per iteration
  static_assert(G <= LPT, "one lane per (token, head) for the exponentials");

  const int kvh = blockIdx.x, seq = blockIdx.y, part = blockIdx.z;
  const int P = gridDim.z;
  const int L = seq_lens[seq];
  // part_len 0: split THIS sequence evenly over the P partitions (multiples of 128 tokens).  The
  // grid of a captured decode graph is sized for max_model_len, so a fixed length would leave the
  // high partitions empty and the low ones doing all the work.
  if (part_len <= 0) part_len = decode_part_len(L, P);
  const int start = part * part_len;
  if (start >= L) return;
  const int end = min(start + part_len, L);
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int Hq = Hkv * G;
  const int j = lane % LPT;  // dim chunk of this lane in K; head it exponentiates

  __shared__ __attribute__((aligned(16))) bf16_t p_s[kWaves][G][TOK];
  __shared__ float red_m[kWaves][G], red_l[kWaves][G];
  __shared__ __attribute__((aligned(16))) float red_o[kWaves][G][D];

  // q for this lane's 8 dims, all G heads, pre-scaled for exp2, as bf16 pairs for v_dot2
  uint32_t qr[G][4];
  {
    const float qs = scale * kLog2e;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint4 v = *reinterpret_cast<const uint4*>(q + (static_cast<size_t>(seq) * Hq + kvh * G + g) * D + 8 * j);
      const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
      for (int k = 0; k < 4; ++k) qr[g][k] = f2bf_rne(bf2f_lo(w[k]) * qs) | (f2bf_rne(bf2f_hi(w[k]) * qs) << 16);
    }
  }
  const int* btp = block_tables + static_cast<size_t>(seq) * bt_stride;
  const char* kbase = reinterpret_cast<const char*>(kv) + static_cast<size_t>(kvh) * kBS * D * EB;
  const char* vbase = reinterpret_cast<const char*>(kv) + static_cast<size_t>(Hkv + kvh) * kBS * D * EB;
  const long bstride_bytes = block_stride * EB;

  const int blk0 = start / kBS;
  const int nblk = (end - 1) / kBS - blk0 + 1;          // blocks touched by this partition
  const int niter = (nblk + kWaves * kBPI - 1) / (kWaves * kBPI);

  float m[G], acc[G][KV];
  float lsum = 0.f;  // partial row sum of head j (lanes with j < G)
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY;
#pragma unroll
    for (int i = 0; i < KV; ++i) acc[g][i] = 0.f;
  }

  KR kr[kBPI][KV], vr[kBPI][KV];
  auto load = [&](int it, KR (&kd)[kBPI][KV], KR (&vd)[kBPI][KV]) {
#pragma unroll
    for (int b = 0; b < kBPI; ++b) {
      const int bi = (it * kWaves + wid) * kBPI + b;
      if (bi < nblk) {
        const long off = static_cast<long>(btp[blk0 + bi]) * bstride_bytes;
        const KRaw* kp = reinterpret_cast<const KRaw*>(kbase + off);
        const KRaw* vp = reinterpret_cast<const KRaw*>(vbase + off);
        // KV bytes are read once per step: non-temporal loads keep them from evicting the
        // weights / block tables from L2 (MI355X_MICROARCH nt-weights: 5-10 % per decode layer)
#pragma unroll
        for (int i = 0; i < KV; ++i) {
          kd[b][i] = __builtin_bit_cast(KR, __builtin_nontemporal_load(kp + lane + 64 * i));
          vd[b][i] = __builtin_bit_cast(KR, __builtin_nontemporal_load(vp + lane + 64 * i));
        }
      }
    }
  };
  if (niter > 0) load(0, kr, vr);

  for (int it = 0; it < niter; ++it) {
    KR kn[kBPI][KV], vn[kBPI][KV];
    if (it + 1 < niter) load(it + 1, kn, vn);  // next iteration's loads in flight under this math
    const int tok0 = (blk0 + (it * kWaves + wid) * kBPI) * kBS;  // first token of this iteration
    if (tok0 < end) {
      // ---- scores: lane holds KT tokens (b, i) -> token tok0 + 16 b + (lane + 64 i) / LPT
      float s[KT][G];
#pragma unroll
      for (int b = 0; b < kBPI; ++b)
#pragma unroll
        for (int i = 0; i < KV; ++i) {
          const uint4 kw = Vec::bf16(kr[b][i]);
          const uint32_t* w = reinterpret_cast<const uint32_t*>(&kw);
#pragma unroll
          for (int g = 0; g < G; ++g) {
            float a = 0.f;
#pragma unroll
            for (int k = 0; k < 4; ++k) a = dot2(w[k], qr[g][k], a);
            s[b * KV + i][g] = token_sum<LPT>(a);
          }
        }
      // mask tokens past the end of the partition
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const int tok = tok0 + (t / KV) * kBS + (lane + 64 * (t % KV)) / LPT;
        if (tok >= end) {
#pragma unroll
          for (int g = 0; g < G; ++g) s[t][g] = -INFINITY;
        }
      }
      // ---- online softmax
      float alpha[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float mx = s[0][g];
#pragma unroll
        for (int t = 1; t < KT; ++t) mx = fmaxf(mx, s[t][g]);
        mx = wave_max_tok<LPT>(mx);
        const float mn = fmaxf(m[g], mx);
        alpha[g] = exp2f(m[g] - mn);
        m[g] = mn;
#pragma unroll
        for (int i = 0; i < KV; ++i) acc[g][i] *= alpha[g];
      }
      if (j < G) {
        float mj = m[0], aj = alpha[0];
#pragma unroll
        for (int g = 1; g < G; ++g)
          if (j == g) {
            mj = m[g];
            aj = alpha[g];
          }
        float ps = 0.f;
#pragma unroll
        for (int t = 0; t < KT; ++t) {
          float sv = s[t][0];
#pragma unroll
          for (int g = 1; g < G; ++g)
            if (j == g) sv = s[t][g];
          const uint32_t pb = f2bf_rne(exp2f(sv - mj));
          ps += __uint_as_float(pb << 16);  // the row sum sees exactly the weights P*V uses
          p_s[wid][j][(t / KV) * kBS + (lane + 64 * (t % KV)) / LPT] = static_cast<bf16_t>(pb);
        }
        // each token is held by one lane per head, so ps counts every token once
        lsum = lsum * aj + ps;
      }
      // ---- P * V  (lane: dims lane/2 + 32 i, tokens 8 (lane % 2) .. +7 of each block)
#pragma unroll
      for (int b = 0; b < kBPI; ++b) {
        const int tb = tok0 + b * kBS;
        if (tb < end) {
          uint4 pv[G];  // 8 bf16 weights: tokens 8 (lane % 2) .. +7 of block b, per head
#pragma unroll
          for (int g = 0; g < G; ++g) pv[g] = *reinterpret_cast<const uint4*>(&p_s[wid][g][b * kBS + 8 * (lane & 1)]);
          const bool full = tb + kBS <= end;
#pragma unroll
          for (int i = 0; i < KV; ++i) {
            const uint4 vb = Vec::bf16(vr[b][i]);
            uint32_t vw[4] = {vb.x, vb.y, vb.z, vb.w};
            if (!full) {  // never let unwritten cache bytes (possibly NaN) reach the sum
#pragma unroll
              for (int u = 0; u < 8; ++u)
                if (tb + 8 * (lane & 1) + u >= end) vw[u / 2] &= (u & 1) ? 0x0000FFFFu : 0xFFFF0000u;
            }
#pragma unroll
            for (int g = 0; g < G; ++g) {
              float a = acc[g][i];
              a = dot2(vw[0], pv[g].x, a);
              a = dot2(vw[1], pv[g].y, a);
              a = dot2(vw[2], pv[g].z, a);
              a = dot2(vw[3], pv[g].w, a);
              acc[g][i] = a;
            }
          }
        }
      }
    }
    if (it + 1 < niter) {
#pragma unroll
      for (int b = 0; b < kBPI; ++b)
#pragma unroll
        for (int i = 0; i < KV; ++i) {
          kr[b][i] = kn[b][i];
          vr[b][i] = vn[b][i];
        }
    }
  }

  // ---- per-wave totals: merge the two token halves of each dim, row sums per head
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int i = 0; i < KV; ++i) acc[g][i] += dpp<0xB1>(acc[g][i]);
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float lg = (j == g) ? lsum : 0.f;
    lg += dpp<0xB1>(lg);
    lg += dpp<0x4E>(lg);
    lg += dpp<0x141>(lg);
    lg += dpp<0x140>(lg);
    lg = perm16_sum(lg);
    lg = perm32_sum(lg);
    if (lane == 0) {
      red_m[wid][g] = m[g];
      red_l[wid][g] = lg;
    }
    if ((lane & 1) == 0) {
#pragma unroll
      for (int i = 0; i < KV; ++i) red_o[wid][g][lane / 2 + 32 * i] = acc[g][i];
    }
  }
  __syncthreads();
  for (int x = threadIdx.x; x < G * D; x += blockDim.x) {
    const int g = x / D, d = x % D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) M = fmaxf(M, red_m[w][g]);
    float Ls = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      const float f = red_m[w][g] == -INFINITY ? 0.f : exp2f(red_m[w][g] - M);
      Ls += red_l[w][g] * f;
      O += red_o[w][g][d] * f;
    }
    const int head = kvh * G + g;
    if (P == 1) {
      out[(static_cast<size_t>(seq) * Hq + head) * D + d] = f2bf(O / Ls * v_scale);
    } else {
      const size_t base = (static_cast<size_t>(seq) * Hq + head) * P + part;
      tmp_out[base * D + d] = O / Ls * v_scale;
      if (d == 0) {
        tmp_ml[base * 2] = M;
        tmp_ml[base * 2 + 1] = Ls;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// MFMA variant: the dot products run on the matrix cores (v_mfma_f32_16x16x32_bf16), which matters
// once VALU, not HBM, is the limit -- wide GQA groups (G = 8: Llama-3-70B at TP 8 keeps one kv
// head per rank, so every K/V byte feeds 8 query heads) and the fp8 cache (half the bytes, same
// math).  Per wave iteration: two KV blocks (32 tokens).
//   S = K . Q^T   A = K rows (token = lane & 15, dims 8 (lane >> 4) + 32 ks ...), B = Q^T with the
//                 G query heads on the columns (zero-padded to 16), kept in registers all along.
//                 C: lane holds tokens 4 (lane >> 4) + i of one block for head lane & 15.
//   online softmax per head (column): max over the lane's 8 scores, then over the 4 lanes of a
//                 column (lane ^ 16, lane ^ 32).
//   O^T += V^T . P^T   B = P^T straight from the S accumulators of the two blocks (k = 8 q + j:
//                 j < 4 -> block 0 token 4 q + j, j >= 4 -> block 1 token 4 q + j - 4), A = V^T
//                 from the dim-major cache: two 4-token pieces per lane, one per block.
// The G x D output of each wave merges through LDS exactly as in the VALU kernel above.
typedef __bf16 bf16x8d_t __attribute__((ext_vector_type(8)));
typedef float f32x4d_t __attribute__((ext_vector_type(4)));

// KV bytes are read once per step: non-temporal loads keep them from evicting the weights and block
// tables from L2 / MALL (as in the VALU kernel)
// The prefetch registers hold the raw cache bytes (fp8: half the VGPRs of bf16); they are widened
// to bf16 right before the MFMA that consumes them.
typedef unsigned int u32x2d_t __attribute__((ext_vector_type(2)));
template <int EB>
struct MfmaKV;
template <>
struct MfmaKV<2> {
  using K8 = uint4;  // 8 bf16 K dims
  using V4 = uint2;  // 4 bf16 V tokens
  __device__ static K8 ldk(const char* p) {
    return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p)));
  }
  __device__ static V4 ldv(const char* p) {
    return __builtin_bit_cast(uint2, __builtin_nontemporal_load(reinterpret_cast<const u32x2d_t*>(p)));
  }
  __device__ static uint4 k(const K8& v) { return v; }
  __device__ static uint2 v(const V4& v) { return v; }
};
template <>
struct MfmaKV<1> {
  using K8 = uint2;     // 8 fp8 K dims
  using V4 = uint32_t;  // 4 fp8 V tokens
  __device__ static K8 ldk(const char* p) {
    return __builtin_bit_cast(uint2, __builtin_nontemporal_load(reinterpret_cast<const u32x2d_t*>(p)));
  }
  __device__ static V4 ldv(const char* p) { return __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(p)); }
  __device__ static uint4 k(const K8& v) { return fp8x8_to_bf16x8(v); }
  __device__ static uint2 v(const V4& v) { return fp8x4_to_bf16x4(v); }
};

template <int D, int G, int EB>
__global__ void __launch_bounds__(256) paged_decode_mfma_kernel(
    bf16_t* __restrict__ out, float* __restrict__ tmp_out, float* __restrict__ tmp_ml,
    const bf16_t* __restrict__ q, const void* __restrict__ kv, long block_stride,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ seq_lens, int Hkv,
    float scale, int part_len, float v_scale, int q_stride, const int64_t* __restrict__ qpos_tab,
    const float* __restrict__ cos_sin) {
  constexpr int KS = D / 32;  // k-steps of S = K Q^T
  constexpr int DT = D / 16;  // 16-dim tiles of O^T
  static_assert(G <= 16, "query heads of a kv head must fit the 16 MFMA columns");
  const int kvh = blockIdx.x, seq = blockIdx.y, part = blockIdx.z;
  const int P = gridDim.z;
  const int L = seq_lens[seq];
  if (part_len <= 0) part_len = decode_part_len(L, P);
  const int start = part * part_len;
  if (start >= L) return;
  const int end = min(start + part_len, L);
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15, qd = lane >> 4;
  const int Hq = Hkv * G;

  __shared__ float red_m[kWaves][G], red_l[kWaves][G];
  __shared__ __attribute__((aligned(16))) float red_o[kWaves][G][D];

  // Q^T (B operand): lane holds dims 32 ks + 8 qd .. +7 of head c, pre-scaled for exp2.  q rows are
  // q_stride elements apart (the fused qkv output when the caller skipped the rope kernel's q write);
  // cos_sin != nullptr rotates them here: chunks ks and ks + KS / 2 are dims d and d + D / 2
  bf16x8d_t qf[KS];
  {
    const float qs = scale * kLog2e;
    float x[KS][8];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (c < G) {
        const uint4 v = *reinterpret_cast<const uint4*>(q + static_cast<size_t>(seq) * q_stride + (kvh * G + c) * D +
                                                        32 * ks + 8 * qd);
        const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          x[ks][2 * k] = bf2f_lo(w[k]);
          x[ks][2 * k + 1] = bf2f_hi(w[k]);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) x[ks][k] = 0.f;
      }
    }
    if (cos_sin != nullptr && c < G) {
      const float* cs = cos_sin + qpos_tab[seq] * D;
#pragma unroll
      for (int ks = 0; ks < KS / 2; ++ks) {
        const int d0 = 32 * ks + 8 * qd;
        float cv[8], sv[8];
        *reinterpret_cast<float4*>(cv) = *reinterpret_cast<const float4*>(cs + d0);
        *reinterpret_cast<float4*>(cv + 4) = *reinterpret_cast<const float4*>(cs + d0 + 4);
        *reinterpret_cast<float4*>(sv) = *reinterpret_cast<const float4*>(cs + D / 2 + d0);
        *reinterpret_cast<float4*>(sv + 4) = *reinterpret_cast<const float4*>(cs + D / 2 + d0 + 4);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x1 = x[ks][j], x2 = x[ks + KS / 2][j];
          x[ks][j] = bf2f(f2bf(x1 * cv[j] - x2 * sv[j]));
          x[ks + KS / 2][j] = bf2f(f2bf(x2 * cv[j] + x1 * sv[j]));
        }
      }
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int k = 0; k < 8; ++k) qf[ks][k] = static_cast<__bf16>(x[ks][k] * qs);
  }
  const int* btp = block_tables + static_cast<size_t>(seq) * bt_stride;
  const char* kbase = reinterpret_cast<const char*>(kv) + static_cast<size_t>(kvh) * kBS * D * EB;
  const char* vbase = reinterpret_cast<const char*>(kv) + static_cast<size_t>(Hkv + kvh) * kBS * D * EB;
  const long bsb = block_stride * EB;
  const int blk0 = start / kBS;
  const int nblk = (end - 1) / kBS - blk0 + 1;
  const int niter = (nblk + kWaves * 2 - 1) / (kWaves * 2);

  f32x4d_t o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = f32x4d_t{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;

  using KVT = MfmaKV<EB>;
  typename KVT::K8 ka[2][KS];
  typename KVT::V4 va[DT][2];
  auto load = [&](int it, typename KVT::K8 (&kd)[2][KS], typename KVT::V4 (&vd)[DT][2]) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int bi = (it * kWaves + wid) * 2 + b;
      // blocks past this partition (a wave's whole pair, or the second block of the last pair) read
      // the partition's last block instead: valid memory, and their tokens are masked or skipped
      const long off = static_cast<long>(btp[blk0 + min(bi, nblk - 1)]) * bsb;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) kd[b][ks] = KVT::ldk(kbase + off + (c * D + 32 * ks + 8 * qd) * EB);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) vd[dt][b] = KVT::ldv(vbase + off + ((16 * dt + c) * kBS + 4 * qd) * EB);
    }
  };
  // software pipeline (next pair's loads in flight under this pair's math) unless it costs a wave
  // of occupancy: D = 128 with an fp8 cache fits 3 waves/SIMD only without the second register set
  constexpr bool kPrefetch = !(D >= 128 && EB == 1);
  if (niter > 0) load(0, ka, va);

  for (int it = 0; it < niter; ++it) {
    typename KVT::K8 kn[2][KS];
    typename KVT::V4 vn[DT][2];
    if constexpr (kPrefetch) {
      if (it + 1 < niter) load(it + 1, kn, vn);
    } else {
      if (it > 0) load(it, ka, va);
    }
    const int tok0 = (blk0 + (it * kWaves + wid) * 2) * kBS;
    if (tok0 < end) {
      f32x4d_t s[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        s[b] = f32x4d_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          s[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8d_t, KVT::k(ka[b][ks])), qf[ks],
                                                          s[b], 0, 0, 0);
      }
      const bool tail = tok0 + 32 > end;
      if (tail) {
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (tok0 + 16 * b + 4 * qd + i >= end) s[b][i] = -INFINITY;
      }
      float mx = s[0][0];
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) mx = fmaxf(mx, s[b][i]);
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m, mx);
      const float alpha = exp2f(m - mn);  // 0 on the first tile
      m = mn;
      lsum *= alpha;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
      bf16x8d_t pf;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const __bf16 pb = static_cast<__bf16>(exp2f(s[j >> 2][j & 3] - m));
        pf[j] = pb;
        lsum += static_cast<float>(pb);  // the row sum sees exactly the weights P V uses
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        uint2 v0 = KVT::v(va[dt][0]), v1 = KVT::v(va[dt][1]);
        if (tail) {  // unwritten cache bytes past the end (possibly NaN) never reach the sum
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t keep = (i & 1) ? 0x0000FFFFu : 0xFFFF0000u;
            if (tok0 + 4 * qd + i >= end) (i < 2 ? v0.x : v0.y) &= keep;
            if (tok0 + 16 + 4 * qd + i >= end) (i < 2 ? v1.x : v1.y) &= keep;
          }
        }
        const uint4 a = make_uint4(v0.x, v0.y, v1.x, v1.y);
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8d_t, a), pf, o[dt], 0, 0, 0);
      }
    }
    if (kPrefetch && it + 1 < niter) {
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) ka[b][ks] = kn[b][ks];
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        va[dt][0] = vn[dt][0];
        va[dt][1] = vn[dt][1];
      }
    }
  }

  // ---- per-wave totals: the row sum of head c is spread over the 4 lanes of its column
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  if (c < G) {
    if (qd == 0) {
      red_m[wid][c] = m;
      red_l[wid][c] = lsum;
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) red_o[wid][c][16 * dt + 4 * qd + i] = o[dt][i];
  }
  __syncthreads();
  for (int x = threadIdx.x; x < G * D; x += blockDim.x) {
    const int g = x / D, d = x % D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) M = fmaxf(M, red_m[w][g]);
    float Ls = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      const float f = red_m[w][g] == -INFINITY ? 0.f : exp2f(red_m[w][g] - M);
      Ls += red_l[w][g] * f;
      O += red_o[w][g][d] * f;
    }
    const int head = kvh * G + g;
    if (P == 1) {
      out[(static_cast<size_t>(seq) * Hq + head) * D + d] = f2bf(O / Ls * v_scale);
    } else {
      const size_t base = (static_cast<size_t>(seq) * Hq + head) * P + part;
      tmp_out[base * D + d] = O / Ls * v_scale;
      if (d == 0) {
        tmp_ml[base * 2] = M;
        tmp_ml[base * 2 + 1] = Ls;
      }
    }
  }
}

// Merge partitions: one workgroup per (head, seq), one thread per dim.
template <int D>
__global__ void __launch_bounds__(D) paged_decode_reduce_kernel(bf16_t* __restrict__ out,
                                                                const float* __restrict__ tmp_out,
                                                                const float* __restrict__ tmp_ml,
                                                                const int* __restrict__ seq_lens, int Hq, int P,
                                                                int part_len) {
  const int head = blockIdx.x, seq = blockIdx.y, d = threadIdx.x;
  if (part_len <= 0) part_len = decode_part_len(seq_lens[seq], P);
  const int np = min(P, (seq_lens[seq] + part_len - 1) / part_len);
  const size_t base = (static_cast<size_t>(seq) * Hq + head) * P;
  float M = -INFINITY;
  for (int p = 0; p < np; ++p) M = fmaxf(M, tmp_ml[(base + p) * 2]);
  float Ls = 0.f, O = 0.f;
  for (int p = 0; p < np; ++p) {
    const float w = tmp_ml[(base + p) * 2 + 1] * exp2f(tmp_ml[(base + p) * 2] - M);
    Ls += w;
    O += w * tmp_out[(base + p) * D + d];
  }
  out[(static_cast<size_t>(seq) * Hq + head) * D + d] = f2bf(np > 0 ? O / Ls : 0.f);
}

// Partition plan: enough workgroups to fill 256 CUs ~8 deep, partitions as long as possible, a
// multiple of one full wave sweep (kWaves * kBPI blocks <= 8 blocks = 128 tokens).
void decode_plan(int B, int Hkv, int max_seq_len, int* P, int* part_len) {
  static const int target = [] {  // MXS_DECODE_TARGET_WGS: the workgroup floor (A/B probes)
    const char* e = std::getenv("MXS_DECODE_TARGET_WGS");
    const int v = e != nullptr ? std::atoi(e) : 0;
    return v > 0 ? v : 2048;
  }();
  const int sweep = kSweepBlocks * kBS;
  int p = (target + B * Hkv - 1) / (B * Hkv);
  const int max_p = (max_seq_len + 255) / 256;  // never below 256 tokens per partition
  if (p > max_p) p = max_p;
  if (p < 1) p = 1;
  int len = (max_seq_len + p - 1) / p;
  len = ((len + sweep - 1) / sweep) * sweep;
  *P = (max_seq_len + len - 1) / len;
  *part_len = len;
}

int decode_num_partitions(int max_seq_len) {
  int P, len;
  decode_plan(1, 1, max_seq_len, &P, &len);
  return P;
}

// impl: 0 = auto, 1 = VALU dot2 kernel, 2 = MFMA kernel.  Auto takes the MFMA kernel from G = 4 query
// heads per kv head up (profiles/r1_v12_decode_attn_probe.jsonl, 4k context: 1B bf16 B 256 0.363 ->
// 0.323 ms = 6.5 TB/s, 8B bf16 0.371 -> 0.324 ms, 1B fp8 0.275 -> 0.202 ms, 70B-TP8 shard (G 8)
// 0.136 -> 0.098 ms); at G <= 2 the MFMA columns are mostly padding and the VALU kernel is as fast
// or faster (Qwen3-0.6B bf16 0.631 vs 0.636 ms, fp8 0.358 vs 0.545 ms).
// q_stride / qpos / cos_sin: see paged_decode_mfma_kernel (the MFMA kernel only; a strided or
// un-rotated q forces it).  Returns false when asked for that with an unsupported shape.
bool launch_paged_decode(bf16_t* out, float* tmp_out, float* tmp_ml, const bf16_t* q, const void* kv, bool kv_fp8,
                         long block_stride, const int* block_tables, int bt_stride, const int* seq_lens, int B,
                         int Hq, int Hkv, int D, int P, int part_len, float scale, float k_scale, float v_scale,
                         int impl, hipStream_t s, int q_stride, const int64_t* qpos, const float* cos_sin) {
  if (B == 0) return true;
  const int G = Hq / Hkv;
  dim3 grid(Hkv, B, P), blk(256);
  if (kv_fp8) scale *= k_scale;
  else v_scale = 1.f;
  if (q_stride <= 0) q_stride = Hq * D;
  const bool fused_q = cos_sin != nullptr || q_stride != Hq * D;
  const bool mfma = fused_q || impl == 2 || (impl == 0 && G >= 4);
  if (mfma) {
#define MXS_DECM(DD, GG)                                                                                   \
    if (D == DD && G == GG) {                                                                              \
      if (kv_fp8)                                                                                          \
        hipLaunchKernelGGL((paged_decode_mfma_kernel<DD, GG, 1>), grid, blk, 0, s, out, tmp_out, tmp_ml, q,  \
                           kv, block_stride, block_tables, bt_stride, seq_lens, Hkv, scale, part_len,      \
                           v_scale, q_stride, qpos, cos_sin);                                              \
      else                                                                                                 \
        hipLaunchKernelGGL((paged_decode_mfma_kernel<DD, GG, 2>), grid, blk, 0, s, out, tmp_out, tmp_ml, q,  \
                           kv, block_stride, block_tables, bt_stride, seq_lens, Hkv, scale, part_len,      \
                           v_scale, q_stride, qpos, cos_sin);                                              \
      if (P > 1)                                                                                           \
        hipLaunchKernelGGL((paged_decode_reduce_kernel<DD>), dim3(Hq, B), dim3(DD), 0, s, out, tmp_out,   \
                           tmp_ml, seq_lens, Hq, P, part_len);                                             \
      MXS_CHECK_LAUNCH();                                                                                  \
      return true;                                                                                         \
    }
    MXS_DECM(64, 1) MXS_DECM(64, 2) MXS_DECM(64, 4) MXS_DECM(64, 8)
    MXS_DECM(128, 1) MXS_DECM(128, 2) MXS_DECM(128, 4) MXS_DECM(128, 8)
#undef MXS_DECM
    if (fused_q) return false;
  }
#define MXS_DEC(DD, GG)                                                                                    \
  if (D == DD && G == GG) {                                                                                \
    if (kv_fp8)                                                                                            \
      hipLaunchKernelGGL((paged_decode_kernel<DD, GG, 1>), grid, blk, 0, s, out, tmp_out, tmp_ml, q, kv,   \
                         block_stride, block_tables, bt_stride, seq_lens, Hkv, scale, part_len, v_scale); \
    else                                                                                                   \
      hipLaunchKernelGGL((paged_decode_kernel<DD, GG, 2>), grid, blk, 0, s, out, tmp_out, tmp_ml, q, kv,   \
                         block_stride, block_tables, bt_stride, seq_lens, Hkv, scale, part_len, v_scale); \
    if (P > 1)                                                                                             \
      hipLaunchKernelGGL((paged_decode_reduce_kernel<DD>), dim3(Hq, B), dim3(DD), 0, s, out, tmp_out,     \
                         tmp_ml, seq_lens, Hq, P, part_len);                                               \
    MXS_CHECK_LAUNCH();                                                                                    \
    return true;                                                                                           \
  }
  MXS_DEC(64, 1) MXS_DEC(64, 2) MXS_DEC(64, 4) MXS_DEC(64, 8)
  MXS_DEC(128, 1) MXS_DEC(128, 2) MXS_DEC(128, 4) MXS_DEC(128, 8)
#undef MXS_DEC
  return false;
}

}  // namespace mxs
