// K12: paged attention, decode (one query token per sequence), GQA-packed, split-KV.
//
// Regime: HBM-bound on the KV read (BASELINE config 2: 128 seqs x 2k context x 32 KiB/token =
// 8.6 GB per step vs 2.5 GB of weights), so the design goal is full-bandwidth streaming with the
// arithmetic hidden under it:
//   * grid (Hkv, B, P): one workgroup per (kv head, sequence, PART-token partition); the G = Hq/Hkv
//     query heads that share a kv head are processed together, so each K/V byte is read once.
//   * 4 waves per workgroup, each streaming 64-token chunks.  QK^T with the TOKEN on the lane: a
//     lane loads its token's K row as D/8 x 16-byte vectors (K cache is token-major), q comes from
//     LDS as broadcast 16-byte reads; P*V with the DIM on the lane: the V cache is dim-major
//     ([D][16] per block), so a lane's 16 tokens of one dim are 2 x 16-byte vectors and a wave reads
//     one block's V as one contiguous 2*D*16-byte sweep.
//   * V loads are issued before the QK^T math so both streams are in flight together; the block
//     table slice of the partition is staged in LDS once (no dependent global load per chunk).
//   * online softmax in base 2 (q pre-scaled by scale*log2 e), per-lane partial row sums, one
//     cross-wave combine through LDS; multi-partition results are merged by a second tiny kernel
//     with the usual max/sum (LSE) rescaling.
#include "common.h"

namespace mxs {

constexpr int kBS = 16;       // tokens per KV block (SGLang --page-size 16, sglang/agg.yaml:38-39)
constexpr int kPart = 512;    // tokens per split-KV partition
constexpr int kWaves = 4;
constexpr float kLog2e = 1.4426950408889634f;

template <int D, int G>
__global__ void __launch_bounds__(256) paged_decode_kernel(
    bf16_t* __restrict__ out, float* __restrict__ tmp_out, float* __restrict__ tmp_ml,
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ kv, long block_stride,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ seq_lens, int Hkv,
    float scale) {
  constexpr int DPL = D / 64;       // dims per lane in the P*V phase
  constexpr int KV16 = D / 8;       // 16-byte vectors per K row
  const int kvh = blockIdx.x, seq = blockIdx.y, part = blockIdx.z;
  const int P = gridDim.z;
  const int L = seq_lens[seq];
  const int start = part * kPart;
  if (start >= L) return;
  const int end = min(start + kPart, L);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int Hq = Hkv * G;

  __shared__ __attribute__((aligned(16))) float q_s[G][D];
  __shared__ __attribute__((aligned(16))) float p_s[kWaves][G][64];
  __shared__ int bt_s[kPart / kBS];
  __shared__ float red_m[kWaves][G], red_l[kWaves][G];
  __shared__ __attribute__((aligned(16))) float red_o[kWaves][G][D];

  const float qscale = scale * kLog2e;
  for (int i = threadIdx.x; i < G * D; i += blockDim.x) {
    const int g = i / D, d = i % D;
    q_s[g][d] = bf2f(q[(static_cast<size_t>(seq) * Hq + kvh * G + g) * D + d]) * qscale;
  }
  const int nblk = (end - start + kBS - 1) / kBS;
  for (int i = threadIdx.x; i < nblk; i += blockDim.x)
    bt_s[i] = block_tables[static_cast<size_t>(seq) * bt_stride + start / kBS + i];
  __syncthreads();

  const size_t k_head_off = static_cast<size_t>(kvh) * kBS * D;
  const size_t v_head_off = static_cast<size_t>(Hkv + kvh) * kBS * D;

  float m[G], lsum[G], acc[G][DPL];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY;
    lsum[g] = 0.f;
#pragma unroll
    for (int j = 0; j < DPL; ++j) acc[g][j] = 0.f;
  }

  for (int c0 = start + wid * 64; c0 < end; c0 += kWaves * 64) {
    // ---- issue K loads (token on lane)
    const int tok = c0 + lane;
    const bool tvalid = tok < end;
    uint4 kr[KV16];
    if (tvalid) {
      const int blk = bt_s[(tok - start) / kBS];
      const uint4* kp = reinterpret_cast<const uint4*>(kv + blk * block_stride + k_head_off +
                                                       static_cast<size_t>(tok % kBS) * D);
#pragma unroll
      for (int i = 0; i < KV16; ++i) kr[i] = kp[i];
    }
    // ---- issue V loads (dim on lane) for the chunk's up-to-4 blocks
    const int nb = min(4, (end - c0 + kBS - 1) / kBS);
    uint4 vr[4][DPL][2];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      if (b < nb) {
        const int blk = bt_s[(c0 - start) / kBS + b];
#pragma unroll
        for (int j = 0; j < DPL; ++j) {
          const uint4* vp = reinterpret_cast<const uint4*>(kv + blk * block_stride + v_head_off +
                                                           static_cast<size_t>(lane + 64 * j) * kBS);
          vr[b][j][0] = vp[0];
          vr[b][j][1] = vp[1];
        }
      }
    }
    // ---- scores
    float s[G];
#pragma unroll
    for (int g = 0; g < G; ++g) s[g] = 0.f;
    if (tvalid) {
#pragma unroll
      for (int i = 0; i < KV16; ++i) {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(&kr[i]);
        float kf[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          kf[2 * k] = bf2f_lo(w[k]);
          kf[2 * k + 1] = bf2f_hi(w[k]);
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const float4_ qa = *reinterpret_cast<const float4_*>(&q_s[g][i * 8]);
          const float4_ qb = *reinterpret_cast<const float4_*>(&q_s[g][i * 8 + 4]);
          s[g] += qa[0] * kf[0] + qa[1] * kf[1] + qa[2] * kf[2] + qa[3] * kf[3] + qb[0] * kf[4] +
                  qb[1] * kf[5] + qb[2] * kf[6] + qb[3] * kf[7];
        }
      }
    }
    // ---- online softmax (base 2)
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float sv = tvalid ? s[g] : -INFINITY;
      const float mx = wave_max(sv);
      const float mn = fmaxf(m[g], mx);
      const float alpha = exp2f(m[g] - mn);
      const float p = tvalid ? exp2f(sv - mn) : 0.f;
      m[g] = mn;
      lsum[g] = lsum[g] * alpha + p;
#pragma unroll
      for (int j = 0; j < DPL; ++j) acc[g][j] *= alpha;
      p_s[wid][g][lane] = p;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- P * V
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      if (b < nb) {
        const int tb = c0 + b * kBS;  // first token of this block
        const bool full = tb + kBS <= end;
#pragma unroll
        for (int t4 = 0; t4 < 4; ++t4) {
          float pv[G][4];
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const float4_ pp = *reinterpret_cast<const float4_*>(&p_s[wid][g][b * kBS + t4 * 4]);
            pv[g][0] = pp[0]; pv[g][1] = pp[1]; pv[g][2] = pp[2]; pv[g][3] = pp[3];
          }
#pragma unroll
          for (int j = 0; j < DPL; ++j) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(&vr[b][j][t4 >> 1]);
            float vf[4] = {bf2f_lo(w[(t4 & 1) * 2]), bf2f_hi(w[(t4 & 1) * 2]), bf2f_lo(w[(t4 & 1) * 2 + 1]),
                           bf2f_hi(w[(t4 & 1) * 2 + 1])};
            if (!full) {
#pragma unroll
              for (int u = 0; u < 4; ++u)
                if (tb + t4 * 4 + u >= end) vf[u] = 0.f;  // never multiply uninitialised cache bytes
            }
#pragma unroll
            for (int g = 0; g < G; ++g)
              acc[g][j] += pv[g][0] * vf[0] + pv[g][1] * vf[1] + pv[g][2] * vf[2] + pv[g][3] * vf[3];
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }

  // ---- combine the 4 waves
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float l = wave_sum(lsum[g]);
    if (lane == 0) {
      red_m[wid][g] = m[g];
      red_l[wid][g] = l;
    }
#pragma unroll
    for (int j = 0; j < DPL; ++j) red_o[wid][g][lane + 64 * j] = acc[g][j];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G * D; i += blockDim.x) {
    const int g = i / D, d = i % D;
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
      out[(static_cast<size_t>(seq) * Hq + head) * D + d] = f2bf(O / Ls);
    } else {
      const size_t base = (static_cast<size_t>(seq) * Hq + head) * P + part;
      tmp_out[base * D + d] = O / Ls;
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
                                                                const int* __restrict__ seq_lens, int Hq, int P) {
  const int head = blockIdx.x, seq = blockIdx.y, d = threadIdx.x;
  const int np = min(P, (seq_lens[seq] + kPart - 1) / kPart);
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

int decode_num_partitions(int max_seq_len) { return (max_seq_len + kPart - 1) / kPart; }

void launch_paged_decode(bf16_t* out, float* tmp_out, float* tmp_ml, const bf16_t* q, const bf16_t* kv,
                         long block_stride, const int* block_tables, int bt_stride, const int* seq_lens, int B,
                         int Hq, int Hkv, int D, int P, float scale, hipStream_t s) {
  if (B == 0) return;
  const int G = Hq / Hkv;
  dim3 grid(Hkv, B, P), blk(256);
#define MXS_DEC(DD, GG)                                                                                    \
  if (D == DD && G == GG) {                                                                                \
    hipLaunchKernelGGL((paged_decode_kernel<DD, GG>), grid, blk, 0, s, out, tmp_out, tmp_ml, q, kv,        \
                       block_stride, block_tables, bt_stride, seq_lens, Hkv, scale);                      \
    if (P > 1)                                                                                             \
      hipLaunchKernelGGL((paged_decode_reduce_kernel<DD>), dim3(Hq, B), dim3(DD), 0, s, out, tmp_out,     \
                         tmp_ml, seq_lens, Hq, P);                                                         \
    MXS_CHECK_LAUNCH();                                                                                    \
    return;                                                                                                \
  }
  MXS_DEC(64, 1) MXS_DEC(64, 2) MXS_DEC(64, 4) MXS_DEC(64, 8)
  MXS_DEC(128, 1) MXS_DEC(128, 2) MXS_DEC(128, 4) MXS_DEC(128, 8)
#undef MXS_DEC
}

}  // namespace mxs
