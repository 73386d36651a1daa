// K11: paged attention, prefill / chunked prefill (varlen, causal, prefix-cache aware), MFMA bf16.
//
// A chunk's own K/V are written into the paged cache first (rope_cache.hip), so this kernel reads
// every key - cached prefix and new tokens alike - from the cache: one code path for prefill,
// chunked prefill and prefix-cache hits.
//
// Work split: workgroup = (query tile, kv head, sequence), 4 waves x 32 rows; a row is a
// (query token, query head of this kv head's GQA group) pair, so the G heads sharing a kv head
// stream its K/V together.  Per 32-key tile, with v_mfma_f32_32x32x16_bf16:
//   S^T = K . Q^T    A = K rows straight from the token-major cache (16 B per lane),
//                    B = Q^T held in registers for the whole loop (pre-scaled by scale*log2 e).
//                    The accumulator has the QUERY ROW on the lane, so the online-softmax max/sum
//                    are per-lane plus one lane^32 exchange (cdna_hip_programming.md T12 idea).
//   O^T += V^T . P^T A = V^T from the dim-major V cache (two 8-byte loads per lane),
//                    B = P^T taken straight from the S^T accumulator registers (§3 "An accumulator
//                    tile as the next MFMA's operand"): no LDS round trip, no shuffles.
// Causal tiles past a workgroup's last query position are skipped; heavy tiles launch first.
#include "common.h"
#include <algorithm>
#include <cstdlib>

namespace mxs {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
constexpr int kPBS = 16;
constexpr float kPLog2e = 1.4426950408889634f;

__device__ __forceinline__ bf16x8_t as_bf16x8(const uint4& v) { return __builtin_bit_cast(bf16x8_t, v); }
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float vmax(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

template <int D, int G>
__global__ void __launch_bounds__(256) paged_prefill_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ q, const bf16_t* __restrict__ kv, long block_stride,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ qsl,
    const int* __restrict__ seq_lens, int Hkv, float scale) {
  constexpr int KS = D / 16;   // k-steps of the QK^T product
  constexpr int DT = D / 32;   // 32-row output tiles of O^T
  constexpr int BQ = 128 / G;  // query tokens per workgroup
  // XCD-aware order: the hardware deals workgroups round-robin over the 8 XCDs, which would spread
  // every (sequence, kv head)'s query tiles over all eight L2s and make each L2 stream the K/V of
  // every head.  Remap so consecutive virtual ids run on one XCD: all query tiles of a (seq, kv head)
  // share one L2, which then holds just that head's K/V.
  const int NT = gridDim.x, total = NT * gridDim.y * gridDim.z;
  const int lin = blockIdx.x + NT * (blockIdx.y + gridDim.y * blockIdx.z);
  const int v = (total % 8 == 0) ? (lin % 8) * (total / 8) + lin / 8 : lin;
  const int pair = v / NT;
  const int kvh = pair % gridDim.y, seq = pair / gridDim.y;
  const int q0 = qsl[seq];
  const int ql = qsl[seq + 1] - q0;
  const int tile = NT - 1 - (v - pair * NT);  // heaviest (latest) tiles first
  const int t0 = tile * BQ;
  if (t0 >= ql) return;
  const int L = seq_lens[seq];
  const int ctx0 = L - ql;
  const int Hq = Hkv * G;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5, c = lane & 31;

  const int r = wid * 32 + c;
  const int tok = t0 + r / G;
  const int head = kvh * G + r % G;
  const bool rvalid = tok < ql;
  const int qpos = ctx0 + (rvalid ? tok : 0);
  const int wg_last_pos = ctx0 + min(t0 + BQ, ql) - 1;
  const int q_stride = Hq * D;  // v2: dense q, no fused RoPE (launch_paged_prefill routes those to v3)
  const int64_t* qpos_tab = nullptr;
  const float* cos_sin = nullptr;
  const int nkeys = wg_last_pos + 1;

  // Q^T fragments (B operand): lane holds Q[row c][16 ks + 8 h + j], pre-scaled
  bf16x8_t qf[KS];
  {
    const int qrow = q0 + (rvalid ? tok : 0);
    const bf16_t* qp = q + static_cast<size_t>(qrow) * q_stride + head * D + 8 * h;
    const float qs = scale * kPLog2e;
    float x[KS][8];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const uint4 v = *reinterpret_cast<const uint4*>(qp + 16 * ks);
      const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        x[ks][2 * k] = bf2f_lo(w[k]);
        x[ks][2 * k + 1] = bf2f_hi(w[k]);
      }
    }
    if (cos_sin != nullptr) {
      const float* cs = cos_sin + qpos_tab[qrow] * D;
#pragma unroll
      for (int ks = 0; ks < KS / 2; ++ks) {
        const int d0 = 16 * ks + 8 * h;  // 8 consecutive dims: two 16-byte loads each of cos and sin
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
      for (int j = 0; j < 8; ++j) qf[ks][j] = static_cast<__bf16>(x[ks][j] * qs);
  }

  const int* bt = block_tables + static_cast<size_t>(seq) * bt_stride;
  const size_t k_head_off = static_cast<size_t>(kvh) * kPBS * D;
  const size_t v_head_off = static_cast<size_t>(Hkv + kvh) * kPBS * D;

  float16_ o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[dt][i] = 0.f;
  float m = -INFINITY, l = 0.f;
  // lowest query position held by this wave: key tiles entirely at or below it need no causal mask
  const int wave_tok0 = t0 + (wid * 32) / G;
  const int wave_min_pos = ctx0 + min(wave_tok0, ql - 1);

  // software pipeline: tile k0 + 32 is loaded while tile k0 is computed.  A 32-key tile spans two
  // cache blocks whose ids are wave-uniform scalar loads (SMEM, lgkmcnt), fetched one tile further
  // ahead still: a per-lane block-table gather would be a VMEM load the K/V addresses depend on, and
  // vmcnt's in-order accounting would then make every iteration wait for the loads just issued.
  uint4 kf[KS];
  uint2 vf[DT][2][2];
  auto tile_blocks = [&](int k0, int& b0, int& b1) {
    b0 = bt[min(k0, L - 1) / kPBS];
    b1 = bt[min(k0 + 16, L - 1) / kPBS];
  };
  auto load_tile = [&](int b0, int b1, uint4 (&kd)[KS], uint2 (&vd)[DT][2][2]) {
    // keys past L read (and later mask) valid bytes of the last block
    const int kblk = c < 16 ? b0 : b1;
    const bf16_t* kp = kv + kblk * block_stride + k_head_off + static_cast<size_t>(c & 15) * D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) kd[ks] = *reinterpret_cast<const uint4*>(kp + 16 * ks);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16_t* vp = kv + (s ? b1 : b0) * block_stride + v_head_off + 4 * h;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const bf16_t* vr = vp + static_cast<size_t>(32 * dt + c) * kPBS;
        vd[dt][s][0] = *reinterpret_cast<const uint2*>(vr);
        vd[dt][s][1] = *reinterpret_cast<const uint2*>(vr + 8);
      }
    }
  };
  int cb0, cb1, nb0, nb1;
  tile_blocks(0, cb0, cb1);
  tile_blocks(32, nb0, nb1);
  load_tile(cb0, cb1, kf, vf);

  // One 32-key tile: S^T = K Q^T, causal mask, online softmax, O^T += V^T P^T.
  auto compute = [&](int k0, uint4 (&kt)[KS], uint2 (&vt)[DT][2][2]) {
    float16_ sacc;
#pragma unroll
    for (int i = 0; i < 16; ++i) sacc[i] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(kt[ks]), qf[ks], sacc, 0, 0, 0);
    // causal mask only on tiles that cross the diagonal of some row of this wave
    if (k0 + 31 > wave_min_pos) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kk = k0 + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (kk > qpos) sacc[i] = -INFINITY;
      }
    }
    // online softmax (row = lane c, keys split across the two lane halves).  Lazy rescale: the
    // running max only moves (and O, l are rescaled) when a tile raises it by more than 2^8, so
    // most tiles skip the D/2 multiplies; both halves of a row see the same max, hence the same
    // decision, and p <= 2^8 stays well inside bf16 / fp32 range.
    float mx = sacc[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) mx = fmaxf(mx, sacc[i]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const bool bump = mx > m + 8.f;
    if (__ballot(bump)) {
      const float mn = bump ? mx : m;
      const float alpha = __builtin_amdgcn_exp2f(m - mn);  // 0 on the first tile (m = -inf)
      m = mn;
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
    }
    float ps = 0.f;
    bf16x8_t pf[2];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = __builtin_amdgcn_exp2f(sacc[i] - m);
      ps += p;
      pf[i >> 3][i & 7] = static_cast<__bf16>(p);
    }
    l += ps;
    // keys >= L in the last tile: zero V so uninitialised cache bytes never reach the sum
    if (k0 + 32 > L) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int kbase = k0 + 16 * s + 8 * half + 4 * h;
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            uint32_t* w = reinterpret_cast<uint32_t*>(&vt[dt][s][half]);
            if (kbase + 0 >= L) w[0] &= 0xFFFF0000u;
            if (kbase + 1 >= L) w[0] &= 0x0000FFFFu;
            if (kbase + 2 >= L) w[1] &= 0xFFFF0000u;
            if (kbase + 3 >= L) w[1] &= 0x0000FFFFu;
          }
        }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const uint4 a = make_uint4(vt[dt][s][0].x, vt[dt][s][0].y, vt[dt][s][1].x, vt[dt][s][1].y);
        o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(a), pf[s], o[dt], 0, 0, 0);
      }
  };

  if constexpr (D <= 64) {
    // two register sets in ping-pong: tile k0 computes from one while k0 + 32 lands in the other
    // (no register copies between iterations)
    uint4 kb[KS];
    uint2 vb[DT][2][2];
    for (int k0 = 0;;) {
      bool more = k0 + 32 < nkeys;
      if (more) {
        load_tile(nb0, nb1, kb, vb);
        tile_blocks(k0 + 64, nb0, nb1);
      }
      compute(k0, kf, vf);
      if (!more) break;
      k0 += 32;
      more = k0 + 32 < nkeys;
      if (more) {
        load_tile(nb0, nb1, kf, vf);
        tile_blocks(k0 + 64, nb0, nb1);
      }
      compute(k0, kb, vb);
      if (!more) break;
      k0 += 32;
    }
  } else {
    // D = 128: a second tile in flight would exceed the 256-VGPR budget; load in place
    for (int k0 = 0; k0 < nkeys; k0 += 32) {
      if (k0 > 0) load_tile(cb0, cb1, kf, vf);
      tile_blocks(k0 + 32, cb0, cb1);
      compute(k0, kf, vf);
    }
  }

  l += __shfl_xor(l, 32, 64);
  if (!rvalid) return;
  const float inv = 1.f / l;
  bf16_t* op = out + (static_cast<size_t>(q0 + tok) * Hq + head) * D;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d0 = 32 * dt + 8 * g4 + 4 * h;
      uint2 v;
      v.x = pack2(o[dt][4 * g4] * inv, o[dt][4 * g4 + 1] * inv);
      v.y = pack2(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv);
      *reinterpret_cast<uint2*>(op + d0) = v;
    }
}

// ---------------------------------------------------------------------------------------------
// v3: K/V tiles shared through LDS.  v2 gives every wave its own copy of each K/V tile straight
// from L2 (4x the load traffic of one workgroup); v3 is the structure of the guide's "Fused
// attention prefill": 8 waves x 32 rows = 256 query rows per workgroup, 64-key tiles double-
// buffered in LDS (global loads for tile i+1 issued before tile i is multiplied, written to the
// other buffer after it), XOR-swizzled 16-byte chunks so the fragment reads of 32 consecutive rows
// spread over the banks.  V is stored per dim with its keys permuted (bits 2 and 3 of the key index
// swapped inside each 16-key group) so the 8 keys a lane needs for the P^T operand taken straight
// from the S^T accumulator are one contiguous ds_read_b128.
// EB = 1: fp8 (e4m3fn) cache.  The staging loads fetch 8 bytes per 8 keys/dims and convert them to
// bf16 words before the LDS store, so LDS layout and MFMA loop are the bf16 ones; k_scale folds
// into q, v_scale into the final normalisation.
template <int EB>
__device__ __forceinline__ uint4 ld8_kv(const char* p) {
  if constexpr (EB == 2)
    return *reinterpret_cast<const uint4*>(p);
  else
    return fp8x8_to_bf16x8(*reinterpret_cast<const uint2*>(p));
}

// Q rows read straight from the fused qkv projection output (row stride q_stride elements) with the
// rotate-half RoPE applied here when cos_sin != nullptr (the rope kernel then writes only K / V: the
// [T, Hq, D] q tensor and its write + re-read disappear).  A lane's chunks ks and ks + KS / 2 hold
// dims d and d + D / 2, i.e. both halves of its rotation pairs.  q is rounded to bf16 after the
// rotation, as the standalone rope kernel stores it.
//
// VAR: softmax variant bits (VALU issue is what bounds a tile at D = 64: per 16 MFMAs of a 64-key
// tile one wave issues 32 v_exp (8 cycles each), 32 row-sum adds, a 32-element max chain, 16 cvt_pk
// and 16 accumulator moves, ~840 issue cycles against 512 matrix-pipe cycles):
//   1  biased reference, overflow check instead of a max: after a row's first tile the reference m
//      sits kBias = 64 above its running max, so every later p = exp2(s - m) <= 2^-64 unless s passes
//      the running max by 65.  That is caught after the exponentials by OR-ing the packed bf16 P words
//      and testing the top exponent bit of each half (p >= 2); the rare tile that trips it is redone
//      with a real max (one more QK^T from the same LDS tile) and a rescale.  f32 / bf16 keep the
//      2^-64-scaled values at full relative precision (normals reach 2^-126), and O / l cancel it.
//   2  row sum on the matrix pipe: lsum = ones^T . P^T (4 MFMAs per tile) instead of 32 VALU adds.
//   4  the QK^T chain starts from a persistent -m register block (C operand) instead of 16 moves.
//   8  256-thread workgroups (4 waves x 32 rows, 128 rows): three per CU at D = 64, so 168 registers
//      a wave instead of 128 (4 waves per SIMD) or 256 (2 per SIMD) -- room for bits 2 / 4 without
//      halving the waves that hide each other's softmax latency.
// Bits 2 / 4 need more than the 128 registers of 4 waves per SIMD: with 512 threads they run 2 per SIMD.
constexpr int kPf3DefaultVar = 0;
constexpr int pf3_threads(int VAR) { return (VAR & 8) ? 256 : 512; }
//  64  Q fragments re-read from LDS each tile (4 ds_read_b128) instead of held in 16 registers, so
//      bit 2 fits the 128 registers of 4 waves per SIMD (VAR 66).
// 128  split-KV for heavy q-tiles (causal load balance): a workgroup owns a q-tile for ALL its keys, so
//      below ~8k tokens per launch the tiles with the most keys set the launch time (1 x 4096: 512
//      workgroups of 1..64 key tiles, mean 32.5).  Every q-tile gets two grid slots; a tile with at
//      least split_min (8) key tiles runs its key range as two halves, each half writes its partial (O
//      normalised to bf16, m, l) with agent-scope atomic stores, takes a ticket on the tile's counter,
//      and the half that arrives second (odd ticket) reads the other half and writes the merged rows
//      (cdna_hip_programming.md §5 "Projection GEMM at M = 256" item 2, the last-arriver form).  Both
//      halves merge from the same rounded partials in a fixed order, so the output does not depend on
//      which half arrives last.  Counters are never reset: each launch adds exactly 2 per split tile, so
//      the ticket parity names the last arriver.  The default launch picks it when the unsplit grid is
//      under ~1.25 waves of resident workgroups (pf3_split_blocks): 1 x 1024 1.29x, 1 x 2048 1.19x,
//      1 x 4096 1.07x at D = 64 (profiles/r5/prefill_attn/split/).
// 1024 the row sum on a 16x16x32 MFMA fed the bf16 P^T fragments (4 MFMAs instead of 33 adds a
//      tile; a lane-group swap at the end): correct, but at D = 64 its 4-register accumulator spills
//      12 VGPRs of the 128 budget and it runs 4-11 % slower; at D = 128 equal (not adopted,
//      profiles/r5/prefill_attn/ms16_row_sum_not_adopted.jsonl).
// 256  paired q-tiles (causal load balance at two waves and up): workgroup s of a sequence's n tiles
//      runs tile n - 1 - s and then tile s, n + 1 key tiles each, half the workgroups; picked when the
//      paired grid fills the resident workgroups at least once: 8 x 1024 1.21x, 4 x 2048 1.11x,
//      2 x 4096 1.09x (883 TF/s), 1 x 8192 1.02x at D = 64 (profiles/r5/prefill_attn/pair/).
constexpr int pf3_wpe(int D, int VAR) {
  return (VAR & 8) ? (D == 64 ? 3 : 2) : (D == 64 ? (((VAR & 6) && !(VAR & 64)) ? 2 : 4) : 0);
}

// one q-tile (`tile` of (kv head, sequence) `pair`; `half` of its key range when split) of the v3
// kernel; NTL: q-tiles per pair (the split workspace's stride)
template <int D, int G, int EB, int VAR>
__device__ __forceinline__ void pf3_tile(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ q, const void* __restrict__ kv, long block_stride,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ qsl,
    const int* __restrict__ seq_lens, int Hkv, float scale, float v_scale, int q_stride,
    const int64_t* __restrict__ qpos_tab, const float* __restrict__ cos_sin, char* __restrict__ split_ws,
    int* __restrict__ split_cnt, int split_min, int tile, int half, int pair, int NTL) {
  constexpr int KS = D / 16, DT = D / 32;
  constexpr int NT = pf3_threads(VAR);
  constexpr bool SPLIT = VAR & 128;
  constexpr int BQ = NT / 2 / G;     // query tokens per workgroup (32 rows per wave)
  constexpr int KT = 64;             // keys per tile
  constexpr int KROW = D * 2;        // bytes of one K row in LDS
  constexpr int KCH = D / 8;         // 16-byte chunks per K row
  constexpr int KBYTES = KT * KROW;
  constexpr int VBYTES = D * KT * 2; // [D][64 keys]
  constexpr int NK = KT * KCH / NT;  // K chunks staged per thread per tile
  constexpr int NV = D * 8 / NT;     // V chunks (8 keys of one dim) staged per thread per tile
  // LDS chunk swizzles: a ds_read_b128 serves 16 lanes = 16 consecutive rows per pass.  128-byte rows
  // (K at D = 64, V always) put rows r and r + 2 on the same banks: XOR the 16-byte chunk with
  // (row >> 1) & 7 so the 16 rows hit 16 distinct slots (rows 2j, 2j + 1 share a swizzle but sit
  // 32 banks apart); 256-byte K rows (D = 128) put every row on the same banks: XOR with row & 15
  // over their 16 chunks.  (row & 7 was 2-way: SQ_LDS_BANK_CONFLICT ~2x the LDS-active cycles,
  // profiles/r3/s3/prefill_attn_counters.json.)
  auto kswz = [](int key) { return D == 64 ? ((key >> 1) & 7) : (key & 15); };
  auto vswz = [](int dim) { return (dim >> 1) & 7; };
  __shared__ __attribute__((aligned(16))) char lds[2][KBYTES + VBYTES];
  constexpr bool QLDS = VAR & 64;
  __shared__ __attribute__((aligned(16))) char qlds[QLDS ? (NT / 64) * KS * 1024 : 16];

  const int kvh = pair % gridDim.y, seq = pair / gridDim.y;
  const int q0 = qsl[seq];
  const int ql = qsl[seq + 1] - q0;
  const int t0 = tile * BQ;
  if (t0 >= ql) return;
  const int L = seq_lens[seq];
  const int ctx0 = L - ql;
  const int Hq = Hkv * G;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, c = lane & 31;

  const int r = wid * 32 + c;
  const int tok = t0 + r / G;
  const int head = kvh * G + r % G;
  const bool rvalid = tok < ql;
  const int qpos = ctx0 + (rvalid ? tok : 0);
  const int nkeys = ctx0 + min(t0 + BQ, ql);
  const int nkt = (nkeys + KT - 1) / KT;
  const int kmid = (nkt / 2) * KT;  // half 0: keys [0, kmid), half 1: [kmid, nkeys)
  // split only where every valid row of the tile has a key in the second half (its first tile then
  // sets m from real scores; padding rows past the sequence end see only masked keys there, and their
  // NaNs stay in their own P columns and are never stored)
  // split_min: low 16 bits, the key-tile floor; bit 16: also require half the sequence's heaviest tile
  const bool heavy = nkt >= (split_min & 0xffff) && (!(split_min >> 16) || 2 * nkt >= (L + KT - 1) / KT);
  const bool split = SPLIT && heavy && ctx0 + t0 >= kmid;
  if (SPLIT && !split && half == 1) return;  // the tile runs unsplit in its first slot
  const int kbeg = split && half == 1 ? kmid : 0, kend = split && half == 0 ? kmid : nkeys;
  const int wave_min_pos = ctx0 + min(t0 + (wid * 32) / G, ql - 1);
  const int wave_max_pos = ctx0 + min(t0 + (wid * 32 + 31) / G, ql - 1);

  bf16x8_t qf[KS];
  {
    const int qrow = q0 + (rvalid ? tok : 0);
    const bf16_t* qp = q + static_cast<size_t>(qrow) * q_stride + head * D + 8 * h;
    const float qs = scale * kPLog2e;
    float x[KS][8];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const uint4 v = *reinterpret_cast<const uint4*>(qp + 16 * ks);
      const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        x[ks][2 * k] = bf2f_lo(w[k]);
        x[ks][2 * k + 1] = bf2f_hi(w[k]);
      }
    }
    if (cos_sin != nullptr) {
      const float* cs = cos_sin + qpos_tab[qrow] * D;
#pragma unroll
      for (int ks = 0; ks < KS / 2; ++ks) {
        const int d0 = 16 * ks + 8 * h;  // 8 consecutive dims: two 16-byte loads each of cos and sin
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
      for (int j = 0; j < 8; ++j) qf[ks][j] = static_cast<__bf16>(x[ks][j] * qs);
  }
  if constexpr (QLDS) {  // this wave's own slice: read back only by the wave itself
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      *reinterpret_cast<uint4*>(qlds + ((wid * KS + ks) * 64 + lane) * 16) = __builtin_bit_cast(uint4, qf[ks]);
  }

  const int* bt = block_tables + static_cast<size_t>(seq) * bt_stride;
  const char* kvb = reinterpret_cast<const char*>(kv);
  const size_t k_head_off = static_cast<size_t>(kvh) * kPBS * D * EB;
  const size_t v_head_off = static_cast<size_t>(Hkv + kvh) * kPBS * D * EB;
  const long bstride = block_stride * EB;
  const int last_blk = (L - 1) / kPBS;

  // ---- staging: global -> registers (tile k0), registers -> LDS buffer
  uint4 sk[NK], sv[NV];
  // A staging chunk's cache block is wave-uniform: chunk ci = tid + NT n covers keys of block
  // ci / (2 D) (2 D >= 128 chunks per block, waves are 64 consecutive threads), so each wave reads its
  // block id with one scalar load and adds a per-lane offset fixed for the whole loop (no per-lane
  // select among the tile's four block ids, no 64-bit multiply per chunk).
  size_t koff[NK], voff[NV];
#pragma unroll
  for (int n = 0; n < NK; ++n) {
    const int ci = tid + NT * n, key = ci / KCH, ch = ci % KCH;
    koff[n] = k_head_off + static_cast<size_t>((key & 15) * (D * EB) + ch * 8 * EB);
  }
#pragma unroll
  for (int n = 0; n < NV; ++n) {
    const int rem = (tid + NT * n) % (2 * D), dim = rem >> 1, half = rem & 1;
    voff[n] = v_head_off + static_cast<size_t>(dim * 16 * EB + half * 8 * EB);
  }
  auto gload = [&](int k0) {
#pragma unroll
    for (int n = 0; n < NK; ++n) {
      const int blk = __builtin_amdgcn_readfirstlane((tid + NT * n) / (2 * D));
      const long b = bt[min(k0 / kPBS + blk, last_blk)];
      sk[n] = ld8_kv<EB>(kvb + b * bstride + koff[n]);
    }
#pragma unroll
    for (int n = 0; n < NV; ++n) {
      const int ci = tid + NT * n, blk = __builtin_amdgcn_readfirstlane(ci / (2 * D)), half = (ci % (2 * D)) & 1;
      const long b = bt[min(k0 / kPBS + blk, last_blk)];
      uint4 v = ld8_kv<EB>(kvb + b * bstride + voff[n]);
      const int kb = k0 + blk * 16 + half * 8;  // keys >= L: zero (unwritten cache bytes may be NaN)
      if (kb + 8 > L) {
        uint32_t* w = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (kb + u >= L) w[u >> 1] &= (u & 1) ? 0x0000FFFFu : 0xFFFF0000u;
      }
      sv[n] = v;
    }
  };
  auto sstore = [&](int buf) {
    char* kl = lds[buf];
    char* vl = lds[buf] + KBYTES;
#pragma unroll
    for (int n = 0; n < NK; ++n) {
      const int ci = tid + NT * n, key = ci / KCH, ch = ci % KCH;
      *reinterpret_cast<uint4*>(kl + key * KROW + ((ch ^ kswz(key)) << 4)) = sk[n];
    }
#pragma unroll
    for (int n = 0; n < NV; ++n) {
      const int ci = tid + NT * n, blk = ci / (2 * D), rem = ci % (2 * D), dim = rem >> 1, half = rem & 1;
      // keys blk*16 + 8 half + j: j < 4 -> group position 4 half + j, j >= 4 -> 8 + 4 half + j - 4
      char* row = vl + dim * (KT * 2);
      const int c0 = blk * 2 + 0, c1 = blk * 2 + 1;  // 16-byte chunks of this block's 16 keys
      uint2 lo = make_uint2(sv[n].x, sv[n].y), hi = make_uint2(sv[n].z, sv[n].w);
      *reinterpret_cast<uint2*>(row + ((c0 ^ vswz(dim)) << 4) + half * 8) = lo;
      *reinterpret_cast<uint2*>(row + ((c1 ^ vswz(dim)) << 4) + half * 8) = hi;
    }
  };

  float16_ o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[dt][i] = 0.f;
  float m = -INFINITY, l = 0.f;
  constexpr bool ORCHK = VAR & 1, MSUM = VAR & 2, CBLK = VAR & 4, MS16 = VAR & 1024;
  constexpr float kBias = 64.f;
  float16_ negm, lsum;  // CBLK: -m in every element; MSUM: the row sum (every element holds it)
  bf16x8_t ones;
#pragma unroll
  for (int i = 0; i < 16; ++i) negm[i] = lsum[i] = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = static_cast<__bf16>(1.f);
  // MS16: the row sum on a 16x16x32 MFMA fed the P^T fragments as its B operand.  That MFMA reads
  // lane l's 8 values as keys 8 (l >> 4) .. + 7 of column l & 15, i.e. query 16 ((l >> 4) & 1) + (l & 15)
  // and key half l >> 5 of ours; an A row m selecting k-groups of parity (m >= 8) sums both key
  // halves of query (l & 15) + 16 (m >= 8): 4 MFMAs a tile instead of 33 adds.  Lane l then holds
  // the sum of query (l & 15) + 16 (l >= 32) in all four accumulator elements.
  // (the selector and the lane's query are rebuilt where used: kept live they spill at D = 64)
  float4_ lsum4 = {0.f, 0.f, 0.f, 0.f};

  // Scores are accumulated relative to the reference m: the QK^T accumulator starts at -m, so exp2
  // reads the MFMA output directly and the per-element subtraction is gone from the VALU stream (at
  // D = 64 the softmax VALU, not the MFMA pipe, bounds a tile).  The first tile of a row starts at 0
  // and sets m from its own max; later tiles move m (lazy rescale) when their max exceeds it by more
  // than 2^8 (VAR 0) or trips the overflow check (VAR & 1, see above).
  // K fragments two reads ahead of their MFMAs (sched_group_barrier pins the order: left alone,
  // hipcc serialises read -> wait -> MFMA eight times per tile; 210.6 -> 205.5 us per layer at an
  // 8192-token chunk).  The softmax stays in scalar f32: packed v_pk_add_f32 beside MFMAs costs more
  // than it saves (MI355X_MICROARCH: an anti-lever; measured 205.5 -> 223.9 us).
  auto qk = [&](const char* kl, float16_ (&sacc)[2], float off) {
    if constexpr (!CBLK) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[kt][i] = off;
    }
    bf16x8_t qv[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      qv[ks] = QLDS ? as_bf16x8(*reinterpret_cast<const uint4*>(qlds + ((wid * KS + ks) * 64 + lane) * 16)) : qf[ks];
    uint4 ka[2 * KS];
#pragma unroll
    for (int idx = 0; idx < 2 * KS; ++idx) {
      const int key = (idx / KS) * 32 + c, ks = idx % KS;
      ka[idx] = *reinterpret_cast<const uint4*>(kl + key * KROW + (((2 * ks + h) ^ kswz(key)) << 4));
    }
#pragma unroll
    for (int idx = 0; idx < 2 * KS; ++idx)
      sacc[idx / KS] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(ka[idx]), qv[idx % KS],
                                                               (CBLK && idx % KS == 0) ? negm : sacc[idx / KS], 0, 0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, QLDS ? 2 + KS : 2, 0);
#pragma unroll
    for (int idx = 0; idx < 2 * KS - 2; ++idx) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
  };
  auto mask = [&](float16_ (&sacc)[2], int k0) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kk = k0 + kt * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (kk > qpos) sacc[kt][i] = -INFINITY;
      }
  };
  auto rowmax = [&](const float16_ (&sacc)[2]) {
    // a balanced max3 tree (depth 4; the 17-deep max chain it replaces was on the critical path from
    // the QK^T MFMAs to the exponentials: 855 -> 954 TF/s at 1 x 8192 with four chains).  Inline asm:
    // fmaxf on MFMA results makes hipcc canonicalise its operands first (an extra v_max each).
    float mx;
    if constexpr (VAR & 16) {  // four fmaxf chains (hipcc's max3 + canonicalising moves)
      float mq[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) mq[j] = fmaxf(sacc[j >> 1][(j & 1) * 8], sacc[j >> 1][(j & 1) * 8 + 1]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 2; i < 8; ++i) mq[j] = fmaxf(mq[j], sacc[j >> 1][(j & 1) * 8 + i]);
      mx = fmaxf(fmaxf(mq[0], mq[1]), fmaxf(mq[2], mq[3]));
    } else {
      float t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kt = j >> 2, i0 = (j & 3) * 4;
        t[j] = vmax(vmax3(sacc[kt][i0], sacc[kt][i0 + 1], sacc[kt][i0 + 2]), sacc[kt][i0 + 3]);
      }
      mx = vmax3(vmax3(t[0], t[1], t[2]), vmax3(t[3], t[4], t[5]), vmax(t[6], t[7]));
    }
    // the row's other half lives 32 lanes away: one permlane32 swap, not an LDS bpermute round trip
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
    return vmax(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
  };
  // move the reference by d (per row; both halves of a row hold the same d): rescale what is already
  // accumulated at the old reference, shift this tile's scores.
  auto move_ref = [&](float16_ (&sacc)[2], float d, bool rescale) {
    if (rescale) {
      const float alpha = __builtin_amdgcn_exp2f(-d);
      if constexpr (MSUM) {
#pragma unroll
        for (int i = 0; i < 16; ++i) lsum[i] *= alpha;
      } else if constexpr (MS16) {
        // the factor of the query this lane sums, (lane & 15) + 16 (lane >= 32); both halves hold it
        lsum4 *= __shfl(alpha, (lane & 15) + ((lane >> 1) & 16), 64);
      } else {
        l *= alpha;
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
    }
    m = rescale ? m + d : d;  // the first tile sets m (m starts at -inf)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) sacc[kt][i] -= d;
    if constexpr (CBLK) {
#pragma unroll
      for (int i = 0; i < 16; ++i) negm[i] = -m;
    }
  };
  auto expcvt = [&](const float16_ (&sacc)[2], bf16x8_t (&pf)[2][2]) {
    // one add chain: split sums keep more exponentials live and spill at 4 waves per SIMD
    float ps = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = __builtin_amdgcn_exp2f(sacc[kt][i]);
        if constexpr (!MSUM && !MS16) ps += p;
        pf[kt][i >> 3][i & 7] = static_cast<__bf16>(p);
      }
    return ps;
  };
  auto overflow = [&](const bf16x8_t (&pf)[2][2]) {  // some p >= 2: the top exponent bit of a half
    uint32_t x = 0;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const uint4 w = __builtin_bit_cast(uint4, pf[kt][s2]);
        x |= w.x | w.y | w.z | w.w;
      }
    return (x & 0x40004000u) != 0u;
  };

  // QK^T + softmax of one tile into P (bf16 fragments pf); pv(): O += V^T . P^T of that tile
  auto softmax_phase = [&](int buf, int k0, bf16x8_t (&pf)[2][2]) {
    const char* kl = lds[buf];
    const bool first = k0 == kbeg;
    const bool diag = k0 + KT - 1 > wave_min_pos;  // tile crosses the diagonal (or the end) of some row
    float16_ sacc[2];
    float ps;
    qk(kl, sacc, first ? 0.f : -m);
    if (diag) mask(sacc, k0);
    if constexpr (ORCHK) {
      if (first) {
        move_ref(sacc, rowmax(sacc) + kBias, false);
        ps = expcvt(sacc, pf);
      } else {
        ps = expcvt(sacc, pf);
        if (__ballot(overflow(pf))) {  // a score passed its row's running max by 65: redo with a real max
          asm volatile("" ::: "memory");  // re-read K from LDS: keeping the first pass's fragments live costs 32 registers
          qk(kl, sacc, -m);
          if (diag) mask(sacc, k0);
          const float mx = rowmax(sacc);
          move_ref(sacc, mx > 0.f ? mx + kBias : 0.f, true);
          ps = expcvt(sacc, pf);
        }
      }
    } else {
      const float mx = rowmax(sacc);  // relative to m (absolute on the first tile)
      // first tile: m := its max; later: lazy rescale when the tile raises the max by more than 2^8.
      // Both halves of a row see the same mx, hence the same decision.
      const bool bump = first || mx > 8.f;
      if (__ballot(bump)) move_ref(sacc, bump ? mx : 0.f, !first);
      ps = expcvt(sacc, pf);
    }
    if constexpr (MSUM) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) lsum = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[kt][s2], lsum, 0, 0, 0);
    } else if constexpr (MS16) {
      // A row m takes the k-groups of parity (m >= 8): one dword pattern per lane, all ones or zero
      const uint32_t w1 = (((lane >> 4) ^ (lane >> 3)) & 1) ? 0u : 0x3F803F80u;
      const bf16x8_t sel = as_bf16x8(make_uint4(w1, w1, w1, w1));
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) lsum4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, pf[kt][s2], lsum4, 0, 0, 0);
    } else {
      l += ps;
    }
  };
  auto pv = [&](int buf, const bf16x8_t (&pf)[2][2]) {
    const char* vl = lds[buf] + KBYTES;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const int dim = 32 * dt + c;
          const uint4 a = *reinterpret_cast<const uint4*>(vl + dim * (KT * 2) + (((4 * kt + 2 * s2 + h) ^ vswz(dim)) << 4));
          o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(a), pf[kt][s2], o[dt], 0, 0, 0);
        }
  };

  auto compute = [&](int buf, int k0) {
    bf16x8_t pf[2][2];
    softmax_phase(buf, k0, pf);
    pv(buf, pf);
  };

  if constexpr (VAR & 32) {
    // Ping-pong (VAR & 32): a tile is two phases, softmax (QK^T MFMAs, then a VALU-dense max / exp /
    // convert) and PV (MFMAs only), one barrier each; waves 4-7 run one phase behind waves 0-3, so on
    // every SIMD (waves w and w + 4) one wave's softmax VALU issues beside the other's PV MFMAs instead
    // of all eight waves alternating MFMA and VALU in step.  Slot s: waves 0-3 run phase s, waves 4-7
    // phase s - 1.  Tile t is loaded from L2 in slot 2t - 2 and written to LDS buffer t & 1 in slot
    // 2t - 1: its previous occupant, tile t - 2, was last read by the late group's PV in slot 2t - 2,
    // and the early group's QK^T of tile t starts in slot 2t.
    const int ntile = (nkeys + KT - 1) / KT, grp = wid >> 2;
    gload(0);
    sstore(0);
    if (ntile > 1) {
      gload(KT);
      sstore(1);
    }
    __syncthreads();
    bf16x8_t pf[2][2];
    for (int sl = 0; sl <= 2 * ntile; ++sl) {
      if (sl > 0) __syncthreads();
      const int tl = sl / 2 + 1;  // even slot: load tile sl / 2 + 1; odd slot: store tile (sl + 1) / 2
      if ((sl & 1) == 0 && sl >= 2 && tl < ntile) gload(tl * KT);
      const int ph = sl - grp;
      if (ph >= 0 && ph < 2 * ntile) {
        const int i = ph >> 1, k0 = i * KT;
        if (k0 <= wave_max_pos) {
          if ((ph & 1) == 0)
            softmax_phase(i & 1, k0, pf);
          else
            pv(i & 1, pf);
        }
      }
      if ((sl & 1) == 1 && sl >= 3 && (sl + 1) / 2 < ntile) sstore(((sl + 1) / 2) & 1);
    }
  } else {
    gload(kbeg);
    sstore(0);
    __syncthreads();
    for (int it = 0, k0 = kbeg; k0 < kend; ++it, k0 += KT) {
      const int buf = it & 1;
      const bool more = k0 + KT < kend;
      if (more) gload(k0 + KT);           // in flight under this tile's MFMAs
      if (k0 <= wave_max_pos) compute(buf, k0);  // waves whose rows all precede the tile skip it
      if (more) sstore(buf ^ 1);
      __syncthreads();
    }
  }

  if constexpr (MSUM) {
    l = lsum[0];  // ones^T . P^T summed both half-waves' keys already
  } else if constexpr (MS16) {
    // lanes 16-31 hold queries 0-15 and lanes 32-47 queries 16-31: swap those two groups
    const int src = (lane >= 16 && lane < 32) ? lane + 16 : (lane >= 32 && lane < 48) ? lane - 16 : lane;
    l = __shfl(lsum4[0], src, 64);
  } else {
    l += __shfl_xor(l, 32, 64);
  }
  if constexpr (SPLIT) {
    if (split) {
      // this half's partial: O / l rounded to bf16 (16 words per lane), then (m, l); a lane's 72 bytes
      // sit at a fixed place per (tile, half, wave, lane), so the other half reads exactly its own lanes
      const int item = pair * NTL + tile;
      const float pin = l > 0.f ? 1.f / l : 0.f;  // rows past the sequence end have no keys
      uint32_t mine[DT * 8];
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int i = 0; i < 8; ++i) mine[dt * 8 + i] = pack2(o[dt][2 * i] * pin, o[dt][2 * i + 1] * pin);
      // agent-scope relaxed atomic stores / loads (write through to, and read from, the cross-XCD
      // coherence point): only the partials bypass the caches.  Release / acquire fences would write
      // back and invalidate this XCD's whole L2 instead, and with it every K/V tile cached for the
      // other workgroups (measured: VAR 128 slower than VAR 0 at every shape that way).
      constexpr int NJ = DT * 4 + 1;  // 8-byte words per lane: O slice, then (m, l); word-major, lane-minor
      uint64_t* wsw = reinterpret_cast<uint64_t*>(split_ws) + ((static_cast<size_t>(item) * 2 + half) * (NT / 64) + wid) * 64 * NJ;
#pragma unroll
      for (int j = 0; j < NJ - 1; ++j)
        __hip_atomic_store(wsw + j * 64 + lane, static_cast<uint64_t>(mine[2 * j]) | (static_cast<uint64_t>(mine[2 * j + 1]) << 32),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(wsw + (NJ - 1) * 64 + lane,
                         static_cast<uint64_t>(__float_as_uint(m)) | (static_cast<uint64_t>(__float_as_uint(l)) << 32),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's partial has reached memory
      __syncthreads();
      int* last_flag = reinterpret_cast<int*>(lds[0]);  // the K/V tiles are no longer read
      if (tid == 0)
        *last_flag = __hip_atomic_fetch_add(split_cnt + item, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1;
      __syncthreads();
      if (!*last_flag) return;
      // the second arriver merges both halves' rounded partials in half order
      const uint64_t* wso = reinterpret_cast<const uint64_t*>(split_ws) +
                            ((static_cast<size_t>(item) * 2 + (half ^ 1)) * (NT / 64) + wid) * 64 * NJ;
      uint32_t other[DT * 8];
#pragma unroll
      for (int j = 0; j < NJ - 1; ++j) {
        const uint64_t v = __hip_atomic_load(wso + j * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        other[2 * j] = static_cast<uint32_t>(v);
        other[2 * j + 1] = static_cast<uint32_t>(v >> 32);
      }
      const uint64_t mlv = __hip_atomic_load(wso + (NJ - 1) * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const float2 mlo = make_float2(__uint_as_float(static_cast<uint32_t>(mlv)), __uint_as_float(static_cast<uint32_t>(mlv >> 32)));
      if (!rvalid) return;
      const float m0 = half == 0 ? m : mlo.x, l0 = half == 0 ? l : mlo.y;
      const float m1 = half == 0 ? mlo.x : m, l1 = half == 0 ? mlo.y : l;
      const uint32_t* p0 = half == 0 ? mine : other;
      const uint32_t* p1 = half == 0 ? other : mine;
      const float mm = fmaxf(m0, m1);
      const float w0 = l0 > 0.f ? l0 * __builtin_amdgcn_exp2f(m0 - mm) : 0.f;
      const float w1 = l1 > 0.f ? l1 * __builtin_amdgcn_exp2f(m1 - mm) : 0.f;
      const float sc = v_scale / (w0 + w1);
      bf16_t* op = out + (static_cast<size_t>(q0 + tok) * Hq + head) * D;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d0 = 32 * dt + 8 * g4 + 4 * h;
          float v[4];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const uint32_t a = p0[dt * 8 + 2 * g4 + e], b = p1[dt * 8 + 2 * g4 + e];
            v[2 * e] = (bf2f_lo(a) * w0 + bf2f_lo(b) * w1) * sc;
            v[2 * e + 1] = (bf2f_hi(a) * w0 + bf2f_hi(b) * w1) * sc;
          }
          *reinterpret_cast<uint2*>(op + d0) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        }
      return;
    }
  }
  if (!rvalid) return;
  const float inv = v_scale / l;
  bf16_t* op = out + (static_cast<size_t>(q0 + tok) * Hq + head) * D;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d0 = 32 * dt + 8 * g4 + 4 * h;
      uint2 v;
      v.x = pack2(o[dt][4 * g4] * inv, o[dt][4 * g4 + 1] * inv);
      v.y = pack2(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv);
      *reinterpret_cast<uint2*>(op + d0) = v;
    }
}

// Grid slots of a (kv head, sequence) pair, heaviest q-tiles first; workgroups visit the pairs
// XCD-aware (the 8 XCDs take contiguous ranges of slots).  VAR & 256 (PAIR): slot s runs q-tile
// n - 1 - s and then q-tile s of its sequence's n tiles, so every workgroup does n + 1 tiles of keys
// (no causal tail); VAR & 128 (SPLIT): two slots per q-tile.
template <int D, int G, int EB, int VAR>
__global__ void __launch_bounds__(pf3_threads(VAR))
__attribute__((amdgpu_waves_per_eu(pf3_wpe(D, VAR) ? pf3_wpe(D, VAR) : 1, pf3_wpe(D, VAR) ? pf3_wpe(D, VAR) : 8)))
paged_prefill_v3_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ q, const void* __restrict__ kv, long block_stride,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ qsl,
    const int* __restrict__ seq_lens, int Hkv, float scale, float v_scale, int q_stride,
    const int64_t* __restrict__ qpos_tab, const float* __restrict__ cos_sin, char* __restrict__ split_ws,
    int* __restrict__ split_cnt, int split_min) {
  constexpr bool SPLIT = VAR & 128, PAIR = VAR & 256;
  static_assert(!(SPLIT && PAIR), "one slot map per variant");
  constexpr int BQ = pf3_threads(VAR) / 2 / G;
  const int NSL = gridDim.x, total = NSL * gridDim.y * gridDim.z;  // grid slots per (kv head, sequence)
  const int lin = blockIdx.x + NSL * (blockIdx.y + gridDim.y * blockIdx.z);
  const int vix = (total % 8 == 0) ? (lin % 8) * (total / 8) + lin / 8 : lin;
  const int pair = vix / NSL, slot = vix - pair * NSL;
#define MXS_PF3_TILE_ARGS out, q, kv, block_stride, block_tables, bt_stride, qsl, seq_lens, Hkv, scale, v_scale, \
                          q_stride, qpos_tab, cos_sin, split_ws, split_cnt, split_min
  if constexpr (PAIR) {
    const int seq = pair / gridDim.y;
    const int n = (qsl[seq + 1] - qsl[seq] + BQ - 1) / BQ;
    if (2 * slot >= n) return;
    pf3_tile<D, G, EB, VAR>(MXS_PF3_TILE_ARGS, n - 1 - slot, 0, pair, NSL);
    if (slot != n - 1 - slot) {
      __syncthreads();  // the first tile's last LDS reads are behind its loop's final barrier; cheap insurance
      pf3_tile<D, G, EB, VAR>(MXS_PF3_TILE_ARGS, slot, 0, pair, NSL);
    }
  } else {
    const int NTL = SPLIT ? NSL / 2 : NSL;
    pf3_tile<D, G, EB, VAR>(MXS_PF3_TILE_ARGS, NTL - 1 - (SPLIT ? slot / 2 : slot), SPLIT ? slot & 1 : 0, pair, NTL);
  }
#undef MXS_PF3_TILE_ARGS
}

// split-variant scratch per q-tile item: 2 halves x waves x 64 lanes x (bf16 O row slice + (m, l))
static constexpr long pf3_split_item_bytes(int D, int VAR) { return 2L * (pf3_threads(VAR) / 64) * 64 * (D * 2 + 8); }

static int pf3_env(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e != nullptr ? std::atoi(e) : dflt;
}
static int pf3_split_min() {
  static const int v = std::max(4, pf3_env("MXS_PF_SPLIT_MIN", 8)) | (pf3_env("MXS_PF_SPLIT_REL", 0) ? 1 << 16 : 0);
  return v;
}
// the default launch splits when its unsplit grid is under this many workgroups (about 1.25 waves of
// resident workgroups: 2 per CU at D = 64, 1 at D = 128)
static int pf3_split_blocks(int D) {
  static const int v = pf3_env("MXS_PF_SPLIT_BLOCKS", -1);
  return v >= 0 ? v : (D == 64 ? 640 : 320);
}

template <int D, int G, int EB, int VAR>
static void pf3_launch(bf16_t* out, const bf16_t* q, const void* kv, long block_stride, const int* block_tables,
                       int bt_stride, const int* qsl, const int* seq_lens, int num_seqs, int max_q_len, int Hkv,
                       float sc, float vs, int q_stride, const int64_t* qpos, const float* cos_sin, hipStream_t s,
                       char* split_ws, int* split_cnt) {
  constexpr int NT = pf3_threads(VAR), BQ = NT / 2 / G;
  constexpr bool SPLIT = VAR & 128, PAIR = VAR & 256;
  const int ntl = (max_q_len + BQ - 1) / BQ;
  const dim3 grid(PAIR ? (ntl + 1) / 2 : ntl * (SPLIT ? 2 : 1), Hkv, num_seqs);
  hipLaunchKernelGGL((paged_prefill_v3_kernel<D, G, EB, VAR>), grid, dim3(NT), 0, s, out, q, kv, block_stride,
                     block_tables, bt_stride, qsl, seq_lens, Hkv, sc, vs, q_stride, qpos, cos_sin, split_ws, split_cnt,
                     pf3_split_min());
}

// the variant a v3 launch runs: explicit (version 0x100 + VAR; other than 128 / 256: bf16 caches, G = 4
// only), else by grid size against the resident workgroups W (2 per CU at D = 64, 1 at D = 128):
// split (128) when the unsplit grid is under ~1.25 W, paired (256) when the paired grid fills at
// least W, else the default (profiles/r5/prefill_attn/split/, pair/).
static int pf3_effective_var(int version, bool fp8, int G, int D, int num_seqs, int max_q_len, int Hkv) {
  if (version >= 0x100) {
    const int var = version - 0x100;
    if (var == 128 || var == 256) return var;
    return !fp8 && G == 4 ? var : kPf3DefaultVar;
  }
  const int BQ = pf3_threads(0) / 2 / G, ntl = (max_q_len + BQ - 1) / BQ;
  const long pairs = static_cast<long>(num_seqs) * Hkv;
  if (pairs * ntl <= pf3_split_blocks(D)) return 128;
  static const int pair_on = pf3_env("MXS_PF_PAIR", 1);
  if (pair_on && pairs * ((ntl + 1) / 2) >= (D == 64 ? 512 : 256)) return 256;
  return kPf3DefaultVar;
}
// the v3 variant a launch would run (host only: the selection of pf3_effective_var, for tests and logs);
// -1 when the launch takes the v2 kernel
// the one v2-vs-v3 decision, shared by the launch, the split-scratch sizing and the variant report:
// fp8 KV and a fused q (RoPE inside the kernel, or q read from the qkv output) exist only on v3
static bool pf_takes_v3(int version, bool kv_fp8, bool fused_q) { return version != 2 || kv_fp8 || fused_q; }
int paged_prefill_variant(int version, bool kv_fp8, bool fused_q, int num_seqs, int max_q_len, int Hq, int Hkv,
                          int D) {
  if (!pf_takes_v3(version, kv_fp8, fused_q)) return -1;
  return pf3_effective_var(version, kv_fp8, Hq / Hkv, D, num_seqs, max_q_len, Hkv);
}
static long pf3_blocks(int num_seqs, int max_q_len, int Hkv, int G) {
  const int BQ = pf3_threads(0) / 2 / G;
  return static_cast<long>(num_seqs) * Hkv * ((max_q_len + BQ - 1) / BQ);
}

template <int D, int G>
static void pf3_dispatch(int var, bool fp8, bf16_t* out, const bf16_t* q, const void* kv, long block_stride,
                         const int* block_tables, int bt_stride, const int* qsl, const int* seq_lens, int num_seqs,
                         int max_q_len, int Hkv, float sc, float vs, int q_stride, const int64_t* qpos,
                         const float* cos_sin, hipStream_t s, char* split_ws, int* split_cnt) {
#define MXS_PF3_ARGS out, q, kv, block_stride, block_tables, bt_stride, qsl, seq_lens, num_seqs, max_q_len, Hkv, sc, vs, \
                     q_stride, qpos, cos_sin, s, split_ws, split_cnt
  if (var == 128 && split_ws != nullptr && split_cnt != nullptr) {
    if (fp8) return pf3_launch<D, G, 1, 128>(MXS_PF3_ARGS);
    return pf3_launch<D, G, 2, 128>(MXS_PF3_ARGS);
  }
  if (var == 256) {
    if (fp8) return pf3_launch<D, G, 1, 256>(MXS_PF3_ARGS);
    return pf3_launch<D, G, 2, 256>(MXS_PF3_ARGS);
  }
  if (fp8) return pf3_launch<D, G, 1, (kPf3DefaultVar & ~128)>(MXS_PF3_ARGS);
  if constexpr (G == 4) {  // the other variants: G = 4 only (A/B probes and tests)
    switch (var) {
      case 1: return pf3_launch<D, G, 2, 1>(MXS_PF3_ARGS);
      case 2: return pf3_launch<D, G, 2, 2>(MXS_PF3_ARGS);
      case 4: return pf3_launch<D, G, 2, 4>(MXS_PF3_ARGS);
      case 6: return pf3_launch<D, G, 2, 6>(MXS_PF3_ARGS);
      case 7: return pf3_launch<D, G, 2, 7>(MXS_PF3_ARGS);
      case 8: return pf3_launch<D, G, 2, 8>(MXS_PF3_ARGS);
      case 10: return pf3_launch<D, G, 2, 10>(MXS_PF3_ARGS);
      case 12: return pf3_launch<D, G, 2, 12>(MXS_PF3_ARGS);
      case 14: return pf3_launch<D, G, 2, 14>(MXS_PF3_ARGS);
      case 16: return pf3_launch<D, G, 2, 16>(MXS_PF3_ARGS);
      case 32: return pf3_launch<D, G, 2, 32>(MXS_PF3_ARGS);
      case 36: return pf3_launch<D, G, 2, 36>(MXS_PF3_ARGS);
      case 64: return pf3_launch<D, G, 2, 64>(MXS_PF3_ARGS);
      case 66: return pf3_launch<D, G, 2, 66>(MXS_PF3_ARGS);
      case 1024: return pf3_launch<D, G, 2, 1024>(MXS_PF3_ARGS);
      case 1280: return pf3_launch<D, G, 2, 1280>(MXS_PF3_ARGS);
      default: break;
    }
  }
  pf3_launch<D, G, 2, (kPf3DefaultVar & ~128)>(MXS_PF3_ARGS);
#undef MXS_PF3_ARGS
}

// Bytes of scratch and int32 counters the launch needs (0 when it does not run the split variant).
// Counters must start at zero once and are never reset (see the split comment above the kernel).
void paged_prefill_split_need(int version, bool kv_fp8, bool fused_q, int num_seqs, int max_q_len, int Hq, int Hkv,
                              int D, long* ws_bytes, long* counters) {
  *ws_bytes = 0;
  *counters = 0;
  if (num_seqs == 0 || max_q_len == 0 || Hkv == 0 || Hq % Hkv != 0 || (D != 64 && D != 128)) return;
  const int G = Hq / Hkv;
  const long items = pf3_blocks(num_seqs, max_q_len, Hkv, G);
  if (!pf_takes_v3(version, kv_fp8, fused_q)) return;  // the v2 kernel has no split form
  if (pf3_effective_var(version, kv_fp8, G, D, num_seqs, max_q_len, Hkv) != 128) return;
  *counters = items;
  *ws_bytes = items * (D == 64 ? pf3_split_item_bytes(64, 128) : pf3_split_item_bytes(128, 128));
}

// q_stride: elements between consecutive q rows (Hq * D for a dense q; (Hq + 2 Hkv) * D when q is
// read from the fused qkv output); cos_sin != nullptr applies RoPE at positions qpos (v3 only).
// version 0x100 + VAR selects a v3 variant explicitly (probes, tests).
void launch_paged_prefill(bf16_t* out, const bf16_t* q, const void* kv_ptr, bool kv_fp8, long block_stride,
                          const int* block_tables, int bt_stride, const int* qsl, const int* seq_lens,
                          int num_seqs, int max_q_len, int Hq, int Hkv, int D, float scale, int version,
                          float k_scale, float v_scale, hipStream_t s, int q_stride, const int64_t* qpos,
                          const float* cos_sin, char* split_ws, int* split_cnt) {
  if (num_seqs == 0 || max_q_len == 0) return;
  const int G = Hq / Hkv;
  const bf16_t* kv = static_cast<const bf16_t*>(kv_ptr);
  if (q_stride <= 0) q_stride = Hq * D;
  if (pf_takes_v3(version, kv_fp8, cos_sin != nullptr || q_stride != Hq * D)) {
    const float sc = kv_fp8 ? scale * k_scale : scale, vs = kv_fp8 ? v_scale : 1.f;
    const int var = pf3_effective_var(version, kv_fp8, G, D, num_seqs, max_q_len, Hkv);
#define MXS_PF3(DD, GG)                                                                                     \
    if (D == DD && G == GG) {                                                                               \
      pf3_dispatch<DD, GG>(var, kv_fp8, out, q, kv_ptr, block_stride, block_tables, bt_stride, qsl, seq_lens, \
                           num_seqs, max_q_len, Hkv, sc, vs, q_stride, qpos, cos_sin, s, split_ws, split_cnt); \
      MXS_CHECK_LAUNCH();                                                                                   \
      return;                                                                                               \
    }
    MXS_PF3(64, 1) MXS_PF3(64, 2) MXS_PF3(64, 4) MXS_PF3(64, 8)
    MXS_PF3(128, 1) MXS_PF3(128, 2) MXS_PF3(128, 4) MXS_PF3(128, 8)
#undef MXS_PF3
  }
  const int BQ = 128 / G;
  dim3 grid((max_q_len + BQ - 1) / BQ, Hkv, num_seqs), blk(256);
#define MXS_PF(DD, GG)                                                                                     \
  if (D == DD && G == GG) {                                                                                \
    hipLaunchKernelGGL((paged_prefill_kernel<DD, GG>), grid, blk, 0, s, out, q, kv, block_stride,          \
                       block_tables, bt_stride, qsl, seq_lens, Hkv, scale);                               \
    MXS_CHECK_LAUNCH();                                                                                    \
    return;                                                                                                \
  }
  MXS_PF(64, 1) MXS_PF(64, 2) MXS_PF(64, 4) MXS_PF(64, 8)
  MXS_PF(128, 1) MXS_PF(128, 2) MXS_PF(128, 4) MXS_PF(128, 8)
#undef MXS_PF
}

}  // namespace mxs
