// Python bindings of the gfx950 kernels (module mxserve._C).  Every op launches on the current HIP
// stream so the model runner can capture decode steps into hipGraphs.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <map>
#include <utility>
#include <mutex>
#include <optional>
#include <vector>

namespace mxs {
typedef unsigned short bf16_t;
void launch_rms_norm(bf16_t*, const bf16_t*, const bf16_t*, int, int, int, float, hipStream_t);
void launch_fused_add_rms_norm(bf16_t*, const bf16_t*, bf16_t*, const bf16_t*, int, int, float, hipStream_t);
void launch_silu_mul(bf16_t*, const bf16_t*, int, int, hipStream_t);
void launch_embed_rms_norm(bf16_t*, bf16_t*, const int64_t*, const bf16_t*, const bf16_t*, int, int, float,
                           hipStream_t);
void launch_rope_and_cache(bf16_t*, const bf16_t*, const int64_t*, const float*, void*, bool, long, const int64_t*,
                           const bf16_t*, const bf16_t*, int, int, int, int, int, float, float, float, hipStream_t);
int decode_num_partitions(int);
void decode_plan(int, int, int, int*, int*);
bool launch_paged_decode(bf16_t*, float*, float*, const bf16_t*, const void*, bool, long, const int*, int, const int*,
                         int, int, int, int, int, int, float, float, float, int, hipStream_t, int = 0,
                         const int64_t* = nullptr, const float* = nullptr);
void launch_paged_prefill(bf16_t*, const bf16_t*, const void*, bool, long, const int*, int, const int*, const int*,
                          int, int, int, int, int, float, int, float, float, hipStream_t, int = 0,
                          const int64_t* = nullptr, const float* = nullptr, char* = nullptr, int* = nullptr);
void paged_prefill_split_need(int, bool, bool, int, int, int, int, int, long*, long*);
int paged_prefill_variant(int, bool, bool, int, int, int, int, int);
void launch_sample(int64_t*, const void*, bool, int, int, long, const float*, const float*, const int*,
                   const int64_t*, const int64_t*, hipStream_t);
void launch_logprobs(float*, int64_t*, float*, const void*, bool, int, int, long, const int64_t*, const int64_t*, int,
                     hipStream_t);
void launch_penalties(void*, bool, int, int, long, const int*, long, const int64_t*, const int*, const int*,
                      const float*, const float*, const float*, int*, hipStream_t);
void launch_moe_topk_softmax(float*, int*, const bf16_t*, int, int, int, hipStream_t);
void launch_moe_align(int*, int*, const int*, int, int, int, int*, hipStream_t);
void launch_moe_combine(bf16_t*, const bf16_t*, const float*, const int*, int, int, int, hipStream_t);
bool launch_gemv_stream(bf16_t*, float*, const bf16_t*, const bf16_t*, int, int, int, int, int, int, int, int, int,
                        bool, hipStream_t);
bool launch_skinny_gemm(bf16_t*, float*, const bf16_t*, const bf16_t*, int, int, int, int, int, int, bool, int,
                        hipStream_t);
bool launch_decode_gemm(bf16_t*, float*, const bf16_t*, const bf16_t*, int, int, int, int, int, int, int, int, int,
                        int, hipStream_t, const int* = nullptr, int = 0, int = 0, int = 0, int = 1);
bool launch_mt_gemm(bf16_t*, float*, const bf16_t*, const bf16_t*, int, int, int, int, int, int, int, int, int, int,
                    int, hipStream_t, int*, int, int = 0, int = 1);
void launch_splitk_add_rms_norm(bf16_t*, bf16_t*, const float*, int, int, int, const bf16_t*, float, hipStream_t);
bool launch_splitk_rope_and_cache(bf16_t*, const float*, int, const int64_t*, const float*, void*, bool, long,
                                  const int64_t*, const bf16_t*, const bf16_t*, int, int, int, int, int, float, float,
                                  float, hipStream_t);
bool launch_prefill_gemm(bf16_t*, float*, const bf16_t*, const bf16_t*, int, int, int, int, int, int, int,
                         hipStream_t);
bool launch_gemm_w4(bf16_t*, const bf16_t*, const bf16_t*, int, int, int, int, int, int, int, hipStream_t,
                    const bf16_t*, int);
bool launch_gemm_pf(bf16_t*, const bf16_t*, const bf16_t*, int, int, int, int, int, int, float*, long, int*, int,
                    const int*, int, int, int, hipStream_t, const bf16_t*, int, bool, float, int);
int pf_plan(int, int, int, int, int, int, int*, int*, int*, int);
bool launch_moe_grouped_gemm(bf16_t*, const bf16_t*, const bf16_t*, const int*, int, int, int, int, int, bool,
                             int, float*, hipStream_t);
void launch_moe_combine_partials(bf16_t*, const float*, const float*, const int*, int, int, int, int, long,
                                 hipStream_t);
void launch_silu_mul_partials(bf16_t*, const float*, int, int, int, long, hipStream_t);
}  // namespace mxs

namespace {

using mxs::bf16_t;

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_CUDA(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_BF16(x) TORCH_CHECK((x).scalar_type() == at::kBFloat16, #x " must be bf16")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")

inline bf16_t* bf(const at::Tensor& t) { return reinterpret_cast<bf16_t*>(t.data_ptr()); }

void rms_norm(at::Tensor out, at::Tensor x, at::Tensor w, double eps) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(out);
  TORCH_CHECK(x.stride(-1) == 1, "x rows must be contiguous");
  const int H = x.size(-1);
  TORCH_CHECK(H % 8 == 0, "hidden size must be a multiple of 8");
  const int rows = x.numel() / H;
  const int x_stride = x.dim() >= 2 ? x.stride(-2) : H;
  mxs::launch_rms_norm(bf(out), bf(x), bf(w), rows, H, x_stride, static_cast<float>(eps), stream());
}

// Split-K slabs [S][M][H] of a residual-stream projection -> residual += their sum (bf16-rounded),
// out = RMSNorm(residual) * w (norm_act.hip splitk_add_rmsnorm_kernel).
void splitk_add_rms_norm(at::Tensor out, at::Tensor residual, at::Tensor part, int64_t S, at::Tensor w, double eps) {
  CHECK_CUDA(out); CHECK_BF16(out); CHECK_BF16(residual); CHECK_BF16(w); CHECK_CONTIG(out); CHECK_CONTIG(residual);
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous(), "part: fp32 CUDA slabs");
  const int64_t H = residual.size(-1), M = residual.numel() / H;
  TORCH_CHECK(out.numel() == M * H && w.numel() == H && H % 8 == 0, "shape mismatch");
  TORCH_CHECK(S >= 1 && part.numel() >= S * M * H, "part holds fewer than S slabs of [M, H]");
  mxs::launch_splitk_add_rms_norm(bf(out), bf(residual), part.data_ptr<float>(), static_cast<int>(S),
                                  static_cast<int>(M), static_cast<int>(H), bf(w), static_cast<float>(eps), stream());
}

void fused_add_rms_norm(at::Tensor out, at::Tensor x, at::Tensor residual, at::Tensor w, double eps) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(residual); CHECK_CONTIG(x); CHECK_CONTIG(residual); CHECK_CONTIG(out);
  const int H = x.size(-1);
  TORCH_CHECK(H % 8 == 0, "hidden size must be a multiple of 8");
  mxs::launch_fused_add_rms_norm(bf(out), bf(x), bf(residual), bf(w), x.numel() / H, H, static_cast<float>(eps),
                                 stream());
}

// K01 + first K02: out = rmsnorm(table[ids]) * w, residual = table[ids]
void embed_rms_norm(at::Tensor out, at::Tensor residual, at::Tensor ids, at::Tensor table, at::Tensor w, double eps) {
  CHECK_CUDA(table); CHECK_BF16(table); CHECK_BF16(w); CHECK_CONTIG(table); CHECK_CONTIG(out); CHECK_CONTIG(residual);
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous(), "ids must be contiguous int64");
  const int H = table.size(1);
  TORCH_CHECK(H % 8 == 0 && out.size(-1) == H && residual.size(-1) == H, "hidden size");
  TORCH_CHECK(out.numel() == ids.numel() * H && residual.numel() == ids.numel() * H, "row count");
  mxs::launch_embed_rms_norm(bf(out), bf(residual), ids.data_ptr<int64_t>(), bf(table), bf(w), ids.numel(), H,
                             static_cast<float>(eps), stream());
}

void silu_mul(at::Tensor out, at::Tensor gu) {
  CHECK_CUDA(gu); CHECK_BF16(gu); CHECK_CONTIG(gu); CHECK_CONTIG(out);
  const int I = gu.size(-1) / 2;
  TORCH_CHECK(I % 8 == 0, "intermediate size must be a multiple of 8");
  mxs::launch_silu_mul(bf(out), bf(gu), gu.numel() / (2 * I), I, stream());
}

// kv_layer: [NB, 2, Hkv, BS, D] view (block stride may exceed 2*Hkv*BS*D); bf16, or fp8 e4m3fn
// (float8_e4m3fn or raw uint8) for the fp8 KV cache.  Returns true for fp8.
bool check_kv(const at::Tensor& kv, int Hkv, int D) {
  CHECK_CUDA(kv);
  const bool fp8 = kv.scalar_type() == at::kFloat8_e4m3fn || kv.scalar_type() == at::kByte;
  TORCH_CHECK(fp8 || kv.scalar_type() == at::kBFloat16, "kv cache must be bf16 or fp8 (e4m3fn)");
  TORCH_CHECK(kv.dim() == 5 && kv.size(1) == 2 && kv.size(2) == Hkv && kv.size(4) == D, "bad kv_layer shape");
  TORCH_CHECK(kv.size(3) == 16, "block size must be 16");
  TORCH_CHECK(kv.stride(4) == 1 && kv.stride(3) == D && kv.stride(2) == 16 * D && kv.stride(1) == Hkv * 16 * D,
              "kv_layer inner dims must be dense");
  return fp8;
}

// q_out None: K / V into the cache only (q stays in the qkv rows for the attention kernels' fused RoPE)
void rope_and_cache(std::optional<at::Tensor> q_out, at::Tensor qkv, at::Tensor positions, at::Tensor cos_sin,
                    at::Tensor kv, at::Tensor slot_mapping, std::optional<at::Tensor> qn, std::optional<at::Tensor> kn,
                    int64_t Hq, int64_t Hkv, int64_t D, double eps, double k_scale, double v_scale) {
  CHECK_CUDA(qkv); CHECK_BF16(qkv); CHECK_CONTIG(qkv);
  if (q_out.has_value()) {
    CHECK_CONTIG((*q_out));
    TORCH_CHECK(q_out->numel() == qkv.size(0) * Hq * D, "q_out shape");
  } else {
    TORCH_CHECK(!qn.has_value(), "q/k norm needs the rope kernel to write q");
  }
  TORCH_CHECK(positions.scalar_type() == at::kLong && slot_mapping.scalar_type() == at::kLong, "int64 indices");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.size(1) == D, "cos_sin must be fp32 [P, D]");
  TORCH_CHECK(qkv.size(1) == (Hq + 2 * Hkv) * D, "qkv width mismatch");
  const bool fp8 = check_kv(kv, Hkv, D);
  const bf16_t* qnp = qn.has_value() ? bf(*qn) : nullptr;
  const bf16_t* knp = kn.has_value() ? bf(*kn) : nullptr;
  mxs::launch_rope_and_cache(q_out.has_value() ? bf(*q_out) : nullptr, bf(qkv), positions.data_ptr<int64_t>(),
                             cos_sin.data_ptr<float>(),
                             kv.data_ptr(), fp8, kv.stride(0), slot_mapping.data_ptr<int64_t>(), qnp, knp, qkv.size(0),
                             Hq, Hkv, D, 16, static_cast<float>(eps), static_cast<float>(k_scale),
                             static_cast<float>(v_scale), stream());
}

// rope_and_cache reading the qkv row from S unreduced fp32 split-K slabs [S][T][(Hq + 2 Hkv) D]
bool splitk_rope_and_cache(at::Tensor q_out, at::Tensor part, int64_t S, int64_t T, at::Tensor positions,
                           at::Tensor cos_sin, at::Tensor kv, at::Tensor slot_mapping, std::optional<at::Tensor> qn,
                           std::optional<at::Tensor> kn, int64_t Hq, int64_t Hkv, int64_t D, double eps, double k_scale,
                           double v_scale) {
  CHECK_CUDA(part); CHECK_CONTIG(q_out);
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.is_contiguous(), "part: fp32 slabs");
  TORCH_CHECK(part.numel() >= S * T * (Hq + 2 * Hkv) * D, "part holds fewer than S slabs of [T, qkv]");
  TORCH_CHECK(positions.scalar_type() == at::kLong && slot_mapping.scalar_type() == at::kLong, "int64 indices");
  TORCH_CHECK(positions.numel() >= T && slot_mapping.numel() >= T && q_out.numel() == T * Hq * D, "shape mismatch");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.size(1) == D, "cos_sin must be fp32 [P, D]");
  const bool fp8 = check_kv(kv, Hkv, D);
  const bf16_t* qnp = qn.has_value() ? bf(*qn) : nullptr;
  const bf16_t* knp = kn.has_value() ? bf(*kn) : nullptr;
  return mxs::launch_splitk_rope_and_cache(bf(q_out), part.data_ptr<float>(), static_cast<int>(S),
                                           positions.data_ptr<int64_t>(), cos_sin.data_ptr<float>(), kv.data_ptr(), fp8,
                                           kv.stride(0), slot_mapping.data_ptr<int64_t>(), qnp, knp,
                                           static_cast<int>(T), Hq, Hkv, D, 16, static_cast<float>(eps),
                                           static_cast<float>(k_scale), static_cast<float>(v_scale), stream());
}

// q [T, Hq, D]: dense, or a row-strided view of the fused qkv output (q = qkv[:, :Hq * D]); with
// rope_pos / cos_sin the kernel applies RoPE to q itself (the rope kernel wrote only K / V).
struct QArg {
  int stride = 0;
  const int64_t* pos = nullptr;
  const float* cs = nullptr;
};
QArg q_arg(const at::Tensor& q, const std::optional<at::Tensor>& rope_pos, const std::optional<at::Tensor>& cos_sin) {
  CHECK_CUDA(q); CHECK_BF16(q);
  TORCH_CHECK(q.dim() == 3 && q.stride(2) == 1 && q.stride(1) == q.size(2), "q rows: [T, Hq, D] with dense heads");
  TORCH_CHECK(q.stride(0) % 8 == 0 && (reinterpret_cast<uintptr_t>(q.data_ptr()) & 15) == 0, "q rows 16-byte aligned");
  QArg a;
  a.stride = static_cast<int>(q.stride(0));
  TORCH_CHECK(rope_pos.has_value() == cos_sin.has_value(), "rope_pos and cos_sin go together");
  if (cos_sin.has_value()) {
    TORCH_CHECK(rope_pos->scalar_type() == at::kLong && rope_pos->is_contiguous() && rope_pos->numel() >= q.size(0),
                "rope_pos: int64 [T]");
    TORCH_CHECK(cos_sin->scalar_type() == at::kFloat && cos_sin->is_contiguous() && cos_sin->size(1) == q.size(2),
                "cos_sin: fp32 [P, D]");
    a.pos = rope_pos->data_ptr<int64_t>();
    a.cs = cos_sin->data_ptr<float>();
  }
  return a;
}

void paged_attention_decode(at::Tensor out, at::Tensor q, at::Tensor kv, at::Tensor block_tables,
                            at::Tensor seq_lens, double scale, int64_t max_seq_len, double k_scale, double v_scale,
                            int64_t impl, std::optional<at::Tensor> rope_pos, std::optional<at::Tensor> cos_sin) {
  const QArg qa = q_arg(q, rope_pos, cos_sin);
  CHECK_CONTIG(out);
  const int B = q.size(0), Hq = q.size(1), D = q.size(2);
  const int Hkv = kv.size(2);
  const bool fp8 = check_kv(kv, Hkv, D);
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && seq_lens.scalar_type() == at::kInt, "int32 tables");
  TORCH_CHECK(block_tables.stride(1) == 1, "block_tables rows must be contiguous");
  TORCH_CHECK(Hq % Hkv == 0, "GQA ratio");
  int P = 1, part_len = 0;
  mxs::decode_plan(B, Hkv, static_cast<int>(std::max<int64_t>(max_seq_len, 1)), &P, &part_len);
  at::Tensor tmp_out, tmp_ml;
  if (P > 1) {
    tmp_out = at::empty({B, Hq, P, D}, q.options().dtype(at::kFloat));
    tmp_ml = at::empty({B, Hq, P, 2}, q.options().dtype(at::kFloat));
  }
  const bool ok = mxs::launch_paged_decode(
      bf(out), P > 1 ? tmp_out.data_ptr<float>() : nullptr, P > 1 ? tmp_ml.data_ptr<float>() : nullptr, bf(q),
      kv.data_ptr(), fp8, kv.stride(0), block_tables.data_ptr<int>(), block_tables.stride(0), seq_lens.data_ptr<int>(),
      B, Hq, Hkv, D, P, /*part_len: split each sequence evenly*/ 0, static_cast<float>(scale),
      static_cast<float>(k_scale), static_cast<float>(v_scale), static_cast<int>(impl), stream(), qa.stride, qa.pos,
      qa.cs);
  TORCH_CHECK(ok, "paged_attention_decode: no kernel for this head shape (fused q needs the MFMA kernel)");
}

void paged_attention_prefill(at::Tensor out, at::Tensor q, at::Tensor kv, at::Tensor block_tables, at::Tensor qsl,
                             at::Tensor seq_lens, double scale, int64_t max_q_len, int64_t version, double k_scale,
                             double v_scale, std::optional<at::Tensor> rope_pos, std::optional<at::Tensor> cos_sin) {
  const QArg qa = q_arg(q, rope_pos, cos_sin);
  CHECK_CONTIG(out);
  const int Hq = q.size(1), D = q.size(2);
  const int Hkv = kv.size(2);
  const bool fp8 = check_kv(kv, Hkv, D);
  TORCH_CHECK(qsl.scalar_type() == at::kInt && seq_lens.scalar_type() == at::kInt, "int32 metadata");
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && block_tables.stride(1) == 1, "block_tables");
  const int S = seq_lens.size(0);
  // the split variant: scratch from the caching allocator per call, tile counters persistent per
  // (device, stream) (zeroed once, never reset: each launch adds 2 per split tile, and launches on one
  // stream run in order, so the ticket parity holds; two streams never share a table)
  long ws_bytes = 0, ncnt = 0;
  const bool fused_q = qa.cs != nullptr || qa.stride != Hq * D;  // as launch_paged_prefill decides v2 / v3
  mxs::paged_prefill_split_need(static_cast<int>(version), fp8, fused_q, S, static_cast<int>(max_q_len), Hq, Hkv,
                                D, &ws_bytes, &ncnt);
  at::Tensor ws;
  int* cnt = nullptr;
  if (ws_bytes > 0) {
    static std::mutex mu;
    // never destroyed: a static tensor's destructor would run after the HIP runtime has shut down
    static auto* counters = new std::map<std::pair<int, hipStream_t>, at::Tensor>();
    std::lock_guard<std::mutex> lock(mu);
    at::Tensor& c = (*counters)[{static_cast<int>(q.get_device()), stream()}];
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    TORCH_CHECK(hipStreamIsCapturing(stream(), &cap) == hipSuccess, "hipStreamIsCapturing");
    if (!c.defined() || c.numel() < ncnt) {
      if (cap == hipStreamCaptureStatusNone) {
        // a grown table's predecessor stays allocated: launches still queued on the stream may use it
        static auto* retired = new std::vector<at::Tensor>();
        if (c.defined()) retired->push_back(c);
        c = at::zeros({std::max<long>(ncnt, 1L << 14)}, q.options().dtype(at::kInt));
      } else {
        ws_bytes = 0;  // no counters outside a graph's pool: run this launch unsplit
      }
    }
    if (ws_bytes > 0) {
      cnt = c.data_ptr<int>();
      ws = at::empty({ws_bytes}, q.options().dtype(at::kByte));
    }
  }
  mxs::launch_paged_prefill(bf(out), bf(q), kv.data_ptr(), fp8, kv.stride(0), block_tables.data_ptr<int>(),
                            block_tables.stride(0), qsl.data_ptr<int>(), seq_lens.data_ptr<int>(), S,
                            static_cast<int>(max_q_len), Hq, Hkv, D, static_cast<float>(scale),
                            static_cast<int>(version), static_cast<float>(k_scale), static_cast<float>(v_scale),
                            stream(), qa.stride, qa.pos, qa.cs,
                            ws_bytes > 0 ? reinterpret_cast<char*>(ws.data_ptr()) : nullptr, cnt);
}

void sample(at::Tensor out, at::Tensor logits, at::Tensor temperature, at::Tensor top_p, at::Tensor top_k,
            at::Tensor seeds, at::Tensor steps) {
  CHECK_CUDA(logits);
  TORCH_CHECK((logits.scalar_type() == at::kFloat || logits.scalar_type() == at::kBFloat16) && logits.stride(1) == 1,
              "logits must be fp32 or bf16 rows");
  TORCH_CHECK(temperature.scalar_type() == at::kFloat && top_p.scalar_type() == at::kFloat, "fp32 params");
  TORCH_CHECK(top_k.scalar_type() == at::kInt && seeds.scalar_type() == at::kLong && steps.scalar_type() == at::kLong,
              "int params");
  mxs::launch_sample(out.data_ptr<int64_t>(), logits.data_ptr(), logits.scalar_type() == at::kBFloat16,
                     logits.size(0), logits.size(1),
                     logits.stride(0), temperature.data_ptr<float>(), top_p.data_ptr<float>(),
                     top_k.data_ptr<int>(), seeds.data_ptr<int64_t>(), steps.data_ptr<int64_t>(), stream());
}

// log-probs of the sampled token + the K best tokens for logits rows `rows`
void logprobs(at::Tensor tok_lp, at::Tensor top_ids, at::Tensor top_lp, at::Tensor logits, at::Tensor rows,
              at::Tensor tokens) {
  CHECK_CUDA(logits);
  TORCH_CHECK((logits.scalar_type() == at::kFloat || logits.scalar_type() == at::kBFloat16) && logits.stride(1) == 1,
              "logits must be fp32 or bf16 rows");
  TORCH_CHECK(rows.scalar_type() == at::kLong && tokens.scalar_type() == at::kLong, "int64 rows / tokens");
  const int n = rows.size(0);
  TORCH_CHECK(tokens.size(0) == n && tok_lp.size(0) == n && top_ids.size(0) == n && top_lp.size(0) == n, "row count");
  TORCH_CHECK(tok_lp.scalar_type() == at::kFloat && top_lp.scalar_type() == at::kFloat &&
                  top_ids.scalar_type() == at::kLong && top_ids.is_contiguous() && top_lp.is_contiguous(),
              "output dtypes");
  const int K = top_ids.dim() == 2 ? top_ids.size(1) : 0;
  TORCH_CHECK(K >= 0 && K <= 20 && top_lp.size(-1) == K, "top_logprobs must be in [0, 20]");
  mxs::launch_logprobs(tok_lp.data_ptr<float>(), top_ids.data_ptr<int64_t>(), top_lp.data_ptr<float>(),
                       logits.data_ptr(), logits.scalar_type() == at::kBFloat16, n, logits.size(1), logits.stride(0),
                       rows.data_ptr<int64_t>(), tokens.data_ptr<int64_t>(), K, stream());
}

// frequency / presence / repetition penalties, in place on logits rows [B, V]
void apply_penalties(at::Tensor logits, at::Tensor hist, at::Tensor srows, at::Tensor hlen, at::Tensor plen,
                     at::Tensor rep, at::Tensor freq, at::Tensor pres, at::Tensor counts) {
  CHECK_CUDA(logits);
  TORCH_CHECK((logits.scalar_type() == at::kFloat || logits.scalar_type() == at::kBFloat16) && logits.stride(1) == 1,
              "logits must be fp32 or bf16 rows");
  const int B = logits.size(0), V = logits.size(1);
  TORCH_CHECK(V <= 163840, "vocab too large for the penalty bitmap");
  TORCH_CHECK(hist.scalar_type() == at::kInt && hist.dim() == 2 && hist.stride(1) == 1, "hist: int32 [rows, L]");
  TORCH_CHECK(srows.scalar_type() == at::kLong && srows.size(0) == B, "srows");
  TORCH_CHECK(hlen.scalar_type() == at::kInt && plen.scalar_type() == at::kInt && hlen.size(0) == B &&
                  plen.size(0) == B, "hlen / plen");
  TORCH_CHECK(rep.scalar_type() == at::kFloat && freq.scalar_type() == at::kFloat && pres.scalar_type() == at::kFloat &&
                  rep.size(0) == B && freq.size(0) == B && pres.size(0) == B, "penalty params");
  TORCH_CHECK(counts.scalar_type() == at::kInt && counts.is_contiguous() && counts.numel() >= static_cast<long>(B) * V,
              "counts scratch");
  mxs::launch_penalties(logits.data_ptr(), logits.scalar_type() == at::kBFloat16, B, V, logits.stride(0),
                        hist.data_ptr<int>(), hist.stride(0), srows.data_ptr<int64_t>(), hlen.data_ptr<int>(),
                        plen.data_ptr<int>(), rep.data_ptr<float>(), freq.data_ptr<float>(), pres.data_ptr<float>(),
                        counts.data_ptr<int>(), stream());
}

// Decode projection (csrc/kernels/gemm_decode.hip): out = x . w^T (epi 0, out [M, N]) or
// out = SiLU(x . w_gate^T) * (x . w_up^T) with w = [gate; up] (epi 1, out [M, N/2]).  `part` is the
// fp32 split-K workspace (>= splitk * M * N floats) when splitk > 1.  False if the configuration
// does not tile the shape (the caller keeps hipBLASLt).
bool decode_gemm(at::Tensor out, at::Tensor x, at::Tensor w, c10::optional<at::Tensor> part, int64_t mf, int64_t nf,
                 int64_t wm, int64_t splitk, int64_t epi, int64_t lu, bool reduce) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "2-D operands");
  const int64_t M = x.size(0), N = w.size(0), K = w.size(1);
  TORCH_CHECK(x.size(1) == K && out.size(0) == M && out.size(1) == (epi == 1 ? N / 2 : N), "shape mismatch");
  TORCH_CHECK(epi == 0 || epi == 1, "epi 0 (none) | 1 (silu*mul)");
  if (x.stride(1) != 1 || out.stride(1) != 1) return false;
  float* p = nullptr;
  if (splitk > 1) {
    TORCH_CHECK(part.has_value() && part->is_cuda() && part->scalar_type() == at::kFloat && part->is_contiguous() &&
                    part->numel() >= splitk * M * N, "split-K needs an fp32 workspace of splitk * M * N");
    p = part->data_ptr<float>();
  }
  return mxs::launch_decode_gemm(bf(out), p, bf(x), bf(w), M, N, K, x.stride(0), out.stride(0), mf, nf, wm, splitk,
                                 epi, stream(), nullptr, 0, 0, lu, reduce ? 1 : 0);
}

// Row-stream form (gemm_decode.hip gemv_stream_kernel): M <= 16 rows, whole W rows streamed once; nr rows
// per wave, kw waves splitting a workgroup's K, kg workgroups splitting K over the grid.  epi 1:
// w = [gate; up], out [M, N / 2] = SiLU(gate) * up.  kg = 1 with part (epi 0): an fp32 [M][N] result
// instead of bf16 out.  kg > 1: fp32 slabs [kg][M][N] in part, summed (with SiLU*mul for epi 1) into out
// when reduce, else left for the caller's fused epilogue.
bool gemv_stream(at::Tensor out, at::Tensor x, at::Tensor w, c10::optional<at::Tensor> part, int64_t nr, int64_t kw,
                 int64_t epi, int64_t kg, bool reduce) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "2-D operands");
  TORCH_CHECK(epi == 0 || epi == 1, "epi 0 (none) or 1 (SiLU*mul)");
  const int64_t M = x.size(0), N = w.size(0), K = w.size(1);
  TORCH_CHECK(x.size(1) == K && out.size(0) == M && out.size(1) == (epi ? N / 2 : N), "shape mismatch");
  if (x.stride(1) != 1 || out.stride(1) != 1 || kg < 1) return false;
  float* p = nullptr;
  if (part.has_value()) {
    TORCH_CHECK(part->is_cuda() && part->scalar_type() == at::kFloat && part->is_contiguous() &&
                    part->numel() >= kg * M * N, "the fp32 result / slabs need a kg * M * N workspace");
    p = part->data_ptr<float>();
  }
  return mxs::launch_gemv_stream(bf(out), p, bf(x), bf(w), M, N, K, x.stride(0), out.stride(0), nr, kw,
                                 static_cast<int>(epi), static_cast<int>(kg), reduce, stream());
}

// Skinny form (gemm_decode.hip skinny_gemm_kernel): M <= 16 rows, 16-column W slices x 4 k-ranges of
// kr per workgroup; K / (4 kr) > 1 groups leave fp32 slabs [groups][M][N] in `part` (summed here when
// reduce, else by the caller's epilogue).  epi 1: w = [gate; up], out [M, N / 2] = SiLU(gate) * up (slabs
// always written, reduce required).
bool skinny_gemm(at::Tensor out, at::Tensor x, at::Tensor w, c10::optional<at::Tensor> part, int64_t kr, bool reduce,
                 int64_t epi) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "2-D operands");
  TORCH_CHECK(epi == 0 || epi == 1, "epi 0 (none) or 1 (SiLU*mul)");
  const int64_t M = x.size(0), N = w.size(0), K = w.size(1);
  TORCH_CHECK(x.size(1) == K && out.size(0) == M && out.size(1) == (epi ? N / 2 : N), "shape mismatch");
  if (x.stride(1) != 1 || out.stride(1) != 1 || kr <= 0 || K % (4 * kr) != 0) return false;
  if (epi && (!reduce || N % 32 != 0)) return false;
  const int64_t groups = K / (4 * kr);
  float* p = nullptr;
  if (groups > 1 || epi) {
    TORCH_CHECK(part.has_value() && part->is_cuda() && part->scalar_type() == at::kFloat && part->is_contiguous() &&
                    part->numel() >= groups * M * N, "split-K needs an fp32 workspace of groups * M * N");
    p = part->data_ptr<float>();
  }
  return mxs::launch_skinny_gemm(bf(out), p, bf(x), bf(w), M, N, K, x.stride(0), out.stride(0), kr, reduce,
                                 static_cast<int>(epi), stream());
}

// Medium-M form of the decode projection (gemm_decode.hip mt_gemm_kernel, M = 64-256 and short
// prefill chunks): WM x WN waves of 32 MR rows x 32 WNF weight rows, same epilogues and workspace rule
// as decode_gemm; with `cnt` (int32 tile counters, zeroed once, left zero by every launch) the split-K
// slabs are summed inside the launch.  False if the configuration does not tile the shape.
bool mt_gemm(at::Tensor out, at::Tensor x, at::Tensor w, c10::optional<at::Tensor> part, int64_t wm, int64_t wn,
             int64_t mr, int64_t wnf, int64_t splitk, int64_t epi, c10::optional<at::Tensor> cnt, int64_t order,
             bool reduce) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "2-D operands");
  const int64_t M = x.size(0), N = w.size(0), K = w.size(1);
  TORCH_CHECK(x.size(1) == K && out.size(0) == M && out.size(1) == (epi == 1 ? N / 2 : N), "shape mismatch");
  TORCH_CHECK(epi == 0 || epi == 1, "epi 0 (none) | 1 (silu*mul)");
  if (x.stride(1) != 1 || out.stride(1) != 1) return false;
  float* p = nullptr;
  if (splitk > 1) {
    TORCH_CHECK(part.has_value() && part->is_cuda() && part->scalar_type() == at::kFloat && part->is_contiguous() &&
                    part->numel() >= splitk * M * N, "split-K needs an fp32 workspace of splitk * M * N");
    p = part->data_ptr<float>();
  }
  int* c = nullptr;
  int clen = 0;
  if (cnt.has_value()) {
    TORCH_CHECK(cnt->is_cuda() && cnt->scalar_type() == at::kInt && cnt->is_contiguous(), "cnt: int32 CUDA tensor");
    c = cnt->data_ptr<int>();
    clen = static_cast<int>(std::min<int64_t>(cnt->numel(), 1 << 30));
  }
  return mxs::launch_mt_gemm(bf(out), p, bf(x), bf(w), M, N, K, x.stride(0), out.stride(0), wm, wn, mr, wnf, splitk,
                             epi, stream(), c, clen, static_cast<int>(order), reduce ? 1 : 0);
}

// K05-K08 at prefill sizes (csrc/kernels/gemm_prefill.hip): out [M, N] = x [M, K] . w [N, K]^T.
// bm in {64, 128}; splitk > 1 needs an fp32 workspace of splitk * M * N.  False if unsupported.
bool prefill_gemm(at::Tensor out, at::Tensor x, at::Tensor w, c10::optional<at::Tensor> part, int64_t bm,
                  int64_t splitk) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "2-D operands");
  const int64_t M = x.size(0), N = w.size(0), K = w.size(1);
  TORCH_CHECK(x.size(1) == K && out.size(0) == M && out.size(1) == N, "shape mismatch");
  if (x.stride(1) != 1 || out.stride(1) != 1) return false;
  float* p = nullptr;
  if (splitk > 1) {
    TORCH_CHECK(part.has_value() && part->is_cuda() && part->scalar_type() == at::kFloat && part->is_contiguous() &&
                    part->numel() >= splitk * M * N, "split-K needs an fp32 workspace of splitk * M * N");
    p = part->data_ptr<float>();
  }
  return mxs::launch_prefill_gemm(bf(out), p, bf(x), bf(w), M, N, K, x.stride(0), out.stride(0), bm, splitk,
                                  stream());
}

// K05-K08 at prefill chunks (csrc/kernels/gemm_pf.hip, persistent stream-K): epi 0 out [M, N] =
// x w^T; epi 1 (SwiGLU) w = [gate; up] [2 I, K], out [M, I]; epi 2 out = resid + x w^T (resid may be
// out).  row_scale (epi 0 / 1): rows scaled by rsqrt(mean(x^2) + eps) (fused RMSNorm, the norm weight
// folded into w).  slab: fp32 stream-K workspace, cnt: int32 tile counters (zero; every launch leaves
// them zero).  False if the shape is unsupported.
bool gemm_pf(at::Tensor out, at::Tensor x, at::Tensor w, int64_t epi, at::Tensor slab, at::Tensor cnt,
             at::Tensor tile_map, int64_t num_cu, int64_t min_iters, c10::optional<at::Tensor> resid,
             bool row_scale, double eps, int64_t trows) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "2-D operands");
  const int64_t M = x.size(0), N = w.size(0), K = w.size(1);
  TORCH_CHECK(x.size(1) == K && out.size(0) == M && out.size(1) == (epi == 1 ? N / 2 : N), "shape mismatch");
  TORCH_CHECK(slab.is_cuda() && slab.scalar_type() == at::kFloat && slab.is_contiguous(), "slab: fp32 CUDA");
  TORCH_CHECK(cnt.is_cuda() && cnt.scalar_type() == at::kInt && cnt.is_contiguous(), "cnt: int32 CUDA");
  TORCH_CHECK(tile_map.is_cuda() && tile_map.scalar_type() == at::kInt && tile_map.is_contiguous(), "tile_map");
  if (x.stride(1) != 1 || out.stride(1) != 1 || M > (1 << 24)) return false;
  const bf16_t* R = nullptr;
  int ldr = 0;
  if (epi == 2) {
    TORCH_CHECK(resid.has_value(), "epi 2 needs resid");
    CHECK_BF16((*resid));
    TORCH_CHECK(resid->dim() == 2 && resid->size(0) == M && resid->size(1) == N && resid->stride(1) == 1,
                "resid shape");
    R = bf(*resid);
    ldr = static_cast<int>(resid->stride(0));
  }
  return mxs::launch_gemm_pf(bf(out), bf(x), bf(w), M, N, K, x.stride(0), out.stride(0), epi, slab.data_ptr<float>(),
                             slab.numel(), cnt.data_ptr<int>(), cnt.numel(), tile_map.data_ptr<int>(),
                             tile_map.numel(), num_cu, min_iters, stream(), R, ldr, row_scale,
                             static_cast<float>(eps), static_cast<int>(trows));
}

// K05-K08 at prefill chunks, four-wave form (csrc/kernels/gemm_w4.hip, data-parallel persistent): the
// epilogues of gemm_pf (epi 0 / 1 SwiGLU / 2 residual), no row scale, no stream-K.
bool gemm_w4(at::Tensor out, at::Tensor x, at::Tensor w, int64_t epi, int64_t num_cu,
             c10::optional<at::Tensor> resid) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "2-D operands");
  const int64_t M = x.size(0), N = w.size(0), K = w.size(1);
  TORCH_CHECK(x.size(1) == K && out.size(0) == M && out.size(1) == (epi == 1 ? N / 2 : N), "shape mismatch");
  if (x.stride(1) != 1 || out.stride(1) != 1 || M > (1 << 24)) return false;
  const bf16_t* R = nullptr;
  int ldr = 0;
  if (epi == 2) {
    TORCH_CHECK(resid.has_value(), "epi 2 needs resid");
    CHECK_BF16((*resid));
    TORCH_CHECK(resid->dim() == 2 && resid->size(0) == M && resid->size(1) == N && resid->stride(1) == 1,
                "resid shape");
    R = bf(*resid);
    ldr = static_cast<int>(resid->stride(0));
  }
  return mxs::launch_gemm_w4(bf(out), bf(x), bf(w), M, N, K, x.stride(0), out.stride(0), epi, num_cu, stream(), R,
                             ldr);
}

// Grouped decode form of decode_gemm (K16 at decode batches): w [E, N, K], x = routed rows sorted by
// expert (offs = moe_align offsets), rows_max = the most rows one expert can hold (tokens).  Output
// as moe_grouped_gemm: out [rows, N or N/2] (splitk 1) or fp32 partials [splitk, rows, N].
bool moe_decode_gemm(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor offs, c10::optional<at::Tensor> part,
                     int64_t rows_max, int64_t mf, int64_t nf, int64_t wm, int64_t splitk, int64_t epi,
                     int64_t lu) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(w); CHECK_CONTIG(x);
  TORCH_CHECK(w.dim() == 3 && x.dim() == 2, "w [E, N, K], x [rows, K]");
  TORCH_CHECK(offs.scalar_type() == at::kInt && offs.is_contiguous() && offs.numel() == w.size(0) + 1,
              "offs: int32 [E + 1]");
  TORCH_CHECK(epi == 0 || epi == 1, "epi 0 (none) | 1 (silu*mul)");
  const int64_t R = x.size(0), E = w.size(0), N = w.size(1), K = w.size(2);
  TORCH_CHECK(x.size(1) == K, "shape mismatch");
  TORCH_CHECK(rows_max >= 1 && rows_max <= R, "rows_max in [1, rows]");
  float* p = nullptr;
  int64_t ldy = epi == 1 ? N / 2 : N;
  if (splitk > 1) {
    TORCH_CHECK(part.has_value() && part->is_cuda() && part->scalar_type() == at::kFloat && part->is_contiguous() &&
                    part->numel() >= splitk * R * N, "split-K needs an fp32 workspace of splitk * rows * N");
    p = part->data_ptr<float>();
  } else {
    CHECK_BF16(out); CHECK_CONTIG(out);
    TORCH_CHECK(out.dim() == 2 && out.size(0) == R && out.size(1) == ldy, "out [rows, N or N/2]");
  }
  return mxs::launch_decode_gemm(splitk > 1 ? nullptr : bf(out), p, bf(x), bf(w), R, N, K, K, ldy, mf, nf, wm, splitk,
                                 epi, stream(), offs.data_ptr<int>(), E, rows_max, lu);
}

// y[r] = x[r] . w[e(r)]^T over expert-sorted rows (offs = moe_align offsets); silu: w rows are
// [gate; up] and y = silu(gate) * up (width N/2).  False if the shape is unsupported.
bool moe_grouped_gemm(at::Tensor y, at::Tensor x, at::Tensor w, at::Tensor offs, bool silu, int64_t split,
                      std::optional<at::Tensor> partial) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(y); CHECK_CONTIG(x); CHECK_CONTIG(w); CHECK_CONTIG(y);
  TORCH_CHECK(w.dim() == 3 && x.dim() == 2 && y.dim() == 2, "w [E, N, K], x [rows, K], y [rows, N']");
  TORCH_CHECK(offs.scalar_type() == at::kInt && offs.numel() == w.size(0) + 1, "offs: int32 [E + 1]");
  const int N = w.size(1), K = w.size(2);
  // split > 1 writes the fp32 partials only: y is not touched (may be empty)
  TORCH_CHECK(x.size(1) == K && (split > 1 || (y.size(0) == x.size(0) && y.size(1) == (silu ? N / 2 : N))),
              "shape mismatch");
  float* pp = nullptr;
  if (split > 1) {
    TORCH_CHECK(partial.has_value() && partial->scalar_type() == at::kFloat && partial->is_contiguous() &&
                    partial->numel() >= split * x.size(0) * N, "partial: fp32 [split, rows, N]");
    pp = partial->data_ptr<float>();
  }
  return mxs::launch_moe_grouped_gemm(bf(y), bf(x), bf(w), offs.data_ptr<int>(), w.size(0), x.size(0), N, K,
                                      y.size(1), silu, static_cast<int>(split), pp, stream());
}

void moe_topk_softmax(at::Tensor w, at::Tensor ids, at::Tensor logits) {
  CHECK_CUDA(logits); CHECK_BF16(logits); CHECK_CONTIG(logits);
  TORCH_CHECK(logits.size(1) <= 64, "at most 64 experts");
  mxs::launch_moe_topk_softmax(w.data_ptr<float>(), ids.data_ptr<int>(), bf(logits), logits.size(0),
                               logits.size(1), w.size(1), stream());
}

void moe_align(at::Tensor expert_offsets, at::Tensor perm, at::Tensor topk_ids, int64_t e_lo, int64_t e_local,
               std::optional<at::Tensor> inv) {
  CHECK_CUDA(topk_ids); CHECK_CONTIG(topk_ids);
  TORCH_CHECK(topk_ids.scalar_type() == at::kInt, "int32 ids");
  TORCH_CHECK(e_local <= 256, "at most 256 local experts");
  if (inv.has_value())
    TORCH_CHECK(inv->scalar_type() == at::kInt && inv->numel() == topk_ids.numel(), "inv: int32 [T K]");
  mxs::launch_moe_align(expert_offsets.data_ptr<int>(), perm.data_ptr<int>(), topk_ids.data_ptr<int>(),
                        topk_ids.numel(), e_lo, e_local, inv.has_value() ? inv->data_ptr<int>() : nullptr, stream());
}

// K17: out[t] = sum_k topk_w[t, k] * ys[inv[t, k]] (inv from moe_align; < 0 = not a local expert)
void moe_combine(at::Tensor out, at::Tensor ys, at::Tensor topk_w, at::Tensor inv) {
  CHECK_CUDA(ys); CHECK_BF16(ys); CHECK_BF16(out); CHECK_CONTIG(ys); CHECK_CONTIG(out);
  TORCH_CHECK(topk_w.scalar_type() == at::kFloat && topk_w.is_contiguous() && topk_w.dim() == 2, "topk_w fp32 [T, K]");
  TORCH_CHECK(inv.scalar_type() == at::kInt && inv.is_contiguous() && inv.numel() == topk_w.numel(), "inv");
  const int T = topk_w.size(0), K = topk_w.size(1), H = ys.size(1);
  TORCH_CHECK(K <= 8 && H % 8 == 0 && out.size(0) == T && out.size(1) == H, "shapes");
  mxs::launch_moe_combine(bf(out), bf(ys), topk_w.data_ptr<float>(), inv.data_ptr<int>(), T, K, H, stream());
}

}  // namespace

void register_comm(pybind11::module_& m);  // comm.cpp: KV transfer agent + custom all-reduce
namespace mxs {
void register_hblt(pybind11::module_& m);  // hblt.cpp: hipBLASLt with a tuned solution
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "mxserve gfx950 HIP kernels";
  m.def("rms_norm", &rms_norm);
  m.def("fused_add_rms_norm", &fused_add_rms_norm);
  m.def("splitk_add_rms_norm", &splitk_add_rms_norm);
  m.def("splitk_rope_and_cache", &splitk_rope_and_cache);
  m.def("silu_mul", &silu_mul);
  m.def("embed_rms_norm", &embed_rms_norm);
  m.def("rope_and_cache", &rope_and_cache, pybind11::arg("q_out"), pybind11::arg("qkv"), pybind11::arg("positions"),
        pybind11::arg("cos_sin"), pybind11::arg("kv"), pybind11::arg("slot_mapping"), pybind11::arg("qn"),
        pybind11::arg("kn"), pybind11::arg("Hq"), pybind11::arg("Hkv"), pybind11::arg("D"), pybind11::arg("eps"),
        pybind11::arg("k_scale") = 1.0, pybind11::arg("v_scale") = 1.0);
  m.def("paged_attention_decode", &paged_attention_decode, pybind11::arg("out"), pybind11::arg("q"),
        pybind11::arg("kv"), pybind11::arg("block_tables"), pybind11::arg("seq_lens"), pybind11::arg("scale"),
        pybind11::arg("max_seq_len"), pybind11::arg("k_scale") = 1.0, pybind11::arg("v_scale") = 1.0,
        pybind11::arg("impl") = 0, pybind11::arg("rope_pos") = pybind11::none(),
        pybind11::arg("cos_sin") = pybind11::none());
  m.def("paged_prefill_variant", &mxs::paged_prefill_variant, pybind11::arg("version"), pybind11::arg("kv_fp8"),
        pybind11::arg("fused_q"), pybind11::arg("num_seqs"), pybind11::arg("max_q_len"), pybind11::arg("hq"),
        pybind11::arg("hkv"), pybind11::arg("head_dim"),
        "prefill attention v3 variant a launch picks (0 default, 128 split-KV, 256 paired tiles; -1: v2)");
  m.def("paged_prefill_split_need",
        [](int version, bool kv_fp8, bool fused_q, int num_seqs, int max_q_len, int hq, int hkv, int head_dim) {
          long ws = 0, cnt = 0;
          mxs::paged_prefill_split_need(version, kv_fp8, fused_q, num_seqs, max_q_len, hq, hkv, head_dim, &ws, &cnt);
          return std::make_pair(ws, cnt);
        },
        pybind11::arg("version"), pybind11::arg("kv_fp8"), pybind11::arg("fused_q"), pybind11::arg("num_seqs"),
        pybind11::arg("max_q_len"), pybind11::arg("hq"), pybind11::arg("hkv"), pybind11::arg("head_dim"),
        "(scratch bytes, tile counters) the split-KV prefill variant of this launch needs (0, 0: unsplit)");
  m.def("paged_attention_prefill", &paged_attention_prefill, pybind11::arg("out"), pybind11::arg("q"),
        pybind11::arg("kv"), pybind11::arg("block_tables"), pybind11::arg("qsl"), pybind11::arg("seq_lens"),
        pybind11::arg("scale"), pybind11::arg("max_q_len"), pybind11::arg("version") = 3,
        pybind11::arg("k_scale") = 1.0, pybind11::arg("v_scale") = 1.0, pybind11::arg("rope_pos") = pybind11::none(),
        pybind11::arg("cos_sin") = pybind11::none());
  m.def("sample", &sample);
  m.def("logprobs", &logprobs);
  m.def("apply_penalties", &apply_penalties);
  m.def("moe_topk_softmax", &moe_topk_softmax);
  m.def("moe_align", &moe_align, pybind11::arg("expert_offsets"), pybind11::arg("perm"), pybind11::arg("topk_ids"),
        pybind11::arg("e_lo"), pybind11::arg("e_local"), pybind11::arg("inv") = pybind11::none());
  m.def("moe_combine", &moe_combine);
  m.def("gemv_stream", &gemv_stream, pybind11::arg("out"), pybind11::arg("x"), pybind11::arg("w"),
        pybind11::arg("part") = c10::nullopt, pybind11::arg("nr") = 2, pybind11::arg("kw") = 1, pybind11::arg("epi") = 0,
        pybind11::arg("kg") = 1, pybind11::arg("reduce") = true);
  m.def("skinny_gemm", &skinny_gemm, pybind11::arg("out"), pybind11::arg("x"), pybind11::arg("w"),
        pybind11::arg("part") = pybind11::none(), pybind11::arg("kr") = 256, pybind11::arg("reduce") = true,
        pybind11::arg("epi") = 0);
  m.def("decode_gemm", &decode_gemm, pybind11::arg("out"), pybind11::arg("x"), pybind11::arg("w"),
        pybind11::arg("part"), pybind11::arg("mf"), pybind11::arg("nf"), pybind11::arg("wm"), pybind11::arg("splitk"),
        pybind11::arg("epi"), pybind11::arg("lu") = 0, pybind11::arg("reduce") = true);
  m.def("mt_gemm", &mt_gemm, pybind11::arg("out"), pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("part"),
        pybind11::arg("wm"), pybind11::arg("wn"), pybind11::arg("mr"), pybind11::arg("wnf"), pybind11::arg("splitk"),
        pybind11::arg("epi"), pybind11::arg("cnt") = pybind11::none(), pybind11::arg("order") = 0,
        pybind11::arg("reduce") = true);
  m.def("prefill_gemm", &prefill_gemm, pybind11::arg("out"), pybind11::arg("x"), pybind11::arg("w"),
        pybind11::arg("part"), pybind11::arg("bm"), pybind11::arg("splitk"));
  m.def("gemm_w4", &gemm_w4, pybind11::arg("out"), pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("epi"),
        pybind11::arg("num_cu"), pybind11::arg("resid") = pybind11::none());
  m.def("gemm_pf", &gemm_pf, pybind11::arg("out"), pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("epi"),
        pybind11::arg("slab"), pybind11::arg("cnt"), pybind11::arg("tile_map"), pybind11::arg("num_cu"),
        pybind11::arg("min_iters") = 16, pybind11::arg("resid") = pybind11::none(),
        pybind11::arg("row_scale") = false, pybind11::arg("eps") = 1e-5, pybind11::arg("trows") = 256);
  m.def("gemm_pf_plan", [](int M, int N, int K, int epi, int num_cu, int min_iters, int trows) {
    int dp = 0, sk = 0, g = 0;
    mxs::pf_plan(M, N, K, epi, num_cu, min_iters, &dp, &sk, &g, trows);
    return std::make_tuple(g, dp, sk);
  });
  m.def("moe_decode_gemm", &moe_decode_gemm, pybind11::arg("out"), pybind11::arg("x"), pybind11::arg("w"),
        pybind11::arg("offs"), pybind11::arg("part"), pybind11::arg("rows_max"), pybind11::arg("mf"),
        pybind11::arg("nf"), pybind11::arg("wm"), pybind11::arg("splitk"), pybind11::arg("epi"),
        pybind11::arg("lu") = 0);
  m.def("moe_grouped_gemm", &moe_grouped_gemm, pybind11::arg("y"), pybind11::arg("x"), pybind11::arg("w"),
        pybind11::arg("offs"), pybind11::arg("silu"), pybind11::arg("split") = 1,
        pybind11::arg("partial") = pybind11::none());
  m.def("silu_mul_partials", [](at::Tensor h, at::Tensor part) {
    CHECK_CUDA(part); CHECK_BF16(h); CHECK_CONTIG(h);
    TORCH_CHECK(part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() == 3, "part fp32 [S, R, 2I]");
    const int R = part.size(1), I = part.size(2) / 2;
    TORCH_CHECK(I % 4 == 0 && h.size(0) == R && h.size(1) == I && part.size(0) <= 8, "shapes (at most 8 slabs)");
    mxs::launch_silu_mul_partials(bf(h), part.data_ptr<float>(), R, I, part.size(0),
                                  part.size(1) * static_cast<long>(part.size(2)), stream());
  });
  m.def("moe_combine_partials", [](at::Tensor out, at::Tensor part, at::Tensor topk_w, at::Tensor inv) {
    CHECK_CUDA(part); CHECK_BF16(out); CHECK_CONTIG(out);
    TORCH_CHECK(part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() == 3, "part fp32 [S, R, H]");
    TORCH_CHECK(topk_w.scalar_type() == at::kFloat && topk_w.is_contiguous() && topk_w.dim() == 2, "topk_w");
    TORCH_CHECK(inv.scalar_type() == at::kInt && inv.is_contiguous() && inv.numel() == topk_w.numel(), "inv");
    const int T = topk_w.size(0), K = topk_w.size(1), H = part.size(2);
    TORCH_CHECK(K <= 8 && H % 4 == 0 && out.size(0) == T && out.size(1) == H && part.size(0) <= 8,
                "shapes (top-k <= 8, at most 8 slabs)");
    mxs::launch_moe_combine_partials(bf(out), part.data_ptr<float>(), topk_w.data_ptr<float>(), inv.data_ptr<int>(),
                                     T, K, H, part.size(0), part.size(1) * static_cast<long>(H), stream());
  });
  m.def("decode_num_partitions", &mxs::decode_num_partitions);
  m.def("decode_plan", [](int B, int Hkv, int max_seq_len) {
    int P = 1, len = 0;
    mxs::decode_plan(B, Hkv, max_seq_len, &P, &len);
    return std::make_pair(P, len);
  });
  register_comm(m);
  mxs::register_hblt(m);
}
