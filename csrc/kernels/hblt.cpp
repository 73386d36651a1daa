// hipBLASLt with a chosen solution: the prefill projections that stay on the library (qkv / o / down
// of the small dense models, where gemm_pf does not win) run the solution a start-up tuner measured
// fastest for their (N, K, row bucket) instead of the library heuristic's pick, which is not monotone
// in the row count (profiles/r3/s3/hipblaslt_m_sweep.jsonl) and is one candidate among hundreds of
// gfx950 solutions.  mxserve/ops/prefill_hblt.py owns the tuning and the table.
//
// Layout: torch's y [M, N] = x [M, K] W^T with W [N, K] row-major is, in hipBLASLt's column-major
// terms, D (N x M, ld ldy) = op_T(A = W: K x N, ld K) * B (x: K x M, ld ldx) -- the TN problem the
// torch path also runs (the Cijk_Alik_Bljk kernels in the headline traces).  The residual form sets
// C = R with beta = 1 (D may alias R: in place on the residual stream).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>

#include <map>
#include <mutex>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace mxs {
namespace {

#define MXS_HBLT_OK(expr)                                                                  \
  do {                                                                                     \
    hipblasStatus_t st_ = (expr);                                                          \
    TORCH_CHECK(st_ == HIPBLAS_STATUS_SUCCESS, "hipBLASLt: ", #expr, " failed: ", (int)st_); \
  } while (0)

// one problem shape's descriptors (created once per (M, N, K, ld*, residual) and kept)
struct Problem {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr, d = nullptr;
  std::map<int, std::pair<bool, hipblasLtMatmulAlgo_t>> algo;  // solution index -> (supported, checked algo)
  std::map<int, size_t> ws;                                    // solution index -> workspace bytes
};

using Key = std::tuple<int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, bool>;

struct Ctx {
  hipblasLtHandle_t h = nullptr;
  std::map<Key, Problem> probs;
  std::unordered_map<int, hipblasLtMatmulAlgo_t> by_index;  // solution index -> algo (getAllAlgos)
  bool listed = false;
};

std::mutex g_mu;
std::map<int, Ctx> g_ctx;  // per device

Ctx& ctx_for(int dev) {
  Ctx& c = g_ctx[dev];
  if (c.h == nullptr) MXS_HBLT_OK(hipblasLtCreate(&c.h));
  return c;
}

void list_all(Ctx& c) {
  if (c.listed) return;
  std::vector<hipblasLtMatmulHeuristicResult_t> all;
  MXS_HBLT_OK(hipblaslt_ext::getAllAlgos(c.h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, HIPBLAS_OP_T, HIPBLAS_OP_N,
                                         HIP_R_16BF, HIP_R_16BF, HIP_R_16BF, HIP_R_16BF, HIPBLAS_COMPUTE_32F, all));
  for (auto& r : all) c.by_index[hipblaslt_ext::getIndexFromAlgo(r.algo)] = r.algo;
  c.listed = true;
}

void destroy(Problem& p) {
  if (p.desc) hipblasLtMatmulDescDestroy(p.desc);
  for (auto l : {p.a, p.b, p.c, p.d})
    if (l) hipblasLtMatrixLayoutDestroy(l);
}

Problem& problem(Ctx& c, int64_t M, int64_t N, int64_t K, int64_t ldx, int64_t ldy, int64_t ldr, bool resid) {
  const Key k{M, N, K, ldx, ldy, resid ? ldr : 0, resid};
  auto it = c.probs.find(k);
  if (it != c.probs.end()) return it->second;
  if (c.probs.size() >= 4096) {  // prefill row counts vary step to step: bound the cache
    for (auto& kv : c.probs) destroy(kv.second);
    c.probs.clear();
  }
  Problem& p = c.probs[k];
  MXS_HBLT_OK(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const int32_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  MXS_HBLT_OK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  MXS_HBLT_OK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  MXS_HBLT_OK(hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, K, N, K));
  MXS_HBLT_OK(hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, K, M, ldx));
  MXS_HBLT_OK(hipblasLtMatrixLayoutCreate(&p.c, HIP_R_16BF, N, M, resid ? ldr : ldy));
  MXS_HBLT_OK(hipblasLtMatrixLayoutCreate(&p.d, HIP_R_16BF, N, M, ldy));
  return p;
}

// the checked algo for this problem (nullptr: the solution does not support it)
const hipblasLtMatmulAlgo_t* checked(Ctx& c, Problem& p, int index, bool resid, size_t* ws) {
  auto it = p.algo.find(index);
  if (it == p.algo.end()) {
    list_all(c);
    auto a = c.by_index.find(index);
    std::pair<bool, hipblasLtMatmulAlgo_t> ent{false, {}};
    size_t need = 0;
    if (a != c.by_index.end()) {
      ent.second = a->second;
      const float alpha = 1.f, beta = resid ? 1.f : 0.f;
      ent.first = hipblaslt_ext::matmulIsAlgoSupported(c.h, p.desc, &alpha, p.a, p.b, &beta, p.c, p.d, ent.second,
                                                       need) == HIPBLAS_STATUS_SUCCESS;
    }
    it = p.algo.emplace(index, ent).first;
    p.ws[index] = need;
  }
  *ws = p.ws[index];
  return it->second.first ? &it->second.second : nullptr;
}

void check_operands(const torch::Tensor& out, const torch::Tensor& x, const torch::Tensor& w) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && out.is_cuda(), "hblt: device tensors");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kBFloat16,
              "hblt: bf16 operands");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2 && x.stride(1) == 1 && w.stride(1) == 1 &&
                  out.stride(1) == 1 && w.stride(0) == w.size(1),
              "hblt: row-major 2-D operands, dense W");
  TORCH_CHECK(x.size(1) == w.size(1) && out.size(0) == x.size(0) && out.size(1) == w.size(0), "hblt: shapes");
}

}  // namespace

// Solution indices that support y[M, N] = x W^T (+ R), in the library heuristic's order first (its
// top `heuristic` picks), then every other supporting solution of the gfx950 library.  ws_max:
// workspace bytes the caller can provide.
std::vector<int64_t> hblt_candidates(int64_t M, int64_t N, int64_t K, bool resid, int64_t heuristic, int64_t ws_max) {
  std::lock_guard<std::mutex> g(g_mu);
  int dev = 0;
  (void)hipGetDevice(&dev);
  Ctx& c = ctx_for(dev);
  Problem& p = problem(c, M, N, K, K, N, N, resid);
  std::vector<int64_t> out;
  {
    hipblasLtMatmulPreference_t pref;
    MXS_HBLT_OK(hipblasLtMatmulPreferenceCreate(&pref));
    const uint64_t wsb = static_cast<uint64_t>(ws_max);
    MXS_HBLT_OK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
    std::vector<hipblasLtMatmulHeuristicResult_t> res(std::max<int64_t>(1, heuristic));
    int got = 0;
    if (hipblasLtMatmulAlgoGetHeuristic(c.h, p.desc, p.a, p.b, p.c, p.d, pref, static_cast<int>(res.size()), res.data(),
                                        &got) == HIPBLAS_STATUS_SUCCESS)
      for (int i = 0; i < got; ++i)
        if (res[i].state == HIPBLAS_STATUS_SUCCESS) out.push_back(hipblaslt_ext::getIndexFromAlgo(res[i].algo));
    hipblasLtMatmulPreferenceDestroy(pref);
  }
  list_all(c);
  for (auto& kv : c.by_index) {
    bool seen = false;
    for (auto v : out) seen |= v == kv.first;
    if (seen) continue;
    size_t ws = 0;
    if (checked(c, p, kv.first, resid, &ws) != nullptr && static_cast<int64_t>(ws) <= ws_max) out.push_back(kv.first);
  }
  return out;
}

// out = x W^T (+ resid, beta 1; out may be resid) with solution `index`; false when the solution does
// not support this problem or needs more workspace than given (the caller falls back)
bool hblt_mm(torch::Tensor out, torch::Tensor x, torch::Tensor w, std::optional<torch::Tensor> resid, int64_t index,
             torch::Tensor workspace) {
  check_operands(out, x, w);
  const bool has_r = resid.has_value();
  if (has_r)
    TORCH_CHECK(resid->scalar_type() == at::kBFloat16 && resid->dim() == 2 && resid->stride(1) == 1 &&
                    resid->size(0) == out.size(0) && resid->size(1) == out.size(1),
                "hblt: residual [M, N] bf16 row-major");
  const int64_t M = x.size(0), N = w.size(0), K = w.size(1);
  if (M == 0) return true;
  std::lock_guard<std::mutex> g(g_mu);
  Ctx& c = ctx_for(x.get_device());
  Problem& p = problem(c, M, N, K, x.stride(0), out.stride(0), has_r ? resid->stride(0) : 0, has_r);
  size_t ws = 0;
  const hipblasLtMatmulAlgo_t* algo = checked(c, p, static_cast<int>(index), has_r, &ws);
  if (algo == nullptr || ws > static_cast<size_t>(workspace.numel() * workspace.element_size())) return false;
  const float alpha = 1.f, beta = has_r ? 1.f : 0.f;
  const void* cptr = has_r ? resid->data_ptr() : out.data_ptr();
  MXS_HBLT_OK(hipblasLtMatmul(c.h, p.desc, &alpha, w.data_ptr(), p.a, x.data_ptr(), p.b, &beta, cptr, p.c,
                              out.data_ptr(), p.d, algo, workspace.data_ptr(), ws,
                              c10::hip::getCurrentHIPStream().stream()));
  return true;
}

std::string hblt_kernel_name(int64_t index) {
  std::lock_guard<std::mutex> g(g_mu);
  int dev = 0;
  (void)hipGetDevice(&dev);
  Ctx& c = ctx_for(dev);
  list_all(c);
  auto a = c.by_index.find(static_cast<int>(index));
  if (a == c.by_index.end()) return "";
  return hipblaslt_ext::getKernelNameFromAlgo(c.h, a->second);
}

void register_hblt(pybind11::module_& m) {
  m.def("hblt_candidates", &hblt_candidates, pybind11::arg("M"), pybind11::arg("N"), pybind11::arg("K"),
        pybind11::arg("resid"), pybind11::arg("heuristic"), pybind11::arg("ws_max"));
  m.def("hblt_mm", &hblt_mm, pybind11::arg("out"), pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("resid"),
        pybind11::arg("index"), pybind11::arg("workspace"));
  m.def("hblt_kernel_name", &hblt_kernel_name);
}

}  // namespace mxs
