// Host side of the KV transfer agent (replaces NIXL):
//   export_pool(tensor)        -> (64-byte hipIpcMemHandle, byte offset of the tensor in its allocation)
//   open_pool(handle, offset)  -> device pointer valid in THIS process (hipIpcOpenMemHandle, lazy
//                                 peer access: over xGMI when the pool lives on another GPU)
//   copy_blocks(dst_ptr, src, src_ids, dst_ids, block_bytes) -> one kernel on the current stream
// The decode worker exports its pool once; the prefill worker opens it once and pushes each
// request's blocks with a single launch.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>
#include <pybind11/stl.h>

namespace mxs {
void launch_copy_blocks(char*, const char*, const int*, const int*, int, long, hipStream_t);
constexpr int kArMaxRanks = 8;
struct ArPeers {  // custom_allreduce.hip
  char* recv[kArMaxRanks];
  unsigned* flags[kArMaxRanks];
  long long timeout_ticks;
};
void launch_custom_allreduce(unsigned short*, const unsigned short*, long, const ArPeers&, int, int, long, unsigned*,
                             hipStream_t);
void launch_custom_allreduce_2shot(unsigned short*, const unsigned short*, long, const ArPeers&, int, int, long,
                                   unsigned*, hipStream_t);
void launch_ipc_all_to_all(void*, const void*, long, const ArPeers&, int, int, long, unsigned*, hipStream_t,
                           const int*, long);
void launch_car_add_rmsnorm(unsigned short*, unsigned short*, const unsigned short*, const float*, int, int, int,
                            const unsigned short*, float, const ArPeers&, int, int, long, unsigned*, bool,
                            hipStream_t);
void launch_car_poll_err(unsigned*, const ArPeers&, int, hipStream_t);
void launch_ep_route(int*, int*, int*, const int*, int, int, int, int, int, int, hipStream_t);
void launch_ep_gather_rows(unsigned short*, const unsigned short*, const int*, int, int, int, int, hipStream_t);
void launch_ep_segment_rows(int*, const int*, int, int, hipStream_t);
}

namespace {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

pybind11::tuple export_pool(at::Tensor t) {
  TORCH_CHECK(t.is_cuda(), "pool must be a GPU tensor");
  void* ptr = t.data_ptr();
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  hip_check(hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(ptr)), "hipMemGetAddressRange");
  hipIpcMemHandle_t h;
  hip_check(hipIpcGetMemHandle(&h, base), "hipIpcGetMemHandle");
  const int64_t off = reinterpret_cast<char*>(ptr) - reinterpret_cast<char*>(base);
  return pybind11::make_tuple(pybind11::bytes(reinterpret_cast<const char*>(&h), sizeof(h)), off);
}

std::mutex g_mu;
// handle bytes -> (mapped base, users): every open_pool takes a reference and every close_handle
// drops one, so two users of one mapping in this process (a KV agent and the custom all-reduce, or
// two agents) cannot unmap it under each other; the last close unmaps
struct Mapping {
  void* base;
  int refs;
};
std::unordered_map<std::string, Mapping> g_open;

int64_t open_pool(const std::string& handle, int64_t offset) {
  TORCH_CHECK(handle.size() == sizeof(hipIpcMemHandle_t), "bad IPC handle size");
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_open.find(handle);
  void* base = nullptr;
  if (it != g_open.end()) {
    base = it->second.base;
    ++it->second.refs;
  } else {
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle.data(), sizeof(h));
    hip_check(hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    g_open.emplace(handle, Mapping{base, 1});
  }
  return reinterpret_cast<int64_t>(reinterpret_cast<char*>(base) + offset);
}

// Drop one reference to an opened handle; the mapping goes away with the last one.
void close_handle(const std::string& handle) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_open.find(handle);
  if (it == g_open.end()) return;
  if (--it->second.refs > 0) return;
  (void)hipIpcCloseMemHandle(it->second.base);
  g_open.erase(it);
}

int64_t open_refs(const std::string& handle) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_open.find(handle);
  return it == g_open.end() ? 0 : it->second.refs;
}

void close_all() {
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& kv : g_open) (void)hipIpcCloseMemHandle(kv.second.base);
  g_open.clear();
}

void copy_blocks(int64_t dst_ptr, at::Tensor src, at::Tensor src_ids, at::Tensor dst_ids, int64_t block_bytes) {
  TORCH_CHECK(src.is_cuda() && src_ids.is_cuda() && dst_ids.is_cuda(), "GPU tensors");
  TORCH_CHECK(src_ids.scalar_type() == at::kInt && dst_ids.scalar_type() == at::kInt, "int32 block ids");
  TORCH_CHECK(src_ids.numel() == dst_ids.numel(), "id count mismatch");
  TORCH_CHECK(block_bytes % 16 == 0, "block bytes must be a multiple of 16");
  mxs::launch_copy_blocks(reinterpret_cast<char*>(dst_ptr), reinterpret_cast<const char*>(src.data_ptr()),
                          src_ids.data_ptr<int>(), dst_ids.data_ptr<int>(), src_ids.numel(), block_bytes,
                          c10::hip::getCurrentHIPStream().stream());
}

// Custom all-reduce buffers: uncached device memory (peers write into it over xGMI and this rank
// polls / reads it without stale L2 lines), zeroed, exported for the peers.
pybind11::tuple car_alloc(int64_t bytes) {
  void* p = nullptr;
  hip_check(hipExtMallocWithFlags(&p, static_cast<size_t>(bytes), hipDeviceMallocUncached), "hipExtMallocWithFlags");
  hip_check(hipMemset(p, 0, static_cast<size_t>(bytes)), "hipMemset");
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  hipIpcMemHandle_t h;
  hip_check(hipIpcGetMemHandle(&h, p), "hipIpcGetMemHandle");
  return pybind11::make_tuple(reinterpret_cast<int64_t>(p),
                              pybind11::bytes(reinterpret_cast<const char*>(&h), sizeof(h)));
}

void car_free(int64_t ptr) { (void)hipFree(reinterpret_cast<void*>(ptr)); }

// Page-lock an existing host mapping (the /dev/shm KV staging arena shared by a prefill and a decode
// worker of one pod): DMA copies to/from it then run at full PCIe/Infinity-Fabric rate.
void host_register(int64_t ptr, int64_t bytes) {
  hip_check(hipHostRegister(reinterpret_cast<void*>(ptr), static_cast<size_t>(bytes), hipHostRegisterDefault),
            "hipHostRegister");
}
void host_unregister(int64_t ptr) { (void)hipHostUnregister(reinterpret_cast<void*>(ptr)); }

mxs::ArPeers make_peers(const std::vector<int64_t>& recv_ptrs, const std::vector<int64_t>& flag_ptrs,
                        int64_t timeout_ticks) {
  const int n = static_cast<int>(recv_ptrs.size());
  TORCH_CHECK(n >= 1 && n <= mxs::kArMaxRanks && static_cast<int>(flag_ptrs.size()) == n, "1..8 ranks");
  TORCH_CHECK(timeout_ticks > 0, "timeout_ticks must be positive");
  mxs::ArPeers peers{};
  for (int r = 0; r < n; ++r) {
    peers.recv[r] = reinterpret_cast<char*>(recv_ptrs[r]);
    peers.flags[r] = reinterpret_cast<unsigned*>(flag_ptrs[r]);
  }
  peers.timeout_ticks = timeout_ticks;
  return peers;
}

void custom_allreduce(at::Tensor out, at::Tensor x, std::vector<int64_t> recv_ptrs, std::vector<int64_t> flag_ptrs,
                      int64_t rank, int64_t slot_elems, int64_t epochs_ptr, int64_t timeout_ticks, bool two_shot) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous(), "x: contiguous bf16 GPU tensor");
  TORCH_CHECK(out.is_contiguous() && out.numel() == x.numel(), "out shape");
  const mxs::ArPeers peers = make_peers(recv_ptrs, flag_ptrs, timeout_ticks);
  const int n = static_cast<int>(recv_ptrs.size());
  TORCH_CHECK(rank >= 0 && rank < n, "rank out of range");
  TORCH_CHECK(x.numel() % 8 == 0 && x.numel() <= slot_elems, "numel must be a multiple of 8 and fit a slot");
  auto launch = two_shot ? mxs::launch_custom_allreduce_2shot : mxs::launch_custom_allreduce;
  launch(reinterpret_cast<unsigned short*>(out.data_ptr()), reinterpret_cast<const unsigned short*>(x.data_ptr()),
         x.numel(), peers, static_cast<int>(rank), n, slot_elems, reinterpret_cast<unsigned*>(epochs_ptr),
         c10::hip::getCurrentHIPStream().stream());
}

// Every rank's error word -> out (uint32 [>= n], host-pinned), ordered on the current stream.
void car_poll_err(at::Tensor out, std::vector<int64_t> recv_ptrs, std::vector<int64_t> flag_ptrs) {
  TORCH_CHECK(out.is_pinned() && out.scalar_type() == at::kInt && out.numel() >= static_cast<int64_t>(flag_ptrs.size()),
              "out: pinned int32 [>= ranks]");
  const mxs::ArPeers peers = make_peers(recv_ptrs, flag_ptrs, 1);
  void* dev = nullptr;
  hip_check(hipHostGetDevicePointer(&dev, out.data_ptr(), 0), "hipHostGetDevicePointer");
  mxs::launch_car_poll_err(static_cast<unsigned*>(dev), peers, static_cast<int>(flag_ptrs.size()),
                           c10::hip::getCurrentHIPStream().stream());
}

// n consecutive uint32 words of device memory (a signal page's error word / give-up record), read
// synchronously: fault diagnosis and tests only, never on the step loop.
std::vector<int64_t> car_read_words(int64_t ptr, int64_t n) {
  TORCH_CHECK(n > 0 && n <= 4096, "1..4096 words");
  std::vector<unsigned> v(static_cast<size_t>(n), 0u);
  hip_check(hipMemcpy(v.data(), reinterpret_cast<void*>(ptr), sizeof(unsigned) * n, hipMemcpyDeviceToHost),
            "hipMemcpy");
  return std::vector<int64_t>(v.begin(), v.end());
}

// Zero n bytes of this rank's signal page (epochs, flags, error word, records) after every rank
// has quiesced: the collective restarts from epoch 1 everywhere.
void car_clear(int64_t ptr, int64_t bytes) {
  hip_check(hipMemset(reinterpret_cast<void*>(ptr), 0, static_cast<size_t>(bytes)), "hipMemset");
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
}

// Wall-clock counter rate of the device (kHz): converts the wait budget to device ticks.
int64_t car_wall_clock_khz() {
  int dev = 0, khz = 0;
  hip_check(hipGetDevice(&dev), "hipGetDevice");
  hip_check(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev), "hipDeviceGetAttribute");
  return khz > 0 ? khz : 100000;
}

// A HIP stream restricted to a subset of the CUs (hipExtStreamCreateWithCUMask): bit i of the mask
// words enables CU i.  Used to run bandwidth-bound and compute-bound kernels side by side on disjoint
// CU sets (mxserve/engine/cu_partition.py); torch wraps the handle with torch.cuda.ExternalStream.
int64_t cu_mask_stream(std::vector<int64_t> mask_words) {
  std::vector<uint32_t> m(mask_words.begin(), mask_words.end());
  hipStream_t s = nullptr;
  hip_check(hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(m.size()), m.data()),
            "hipExtStreamCreateWithCUMask");
  return reinterpret_cast<int64_t>(s);
}

std::vector<int64_t> stream_cu_mask(int64_t stream, int64_t words) {
  std::vector<uint32_t> m(static_cast<size_t>(words), 0u);
  hip_check(hipExtStreamGetCUMask(reinterpret_cast<hipStream_t>(stream), static_cast<uint32_t>(words), m.data()),
            "hipExtStreamGetCUMask");
  return std::vector<int64_t>(m.begin(), m.end());
}

void stream_destroy(int64_t stream) { (void)hipStreamDestroy(reinterpret_cast<hipStream_t>(stream)); }

// Fused TP epilogue: h = RMSNorm(residual += AllReduce(partial)) * w.  The partial is x (bf16 [M, H])
// or part (fp32 split-K slabs [S][M][H]); residual [M, H] is updated in place.
void car_add_rms_norm(at::Tensor h, at::Tensor residual, c10::optional<at::Tensor> x, c10::optional<at::Tensor> part,
                      at::Tensor w, double eps, std::vector<int64_t> recv_ptrs, std::vector<int64_t> flag_ptrs,
                      int64_t rank, int64_t slot_elems, int64_t epochs_ptr, int64_t timeout_ticks, bool two_shot) {
  TORCH_CHECK(residual.is_cuda() && residual.scalar_type() == at::kBFloat16 && residual.is_contiguous() &&
                  residual.dim() == 2, "residual: contiguous bf16 [M, H] GPU tensor");
  const int M = residual.size(0), H = residual.size(1);
  TORCH_CHECK(h.is_contiguous() && h.scalar_type() == at::kBFloat16 && h.numel() == residual.numel(), "h shape");
  TORCH_CHECK(w.is_contiguous() && w.scalar_type() == at::kBFloat16 && w.numel() == H, "w: bf16 [H]");
  TORCH_CHECK(H % 8 == 0 && H <= 16384, "H must be a multiple of 8, at most 16384");
  TORCH_CHECK(static_cast<int64_t>(M) * H <= slot_elems, "M * H must fit a slot");
  TORCH_CHECK(x.has_value() != part.has_value(), "exactly one of x (bf16 partial) / part (fp32 slabs)");
  const unsigned short* xp = nullptr;
  const float* pp = nullptr;
  int S = 1;
  if (x.has_value()) {
    TORCH_CHECK(x->is_contiguous() && x->scalar_type() == at::kBFloat16 && x->numel() == residual.numel(), "x shape");
    xp = reinterpret_cast<const unsigned short*>(x->data_ptr());
  } else {
    TORCH_CHECK(part->is_contiguous() && part->scalar_type() == at::kFloat && part->numel() % residual.numel() == 0,
                "part: fp32 [S, M, H]");
    S = static_cast<int>(part->numel() / residual.numel());
    TORCH_CHECK(S >= 1, "at least one slab");
    pp = part->data_ptr<float>();
  }
  const mxs::ArPeers peers = make_peers(recv_ptrs, flag_ptrs, timeout_ticks);
  const int n = static_cast<int>(recv_ptrs.size());
  TORCH_CHECK(rank >= 0 && rank < n, "rank out of range");
  if (M == 0) return;
  mxs::launch_car_add_rmsnorm(reinterpret_cast<unsigned short*>(h.data_ptr()),
                              reinterpret_cast<unsigned short*>(residual.data_ptr()), xp, pp, S, M, H,
                              reinterpret_cast<const unsigned short*>(w.data_ptr()), static_cast<float>(eps), peers,
                              static_cast<int>(rank), n, slot_elems, reinterpret_cast<unsigned*>(epochs_ptr), two_shot,
                              c10::hip::getCurrentHIPStream().stream());
}

// equal splits: out/in hold N segments of seg_bytes each; segment d of `in` goes to rank d
void ipc_all_to_all(at::Tensor out, at::Tensor in, std::vector<int64_t> recv_ptrs, std::vector<int64_t> flag_ptrs,
                    int64_t rank, int64_t slot_bytes, int64_t epochs_ptr, int64_t timeout_ticks,
                    c10::optional<at::Tensor> push_rows, int64_t row_bytes) {
  TORCH_CHECK(in.is_cuda() && in.is_contiguous() && out.is_contiguous(), "contiguous GPU tensors");
  TORCH_CHECK(in.scalar_type() == out.scalar_type() && in.numel() == out.numel(), "in/out shape");
  const mxs::ArPeers peers = make_peers(recv_ptrs, flag_ptrs, timeout_ticks);
  const int n = static_cast<int>(recv_ptrs.size());
  TORCH_CHECK(rank >= 0 && rank < n, "rank out of range");
  const long bytes = in.numel() * in.element_size();
  TORCH_CHECK(bytes % n == 0, "equal splits");
  const long seg = bytes / n;
  TORCH_CHECK(seg % 4 == 0 && seg <= slot_bytes, "segment must be a multiple of 4 bytes and fit a slot");
  const int* pr = nullptr;
  if (push_rows.has_value()) {
    const at::Tensor& t = *push_rows;
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kInt && t.numel() == n && t.is_contiguous(),
                "push_rows: int32 GPU tensor, one count per rank");
    TORCH_CHECK(row_bytes > 0 && seg % row_bytes == 0 && row_bytes % 4 == 0, "row_bytes must divide the segment");
    pr = t.data_ptr<int>();
  }
  mxs::launch_ipc_all_to_all(out.data_ptr(), in.data_ptr(), seg, peers, static_cast<int>(rank), n, slot_bytes,
                             reinterpret_cast<unsigned*>(epochs_ptr), c10::hip::getCurrentHIPStream().stream(), pr,
                             row_bytes);
}

// ---- EP dispatch (csrc/kernels/ep.hip)
void ep_route(at::Tensor slot, at::Tensor send_e, at::Tensor counts, at::Tensor topk_ids, int64_t valid_rows,
              int64_t e_local, int64_t nranks, int64_t C) {
  TORCH_CHECK(topk_ids.is_cuda() && topk_ids.scalar_type() == at::kInt && topk_ids.dim() == 2 &&
                  topk_ids.is_contiguous(), "topk_ids: int32 [S, k] GPU tensor");
  const int P = topk_ids.numel(), k = topk_ids.size(1);
  TORCH_CHECK(nranks >= 1 && nranks <= 8 && e_local >= 1 && C >= 0, "1..8 ranks");
  TORCH_CHECK(slot.scalar_type() == at::kInt && slot.numel() == P, "slot: int32 [P]");
  TORCH_CHECK(send_e.scalar_type() == at::kInt && send_e.numel() == nranks * C, "send_e: int32 [nranks * C]");
  TORCH_CHECK(counts.scalar_type() == at::kInt && counts.numel() == nranks, "counts: int32 [nranks]");
  mxs::launch_ep_route(slot.data_ptr<int>(), send_e.data_ptr<int>(), counts.data_ptr<int>(), topk_ids.data_ptr<int>(),
                       P, k, static_cast<int>(valid_rows), static_cast<int>(e_local), static_cast<int>(nranks),
                       static_cast<int>(C), c10::hip::getCurrentHIPStream().stream());
}

void ep_gather_rows(at::Tensor send_x, at::Tensor hs, at::Tensor slot, int64_t k) {
  TORCH_CHECK(send_x.is_cuda() && hs.is_cuda() && slot.is_cuda(), "GPU tensors");
  TORCH_CHECK(send_x.scalar_type() == at::kBFloat16 && hs.scalar_type() == at::kBFloat16, "bf16 rows");
  TORCH_CHECK(send_x.is_contiguous() && hs.is_contiguous() && slot.scalar_type() == at::kInt, "layout");
  const int H = hs.size(1);
  TORCH_CHECK(H % 8 == 0 && send_x.size(1) == H && slot.numel() == hs.size(0) * k, "shapes");
  mxs::launch_ep_gather_rows(reinterpret_cast<unsigned short*>(send_x.data_ptr()),
                             reinterpret_cast<const unsigned short*>(hs.data_ptr()), slot.data_ptr<int>(),
                             static_cast<int>(slot.numel()), static_cast<int>(k), H,
                             static_cast<int>(send_x.size(0)), c10::hip::getCurrentHIPStream().stream());
}

void ep_segment_rows(at::Tensor counts, at::Tensor ids, int64_t C) {
  TORCH_CHECK(ids.is_cuda() && ids.scalar_type() == at::kInt && counts.scalar_type() == at::kInt, "int32 GPU");
  const int nseg = counts.numel();
  TORCH_CHECK(ids.numel() == nseg * C, "ids: [nseg * C]");
  mxs::launch_ep_segment_rows(counts.data_ptr<int>(), ids.data_ptr<int>(), nseg, static_cast<int>(C),
                              c10::hip::getCurrentHIPStream().stream());
}

}  // namespace

void register_comm(pybind11::module_& m) {
  m.def("car_alloc", &car_alloc);
  m.def("car_free", &car_free);
  m.def("car_read_words", &car_read_words);
  m.def("car_clear", &car_clear);
  m.def("car_wall_clock_khz", &car_wall_clock_khz);
  m.def("car_poll_err", &car_poll_err);
  m.def("host_register", &host_register);
  m.def("host_unregister", &host_unregister);
  m.def("custom_allreduce", &custom_allreduce, pybind11::arg("out"), pybind11::arg("x"), pybind11::arg("recv_ptrs"),
        pybind11::arg("flag_ptrs"), pybind11::arg("rank"), pybind11::arg("slot_elems"), pybind11::arg("epochs_ptr"),
        pybind11::arg("timeout_ticks"), pybind11::arg("two_shot") = false);
  m.def("cu_mask_stream", &cu_mask_stream);
  m.def("stream_cu_mask", &stream_cu_mask);
  m.def("stream_destroy", &stream_destroy);
  m.def("car_add_rms_norm", &car_add_rms_norm, pybind11::arg("h"), pybind11::arg("residual"), pybind11::arg("x"),
        pybind11::arg("part"), pybind11::arg("w"), pybind11::arg("eps"), pybind11::arg("recv_ptrs"),
        pybind11::arg("flag_ptrs"), pybind11::arg("rank"), pybind11::arg("slot_elems"), pybind11::arg("epochs_ptr"),
        pybind11::arg("timeout_ticks"), pybind11::arg("two_shot") = false);
  m.def("ipc_all_to_all", &ipc_all_to_all, pybind11::arg("out"), pybind11::arg("in"), pybind11::arg("recv_ptrs"),
        pybind11::arg("flag_ptrs"), pybind11::arg("rank"), pybind11::arg("slot_bytes"), pybind11::arg("epochs_ptr"),
        pybind11::arg("timeout_ticks"), pybind11::arg("push_rows") = pybind11::none(), pybind11::arg("row_bytes") = 0);
  m.def("ep_route", &ep_route);
  m.def("ep_gather_rows", &ep_gather_rows);
  m.def("ep_segment_rows", &ep_segment_rows);
  m.def("ipc_export_pool", &export_pool);
  // may block on the peer driver: let watchdog threads run meanwhile
  m.def("ipc_open_pool", &open_pool, pybind11::call_guard<pybind11::gil_scoped_release>());
  m.def("ipc_close_all", &close_all);
  m.def("ipc_close", &close_handle);
  m.def("ipc_open_refs", &open_refs);
  m.def("copy_blocks", &copy_blocks);
}
