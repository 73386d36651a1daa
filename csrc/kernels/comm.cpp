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

namespace mxs {
void launch_copy_blocks(char*, const char*, const int*, const int*, int, long, hipStream_t);
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
std::unordered_map<std::string, void*> g_open;  // handle bytes -> mapped base

int64_t open_pool(const std::string& handle, int64_t offset) {
  TORCH_CHECK(handle.size() == sizeof(hipIpcMemHandle_t), "bad IPC handle size");
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_open.find(handle);
  void* base = nullptr;
  if (it != g_open.end()) {
    base = it->second;
  } else {
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle.data(), sizeof(h));
    hip_check(hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    g_open.emplace(handle, base);
  }
  return reinterpret_cast<int64_t>(reinterpret_cast<char*>(base) + offset);
}

void close_all() {
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& kv : g_open) (void)hipIpcCloseMemHandle(kv.second);
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

}  // namespace

void register_comm(pybind11::module_& m) {
  m.def("ipc_export_pool", &export_pool);
  m.def("ipc_open_pool", &open_pool);
  m.def("ipc_close_all", &close_all);
  m.def("copy_blocks", &copy_blocks);
}
