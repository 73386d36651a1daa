// K19: KV-block copy between two paged pools (local->local or local->peer-mapped over xGMI).
// One workgroup per block pair; 16-byte vector loads/stores.  The destination may be an IPC-opened
// allocation on another GPU (hipIpcOpenMemHandle): stores from this GPU then travel over xGMI
// (push model: the prefill GPU writes straight into the decode GPU's KV pool).
#include "common.h"

namespace mxs {

__global__ void __launch_bounds__(256) copy_blocks_kernel(char* __restrict__ dst, const char* __restrict__ src,
                                                          const int* __restrict__ src_ids,
                                                          const int* __restrict__ dst_ids, long block_bytes) {
  MXS_KCHECK(src_ids[blockIdx.x] >= 0 && dst_ids[blockIdx.x] >= 0);
  // the source may have been written by ANOTHER GPU over xGMI (a decode worker landing its staging
  // arena after the prefill GPU's push, published through the host): acquire at system scope so no
  // stale line of an earlier use of the arena is read from this GPU's caches
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const long s = static_cast<long>(src_ids[blockIdx.x]) * block_bytes;
  const long d = static_cast<long>(dst_ids[blockIdx.x]) * block_bytes;
  const uint4* sp = reinterpret_cast<const uint4*>(src + s);
  uint4* dp = reinterpret_cast<uint4*>(dst + d);
  const long n = block_bytes >> 4;
  long i = threadIdx.x;
  // 4 independent 16-byte loads in flight per thread before the stores
  for (; i + 3 * 256 < n; i += 4 * 256) {
    const uint4 a = sp[i], b = sp[i + 256], c = sp[i + 512], e = sp[i + 768];
    dp[i] = a;
    dp[i + 256] = b;
    dp[i + 512] = c;
    dp[i + 768] = e;
  }
  for (; i < n; i += 256) dp[i] = sp[i];
  // the destination may be another GPU's memory: make the stores visible at system scope before this
  // wave retires, so the host's completion of the launch means the peer can read them
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

void launch_copy_blocks(char* dst, const char* src, const int* src_ids, const int* dst_ids, int n,
                        long block_bytes, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(copy_blocks_kernel, dim3(n), dim3(256), 0, s, dst, src, src_ids, dst_ids, block_bytes);
  MXS_CHECK_LAUNCH();
}

}  // namespace mxs
