// How long was the round-4 custom all-reduce wait budget in wall-clock time?  It was a spin COUNT:
// 2^26 polls of a system-scope atomic load on uncached device memory, each followed by s_sleep 1.
// This times 2^20 such polls (one lane per block, like the waiters) on the device's constant clock
// and extrapolates to 2^26.  Build: hipcc --offload-arch=gfx950 -O3 car_spin_probe.hip -o car_spin_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void spin(unsigned* flag, unsigned long long* out, long iters) {
  if (threadIdx.x != 0) return;
  const long long t0 = wall_clock64();
  unsigned acc = 0;
  for (long i = 0; i < iters; ++i) {
    acc += __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_s_sleep(1);
  }
  const long long t1 = wall_clock64();
  out[blockIdx.x] = static_cast<unsigned long long>(t1 - t0) + (acc == 0xFFFFFFFFu ? 1 : 0);
}

int main() {
  unsigned* flag = nullptr;
  unsigned long long* out = nullptr;
  if (hipExtMallocWithFlags(reinterpret_cast<void**>(&flag), 4096, hipDeviceMallocUncached) != hipSuccess) return 1;
  if (hipMemset(flag, 0, 4096) != hipSuccess) return 1;
  if (hipMallocManaged(reinterpret_cast<void**>(&out), 256 * sizeof(unsigned long long)) != hipSuccess) return 1;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0) != hipSuccess || khz <= 0) khz = 100000;
  const long iters = 1L << 20;
  for (int blocks : {1, 64, 256}) {
    hipLaunchKernelGGL(spin, dim3(blocks), dim3(64), 0, 0, flag, out, iters);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    double mx = 0;
    for (int b = 0; b < blocks; ++b) mx = out[b] > mx ? out[b] : mx;
    const double ms = mx / khz;
    printf("{\"blocks\": %d, \"polls\": %ld, \"ms\": %.3f, \"ns_per_poll\": %.1f, \"round4_budget_2pow26_s\": %.2f}\n",
           blocks, iters, ms, ms * 1e6 / iters, ms * 64.0 / 1e3);
  }
  return 0;
}
