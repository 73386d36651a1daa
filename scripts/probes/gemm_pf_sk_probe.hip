// Stream-K cost probe for gemm_pf (csrc/kernels/gemm_pf.hip), standalone (no torch): times one shape
// at data-parallel (min_iters 0) and stream-K (min_iters 8) settings with hipEvents.  Built twice by
// the caller: as is, and with -DPF_PROBE_NO_FIXUP (the stream-K hand-off compiled out: wrong results,
// the schedule's own time) to price the fixup.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc/kernels gemm_pf_sk_probe.hip -o probe
//   ./probe M N K
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../csrc/kernels/gemm_pf.hip"

static void check(hipError_t e, const char* w) {
  if (e != hipSuccess) {
    fprintf(stderr, "%s: %s\n", w, hipGetErrorString(e));
    exit(1);
  }
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 6656, N = argc > 2 ? atoi(argv[2]) : 2048, K = argc > 3 ? atoi(argv[3]) : 8192;
  int dev = 0, ncu = 0;
  check(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev), "attr");
  mxs::bf16_t *X, *W, *Y;
  float* slab;
  int *cnt, *map;
  check(hipMalloc(&X, sizeof(mxs::bf16_t) * M * K), "X");
  check(hipMalloc(&W, sizeof(mxs::bf16_t) * N * K), "W");
  check(hipMalloc(&Y, sizeof(mxs::bf16_t) * M * N), "Y");
  const long slab_floats = 2L * ncu * mxs::PF_SLAB_FRAGS * 512 * 4;
  check(hipMalloc(&slab, sizeof(float) * slab_floats), "slab");
  check(hipMalloc(&cnt, sizeof(int) * 65536), "cnt");
  check(hipMemset(cnt, 0, sizeof(int) * 65536), "cnt0");
  check(hipMemset(X, 0x3c, sizeof(mxs::bf16_t) * M * K), "Xfill");
  check(hipMemset(W, 0x3c, sizeof(mxs::bf16_t) * N * K), "Wfill");
  const int ntn = N / 256;
  check(hipMalloc(&map, sizeof(int) * 65536), "map");
  hipEvent_t e0, e1;
  check(hipEventCreate(&e0), "ev");
  check(hipEventCreate(&e1), "ev");
  for (int trows : {256, 192, 160, 128})
  for (int mi : {0, 8}) {
    const int ntm = (M + trows - 1) / trows;
    std::vector<int> hmap(ntm * ntn);
    const int gm = 8;  // ops.pf_tile_map: GM token tiles per weight-column sweep
    for (int L = 0; L < ntm * ntn; ++L) {
      const int per = gm * ntn, grp = L / per, first = grp * gm, gsz = std::min(ntm - first, gm), ing = L - grp * per;
      hmap[L] = (first + ing % gsz) | ((ing / gsz) << 16);
    }
    check(hipMemcpy(map, hmap.data(), sizeof(int) * hmap.size(), hipMemcpyHostToDevice), "mapcpy");
    int dp, sk, G;
    mxs::pf_plan(M, N, K, 0, ncu, mi, &dp, &sk, &G, trows);
    auto run = [&]() {
      if (!mxs::launch_gemm_pf(Y, X, W, M, N, K, K, N, 0, slab, slab_floats, cnt, 65536, map, ntm * ntn, ncu, mi, 0,
                               nullptr, 0, false, 1e-5f, trows))
        exit(2);
    };
    for (int i = 0; i < 5; ++i) run();
    check(hipDeviceSynchronize(), "warm");
    check(hipEventRecord(e0, 0), "rec");
    const int it = 20;
    for (int i = 0; i < it; ++i) run();
    check(hipEventRecord(e1, 0), "rec");
    check(hipEventSynchronize(e1), "sync");
    float ms = 0;
    check(hipEventElapsedTime(&ms, e0, e1), "el");
    const double us = ms * 1e3 / it;
    printf("{\"M\": %d, \"N\": %d, \"K\": %d, \"trows\": %d, \"min_iters\": %d, \"grid\": %d, \"dp_rounds\": %d, \"sk_tiles\": %d, "
           "\"us\": %.2f, \"TF\": %.1f, \"fixup\": %s}\n",
           M, N, K, trows, mi, G, dp, sk, us, 2.0 * M * N * K / us / 1e6,
#ifdef PF_PROBE_NO_FIXUP
           "false"
#else
           "true"
#endif
    );
  }
  return 0;
}
