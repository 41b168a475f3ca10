// cumask_probe.hip -- which CUs the workgroups of a CU-masked stream (hipExtStreamCreateWithCUMask) run
// on, on a multi-XCD MI355X: does a mask of 32 CUs keep a kernel on one XCD, and do 8 streams with
// disjoint masks run side by side?  (Round 5: a rehearsal of run()'s pieces on separate devices, each
// piece on its own slice of one GPU.)  Every wait is bounded; a kernel that does not finish in 20 s is
// reported and the process exits.
//   hipcc --offload-arch=gfx950 -O2 -o tools/diag/cumask_probe tools/diag/cumask_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>
#include <chrono>
#include <map>
#include <set>
#include <thread>
#include <vector>

__global__ __launch_bounds__(256) void probe(uint32_t* out, uint32_t spin) {
  const uint32_t hw = __builtin_amdgcn_s_getreg((31u << 11) | (0u << 6) | 4u);   // HW_REG_HW_ID
  const uint32_t xcc = __builtin_amdgcn_s_getreg((15u << 11) | (0u << 6) | 20u); // HW_REG_XCC_ID
  uint32_t x = threadIdx.x;
  for (uint32_t i = 0; i < spin; ++i) x = x * 1664525u + 1013904223u;
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = (xcc & 0xF) | (x & 0x80000000u);
  }
}

static bool wait(hipStream_t s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return true;
    if (e != hipErrorNotReady) {
      printf("{\"error\": \"%s\"}\n", hipGetErrorString(e));
      return false;
    }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(20)) {
      printf("{\"error\": \"kernel did not finish in 20 s\"}\n");
      fflush(stdout);
      _exit(3);
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int nwg = 1024;
  const uint32_t spin = 200000;
  std::vector<uint32_t*> d(8);
  for (auto& p : d)
    if (hipMalloc(&p, nwg * 2 * 4) != hipSuccess) return 1;
  auto report = [&](const char* name, int k, uint32_t* dp, double ms) {
    std::vector<uint32_t> h(nwg * 2);
    hipMemcpy(h.data(), dp, h.size() * 4, hipMemcpyDeviceToHost);
    std::set<uint32_t> cus;
    std::map<uint32_t, int> per_xcc;
    for (int g = 0; g < nwg; ++g) {
      const uint32_t hw = h[2 * g], xcc = h[2 * g + 1] & 0xF;
      cus.insert((xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15));
      per_xcc[xcc]++;
    }
    printf("{\"mode\": \"%s\", \"stream\": %d, \"ms\": %.3f, \"distinct_cus\": %zu, \"wg_per_xcc\": {", name, k, ms,
           cus.size());
    bool first = true;
    for (auto& x : per_xcc) {
      printf("%s\"%u\": %d", first ? "" : ", ", x.first, x.second);
      first = false;
    }
    printf("}}\n");
    fflush(stdout);
  };
  // the whole GPU on a plain stream, for the timing reference
  {
    hipStream_t s;
    hipStreamCreate(&s);
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(probe, dim3(nwg), dim3(256), 0, s, d[0], spin);
    if (!wait(s)) return 1;
    report("unmasked", 0, d[0], std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    hipStreamDestroy(s);
  }
  const int words = (ncu + 31) / 32;
  for (int mode = 0; mode < 2; ++mode) {
    // mode 0: CUs [32k, 32k + 32); mode 1: CUs k, k + 8, k + 16, ...
    std::vector<hipStream_t> st(8);
    for (int k = 0; k < 8; ++k) {
      std::vector<uint32_t> m(words, 0);
      for (int c = 0; c < ncu; ++c)
        if (mode == 0 ? c / (ncu / 8) == k : c % 8 == k) m[c / 32] |= 1u << (c % 32);
      const hipError_t e = hipExtStreamCreateWithCUMask(&st[k], (uint32_t)words, m.data());
      if (e != hipSuccess) {
        printf("{\"mode\": %d, \"error\": \"hipExtStreamCreateWithCUMask: %s\"}\n", mode, hipGetErrorString(e));
        return 1;
      }
    }
    // one masked stream alone
    auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(probe, dim3(nwg), dim3(256), 0, st[0], d[0], spin);
    if (!wait(st[0])) return 1;
    report(mode ? "strided_alone" : "block_alone", 0, d[0],
           std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    // eight at once
    t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < 8; ++k) hipLaunchKernelGGL(probe, dim3(nwg), dim3(256), 0, st[k], d[k], spin);
    for (int k = 0; k < 8; ++k)
      if (!wait(st[k])) return 1;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (int k = 0; k < 8; ++k) report(mode ? "strided_8" : "block_8", k, d[k], ms);
    for (auto& s : st) hipStreamDestroy(s);
  }
  return 0;
}
