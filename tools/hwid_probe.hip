// hwid_probe.hip -- where the waves of a 1024-thread workgroup run: HW_ID (SIMD, CU, SE) and XCC_ID of
// every wave of a 256-workgroup launch with the binned verification kernel's shape (96 KiB of LDS,
// so one workgroup per CU).  Prints per-workgroup counts of waves per SIMD id and a CU histogram.
//   hipcc --offload-arch=gfx950 -O2 -o tools/hwid_probe tools/hwid_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <map>
#include <vector>

__global__ __launch_bounds__(1024) void probe(uint32_t* out, uint32_t spin) {
  __shared__ uint32_t lds[(96u << 10) / 4];
  if (threadIdx.x < 4) lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const uint32_t hw = __builtin_amdgcn_s_getreg((31u << 11) | (0u << 6) | 4u);   // HW_REG_HW_ID, all 32 bits
  const uint32_t xcc = __builtin_amdgcn_s_getreg((15u << 11) | (0u << 6) | 20u); // HW_REG_XCC_ID
  uint32_t x = lds[threadIdx.x & 3];
  for (uint32_t i = 0; i < spin; ++i) x = x * 1664525u + 1013904223u;  // keep every wave resident a while
  if ((threadIdx.x & 63) == 0) {
    const uint32_t w = blockIdx.x * 16 + threadIdx.x / 64;
    out[2 * w] = hw;
    out[2 * w + 1] = xcc | (x & 0x80000000u);
  }
}

int main() {
  const int nwg = 256;
  uint32_t* d;
  if (hipMalloc(&d, nwg * 16 * 2 * 4) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(nwg), dim3(1024), 0, 0, d, 200000u);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::vector<uint32_t> h(nwg * 16 * 2);
  if (hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  std::map<std::vector<int>, int> patterns;
  std::map<uint64_t, int> cus;  // (xcc, se, sh, cu) -> workgroups
  for (int g = 0; g < nwg; ++g) {
    std::vector<int> per(4, 0);
    uint64_t key = 0;
    for (int w = 0; w < 16; ++w) {
      const uint32_t hw = h[2 * (g * 16 + w)], xcc = h[2 * (g * 16 + w) + 1] & 0xF;
      per[(hw >> 4) & 3]++;
      key = ((uint64_t)xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15);
    }
    patterns[per]++;
    cus[key]++;
    if (g < 4) {
      printf("wg %d:", g);
      for (int w = 0; w < 16; ++w) printf(" %u", (h[2 * (g * 16 + w)] >> 4) & 3);
      printf("\n");
    }
  }
  for (auto& p : patterns) printf("waves per SIMD id {%d,%d,%d,%d}: %d workgroups\n", p.first[0], p.first[1],
                                  p.first[2], p.first[3], p.second);
  int maxc = 0;
  for (auto& c : cus) maxc = c.second > maxc ? c.second : maxc;
  printf("distinct CUs: %zu, most workgroups on one CU: %d\n", cus.size(), maxc);
  return 0;
}
