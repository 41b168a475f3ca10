// atomic_rate.hip -- device-scope atomicAdd-with-return on ONE address from many workgroups (the
// block queue a persistent sweep would use): per-op latency under contention and total rate.
//   hipcc --offload-arch=gfx950 -O2 -o tools/diag/atomic_rate tools/diag/atomic_rate.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void spin_add(unsigned long long* ctr, unsigned long long* sink, int ops, int gap) {
  if (threadIdx.x != 0) return;
  unsigned long long acc = 0;
  for (int i = 0; i < ops; ++i) {
    acc += atomicAdd(ctr, 1ull);
    for (int z = 0; z < gap; ++z) __builtin_amdgcn_s_sleep(127);
  }
  sink[blockIdx.x] = acc;
}

int main() {
  unsigned long long *ctr, *sink;
  hipMalloc(&ctr, 8);
  hipMalloc(&sink, 8 * 65536);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int wgs[] = {256, 1280, 5120};
  const int gaps[] = {0, 4};
  for (int g : gaps)
    for (int nwg : wgs) {
      const int ops = 200;
      hipMemset(ctr, 0, 8);
      hipLaunchKernelGGL(spin_add, dim3(nwg), dim3(256), 0, 0, ctr, sink, 4, g);  // warm
      hipDeviceSynchronize();
      hipEventRecord(a, 0);
      hipLaunchKernelGGL(spin_add, dim3(nwg), dim3(256), 0, 0, ctr, sink, ops, g);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const double total = (double)nwg * ops;
      printf("{\"wgs\": %d, \"gap_sleeps\": %d, \"ops\": %.0f, \"ms\": %.4f, \"Mops_per_s\": %.2f, \"ns_per_op_per_wg\": %.1f}\n",
             nwg, g, total, ms, total / (ms * 1e3), ms * 1e6 / ops);
    }
  return 0;
}
