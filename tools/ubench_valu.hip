// ubench_valu.hip -- measured issue rate of the integer VALU instructions the trial
// function is built from, on the MI355X it runs on.  Establishes the integer-op peak
// used for the roofline in DESIGN.md (the guides list only the FP32 vector peak).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_valu tools/ubench_valu.hip
//   ./tools/ubench_valu            (prints one JSON line per instruction)
//
// Each kernel runs NCH independent dependency chains per lane (ILP) at full occupancy
// (2048 blocks x 256 threads), instruction pinned by inline asm.  lane-ops/s =
// threads x ITERS x UNROLL x NCH / time.  The in-kernel clock comes from
// s_memtime / s_memrealtime (100 MHz) around the loop on block 0.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 2048;
constexpr int UNROLL = 8;

#define CHAINS8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ __launch_bounds__(256) void kern(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, a5 = a0 * 11,
           a6 = a0 * 13, a7 = a0 * 15;
  uint32_t b = seed * 17 + threadIdx.x, c = seed * 29 + blockIdx.x;
  uint32_t h0 = a0 * 19, h1 = a0 * 21, h2 = a0 * 23, h3 = a0 * 25, h4 = a0 * 27, h5 = a0 * 29,
           h6 = a0 * 31, h7 = a0 * 33;
  uint64_t q0 = a0, q1 = a1, q2 = a2, q3 = a3, q4 = a4, q5 = a5, q6 = a6, q7 = a7;
  uint64_t qb = ((uint64_t)b << 32) | c;
  uint64_t t0 = 0, r0 = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if constexpr (OP == 0) {
#define X(i) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a##i) : "v"(b));
        CHAINS8(X)
#undef X
      } else if constexpr (OP == 1) {
#define X(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a##i) : "v"(b));
        CHAINS8(X)
#undef X
      } else if constexpr (OP == 2) {
#define X(i) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a##i) : "v"(b), "v"(c));
        CHAINS8(X)
#undef X
      } else if constexpr (OP == 3) {
#define X(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(q##i) : "v"(qb));
        CHAINS8(X)
#undef X
      } else if constexpr (OP == 4) {
        // 64-bit add as a carry pair: counts as 2 instructions per chain step
#define X(i) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %2, vcc, %2, %3, vcc" \
                          : "+v"(a##i), "+v"(h##i) : "v"(b), "v"(b) : "vcc");
        CHAINS8(X)
#undef X
      } else if constexpr (OP == 5) {
#define X(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##i) : "v"(b));
        CHAINS8(X)
#undef X
      } else if constexpr (OP == 6) {
#define X(i) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(a##i) : "v"(b), "v"(c));
        CHAINS8(X)
#undef X
      } else if constexpr (OP == 7) {
#define X(i) asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(q##i));
        CHAINS8(X)
#undef X
      } else if constexpr (OP == 8) {
#define X(i) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a##i) : "v"(b), "v"(c));
        CHAINS8(X)
#undef X
      } else if constexpr (OP == 9) {
        // alignbit with an SGPR operand (constant-bus read)
        uint32_t sb = __builtin_amdgcn_readfirstlane(b);
#define X(i) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a##i) : "s"(sb));
        CHAINS8(X)
#undef X
      } else if constexpr (OP == 11) {
        // the address search's field products: 32x32 -> 64 multiply-add
        uint64_t cc;
#define X(i) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(q##i), "=s"(cc) : "v"(b), "v"(c));
        CHAINS8(X)
#undef X
      } else if constexpr (OP == 12) {
#define X(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a##i) : "v"(b));
        CHAINS8(X)
#undef X
      } else if constexpr (OP == 13) {
#define X(i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(q##i) : "v"(qb), "v"(qb));
        CHAINS8(X)
#undef X
      } else if constexpr (OP == 10) {
#define X(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %2\n\tv_alignbit_b32 %1, %1, %3, 7" \
                          : "+v"(q##i), "+v"(a##i) : "v"(qb), "v"(b));
        CHAINS8(X)
#undef X
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  uint32_t s = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ c ^ h0 ^ h1 ^ h2 ^ h3 ^ h4 ^ h5 ^ h6 ^ h7;
  s ^= (uint32_t)(q0 ^ q1 ^ q2 ^ q3 ^ q4 ^ q5 ^ q6 ^ q7) ^ (uint32_t)((q0 + q7) >> 32);
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
int run(const char* name, int instr_per_step, int blocks, uint32_t* dout, uint64_t* dclk) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, dout, dclk, 1u);  // warm-up
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  uint64_t clk[2] = {0, 0};
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, dout, dclk, 2u + r);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) {
      best = ms;
      CHECK(hipMemcpy(clk, dclk, sizeof clk, hipMemcpyDeviceToHost));
    }
  }
  const double lane_ops = (double)blocks * 256 * ITERS * UNROLL * 8 * instr_per_step;
  const double ghz = clk[1] ? (double)clk[0] / (double)clk[1] * 0.1 : 0.0;
  printf("{\"instr\": \"%s\", \"ms\": %.3f, \"T_lane_ops_per_s\": %.2f, \"clock_ghz\": %.3f, "
         "\"lane_ops_per_clk_per_cu\": %.1f}\n",
         name, best, lane_ops / (best * 1e-3) / 1e12, ghz,
         ghz > 0 ? lane_ops / (best * 1e-3) / (ghz * 1e9) / 256.0 : 0.0);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  printf("{\"device\": \"%s\", \"arch\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", p.name, p.gcnArchName,
         p.multiProcessorCount, p.clockRate);
  const int blocks = p.multiProcessorCount * 8 * 4;  // 8 blocks/CU x 4 rounds
  uint32_t* dout;
  uint64_t* dclk;
  CHECK(hipMalloc(&dout, (size_t)blocks * 256 * 4));
  CHECK(hipMalloc(&dclk, 16));
  int rc = 0;
  rc |= run<0>("v_alignbit_b32", 1, blocks, dout, dclk);
  rc |= run<1>("v_xor_b32", 1, blocks, dout, dclk);
  rc |= run<2>("v_bitop3_b32", 1, blocks, dout, dclk);
  rc |= run<3>("v_lshl_add_u64", 1, blocks, dout, dclk);
  rc |= run<4>("v_add_co_u32+v_addc_co_u32 (per instr)", 2, blocks, dout, dclk);
  rc |= run<5>("v_add_u32", 1, blocks, dout, dclk);
  rc |= run<6>("v_bfi_b32", 1, blocks, dout, dclk);
  rc |= run<7>("v_lshrrev_b64", 1, blocks, dout, dclk);
  rc |= run<8>("v_add3_u32", 1, blocks, dout, dclk);
  rc |= run<9>("v_alignbit_b32 (sgpr operand)", 1, blocks, dout, dclk);
  rc |= run<10>("v_lshl_add_u64+v_alignbit_b32 (per instr)", 2, blocks, dout, dclk);
  rc |= run<11>("v_mad_u64_u32", 1, blocks, dout, dclk);
  rc |= run<12>("v_mul_lo_u32", 1, blocks, dout, dclk);
  rc |= run<13>("v_fma_f64", 1, blocks, dout, dclk);
  CHECK(hipFree(dout));
  CHECK(hipFree(dclk));
  return rc;
}
