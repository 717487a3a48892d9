// VALU issue cost per instruction class on MI355X (gfx950): the microbenchmark
// behind the cycles-per-class table of DESIGN.md and the cycle-weighted VALU
// fraction bench.py reports.  Build and run:
//   hipcc --offload-arch=gfx950 -O3 -o profiles/valu_issue_bench profiles/valu_issue_bench.hip
//   profiles/valu_issue_bench > profiles/valu_issue_cycles.json
//
// Every lane runs 8 independent register chains of ONE instruction (so the
// measurement is issue throughput, not latency), 16-way unrolled, for `iters`
// loop trips.  The grid is 1024 workgroups of 256 threads: 4 waves on every one
// of the 1024 SIMDs, the detector kernel's occupancy.  Cycles per wave64
// instruction per SIMD = elapsed time x clock / (instructions per SIMD).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CHAIN8(STMT) STMT(a0) STMT(a1) STMT(a2) STMT(a3) STMT(a4) STMT(a5) STMT(a6) STMT(a7)

template <int OP>
__global__ __launch_bounds__(256) void issue_kernel(uint32_t* out, int iters, uint32_t s0) {
  uint32_t a0 = threadIdx.x, a1 = a0 * 3u + 1u, a2 = a0 ^ 0x55u, a3 = a0 + 7u, a4 = a0 * 5u, a5 = ~a0, a6 = a0 << 3,
           a7 = a0 + 0x1234u;
  const uint32_t b = blockIdx.x | 1u;
  uint64_t w0 = a0, w1 = a1, w2 = a2, w3 = a3, w4 = a4, w5 = a5, w6 = a6, w7 = a7;
  const uint64_t m64 = 0x5555555555555555ull ^ s0;
  double d0 = a0, d1 = a1, d2 = a2, d3 = a3, d4 = a4, d5 = a5, d6 = a6, d7 = a7;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if constexpr (OP == 0) {
#define S(x) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(x) : "v"(b));
        CHAIN8(S)
#undef S
      } else if constexpr (OP == 1) {
#define S(x) asm volatile("v_xor_b32_e32 %0, %1, %0" : "+v"(x) : "v"(b));
        CHAIN8(S)
#undef S
      } else if constexpr (OP == 2) {
#define S(x) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(b));
        CHAIN8(S)
#undef S
      } else if constexpr (OP == 3) {
#define S(x) asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(x) : "v"(b));
        CHAIN8(S)
#undef S
      } else if constexpr (OP == 4) {
#define S(x) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "s"(s0));
        CHAIN8(S)
#undef S
      } else if constexpr (OP == 5) {
#define S(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(b), "s"(s0));
        CHAIN8(S)
#undef S
      } else if constexpr (OP == 6) {
#define S(x) asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(x) : "v"(b));
        CHAIN8(S)
#undef S
      } else if constexpr (OP == 7) {
#define S(x) asm volatile("v_lshlrev_b32_e32 %0, %1, %0" : "+v"(x) : "v"(b));
        CHAIN8(S)
#undef S
      } else if constexpr (OP == 8) {
#define S(x) { uint64_t sd; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(x), "=s"(sd) : "v"(b), "v"(s0 | 1u)); }
        S(w0) S(w1) S(w2) S(w3) S(w4) S(w5) S(w6) S(w7)
#undef S
      } else if constexpr (OP == 9) {
#define S(x) asm volatile("v_add_f64 %0, %0, %1" : "+v"(x) : "v"(d7));
        S(d0) S(d1) S(d2) S(d3) S(d4) S(d5) S(d6) S(d0)
#undef S
      } else if constexpr (OP == 10) {
#define S(x) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x) : "v"(b), "s"(m64));
        CHAIN8(S)
#undef S
      } else if constexpr (OP == 11) {
#define S(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));
        CHAIN8(S)
#undef S
      } else if constexpr (OP == 12) {
#define S(x) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "s"(s0));
        CHAIN8(S)
#undef S
      } else if constexpr (OP == 13) {
#define S(x) asm volatile("v_sub_u32_e32 %0, %0, %1" : "+v"(x) : "v"(b));
        CHAIN8(S)
#undef S
      }
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(w0 ^ w1 ^ w2 ^ w3) ^
                                        (uint32_t)(w4 ^ w5 ^ w6 ^ w7) ^ (uint32_t)(d0 + d1 + d2 + d3 + d4 + d5 + d6);
}

static const char* kNames[] = {"v_add_u32 (VOP2)", "v_xor_b32 (VOP2)", "v_pk_add_u16 (VOP3P)",
                               "v_pk_min_u16 (VOP3P)", "v_perm_b32 (VOP3)", "v_bitop3_b32 (VOP3)",
                               "v_lshl_add_u32 (VOP3)", "v_lshlrev_b32 (VOP2)", "v_mad_u64_u32 (VOP3)",
                               "v_add_f64", "v_cndmask_b32_e64 (VOP3)", "v_mul_lo_u32 (VOP3)",
                               "v_or3_b32 (VOP3)", "v_sub_u32 (VOP2)"};

template <int OP>
static double run(uint32_t* d, int iters, int blocks) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(issue_kernel<OP>, dim3(blocks), dim3(256), 0, 0, d, 4, 0x05040100u);   // warm
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(issue_kernel<OP>, dim3(blocks), dim3(256), 0, 0, d, iters, 0x05040100u);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

template <int OP>
static void report(uint32_t* d, int iters, int blocks, double ghz, int simds, bool last) {
  const double ms = run<OP>(d, iters, blocks);
  const double waves = blocks * 4.0;
  const double inst_per_simd = waves / simds * iters * 16.0 * 8.0;
  const double cyc = ms * 1e-3 * ghz * 1e9 / inst_per_simd;
  std::printf("  {\"op\": \"%s\", \"ms\": %.3f, \"cycles_per_wave_inst_per_simd\": %.3f}%s\n", kNames[OP], ms, cyc,
              last ? "" : ",");
}

int main(int argc, char** argv) {
  const double ghz = argc > 1 ? std::atof(argv[1]) : 2.4;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 4096;
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int simds = prop.multiProcessorCount * 4;
  const int blocks = prop.multiProcessorCount * 4;   // 4 waves per SIMD
  uint32_t* d = nullptr;
  (void)hipMalloc(&d, (size_t)blocks * 256 * sizeof(uint32_t));
  std::printf("{\"device\": \"%s\", \"cus\": %d, \"clock_ghz_assumed\": %.2f, \"waves_per_simd\": 4, "
              "\"chains_per_lane\": 8, \"iters\": %d, \"results\": [\n",
              prop.gcnArchName, prop.multiProcessorCount, ghz, iters);
  report<0>(d, iters, blocks, ghz, simds, false);
  report<1>(d, iters, blocks, ghz, simds, false);
  report<2>(d, iters, blocks, ghz, simds, false);
  report<3>(d, iters, blocks, ghz, simds, false);
  report<4>(d, iters, blocks, ghz, simds, false);
  report<5>(d, iters, blocks, ghz, simds, false);
  report<6>(d, iters, blocks, ghz, simds, false);
  report<7>(d, iters, blocks, ghz, simds, false);
  report<8>(d, iters, blocks, ghz, simds, false);
  report<9>(d, iters, blocks, ghz, simds, false);
  report<10>(d, iters, blocks, ghz, simds, false);
  report<11>(d, iters, blocks, ghz, simds, false);
  report<12>(d, iters, blocks, ghz, simds, false);
  report<13>(d, iters, blocks, ghz, simds, true);
  std::printf("]}\n");
  (void)hipFree(d);
  return 0;
}
