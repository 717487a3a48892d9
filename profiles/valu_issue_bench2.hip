// VALU issue cost per opcode on MI355X (gfx950), second table: the opcodes of the bit-sliced
// m = 6 detector's step loop (profiles/valu_issue_bench.hip measured the first 14; there add,
// xor and sub ran at ~2.6 cycles per wave64 instruction and shifts, bitop3, perm and cndmask
// at ~4.2).  Same method: 8 independent chains per lane, 16-way unrolled, 4 waves on every
// SIMD; cycles per wave64 instruction per SIMD = time x clock / instructions per SIMD.  The
// "mix" rows alternate two opcodes (cycles per instruction of the pair's average): additive
// costs give the mean of the two rows, co-issue less.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/vib2 profiles/valu_issue_bench2.hip && /tmp/vib2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHAIN8(STMT) STMT(a0) STMT(a1) STMT(a2) STMT(a3) STMT(a4) STMT(a5) STMT(a6) STMT(a7)
#define MIX8(S1, S2) S1(a0) S2(a1) S1(a2) S2(a3) S1(a4) S2(a5) S1(a6) S2(a7)

#define OPS(X)                                                                                   \
  X(0, "v_and_b32_e32", "v_and_b32_e32 %0, %1, %0")                                           \
  X(1, "v_or_b32_e32", "v_or_b32_e32 %0, %1, %0")                                             \
  X(2, "v_xor_b32_e32", "v_xor_b32_e32 %0, %1, %0")                                           \
  X(3, "v_xor_b32_e64 (VOP3, VGPRs)", "v_xor_b32_e64 %0, %1, %0")                            \
  X(4, "v_add_u32_e32", "v_add_u32_e32 %0, %1, %0")                                           \
  X(5, "v_add_u32_e64 (VOP3)", "v_add_u32_e64 %0, %1, %0")                                    \
  X(6, "v_not_b32", "v_not_b32_e32 %0, %0")                                                   \
  X(7, "v_mov_b32 (from chain)", "v_mov_b32_e32 %0, %0")                                      \
  X(8, "v_lshrrev_b32_e32", "v_lshrrev_b32_e32 %0, %1, %0")                                   \
  X(9, "v_lshlrev_b32_e32 imm", "v_lshlrev_b32_e32 %0, 3, %0")                                \
  X(10, "v_bitop3_b32 (VGPRs)", "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")                   \
  X(11, "v_bitop3_b32 0xE8 (VGPRs)", "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8")              \
  X(12, "v_med3_u32", "v_med3_u32 %0, %0, %1, %2")                                            \
  X(13, "v_bfi_b32", "v_bfi_b32 %0, %1, %0, %2")                                              \
  X(14, "v_perm_b32 (VGPRs)", "v_perm_b32 %0, %0, %1, %2")                                    \
  X(15, "v_alignbit_b32", "v_alignbit_b32 %0, %0, %1, 16")                                    \
  X(16, "v_bfe_u32", "v_bfe_u32 %0, %0, 3, 12")                                               \
  X(17, "v_cndmask_b32_e32 (vcc)", "v_cndmask_b32_e32 %0, %1, %0, vcc")                       \
  X(18, "v_add3_u32", "v_add3_u32 %0, %0, %1, %2")                                            \
  X(19, "v_lshl_or_b32", "v_lshl_or_b32 %0, %0, 3, %1")                                      \
  X(20, "v_and_or_b32", "v_and_or_b32 %0, %0, %1, %2")                                        \
  X(21, "v_min_u32_e32", "v_min_u32_e32 %0, %1, %0")                                          \
  X(22, "v_mul_u32_u24_e32", "v_mul_u32_u24_e32 %0, %1, %0")                                  \
  X(23, "v_mul_hi_u32", "v_mul_hi_u32 %0, %0, %1")                                            \
  X(24, "v_sub_u32_e32", "v_sub_u32_e32 %0, %0, %1")                                          \
  X(25, "v_pk_add_u16", "v_pk_add_u16 %0, %0, %1")                                            \
  X(26, "v_pk_mov_b32 (2 regs)", "")                                                          \
  X(27, "mix bitop3 + xor_e32", "")                                                           \
  X(28, "mix bitop3 + and_e32", "")                                                           \
  X(29, "mix bitop3 + lshrrev", "")                                                           \
  X(30, "v_mad_u64_u32", "")                                                                  \
  X(31, "v_cndmask_b32_e64 (sgpr pair)", "v_cndmask_b32_e64 %0, %0, %1, %3")

#define NAME(i, n, s) n,
static const char* kNames[] = {OPS(NAME)};
constexpr int kOps = sizeof(kNames) / sizeof(kNames[0]);

template <int OP>
__global__ __launch_bounds__(256) void issue_kernel(uint32_t* out, int iters, uint32_t s0) {
  uint32_t a0 = threadIdx.x, a1 = a0 * 3u + 1u, a2 = a0 ^ 0x55u, a3 = a0 + 7u, a4 = a0 * 5u, a5 = ~a0, a6 = a0 << 3,
           a7 = a0 + 0x1234u;
  const uint32_t b = blockIdx.x | 1u, c = (blockIdx.x * 0x9E3779B9u) ^ threadIdx.x;
  const uint64_t m64 = 0x5555555555555555ull ^ s0;
  uint64_t w0 = a0, w1 = a1, w2 = a2, w3 = a3, w4 = a4, w5 = a5, w6 = a6, w7 = a7;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
#define GEN(i, n, s) if constexpr (OP == i && sizeof(s) > 1) { \
        asm volatile(s : "+v"(a0) : "v"(b), "v"(c), "s"(m64)); asm volatile(s : "+v"(a1) : "v"(b), "v"(c), "s"(m64)); \
        asm volatile(s : "+v"(a2) : "v"(b), "v"(c), "s"(m64)); asm volatile(s : "+v"(a3) : "v"(b), "v"(c), "s"(m64)); \
        asm volatile(s : "+v"(a4) : "v"(b), "v"(c), "s"(m64)); asm volatile(s : "+v"(a5) : "v"(b), "v"(c), "s"(m64)); \
        asm volatile(s : "+v"(a6) : "v"(b), "v"(c), "s"(m64)); asm volatile(s : "+v"(a7) : "v"(b), "v"(c), "s"(m64)); }
      OPS(GEN)
#undef GEN
      if constexpr (OP == 26) {
#define S(x) asm volatile("v_pk_mov_b32 %0, %0, %0 op_sel:[1,0]" : "+v"(x));
        S(w0) S(w1) S(w2) S(w3) S(w4) S(w5) S(w6) S(w7)
#undef S
      } else if constexpr (OP == 27) {
#define SA(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(b), "v"(c));
#define SB(x) asm volatile("v_xor_b32_e32 %0, %1, %0" : "+v"(x) : "v"(b));
        MIX8(SA, SB)
#undef SB
      } else if constexpr (OP == 28) {
#define SB(x) asm volatile("v_and_b32_e32 %0, %1, %0" : "+v"(x) : "v"(b));
        MIX8(SA, SB)
#undef SB
      } else if constexpr (OP == 29) {
#define SB(x) asm volatile("v_lshrrev_b32_e32 %0, %1, %0" : "+v"(x) : "v"(b));
        MIX8(SA, SB)
#undef SB
#undef SA
      } else if constexpr (OP == 30) {
#define S(x) { uint64_t sd; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(x), "=s"(sd) : "v"(b), "v"(c | 1u)); }
        S(w0) S(w1) S(w2) S(w3) S(w4) S(w5) S(w6) S(w7)
#undef S
      }
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(w0 ^ w1 ^ w2 ^ w3) ^
                                        (uint32_t)(w4 ^ w5 ^ w6 ^ w7);
}

template <int OP>
static void report(uint32_t* d, int iters, int blocks, double ghz, int simds) {
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
  const double inst_per_simd = blocks * 4.0 / simds * iters * 16.0 * 8.0;
  std::printf("  {\"op\": \"%s\", \"ms\": %.3f, \"cycles_per_wave_inst_per_simd\": %.3f}%s\n", kNames[OP], ms,
              ms * 1e-3 * ghz * 1e9 / inst_per_simd, OP + 1 == kOps ? "" : ",");
  if constexpr (OP + 1 < kOps) report<OP + 1>(d, iters, blocks, ghz, simds);
}

int main(int argc, char** argv) {
  const double ghz = argc > 1 ? std::atof(argv[1]) : 2.4;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 4096;
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int simds = prop.multiProcessorCount * 4;
  const int blocks = prop.multiProcessorCount * 4;
  uint32_t* d = nullptr;
  (void)hipMalloc(&d, (size_t)blocks * 256 * sizeof(uint32_t));
  std::printf("{\"device\": \"%s\", \"cus\": %d, \"clock_ghz_assumed\": %.2f, \"waves_per_simd\": 4, "
              "\"chains_per_lane\": 8, \"iters\": %d, \"results\": [\n",
              prop.gcnArchName, prop.multiProcessorCount, ghz, iters);
  report<0>(d, iters, blocks, ghz, simds);
  std::printf("]}\n");
  (void)hipFree(d);
  return 0;
}
