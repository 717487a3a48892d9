// VALU issue cost per opcode on MI355X (gfx950), third table (operand kinds): the opcodes of the bit-sliced
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
  X(0, "xor_e32 (v, v)", "v_xor_b32_e32 %0, %1, %0")                                          \
  X(1, "xor_e32 (s, v)", "v_xor_b32_e32 %0, %4, %0")                                          \
  X(2, "xor_e32 (inline 3, v)", "v_xor_b32_e32 %0, 3, %0")                                    \
  X(3, "xor_e32 (literal, v)", "v_xor_b32_e32 %0, 0x55555555, %0")                            \
  X(4, "lshrrev_e32 (v, v)", "v_lshrrev_b32_e32 %0, %1, %0")                                  \
  X(5, "lshrrev_e32 (inline 3, v)", "v_lshrrev_b32_e32 %0, 3, %0")                            \
  X(6, "lshrrev_e32 (s, v)", "v_lshrrev_b32_e32 %0, %4, %0")                                  \
  X(7, "lshlrev_e32 (v, v)", "v_lshlrev_b32_e32 %0, %1, %0")                                  \
  X(8, "lshlrev_e32 (inline 3, v)", "v_lshlrev_b32_e32 %0, 3, %0")                            \
  X(9, "bitop3 (v, v, v)", "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca")                        \
  X(10, "bitop3 (v, v, s)", "v_bitop3_b32 %0, %0, %1, %4 bitop3:0xca")                       \
  X(11, "bitop3 (v, v, inline 3)", "v_bitop3_b32 %0, %0, %1, 3 bitop3:0xca")                 \
  X(12, "bitop3 (s, v, v)", "v_bitop3_b32 %0, %4, %0, %1 bitop3:0xca")                       \
  X(13, "bfi (v, v, v)", "v_bfi_b32 %0, %1, %0, %2")                                          \
  X(14, "alignbit (v, v, v)", "v_alignbit_b32 %0, %0, %1, %2")                                \
  X(15, "and_e32 (s, v)", "v_and_b32_e32 %0, %4, %0")                                         \
  X(16, "add_e32 (inline 3, v)", "v_add_u32_e32 %0, 3, %0")                                   \
  X(17, "perm (v, v, v)", "v_perm_b32 %0, %0, %1, %2")                                        \
  X(18, "lshrrev_e64 (v, v)", "v_lshrrev_b32_e64 %0, %1, %0")                                 \
  X(19, "xor_e64 (v, s)", "v_xor_b32_e64 %0, %0, %4")                                         \
  X(20, "cndmask_e64 (v, v, s[2])", "v_cndmask_b32_e64 %0, %0, %1, %3")                       \
  X(21, "bitop3 0xE8 (v, v, v), 4 waves x 8 chains, repeat of bench2", "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8") \
  X(22, "lshlrev_b64 (v, v)", "")                                                             \
  X(23, "v_mov_b32 (s)", "v_mov_b32_e32 %0, %4")                                              \
  X(24, "bitop3 (v, v, v) dst != srcs", "")                                                  \
  X(25, "bitop3 (v, v, v), 1 chain per lane", "")                                             \
  X(26, "bitop3 (v, v, v), 2 chains per lane", "")                                            \
  X(27, "bitop3 (v, v, v), 4 chains per lane", "")                                            \
  X(28, "lshrrev (inline) + lshlrev (inline) + bitop3 (s, v, v): one flip", "")               \
  X(29, "lshrrev (v) + lshrrev (v) + bitop3 (v, v, v): flip, right shifts, VGPR mask", "")

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
        asm volatile(s : "+v"(a0) : "v"(b), "v"(c), "s"(m64), "s"(s0)); asm volatile(s : "+v"(a1) : "v"(b), "v"(c), "s"(m64), "s"(s0)); \
        asm volatile(s : "+v"(a2) : "v"(b), "v"(c), "s"(m64), "s"(s0)); asm volatile(s : "+v"(a3) : "v"(b), "v"(c), "s"(m64), "s"(s0)); \
        asm volatile(s : "+v"(a4) : "v"(b), "v"(c), "s"(m64), "s"(s0)); asm volatile(s : "+v"(a5) : "v"(b), "v"(c), "s"(m64), "s"(s0)); \
        asm volatile(s : "+v"(a6) : "v"(b), "v"(c), "s"(m64), "s"(s0)); asm volatile(s : "+v"(a7) : "v"(b), "v"(c), "s"(m64), "s"(s0)); }
      OPS(GEN)
#undef GEN
      if constexpr (OP == 22) {
#define S(x) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(x) : "v"(b));
        S(w0) S(w1) S(w2) S(w3) S(w4) S(w5) S(w6) S(w7)
#undef S
      } else if constexpr (OP == 24) {
        // results into fresh registers: t = f(a_i, b, c), then a_i = t via the next op's use
#define S(x, y) asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(x) : "v"(y), "v"(b), "v"(c));
        S(a0, a0) S(a1, a1) S(a2, a2) S(a3, a3) S(a4, a4) S(a5, a5) S(a6, a6) S(a7, a7)
#undef S
      } else if constexpr (OP >= 25 && OP <= 27) {
#define S(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(x) : "v"(b), "v"(c));
        if constexpr (OP == 25) { S(a0) S(a0) S(a0) S(a0) S(a0) S(a0) S(a0) S(a0) }
        if constexpr (OP == 26) { S(a0) S(a1) S(a0) S(a1) S(a0) S(a1) S(a0) S(a1) }
        if constexpr (OP == 27) { S(a0) S(a1) S(a2) S(a3) S(a0) S(a1) S(a2) S(a3) }
#undef S
      } else if constexpr (OP == 28) {   // 8 ops per 3-op flip group approx: 3 flips minus one op (counted as 8)
#define F(x) { uint32_t h, l; asm volatile("v_lshrrev_b32_e32 %0, 4, %1" : "=v"(h) : "v"(x)); \
        asm volatile("v_lshlrev_b32_e32 %0, 4, %1" : "=v"(l) : "v"(x)); \
        asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(x) : "s"(s0), "v"(h), "v"(l)); }
        F(a0) F(a1) F(a2) F(a3) F(a4) F(a5) F(a6) F(a7)
#undef F
      } else if constexpr (OP == 29) {
#define F(x) { uint32_t h, l; asm volatile("v_lshrrev_b32_e32 %0, %1, %2" : "=v"(h) : "v"(b), "v"(x)); \
        asm volatile("v_lshrrev_b32_e32 %0, %1, %2" : "=v"(l) : "v"(c), "v"(x)); \
        asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(x) : "v"(b), "v"(h), "v"(l)); }
        F(a0) F(a1) F(a2) F(a3) F(a4) F(a5) F(a6) F(a7)
#undef F
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
