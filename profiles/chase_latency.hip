// Dependent-load latency on MI355X (measurement tool, not product code): every lane
// chases its own random cycle through a table of 16-byte records, one load per step,
// the next index taken from the loaded record -- the access pattern of k1b_walk's table
// walks.  Table sizes from L2-resident to far past the Infinity Cache; WAVES waves per
// SIMD on every CU.
//   hipcc -O3 --offload-arch=gfx950 -o chase_latency chase_latency.hip && ./chase_latency
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <numeric>
#include <random>

__global__ void chase(const uint4* tab, uint32_t mask, int steps, uint32_t* out) {
  uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u & mask;
  uint32_t acc = 0;
  for (int s = 0; s < steps; ++s) {
    const uint4 v = tab[i];
    i = v.x;
    acc += v.y;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc + i;
}

int main() {
  const size_t sizes_mb[] = {1, 2, 8, 32, 128, 512, 2048};
  const int wps[] = {1, 4};
  const int steps = 4096;
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  printf("{\"device\": \"%s\", \"cus\": %d, \"record_bytes\": 16, \"steps\": %d, \"results\": [\n", prop.gcnArchName, cus, steps);
  bool first = true;
  for (size_t mb : sizes_mb) {
    const size_t n = (mb << 20) / 16;   // power of two
    std::vector<uint32_t> perm(n);
    std::iota(perm.begin(), perm.end(), 0u);
    std::mt19937 rng(12345);
    std::shuffle(perm.begin(), perm.end(), rng);
    std::vector<uint4> h(n);
    for (size_t k = 0; k < n; ++k) h[perm[k]] = make_uint4(perm[(k + 1) % n], 1u, 0u, 0u);   // one cycle
    uint4* d;
    uint32_t* o;
    hipMalloc(&d, n * 16);
    hipMemcpy(d, h.data(), n * 16, hipMemcpyHostToDevice);
    hipMalloc(&o, (size_t)cus * 4 * 4 * 64 * 4);
    for (int w : wps) {
      const int block = 64 * 4 * w;   // w waves per SIMD (4 SIMDs per CU), one block per CU
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      chase<<<cus, block>>>(d, (uint32_t)(n - 1), 64, o);
      hipEventRecord(e0);
      chase<<<cus, block>>>(d, (uint32_t)(n - 1), steps, o);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      printf("%s  {\"table_mb\": %zu, \"waves_per_simd\": %d, \"ns_per_dependent_load\": %.1f}", first ? "" : ",\n", mb, w,
             ms * 1e6 / steps);
      first = false;
      hipEventDestroy(e0);
      hipEventDestroy(e1);
    }
    hipFree(d);
    hipFree(o);
  }
  printf("\n]}\n");
  return 0;
}
