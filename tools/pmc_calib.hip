// FETCH_SIZE calibration for the MSM accumulate's access pattern (MI355X_MICROARCH.md §HBM:
// "other access widths are uncalibrated: calibrate on a known byte count in your own access
// pattern").  Each lane gathers ONE record of RB bytes (RB = 64: G1 affine point, 128: G2) at a
// pseudo-random index of a 4 GiB table (>> the 256 MiB Infinity Cache) with the same
// global_load_dwordx4 sequence the accumulate kernel emits; known bytes = lanes x RB.
// Run under: rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./pmc_calib
#include <hip/hip_runtime.h>
#include <cstdio>

template <int RB>
struct Rec { uint4 q[RB / 16]; };

template <int RB>
__global__ __launch_bounds__(64) void k_gather(const Rec<RB>* table, size_t nrec, size_t lanes, uint4* sink) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= lanes) return;
  uint64_t h = (i + 1) * 0x9E3779B97F4A7C15ull;
  h ^= h >> 29; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 32;
  Rec<RB> r = table[h % nrec];
  uint4 acc = r.q[0];
#pragma unroll
  for (int k = 1; k < RB / 16; k++) { acc.x ^= r.q[k].x; acc.y ^= r.q[k].y; acc.z ^= r.q[k].z; acc.w ^= r.q[k].w; }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = acc;  // keep the loads alive
}

int main() {
  const size_t table_bytes = 4ull << 30, lanes = 4u << 20;
  void* t;
  uint4* sink;
  if (hipMalloc(&t, table_bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
  hipMemset(t, 0x5a, table_bytes);
  unsigned g = (unsigned)((lanes + 63) / 64);
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_gather<64>, dim3(g), dim3(64), 0, 0, (const Rec<64>*)t, table_bytes / 64, lanes, sink);
    hipLaunchKernelGGL(k_gather<128>, dim3(g), dim3(64), 0, 0, (const Rec<128>*)t, table_bytes / 128, lanes, sink);
  }
  hipDeviceSynchronize();
  printf("known bytes: k_gather<64> %.2f MiB, k_gather<128> %.2f MiB per launch\n", lanes * 64 / 1048576.0,
         lanes * 128 / 1048576.0);
  return 0;
}
