// How many kernels run concurrently on MI355X from one process?  S streams each launch one
// single-wave kernel that spins for ~T us (s_sleep loop on the wall clock); the elapsed time
// divided by T gives the serialization factor.  Run with GPU_MAX_HW_QUEUES set as bench.py does.
//   ./concurrency_probe [streams...]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_spin(long long cycles, int* out) {
  long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(10);
  if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

int main(int argc, char** argv) {
  int* d;
  if (hipMalloc(&d, 1 << 20) != hipSuccess) return 1;
  int rate_khz = 0;
  (void)hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0);
  const long long cycles = (long long)rate_khz * 20;  // 20 ms
  std::vector<int> counts = {1, 2, 4, 8, 12, 16, 24, 32};
  if (argc > 1) {
    counts.clear();
    for (int i = 1; i < argc; i++) counts.push_back(atoi(argv[i]));
  }
  std::vector<hipStream_t> st(64);
  for (auto& s : st) (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, st[0], cycles / 20, d);
  (void)hipDeviceSynchronize();
  for (int n : counts) {
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, st[i], cycles, d);
    (void)hipDeviceSynchronize();
    double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    printf("streams %2d: %.1f ms for %d x 20 ms single-wave kernels -> %.2f concurrent\n", n, ms, n, n * 20.0 / ms);
  }
  return 0;
}
