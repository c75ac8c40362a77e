// Kernel dispatch rate of one process on MI355X: S streams, each a chain of K tiny kernels (one
// 64-thread block that stores one word), launched one by one or replayed from a captured graph.
// Prints launches per second for each S: if the rate stops growing with S, the front end (the
// command processor's packet handling), not the CUs, bounds a workload of many small kernels --
// config 5's ~50 launches per proof.  Run with GPU_MAX_HW_QUEUES set as bench.py does.
//   ./dispatch_probe [K] [streams...]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_tiny(int* out, int i) {
  if (threadIdx.x == 0) out[blockIdx.x + i] = i;
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 2000;
  std::vector<int> counts = {1, 2, 4, 8, 16, 24};
  if (argc > 2) {
    counts.clear();
    for (int i = 2; i < argc; i++) counts.push_back(atoi(argv[i]));
  }
  int* d;
  CK(hipMalloc(&d, 1 << 20));
  std::vector<hipStream_t> st(64);
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int S : counts) {
    if (S > 64) continue;
    // direct launches
    for (int w = 0; w < 2; w++) {
      CK(hipDeviceSynchronize());
      const auto t0 = std::chrono::steady_clock::now();
      for (int k = 0; k < K; k++)
        for (int s = 0; s < S; s++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, st[s], d, s * 8);
      CK(hipGetLastError());
      const auto t1 = std::chrono::steady_clock::now();
      CK(hipDeviceSynchronize());
      const auto t2 = std::chrono::steady_clock::now();
      const double host = std::chrono::duration<double>(t1 - t0).count();
      const double all = std::chrono::duration<double>(t2 - t0).count();
      if (w) printf("streams %2d  direct: %8.0f launches/s (host enqueue %.2f us per launch)\n", S, S * K / all,
                    host * 1e6 / (S * K));
    }
    // graphs: each stream replays a captured chain of 50 kernels (a config-5 proof's count)
    const int G = 50;
    std::vector<hipGraphExec_t> ex(S);
    for (int s = 0; s < S; s++) {
      hipGraph_t g;
      CK(hipStreamBeginCapture(st[s], hipStreamCaptureModeThreadLocal));
      for (int k = 0; k < G; k++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, st[s], d, s * 8);
      CK(hipStreamEndCapture(st[s], &g));
      CK(hipGraphInstantiate(&ex[s], g, nullptr, nullptr, 0));
      CK(hipGraphDestroy(g));
    }
    for (int w = 0; w < 2; w++) {
      CK(hipDeviceSynchronize());
      const auto t0 = std::chrono::steady_clock::now();
      for (int k = 0; k < K / G; k++)
        for (int s = 0; s < S; s++) CK(hipGraphLaunch(ex[s], st[s]));
      const auto t1 = std::chrono::steady_clock::now();
      CK(hipDeviceSynchronize());
      const auto t2 = std::chrono::steady_clock::now();
      const double host = std::chrono::duration<double>(t1 - t0).count();
      const double all = std::chrono::duration<double>(t2 - t0).count();
      if (w) printf("streams %2d  graphs: %8.0f launches/s (host %.2f us per kernel node)\n", S, S * (K / G) * G / all,
                    host * 1e6 / (S * (K / G) * G));
    }
    for (auto& e : ex) CK(hipGraphExecDestroy(e));
  }
  CK(hipDeviceSynchronize());
  CK(hipFree(d));
  for (auto& s : st) CK(hipStreamDestroy(s));
  return 0;
}
