// Where a fresh process's first milliseconds go (the CLI's context_wait): HIP runtime
// initialization (hipGetDeviceCount), device + stream, the first allocation, and -- with libzkfl.so
// loaded -- zkfl_ctx_create and the first kernel launched from libzkfl's code object
// (zkfl_poseidon_batch on one input).  One JSON line of milliseconds.
//   ctx_probe            HIP runtime only (libamdhip64, no libzkfl code object registered)
//   ctx_probe <lib.so>   dlopen libzkfl.so first (its fatbin registers at load), then the same
// Build: make -C tools ctx_probe
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main(int argc, char** argv) {
  auto t = std::chrono::steady_clock::now();
  double t_dl = 0, t_init = 0, t_dev = 0, t_malloc = 0, t_ctx = 0, t_kernel = 0;
  void* lib = nullptr;
  if (argc > 1) {
    lib = dlopen(argv[1], RTLD_NOW | RTLD_GLOBAL);
    if (!lib) {
      fprintf(stderr, "dlopen: %s\n", dlerror());
      return 1;
    }
    t_dl = ms_since(t);
  }
  t = std::chrono::steady_clock::now();
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return 2;
  t_init = ms_since(t);
  t = std::chrono::steady_clock::now();
  hipStream_t st;
  if (hipSetDevice(0) != hipSuccess || hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 3;
  t_dev = ms_since(t);
  t = std::chrono::steady_clock::now();
  void* p = nullptr;
  if (hipMalloc(&p, 1 << 20) != hipSuccess) return 4;
  t_malloc = ms_since(t);
  if (lib) {
    using CtxCreate = int (*)(int, void**);
    using Pos = int (*)(void*, uint32_t, size_t, const uint8_t*, uint8_t*);
    auto cc = reinterpret_cast<CtxCreate>(dlsym(lib, "zkfl_ctx_create"));
    auto pb = reinterpret_cast<Pos>(dlsym(lib, "zkfl_poseidon_batch"));
    if (!cc || !pb) return 5;
    t = std::chrono::steady_clock::now();
    void* ctx = nullptr;
    if (cc(0, &ctx)) return 6;
    t_ctx = ms_since(t);
    uint8_t in[64] = {1}, out[32];
    t = std::chrono::steady_clock::now();
    if (pb(ctx, 2, 1, in, out)) return 7;
    t_kernel = ms_since(t);
  }
  printf("{\"dlopen_libzkfl\": %.2f, \"hip_init\": %.2f, \"device_and_stream\": %.2f, \"first_malloc\": %.2f, "
         "\"zkfl_ctx_create\": %.2f, \"first_libzkfl_kernel\": %.2f}\n",
         t_dl, t_init, t_dev, t_malloc, t_ctx, t_kernel);
  (void)hipFree(p);
  return 0;
}
