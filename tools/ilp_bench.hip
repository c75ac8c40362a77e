// Does a second independent multiplication chain per lane help at the accumulate kernel's
// occupancy (4 waves/SIMD, forced with 10 KiB of dynamic LDS per 64-thread block)?
// V=0: library fp_mul (carry through VCC: every MAC asm clobbers VCC, so two chains cannot
//      interleave); V=1: carry in a compiler-allocated SGPR pair (chains may interleave).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "field.h"
#include "fp_mul_asm.h"
using namespace zkfl;

#define MACV_S(x, y) asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, %2, 0, %1" : "+v"(lo), "=&s"(cc), "+v"(hi) : "v"(x), "v"(y));
#define MACS_S(x, y) asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, %2, 0, %1" : "+v"(lo), "=&s"(cc), "+v"(hi) : "v"(x), "s"(y));

template <class PR>
__device__ __forceinline__ Fp<PR> mul_sgpr(const Fp<PR>& a, const Fp<PR>& b) {
  uint32_t m[8], u[9];
  uint64_t lo = 0, cc;
  uint32_t hi = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) { MACV_S(a.v[j], b.v[i - j]); MACS_S(m[j], PR::P[i - j]); }
    MACV_S(a.v[i], b.v[0]);
    m[i] = (uint32_t)lo * PR::INV;
    MACS_S(m[i], PR::P[0]);
    lo = (lo >> 32) | ((uint64_t)hi << 32); hi = 0;
  }
#pragma unroll
  for (int i = 8; i < 16; i++) {
#pragma unroll
    for (int j = i - 7; j < 8; j++) { MACV_S(a.v[j], b.v[i - j]); MACS_S(m[j], PR::P[i - j]); }
    u[i - 8] = (uint32_t)lo;
    lo = (lo >> 32) | ((uint64_t)hi << 32); hi = 0;
  }
  u[8] = (uint32_t)lo;
  Fp<PR> r;
  fp_reduce_once<PR>(r.v, u);
  return r;
}

__device__ __forceinline__ Fq mul_whole(const Fq& a, const Fq& b) {
  uint32_t u[8];
  ZK_FP_MUL_ASM(u, a.v, b.v, FqP::P, FqP::INV);
  Fq r;
  fp_reduce_once<FqP>(r.v, u);
  return r;
}

template <int V>
__device__ __forceinline__ Fq mulv(const Fq& a, const Fq& b) {
  return V == 0 ? fp_mul(a, b) : (V == 1 ? mul_sgpr(a, b) : mul_whole(a, b));
}

__global__ void kcheck2(const Fq* a, const Fq* b, int n, int* bad) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (!fp_eq(mul_whole(a[i], b[i]), fp_mul(a[i], b[i]))) atomicAdd(bad, 1);
}

__global__ void klat1(Fq* data, int iters, int v) {
  Fq x = data[1];
  const Fq y = data[0];
  if (v == 0) for (int k = 0; k < iters; k++) x = fp_mul(x, y);
  else for (int k = 0; k < iters; k++) x = mul_whole(x, y);
  data[1] = x;
}

template <int V, int CH>
__global__ __launch_bounds__(64) void kchain(Fq* data, int iters) {
  extern __shared__ uint32_t lds[];
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  Fq x = data[i], z = data[i + 1];
  const Fq y = data[0], w = data[2];
  for (int k = 0; k < iters; k++) {
    x = mulv<V>(x, y);
    if (CH == 2) z = mulv<V>(z, w);
  }
  if (threadIdx.x == 999) lds[0] = 1;
  data[i] = CH == 2 ? fp_add(x, z) : x;
}

int main() {
  const int blocks = 256 * 16, threads = 64, iters = 1000;
  Fq* d;
  (void)hipMalloc(&d, (size_t)(blocks * threads + 8) * sizeof(Fq));
  (void)hipMemset(d, 0x11, (size_t)(blocks * threads + 8) * sizeof(Fq));
  void (*ks[6])(Fq*, int) = {kchain<0, 1>, kchain<0, 2>, kchain<1, 1>, kchain<1, 2>, kchain<2, 1>, kchain<2, 2>};
  const char* names[6] = {"lib   1 chain ", "lib   2 chains", "sgpr  1 chain ", "sgpr  2 chains", "whole 1 chain ",
                          "whole 2 chains"};
  {
    const int m = 1 << 20;
    Fq* h = (Fq*)malloc(2 * m * sizeof(Fq));
    uint64_t st = 88172645463325252ull;
    for (int i = 0; i < 2 * m; i++)
      for (int j = 0; j < 8; j++) {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        h[i].v[j] = (uint32_t)st & (j == 7 ? 0x1fffffffu : 0xffffffffu);
      }
    Fq* dd; int* bad; int hb = 0;
    (void)hipMalloc(&dd, 2 * m * sizeof(Fq)); (void)hipMalloc(&bad, 4);
    (void)hipMemcpy(dd, h, 2 * m * sizeof(Fq), hipMemcpyHostToDevice); (void)hipMemset(bad, 0, 4);
    hipLaunchKernelGGL(kcheck2, dim3(m / 256), dim3(256), 0, 0, dd, dd + m, m, bad);
    (void)hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    printf("whole-asm mismatches vs library: %d of %d\n", hb, m);
  }
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int lds_kib : {10, 0}) {
    for (int v = 0; v < 6; v++) {
      float ms = 0;
      for (int rep = 0; rep < 2; rep++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(threads), lds_kib * 1024, 0, d, iters);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
      }
      double muls = (double)blocks * threads * iters * ((v & 1) ? 2 : 1);
      printf("LDS %2d KiB/block  %s: %6.1f G Fq-mul/s\n", lds_kib, names[v], muls / ms / 1e6);
    }
  }
  for (int v = 0; v < 2; v++) {
    float ms = 0;
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(klat1, dim3(1), dim3(1), 0, 0, d, 10000, v);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
    printf("%s single-lane latency: %.1f ns / mul\n", v ? "whole" : "lib  ", ms * 1e6 / 10000);
  }
  return 0;
}
