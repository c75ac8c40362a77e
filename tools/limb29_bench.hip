// Microbenchmark: Fq Montgomery multiplication in nine 29-bit limbs (R = 2^261) against the
// 8 x 32-bit whole-asm product of the G1 MSM kernels (FqOpsLazy::mul).
//
// With 29-bit limbs every 32x32 product is < 2^58 (< 2^60 for limbs < 2^30), so a column of up
// to 18 products plus the carry fits a 64-bit accumulator: each product is ONE v_mad_u64_u32,
// with no v_addc_co for a third accumulator word.  81 + 81 mads against 64 + 64 (mad, addc)
// pairs: ~356 issue units against ~512 (tools/isa_rate.hip: mad 2.2x, addc 1.8x).
// A product of inputs < 2^257 is < p + 2^253 < 2p (no final subtraction).
// Build: make -C tools limb29_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "field.h"
using namespace zkfl;

struct F29 {
  uint32_t v[9];
};
constexpr uint32_t M29 = (1u << 29) - 1;
__constant__ constexpr uint32_t P29[9] = {0x187cfd47u, 0x010460b6u, 0x1c72a34fu, 0x02d522d0u, 0x1585d978u,
                                          0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
constexpr uint32_t NINV29 = 0x4866389u;  // -p^-1 mod 2^29

__device__ __forceinline__ F29 pack29(const Fq& a) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int b = 29 * i, w = b >> 5, s = b & 31;
    uint32_t x = a.v[w] >> s;
    if (s > 3 && w + 1 < 8) x |= a.v[w + 1] << (32 - s);
    r.v[i] = x & M29;
  }
  return r;
}

__device__ __forceinline__ Fq unpack29(const F29& a) {  // normalized limbs, value < 2^256
  Fq r;
#pragma unroll
  for (int w = 0; w < 8; w++) {
    const int b = 32 * w, i = b / 29, s = b % 29;
    uint32_t x = a.v[i] >> s;
    if (i + 1 < 9) x |= a.v[i + 1] << (29 - s);
    if (s > 26 && i + 2 < 9) x |= a.v[i + 2] << (58 - s);
    r.v[w] = x;
  }
  return r;
}

// product scanning; ACC2: the a*b and m*p products of a column in two accumulators (ILP)
template <bool ACC2>
__device__ __forceinline__ F29 mul29(const F29& a, const F29& b) {
  uint32_t m[9];
  F29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    uint64_t acc2 = 0;
#pragma unroll
    for (int i = 0; i < k; i++) {
      acc += (uint64_t)a.v[i] * b.v[k - i];
      if (ACC2) acc2 += (uint64_t)m[i] * P29[k - i];
      else acc += (uint64_t)m[i] * P29[k - i];
    }
    acc += (uint64_t)a.v[k] * b.v[0];
    if (ACC2) acc += acc2;
    m[k] = ((uint32_t)acc * NINV29) & M29;
    acc += (uint64_t)m[k] * P29[0];
    acc >>= 29;
  }
#pragma unroll
  for (int k = 9; k < 17; k++) {
    uint64_t acc2 = 0;
#pragma unroll
    for (int i = k - 8; i < 9; i++) {
      acc += (uint64_t)a.v[i] * b.v[k - i];
      if (ACC2) acc2 += (uint64_t)m[i] * P29[k - i];
      else acc += (uint64_t)m[i] * P29[k - i];
    }
    if (ACC2) acc += acc2;
    r.v[k - 9] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  r.v[8] = (uint32_t)acc;
  return r;
}

// NACC independent column accumulators (products dealt round-robin), kept apart by empty asm
// barriers so the compiler cannot re-associate them into one dependency chain
template <int NACC>
__device__ __forceinline__ F29 mul29_split(const F29& a, const F29& b) {
  uint32_t m[9];
  F29 r;
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
    uint64_t acc[NACC];
#pragma unroll
    for (int j = 0; j < NACC; j++) acc[j] = 0;
    acc[0] = carry;
    int t = 0;
    const int lo = k < 9 ? 0 : k - 8, hi = k < 9 ? k : 8;
#pragma unroll
    for (int i = lo; i <= hi; i++) {
      acc[t % NACC] += (uint64_t)a.v[i] * b.v[k - i];
      t++;
      if (i < k) {  // m_i p_(k-i); m_k is not known yet
        acc[t % NACC] += (uint64_t)m[i] * P29[k - i];
        t++;
      }
    }
#pragma unroll
    for (int j = 0; j < NACC; j++) asm volatile("" : "+v"(acc[j]));
    uint64_t s = acc[0];
#pragma unroll
    for (int j = 1; j < NACC; j++) s += acc[j];
    if (k < 9) {
      m[k] = ((uint32_t)s * NINV29) & M29;
      s += (uint64_t)m[k] * P29[0];
    } else {
      r.v[k - 9] = (uint32_t)s & M29;
    }
    carry = s >> 29;
  }
  r.v[8] = (uint32_t)carry;
  return r;
}

template <int V, class T>
__device__ __forceinline__ T vmul(const T& x, const T& y);
template <>
__device__ __forceinline__ Fq vmul<0, Fq>(const Fq& x, const Fq& y) { return FqOpsLazy::mul(x, y); }
template <>
__device__ __forceinline__ F29 vmul<1, F29>(const F29& x, const F29& y) { return mul29<false>(x, y); }
template <>
__device__ __forceinline__ F29 vmul<2, F29>(const F29& x, const F29& y) { return mul29<true>(x, y); }
template <>
__device__ __forceinline__ F29 vmul<3, F29>(const F29& x, const F29& y) { return mul29_split<2>(x, y); }
template <>
__device__ __forceinline__ F29 vmul<4, F29>(const F29& x, const F29& y) { return mul29_split<3>(x, y); }

template <int V, class T>
__global__ void __launch_bounds__(256) kbench(T* data, int iters) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  T x0 = data[i], x1 = data[i + 1], x2 = data[i + 2], x3 = data[i + 3];
  const T y = data[0];
  for (int k = 0; k < iters; k++) {
    x0 = vmul<V>(x0, y); x1 = vmul<V>(x1, y); x2 = vmul<V>(x2, y); x3 = vmul<V>(x3, y);
  }
#pragma unroll
  for (int j = 0; j < (int)(sizeof(T) / 4); j++) x0.v[j] ^= x1.v[j] ^ x2.v[j] ^ x3.v[j];
  data[i] = x0;
}

template <int V, class T>
__global__ void klat(T* data, int iters) {
  T x = data[1];
  const T y = data[0];
  for (int k = 0; k < iters; k++) x = vmul<V>(x, y);
  data[1] = x;
}

// mode 0: a, b < p; mode 1: a + p (< 2p); mode 2: limb-wise a + b' (limbs < 2^30, no carries)
__global__ void kcheck(const Fq* a, const Fq* b, const Fq* c, int n, int* bad) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fq c251 = fp_zero<FqP>();
  c251.v[7] = 1u << 27;  // 2^251: fp_mul(x, 2^251) = x 2^-5
  Fq ref = fp_mul(fp_mul(a[i], b[i]), c251);
  F29 a29 = pack29(a[i]), b29 = pack29(b[i]);
  for (int mode = 0; mode < 3; mode++) {
    F29 x = a29;
    Fq want = ref;
    if (mode == 1) {
      x = pack29(fp_add(a[i], fp_zero<FqP>()));
#pragma unroll
      for (int j = 0; j < 9; j++) x.v[j] = 0;
      Fq ap;  // a + p as a 256-bit integer
      uint64_t cc = 0;
      for (int j = 0; j < 8; j++) {
        cc += (uint64_t)a[i].v[j] + FqP::P[j];
        ap.v[j] = (uint32_t)cc;
        cc >>= 32;
      }
      x = pack29(ap);
    } else if (mode == 2) {
      F29 c29 = pack29(c[i]);
#pragma unroll
      for (int j = 0; j < 9; j++) x.v[j] = a29.v[j] + c29.v[j];
      want = fp_mul(fp_mul(fp_add(a[i], c[i]), b[i]), c251);
    }
    for (int v = 1; v <= 4; v++) {
      F29 r = v == 1 ? mul29<false>(x, b29) : v == 2 ? mul29<true>(x, b29) : v == 3 ? mul29_split<2>(x, b29) : mul29_split<3>(x, b29);
      Fq u = unpack29(r);
      Fq red;
      fp_reduce_once<FqP>(red.v, u.v);
      bool lim = true;
      for (int j = 0; j < 9; j++) lim &= r.v[j] <= (j < 8 ? M29 : 0xFFFFFFu);
      if (!fp_eq(red, want) || !lim) atomicAdd(bad + mode * 4 + (v - 1), 1);
    }
  }
}

int main() {
  const int blocks = 256 * 8, threads = 256, iters = 2000;
  size_t n = (size_t)blocks * threads + 8;
  {
    const int m = 1 << 20;
    Fq* h = (Fq*)malloc(3 * m * sizeof(Fq));
    uint64_t st = 88172645463325252ull;
    for (int i = 0; i < 3 * m; i++)
      for (int j = 0; j < 8; j++) {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        h[i].v[j] = (uint32_t)st & (j == 7 ? 0x1fffffffu : 0xffffffffu);  // < 2^253 < p
      }
    Fq* dd; int* bad; int hb[12] = {0};
    hipMalloc(&dd, 3 * m * sizeof(Fq)); hipMalloc(&bad, sizeof(hb));
    hipMemcpy(dd, h, 3 * m * sizeof(Fq), hipMemcpyHostToDevice); hipMemset(bad, 0, sizeof(hb));
    hipLaunchKernelGGL(kcheck, dim3(m / 256), dim3(256), 0, 0, dd, dd + m, dd + 2 * m, m, bad);
    hipMemcpy(hb, bad, sizeof(hb), hipMemcpyDeviceToHost);
    printf("mismatches (a<p, a<2p, lazy limbs) x (1 acc, ab|mp acc, split2, split3):");
    for (int k = 0; k < 12; k++) printf(" %d", hb[k]);
    printf(" (of %d)\n", m);
    free(h);
  }
  Fq* d32;
  F29* d29;
  hipMalloc(&d32, n * sizeof(Fq));
  hipMalloc(&d29, n * sizeof(F29));
  hipMemset(d32, 0x11, n * sizeof(Fq));
  hipMemset(d29, 0x05, n * sizeof(F29));  // limbs 0x05050505 < 2^29
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[5] = {"8x32 whole-asm (FqOpsLazy::mul)", "9x29, one accumulator", "9x29, ab | mp accumulators",
                          "9x29, 2 split accumulators", "9x29, 3 split accumulators"};
  for (int v = 0; v < 5; v++) {
    float ms = 0, lat = 0;
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(a);
      if (v == 0) hipLaunchKernelGGL((kbench<0, Fq>), dim3(blocks), dim3(threads), 0, 0, d32, iters);
      if (v == 1) hipLaunchKernelGGL((kbench<1, F29>), dim3(blocks), dim3(threads), 0, 0, d29, iters);
      if (v == 2) hipLaunchKernelGGL((kbench<2, F29>), dim3(blocks), dim3(threads), 0, 0, d29, iters);
      if (v == 3) hipLaunchKernelGGL((kbench<3, F29>), dim3(blocks), dim3(threads), 0, 0, d29, iters);
      if (v == 4) hipLaunchKernelGGL((kbench<4, F29>), dim3(blocks), dim3(threads), 0, 0, d29, iters);
      hipEventRecord(b);
      hipEventSynchronize(b);
      hipEventElapsedTime(&ms, a, b);
    }
    hipEventRecord(a);
    if (v == 0) hipLaunchKernelGGL((klat<0, Fq>), dim3(1), dim3(1), 0, 0, d32, 10000);
    if (v == 1) hipLaunchKernelGGL((klat<1, F29>), dim3(1), dim3(1), 0, 0, d29, 10000);
    if (v == 2) hipLaunchKernelGGL((klat<2, F29>), dim3(1), dim3(1), 0, 0, d29, 10000);
    if (v == 3) hipLaunchKernelGGL((klat<3, F29>), dim3(1), dim3(1), 0, 0, d29, 10000);
    if (v == 4) hipLaunchKernelGGL((klat<4, F29>), dim3(1), dim3(1), 0, 0, d29, 10000);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&lat, a, b);
    const double muls = (double)blocks * threads * iters * 4;
    printf("%-34s %.1f G Fq-mul/s, single-lane latency %.1f ns\n", names[v], muls / ms / 1e6, lat * 1e6 / 10000);
  }
  return 0;
}
