// Microbenchmark: Fq Montgomery multiplication throughput variants on gfx950.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I<pkg>/csrc -o fp_microbench fp_microbench.hip
// `fp_microbench` runs the round-1 32-bit variants; `fp_microbench f64` (round 6) the FP64-FMA
// 52-bit-limb multiply (tools/f64mont.h) against the shipped 29-bit engine (csrc/field29.h).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include "field.h"
#include "field29.h"
#include "f64mont.h"
using namespace zkfl;

// the original compiler-lowered CIOS (baseline)
template <class PR>
__device__ __forceinline__ Fp<PR> cios_mul(const Fp<PR>& a, const Fp<PR>& b) {
  uint32_t t[9];
#pragma unroll
  for (int i = 0; i < 9; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t c = 0;
    const uint32_t bi = b.v[i];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      c = (uint64_t)a.v[j] * bi + t[j] + c;
      t[j] = (uint32_t)c;
      c >>= 32;
    }
    uint32_t t8 = t[8] + (uint32_t)c;
    const uint32_t m = t[0] * PR::INV;
    c = ((uint64_t)m * PR::P[0] + t[0]) >> 32;
#pragma unroll
    for (int j = 1; j < 8; j++) {
      c = (uint64_t)m * PR::P[j] + t[j] + c;
      t[j - 1] = (uint32_t)c;
      c >>= 32;
    }
    c += t8;
    t[7] = (uint32_t)c;
    t[8] = (uint32_t)(c >> 32);
  }
  Fp<PR> r;
  fp_reduce_once<PR>(r.v, t);
  return r;
}

template <class PR>
__device__ __forceinline__ Fp<PR> fips_mul(const Fp<PR>& a, const Fp<PR>& b) {
  uint32_t m[8], u[9];
  uint64_t lo = 0;
  uint32_t hi = 0;
  uint64_t cc;
#define MACV(x, y) asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, %2, 0, %1" : "+v"(lo), "=&s"(cc), "+v"(hi) : "v"(x), "v"(y) : "vcc");
#define MACS(x, y) asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, %2, 0, %1" : "+v"(lo), "=&s"(cc), "+v"(hi) : "v"(x), "s"(y) : "vcc");
#define SHIFT() { lo = (lo >> 32) | ((uint64_t)hi << 32); hi = 0; }
#pragma unroll
  for (int i = 0; i < 8; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) { MACV(a.v[j], b.v[i - j]); MACS(m[j], PR::P[i - j]); }
    MACV(a.v[i], b.v[0]);
    m[i] = (uint32_t)lo * PR::INV;
    MACS(m[i], PR::P[0]);
    SHIFT();
  }
#pragma unroll
  for (int i = 8; i < 16; i++) {
#pragma unroll
    for (int j = i - 7; j < 8; j++) { MACV(a.v[j], b.v[i - j]); MACS(m[j], PR::P[i - j]); }
    u[i - 8] = (uint32_t)lo;
    SHIFT();
  }
  u[8] = (uint32_t)lo;
  Fp<PR> r;
  fp_reduce_once<PR>(r.v, u);
  return r;
}


template <class PR>
__device__ __forceinline__ Fp<PR> fips_mul_vcc(const Fp<PR>& a, const Fp<PR>& b) {
  uint32_t m[8], u[9];
  uint64_t lo = 0;
  uint32_t hi = 0;
#define MACV2(x, y) asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc" : "+v"(lo), "+v"(hi) : "v"(x), "v"(y) : "vcc");
#define MACS2(x, y) asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc" : "+v"(lo), "+v"(hi) : "v"(x), "s"(y) : "vcc");
#define SHIFT2() { lo = (lo >> 32) | ((uint64_t)hi << 32); hi = 0; }
#pragma unroll
  for (int i = 0; i < 8; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) { MACV2(a.v[j], b.v[i - j]); MACS2(m[j], PR::P[i - j]); }
    MACV2(a.v[i], b.v[0]);
    m[i] = (uint32_t)lo * PR::INV;
    MACS2(m[i], PR::P[0]);
    SHIFT2();
  }
#pragma unroll
  for (int i = 8; i < 16; i++) {
#pragma unroll
    for (int j = i - 7; j < 8; j++) { MACV2(a.v[j], b.v[i - j]); MACS2(m[j], PR::P[i - j]); }
    u[i - 8] = (uint32_t)lo;
    SHIFT2();
  }
  u[8] = (uint32_t)lo;
  Fp<PR> r;
  fp_reduce_once<PR>(r.v, u);
  return r;
}


// V3: library form plus one explicit s_nop per MAC (what does a wait state cost?)
// V4: both products of one FIPS step in ONE asm statement (half the asm boundaries)
#define MAC_NOP_V(x, y) asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\ts_nop 0" : "+v"(lo), "+v"(hi) : "v"(x), "v"(y) : "vcc");
#define MAC_NOP_S(x, y) asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\ts_nop 0" : "+v"(lo), "+v"(hi) : "v"(x), "s"(y) : "vcc");
#define MAC_PAIR(x1, y1, x2, y2) asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t" \
                                     "v_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc" \
                                     : "+v"(lo), "+v"(hi) : "v"(x1), "v"(y1), "v"(x2), "s"(y2) : "vcc");

template <class PR, int MODE>
__device__ __forceinline__ Fp<PR> fips_mul_x(const Fp<PR>& a, const Fp<PR>& b) {
  uint32_t m[8], u[9];
  uint64_t lo = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
      if (MODE == 0) { MAC_NOP_V(a.v[j], b.v[i - j]); MAC_NOP_S(m[j], PR::P[i - j]); }
      else { MAC_PAIR(a.v[j], b.v[i - j], m[j], PR::P[i - j]); }
    }
    if (MODE == 0) { MAC_NOP_V(a.v[i], b.v[0]); } else { MACV2(a.v[i], b.v[0]); }
    m[i] = (uint32_t)lo * PR::INV;
    if (MODE == 0) { MAC_NOP_S(m[i], PR::P[0]); } else { MACS2(m[i], PR::P[0]); }
    SHIFT2();
  }
#pragma unroll
  for (int i = 8; i < 16; i++) {
#pragma unroll
    for (int j = i - 7; j < 8; j++) {
      if (MODE == 0) { MAC_NOP_V(a.v[j], b.v[i - j]); MAC_NOP_S(m[j], PR::P[i - j]); }
      else { MAC_PAIR(a.v[j], b.v[i - j], m[j], PR::P[i - j]); }
    }
    u[i - 8] = (uint32_t)lo;
    SHIFT2();
  }
  u[8] = (uint32_t)lo;
  Fp<PR> r;
  fp_reduce_once<PR>(r.v, u);
  return r;
}

template <int V>
__device__ __forceinline__ Fq vmul(const Fq& x, const Fq& y) {
  if (V == 0) return cios_mul(x, y);
  if (V == 1) return fips_mul(x, y);
  if (V == 2) return fips_mul_vcc(x, y);
  if (V == 3) return fips_mul_x<FqP, 0>(x, y);
  if (V == 4) return fips_mul_x<FqP, 1>(x, y);
  return fp_mul(x, y);
}

template <int V>
__global__ void __launch_bounds__(256) kbench(Fq* data, int iters) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  Fq x0 = data[i], x1 = data[i + 1], x2 = data[i + 2], x3 = data[i + 3];
  const Fq y = data[0];
  for (int k = 0; k < iters; k++) {
    x0 = vmul<V>(x0, y); x1 = vmul<V>(x1, y); x2 = vmul<V>(x2, y); x3 = vmul<V>(x3, y);
  }
  data[i] = fp_add(fp_add(x0, x1), fp_add(x2, x3));
}

// latency: one lane, one dependent chain
template <int V>
__global__ void klat(Fq* data, int iters) {
  Fq x = data[1];
  const Fq y = data[0];
  for (int k = 0; k < iters; k++) x = vmul<V>(x, y);
  data[1] = x;
}

__global__ void kcheck(const Fq* a, const Fq* b, int n, int* bad) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fq r0 = cios_mul(a[i], b[i]);
  if (!fp_eq(r0, vmul<1>(a[i], b[i]))) atomicAdd(bad, 1);
  if (!fp_eq(r0, vmul<2>(a[i], b[i]))) atomicAdd(bad + 1, 1);
  if (!fp_eq(r0, vmul<3>(a[i], b[i]))) atomicAdd(bad + 2, 1);
  if (!fp_eq(r0, vmul<4>(a[i], b[i]))) atomicAdd(bad + 3, 1);
  if (!fp_eq(r0, vmul<5>(a[i], b[i]))) atomicAdd(bad + 4, 1);
}


// ---- round 6: FP64-FMA limbs (f64m::mul, R = 2^260) vs 29-bit limbs (f29_mul, R = 2^261) ----
// V 0: f29_mul (two accumulators per column, the MSM's single product); 1: f29_mul2 (two
// independent products interleaved, the madd's paired form); 2: f64m::mul; 3: two f64m::mul
// side by side (the same pairing, left to the scheduler).  CH = 4 independent chains per lane.
template <int V>
struct Chain;
template <>
struct Chain<0> {
  using T = F29;
  static __device__ T load(const uint32_t* p) { uint32_t a[8]; for (int j = 0; j < 8; j++) a[j] = p[j]; return f29_pack(a); }
  static __device__ void step(T* x, const T& y) {
#pragma unroll
    for (int c = 0; c < 4; c++) x[c] = f29_mul(x[c], y); }
  static __device__ uint32_t fold(const T& x) { uint32_t s = 0; for (int j = 0; j < 9; j++) s ^= x.v[j]; return s; }
};
template <>
struct Chain<1> : Chain<0> {
  static __device__ void step(T* x, const T& y) {
    F29x2 r = f29_mul2(x[0], y, x[1], y); x[0] = r.a; x[1] = r.b;
    r = f29_mul2(x[2], y, x[3], y); x[2] = r.a; x[3] = r.b;
  }
};
template <>
struct Chain<2> {
  using T = f64m::D52;
  static __device__ T load(const uint32_t* p) { uint32_t a[8]; for (int j = 0; j < 8; j++) a[j] = p[j]; return f64m::pack(a); }
  static __device__ void step(T* x, const T& y) {
#pragma unroll
    for (int c = 0; c < 4; c++) x[c] = f64m::mul(x[c], y); }
  static __device__ uint32_t fold(const T& x) { uint32_t s = 0; for (int j = 0; j < 5; j++) s ^= (uint32_t)f64m::dbits(x.v[j]); return s; }
};
template <>
struct Chain<3> : Chain<2> {
  static __device__ void step(T* x, const T& y) {
#pragma unroll
    for (int c = 0; c < 4; c += 2) {
      const T a = f64m::mul(x[c], y), b = f64m::mul(x[c + 1], y);
      x[c] = a; x[c + 1] = b;
    }
  }
};

template <int V>
__global__ void __launch_bounds__(256) kf(uint32_t* data, int iters) {
  extern __shared__ uint32_t pad_lds[];  // occupancy control only
  if (V >= 2) f64m::set_rz();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  typename Chain<V>::T x[4];
#pragma unroll
  for (int c = 0; c < 4; c++) x[c] = Chain<V>::load(data + 8 * (i + c));
  const typename Chain<V>::T y = Chain<V>::load(data);
  for (int k = 0; k < iters; k++) Chain<V>::step(x, y);
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < 4; c++) s ^= Chain<V>::fold(x[c]);
  if (s == 0x9e3779b9u) pad_lds[threadIdx.x] = s;  // keep the chains live
  data[8 * i] ^= (s == 0x9e3779b9u);
}

// 2^20 random pairs: both engines against fp_mul (32-bit limbs, R = 2^256) scaled into their
// Montgomery domains (x 2^251 -> 2^-261, x 2^252 -> 2^-260), every result reduced once and
// compared; mode 1 takes a from [2^255, 2^256) (lazy operand ~5-9p, as in the madd).
__global__ void kcheck64(const Fq* a, const Fq* b, int n, int* bad) {
  f64m::set_rz();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for (int mode = 0; mode < 2; mode++) {
    Fq x = a[i];
    if (mode == 1) x.v[7] |= 0x80000000u;
    Fq ab = fp_mul(x, b[i]);  // x may exceed p: fp_mul's result is still the residue
    Fq c251 = fp_zero<FqP>(), c252 = fp_zero<FqP>();
    c251.v[7] = 1u << 27;
    c252.v[7] = 1u << 28;
    const Fq w29 = fp_mul(ab, c251), w64 = fp_mul(ab, c252);
    // 29-bit
    F29 r29 = f29_mul(f29_pack(x.v), f29_pack(b[i].v));
    Fq u;
    f29_unpack(u.v, r29);
    Fq red;
    fp_reduce_once<FqP>(red.v, u.v);
    if (!fp_eq(red, w29)) atomicAdd(bad + 2 * mode, 1);
    // FP64
    f64m::D52 r64 = f64m::mul(f64m::pack(x.v), f64m::pack(b[i].v));
    bool norm = true;
    for (int j = 0; j < 5; j++) {  // an integer in [0, 2^52): 2^52 + v has v as its mantissa
      const uint64_t u = f64m::dbits(f64m::ffma(r64.v[j], 1.0, 0x1p52));
      norm &= (f64m::dbits(r64.v[j]) >> 63) == 0 && (u >> 52) == 0x433 && f64m::dbits(f64m::ffma(f64m::bitsd(u), 1.0, -0x1p52)) == f64m::dbits(r64.v[j]);
    }
    f64m::unpack(u.v, r64);
    fp_reduce_once<FqP>(red.v, u.v);
    if (!fp_eq(red, w64) || !norm) atomicAdd(bad + 2 * mode + 1, 1);
  }
}

static int run_f64() {
  const int m = 1 << 20;
  {
    Fq* h = (Fq*)malloc(2 * m * sizeof(Fq));
    uint64_t st = 88172645463325252ull;
    for (int i = 0; i < 2 * m; i++)
      for (int j = 0; j < 8; j++) {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        h[i].v[j] = (uint32_t)st & (j == 7 ? 0x1fffffffu : 0xffffffffu);  // < 2^253 < p
      }
    Fq* dd; int* bad; int hb[4] = {0, 0, 0, 0};
    hipMalloc(&dd, 2 * m * sizeof(Fq)); hipMalloc(&bad, sizeof(hb));
    hipMemcpy(dd, h, 2 * m * sizeof(Fq), hipMemcpyHostToDevice); hipMemset(bad, 0, sizeof(hb));
    hipLaunchKernelGGL(kcheck64, dim3(m / 256), dim3(256), 0, 0, dd, dd + m, m, bad);
    hipMemcpy(hb, bad, sizeof(hb), hipMemcpyDeviceToHost);
    printf("bit-exactness, %d random pairs: mismatches 29-bit %d, FP64 %d (a < p); 29-bit %d, FP64 %d (a in [2^255, 2^256))\n",
           m, hb[0], hb[1], hb[2], hb[3]);
    free(h); hipFree(dd); hipFree(bad);
    if (hb[0] | hb[1] | hb[2] | hb[3]) return 1;
  }
  const int threads = 256, iters = 400;
  const int blocks = 256 * 3 * 8;  // 8 rounds of 3 blocks per CU
  uint32_t* d;
  hipMalloc(&d, ((size_t)blocks * threads + 8) * 32);
  hipMemset(d, 0x05, ((size_t)blocks * threads + 8) * 32);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const char* names[4] = {"29-bit f29_mul (shipped single product)", "29-bit f29_mul2 (shipped paired form)",
                          "FP64 52-bit f64m::mul", "FP64 52-bit, two products side by side"};
  void (*ks[4])(uint32_t*, int) = {kf<0>, kf<1>, kf<2>, kf<3>};
  for (int occ = 0; occ < 2; occ++) {
    const size_t lds = occ == 0 ? 46 * 1024 : 0;  // 3 blocks (3 waves/SIMD) per CU, or registers decide
    printf("-- %s\n", occ == 0 ? "3 waves/SIMD (LDS-limited, the G1 accumulation's occupancy)" : "occupancy set by registers");
    for (int v = 0; v < 4; v++) {
      hipFuncAttributes fa;
      hipFuncGetAttributes(&fa, (const void*)ks[v]);
      float best = 1e30f;
      for (int rep = 0; rep < 3; rep++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(threads), lds, 0, d, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep && ms < best) best = ms;
      }
      const double muls = (double)blocks * threads * iters * 4;
      const double simd_cyc = best * 1e-3 * 2.4e9 * 1024 / (muls / 64);  // per wave64 product
      printf("%-44s VGPRs %3d  %7.1f G Fq-mul/s  %7.1f SIMD-cycles per wave64 product @2.4GHz\n", names[v],
             fa.numRegs, muls / best / 1e6, simd_cyc);
    }
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && !strcmp(argv[1], "f64")) return run_f64();
  const int blocks = 256 * 8, threads = 256, iters = 2000;
  size_t n = (size_t)blocks * threads + 8;
  Fq* d;
  hipMalloc(&d, n * sizeof(Fq));
  hipMemset(d, 0x11, n * sizeof(Fq));
  {
    // correctness on pseudo-random inputs < q
    const int m = 1 << 20;
    Fq* h = (Fq*)malloc(2 * m * sizeof(Fq));
    uint64_t st = 88172645463325252ull;
    for (int i = 0; i < 2 * m; i++)
      for (int j = 0; j < 8; j++) {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        h[i].v[j] = (uint32_t)st & (j == 7 ? 0x1fffffffu : 0xffffffffu);
      }
    Fq* dd; int* bad; int hb[5] = {0, 0, 0, 0, 0};
    hipMalloc(&dd, 2 * m * sizeof(Fq)); hipMalloc(&bad, 20);
    hipMemcpy(dd, h, 2 * m * sizeof(Fq), hipMemcpyHostToDevice); hipMemset(bad, 0, 20);
    hipLaunchKernelGGL(kcheck, dim3(m / 256), dim3(256), 0, 0, dd, dd + m, m, bad);
    hipMemcpy(hb, bad, 20, hipMemcpyDeviceToHost);
    printf("mismatches vs CIOS (variants 1..5): %d %d %d %d %d (of %d)\n", hb[0], hb[1], hb[2], hb[3], hb[4], m);
  }
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int v = 0; v < 6; v++) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(a);
      void (*kb[6])(Fq*, int) = {kbench<0>, kbench<1>, kbench<2>, kbench<3>, kbench<4>, kbench<5>};
      hipLaunchKernelGGL(kb[v], dim3(blocks), dim3(threads), 0, 0, d, iters);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      double muls = (double)blocks * threads * iters * 4;
      if (rep) printf("variant %d throughput: %.1f G Fq-mul/s (%.2f ms)\n", v, muls / ms / 1e6, ms);
    }
    hipEventRecord(a);
    void (*kl[6])(Fq*, int) = {klat<0>, klat<1>, klat<2>, klat<3>, klat<4>, klat<5>};
    hipLaunchKernelGGL(kl[v], dim3(1), dim3(1), 0, 0, d, 10000);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("variant %d single-lane latency: %.1f ns / mul\n", v, ms * 1e6 / 10000);
  }
  return 0;
}

