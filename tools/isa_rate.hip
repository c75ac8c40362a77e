// Issue-rate microbenchmark for the integer / FP64 instructions relevant to 254-bit Montgomery
// multiplication on gfx950.  8 waves per SIMD, 8 independent dependency chains per lane, so the
// figure is throughput (SIMD cycles per wave64 instruction, assuming 2.4 GHz).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(S) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)

template <int KIND>
__global__ void __launch_bounds__(256) krate(uint64_t* out, double* dout, int iters) {
  uint64_t a[8];
  uint32_t h[8];
  double f[8];
  uint32_t x = threadIdx.x * 2654435761u, y = x ^ 0x9e3779b9u;
  double fx = 1.0000001 + threadIdx.x * 1e-9, fy = 0.9999999;
#define INIT(i) a[i] = threadIdx.x * (i + 3); h[i] = i; f[i] = 1.0 + i * 1e-3;
  REP8(INIT)
  for (int k = 0; k < iters; k++) {
    if (KIND == 0) {
#define MAD(i) asm volatile("v_mad_u64_u32 %0, s[%2:%3], %1, %4, %0" : "+v"(a[i]) : "v"(x), "n"(20 + 2 * i), "n"(21 + 2 * i), "v"(y) : "s20","s21","s22","s23","s24","s25","s26","s27","s28","s29","s30","s31","s32","s33","s34","s35");
      REP8(MAD)
    } else if (KIND == 1) {
#define ADDC(i) asm volatile("v_addc_co_u32 %0, s[%1:%2], %0, %3, s[%1:%2]" : "+v"(h[i]) : "n"(20 + 2 * i), "n"(21 + 2 * i), "v"(x) : "s20","s21","s22","s23","s24","s25","s26","s27","s28","s29","s30","s31","s32","s33","s34","s35");
      REP8(ADDC)
    } else if (KIND == 2) {
#define MULLO(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(h[i]) : "v"(y));
      REP8(MULLO)
    } else if (KIND == 3) {
#define FMA64(i) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(f[i]) : "v"(fx), "v"(fy));
      REP8(FMA64)
    } else if (KIND == 6) {
#define ADDF64(i) asm volatile("v_add_f64 %0, %1, %0" : "+v"(f[i]) : "v"(fx));
      REP8(ADDF64)
    } else if (KIND == 4) {
#define ADD64(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
      REP8(ADD64)
    } else {
#define ADD32(i) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(h[i]) : "v"(x));
      REP8(ADD32)
    }
  }
  uint64_t s = 0;
  double ds = 0;
#define SUM(i) s += a[i] + h[i]; ds += f[i];
  REP8(SUM)
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  dout[blockIdx.x * blockDim.x + threadIdx.x] = ds;
}

int main() {
  const int blocks = 256 * 8, threads = 256, iters = 10000;
  uint64_t* d;
  double* dd;
  hipMalloc(&d, (size_t)blocks * threads * 8);
  hipMalloc(&dd, (size_t)blocks * threads * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[7] = {"v_mad_u64_u32", "v_addc_co_u32", "v_mul_lo_u32", "v_fma_f64", "v_lshl_add_u64", "v_add_u32", "v_add_f64"};
  for (int k = 0; k < 7; k++) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(a);
      switch (k) {
        case 0: hipLaunchKernelGGL(krate<0>, dim3(blocks), dim3(threads), 0, 0, d, dd, iters); break;
        case 1: hipLaunchKernelGGL(krate<1>, dim3(blocks), dim3(threads), 0, 0, d, dd, iters); break;
        case 2: hipLaunchKernelGGL(krate<2>, dim3(blocks), dim3(threads), 0, 0, d, dd, iters); break;
        case 3: hipLaunchKernelGGL(krate<3>, dim3(blocks), dim3(threads), 0, 0, d, dd, iters); break;
        case 4: hipLaunchKernelGGL(krate<4>, dim3(blocks), dim3(threads), 0, 0, d, dd, iters); break;
        case 6: hipLaunchKernelGGL(krate<6>, dim3(blocks), dim3(threads), 0, 0, d, dd, iters); break;
        default: hipLaunchKernelGGL(krate<5>, dim3(blocks), dim3(threads), 0, 0, d, dd, iters); break;
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      double wave_instr = (double)iters * 8 * blocks * threads / 64.0;
      double cyc = ms * 1e-3 * 2.4e9 * 1024 / wave_instr;
      if (rep) printf("%-16s %8.2f ms  %6.2f SIMD-cycles per wave64 instruction (@2.4GHz)\n", names[k], ms, cyc);
    }
  }
  return 0;
}
