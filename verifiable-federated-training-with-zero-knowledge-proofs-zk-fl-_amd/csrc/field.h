// BN254 prime-field arithmetic for gfx950 (CDNA4), 8 x 32-bit limbs, Montgomery R = 2^256.
//
// Replaces the ffjavascript/wasmcurves Fq/Fr kernels (reference dependency ffjavascript
// ^0.2.63, package.json:44; used by `snarkjs groth16 prove`, tests/full_system_simulation.mjs:773).
// Representation: little-endian 32-bit limbs, values kept fully reduced (< p) between
// operations.  Montgomery multiplication is product scanning (FIPS) on v_mad_u64_u32 with the
// column carry routed through VCC (see fp_mul).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zkfl {

#define ZK_DEV __device__ __forceinline__

struct FqP {  // base field q
  static constexpr uint32_t P[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t ONE[8] = {0xc58f0d9du, 0xd35d438du, 0xf5c70b3du, 0x0a78eb28u,
                                      0x7879462cu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
  static constexpr uint32_t R2[8] = {0x538afa89u, 0xf32cfc5bu, 0xd44501fbu, 0xb5e71911u,
                                     0x0a417ff6u, 0x47ab1effu, 0xcab8351fu, 0x06d89f71u};
  static constexpr uint32_t INV = 0xe4866389u;  // -q^-1 mod 2^32
};

struct FrP {  // scalar field r
  static constexpr uint32_t P[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t ONE[8] = {0x4ffffffbu, 0xac96341cu, 0x9f60cd29u, 0x36fc7695u,
                                      0x7879462eu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
  static constexpr uint32_t R2[8] = {0xae216da7u, 0x1bb8e645u, 0xe35c59e3u, 0x53fe3ab1u,
                                     0x53bb8085u, 0x8c49833du, 0x7f4e44a5u, 0x0216d0b1u};
  static constexpr uint32_t INV = 0xefffffffu;  // -r^-1 mod 2^32
};

template <class PR>
struct Fp {
  uint32_t v[8];
};

using Fq = Fp<FqP>;
using Fr = Fp<FrP>;

template <class PR>
ZK_DEV Fp<PR> fp_zero() {
  Fp<PR> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = 0;
  return r;
}

template <class PR>
ZK_DEV Fp<PR> fp_one() {  // Montgomery one
  Fp<PR> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = PR::ONE[i];
  return r;
}

template <class PR>
ZK_DEV bool fp_is_zero(const Fp<PR>& a) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x |= a.v[i];
  return x == 0;
}

template <class PR>
ZK_DEV bool fp_eq(const Fp<PR>& a, const Fp<PR>& b) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x |= a.v[i] ^ b.v[i];
  return x == 0;
}

// r = a - p if a >= p else a   (a < 2p)
template <class PR>
ZK_DEV void fp_reduce_once(uint32_t r[8], const uint32_t a[8]) {
  uint32_t t[8];
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t d = (uint64_t)a[i] - PR::P[i] - borrow;
    t[i] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = borrow ? a[i] : t[i];
}

template <class PR>
ZK_DEV Fp<PR> fp_add(const Fp<PR>& a, const Fp<PR>& b) {
  uint32_t s[8];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c += (uint64_t)a.v[i] + b.v[i];
    s[i] = (uint32_t)c;
    c >>= 32;
  }
  Fp<PR> r;
  fp_reduce_once<PR>(r.v, s);
  return r;
}

template <class PR>
ZK_DEV Fp<PR> fp_sub(const Fp<PR>& a, const Fp<PR>& b) {
  uint32_t d[8];
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t t = (uint64_t)a.v[i] - b.v[i] - borrow;
    d[i] = (uint32_t)t;
    borrow = (uint32_t)(t >> 63);
  }
  // if borrow, add p back
  uint32_t mask = 0u - borrow;
  uint64_t c = 0;
  Fp<PR> r;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c += (uint64_t)d[i] + (PR::P[i] & mask);
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
  return r;
}

template <class PR>
ZK_DEV Fp<PR> fp_neg(const Fp<PR>& a) {
  return fp_sub<PR>(fp_zero<PR>(), a);
}

template <class PR>
ZK_DEV Fp<PR> fp_dbl(const Fp<PR>& a) {
  return fp_add<PR>(a, a);
}

// Montgomery multiplication, finely integrated product scanning (FIPS).  a, b < p  ->
// a*b*2^-256 mod p, < p.  Column sums are accumulated in a 3-word register triple
// (lo:64 | hi:32): each 32x32 product is ONE v_mad_u64_u32 whose 64-bit addend is the running
// column and whose carry-out goes, through an SGPR pair the compiler allocates, into `hi`
// (v_addc_co_u32).  The compiler's own lowering of the same C++ needs a v_cmp + v_cndmask per
// product and ~270 v_mov per multiply for 64-bit zero-extension; measured on MI355X
// (tools/fp_microbench.hip, tools/ilp_bench.hip): 125 vs 94 G Fq-mul/s at full occupancy, and at
// the MSM kernel's 4 waves/SIMD 118 G/s with the SGPR carry vs 109 G/s with the carry pinned
// to VCC (a fixed VCC clobber serializes independent multiplications).  Both moduli are 254-bit
// so the column accumulator never exceeds 3 words.
#define ZK_MAC_VV(lo, hi, x, y)                                                                             \
  do {                                                                                                      \
    uint64_t cc_;                                                                                           \
    asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, %2, 0, %1" : "+v"(lo), "=&s"(cc_), "+v"(hi) \
        : "v"(x), "v"(y));                                                                                  \
  } while (0)
#define ZK_MAC_VS(lo, hi, x, y)                                                                             \
  do {                                                                                                      \
    uint64_t cc_;                                                                                           \
    asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, %2, 0, %1" : "+v"(lo), "=&s"(cc_), "+v"(hi) \
        : "v"(x), "s"(y));                                                                                  \
  } while (0)

template <class PR>
ZK_DEV Fp<PR> fp_mul(const Fp<PR>& a, const Fp<PR>& b) {
  uint32_t m[8], u[9];
  uint64_t lo = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
      ZK_MAC_VV(lo, hi, a.v[j], b.v[i - j]);
      ZK_MAC_VS(lo, hi, m[j], PR::P[i - j]);
    }
    ZK_MAC_VV(lo, hi, a.v[i], b.v[0]);
    m[i] = (uint32_t)lo * PR::INV;
    ZK_MAC_VS(lo, hi, m[i], PR::P[0]);
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
#pragma unroll
  for (int i = 8; i < 16; i++) {
#pragma unroll
    for (int j = i - 7; j < 8; j++) {
      ZK_MAC_VV(lo, hi, a.v[j], b.v[i - j]);
      ZK_MAC_VS(lo, hi, m[j], PR::P[i - j]);
    }
    u[i - 8] = (uint32_t)lo;
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  u[8] = (uint32_t)lo;
  Fp<PR> r;
  fp_reduce_once<PR>(r.v, u);
  return r;
}

// (a*b + c*d) * 2^-256 mod p with ONE Montgomery reduction (a, b, c, d < p): both products
// accumulate into the same FIPS columns (<= 24 terms per column, < 2^69: the 96-bit column
// accumulator holds it); a*b + c*d < 2p^2 < 2^256 p, so the result is < 2p before the final
// subtraction.  200 multiply-adds instead of 2 x 136 (the lane-pair Fq2 product).
template <class PR>
ZK_DEV Fp<PR> fp_mul_sum2(const Fp<PR>& a, const Fp<PR>& b, const Fp<PR>& c, const Fp<PR>& d) {
  uint32_t m[8], u[9];
  uint64_t lo = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
      ZK_MAC_VV(lo, hi, a.v[j], b.v[i - j]);
      ZK_MAC_VV(lo, hi, c.v[j], d.v[i - j]);
      ZK_MAC_VS(lo, hi, m[j], PR::P[i - j]);
    }
    ZK_MAC_VV(lo, hi, a.v[i], b.v[0]);
    ZK_MAC_VV(lo, hi, c.v[i], d.v[0]);
    m[i] = (uint32_t)lo * PR::INV;
    ZK_MAC_VS(lo, hi, m[i], PR::P[0]);
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
#pragma unroll
  for (int i = 8; i < 16; i++) {
#pragma unroll
    for (int j = i - 7; j < 8; j++) {
      ZK_MAC_VV(lo, hi, a.v[j], b.v[i - j]);
      ZK_MAC_VV(lo, hi, c.v[j], d.v[i - j]);
      ZK_MAC_VS(lo, hi, m[j], PR::P[i - j]);
    }
    u[i - 8] = (uint32_t)lo;
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  u[8] = (uint32_t)lo;
  Fp<PR> r;
  fp_reduce_once<PR>(r.v, u);
  return r;
}

// sum_{k<4} x_k * y_k * 2^-256 mod p with one reduction (inputs < p): <= 40 terms per column
// (< 2^70), the sum < 4p^2 gives a result < 1.76p before the final subtraction.
template <class PR>
ZK_DEV Fp<PR> fp_mul_sum4(const Fp<PR>* x, const Fp<PR>* y) {
  uint32_t m[8], u[9];
  uint64_t lo = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
#pragma unroll
      for (int k = 0; k < 4; k++) ZK_MAC_VV(lo, hi, x[k].v[j], y[k].v[i - j]);
      ZK_MAC_VS(lo, hi, m[j], PR::P[i - j]);
    }
#pragma unroll
    for (int k = 0; k < 4; k++) ZK_MAC_VV(lo, hi, x[k].v[i], y[k].v[0]);
    m[i] = (uint32_t)lo * PR::INV;
    ZK_MAC_VS(lo, hi, m[i], PR::P[0]);
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
#pragma unroll
  for (int i = 8; i < 16; i++) {
#pragma unroll
    for (int j = i - 7; j < 8; j++) {
#pragma unroll
      for (int k = 0; k < 4; k++) ZK_MAC_VV(lo, hi, x[k].v[j], y[k].v[i - j]);
      ZK_MAC_VS(lo, hi, m[j], PR::P[i - j]);
    }
    u[i - 8] = (uint32_t)lo;
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  u[8] = (uint32_t)lo;
  Fp<PR> r;
  fp_reduce_once<PR>(r.v, u);
  return r;
}

template <class PR>
ZK_DEV Fp<PR> fp_sqr(const Fp<PR>& a) {
  return fp_mul<PR>(a, a);
}

// Standard <-> Montgomery
template <class PR>
ZK_DEV Fp<PR> fp_to_mont(const Fp<PR>& a) {
  Fp<PR> r2;
#pragma unroll
  for (int i = 0; i < 8; i++) r2.v[i] = PR::R2[i];
  return fp_mul<PR>(a, r2);
}

template <class PR>
ZK_DEV Fp<PR> fp_from_mont(const Fp<PR>& a) {
  Fp<PR> one;
  one.v[0] = 1;
#pragma unroll
  for (int i = 1; i < 8; i++) one.v[i] = 0;
  return fp_mul<PR>(a, one);
}

// a^e for a public exponent given as 8 little-endian limbs (left-to-right binary).
template <class PR>
ZK_DEV Fp<PR> fp_pow(const Fp<PR>& a, const uint32_t e[8]) {
  Fp<PR> r = fp_one<PR>();
#pragma unroll
  for (int i = 7; i >= 0; i--) {  // constant limb index: e stays in registers
#pragma unroll 1
    for (int b = 31; b >= 0; b--) {
      r = fp_sqr<PR>(r);
      if ((e[i] >> b) & 1u) r = fp_mul<PR>(r, a);
    }
  }
  return r;
}

// Inverse by Fermat (p - 2).  inv(0) = 0.
template <class PR>
ZK_DEV Fp<PR> fp_inv(const Fp<PR>& a) {
  uint32_t e[8];
  uint32_t borrow = 2;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t d = (uint64_t)PR::P[i] - borrow;
    e[i] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
  return fp_pow<PR>(a, e);
}

// ---------------------------------------------------------------------------
// Fq2 = Fq[u] / (u^2 + 1)
// ---------------------------------------------------------------------------
struct Fq2 {
  Fq c0, c1;
};

ZK_DEV Fq2 f2_zero() { return {fp_zero<FqP>(), fp_zero<FqP>()}; }
ZK_DEV Fq2 f2_one() { return {fp_one<FqP>(), fp_zero<FqP>()}; }
ZK_DEV bool f2_is_zero(const Fq2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
ZK_DEV bool f2_eq(const Fq2& a, const Fq2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
ZK_DEV Fq2 f2_add(const Fq2& a, const Fq2& b) { return {fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
ZK_DEV Fq2 f2_sub(const Fq2& a, const Fq2& b) { return {fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
ZK_DEV Fq2 f2_neg(const Fq2& a) { return {fp_neg(a.c0), fp_neg(a.c1)}; }
ZK_DEV Fq2 f2_dbl(const Fq2& a) { return {fp_dbl(a.c0), fp_dbl(a.c1)}; }
ZK_DEV Fq2 f2_mul(const Fq2& a, const Fq2& b) {
  Fq t0 = fp_mul(a.c0, b.c0);
  Fq t1 = fp_mul(a.c1, b.c1);
  Fq t2 = fp_mul(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1));
  return {fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}
ZK_DEV Fq2 f2_sqr(const Fq2& a) {
  // (a0 + a1 u)^2 = (a0+a1)(a0-a1) + 2 a0 a1 u
  Fq t0 = fp_mul(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1));
  Fq t1 = fp_mul(a.c0, a.c1);
  return {t0, fp_dbl(t1)};
}
ZK_DEV Fq2 f2_inv(const Fq2& a) {
  Fq n = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  Fq ni = fp_inv(n);
  return {fp_mul(a.c0, ni), fp_neg(fp_mul(a.c1, ni))};
}
ZK_DEV Fq2 f2_from_mont(const Fq2& a) { return {fp_from_mont(a.c0), fp_from_mont(a.c1)}; }

// ---------------------------------------------------------------------------
// Uniform field interface used by the curve templates (G1 over Fq, G2 over Fq2)
// ---------------------------------------------------------------------------
struct FqOps {
  using T = Fq;
  static ZK_DEV T zero() { return fp_zero<FqP>(); }
  static ZK_DEV T one() { return fp_one<FqP>(); }
  static ZK_DEV bool is_zero(const T& a) { return fp_is_zero(a); }
  static ZK_DEV bool eq(const T& a, const T& b) { return fp_eq(a, b); }
  static ZK_DEV T add(const T& a, const T& b) { return fp_add(a, b); }
  static ZK_DEV T sub(const T& a, const T& b) { return fp_sub(a, b); }
  static ZK_DEV T neg(const T& a) { return fp_neg(a); }
  static ZK_DEV T dbl(const T& a) { return fp_dbl(a); }
  static ZK_DEV T mul(const T& a, const T& b) { return fp_mul(a, b); }
  static ZK_DEV T sqr(const T& a) { return fp_sqr(a); }
  // a*b - c*d with one reduction
  static ZK_DEV T mul_sub(const T& a, const T& b, const T& c, const T& d) {
    return fp_mul_sum2(a, b, fp_neg(c), d);
  }
  static ZK_DEV T inv(const T& a) { return fp_inv(a); }
  static ZK_DEV T from_mont(const T& a) { return fp_from_mont(a); }
  static ZK_DEV T canon(const T& a) { return a; }  // values are kept in [0, p)
};

struct Fq2Ops {
  using T = Fq2;
  static ZK_DEV T zero() { return f2_zero(); }
  static ZK_DEV T one() { return f2_one(); }
  static ZK_DEV bool is_zero(const T& a) { return f2_is_zero(a); }
  static ZK_DEV bool eq(const T& a, const T& b) { return f2_eq(a, b); }
  static ZK_DEV T add(const T& a, const T& b) { return f2_add(a, b); }
  static ZK_DEV T sub(const T& a, const T& b) { return f2_sub(a, b); }
  static ZK_DEV T neg(const T& a) { return f2_neg(a); }
  static ZK_DEV T dbl(const T& a) { return f2_dbl(a); }
  static ZK_DEV T mul(const T& a, const T& b) { return f2_mul(a, b); }
  static ZK_DEV T sqr(const T& a) { return f2_sqr(a); }
  static ZK_DEV T mul_sub(const T& a, const T& b, const T& c, const T& d) { return f2_sub(f2_mul(a, b), f2_mul(c, d)); }
  static ZK_DEV T canon(const T& a) { return a; }
  static ZK_DEV T inv(const T& a) { return f2_inv(a); }
  static ZK_DEV T from_mont(const T& a) { return f2_from_mont(a); }
};

// ---------------------------------------------------------------------------
// Compact-code Fq multiplication for the G1 accumulation loop: the whole product as one asm
// statement (tools/gen_fp_mul_asm.py: VOP2 carries through VCC, no hazard nops or register-pair
// shuffles between statements) is ~1.7 KB instead of ~2.9 KB.  The mixed addition inlines ten
// products, and the loop outgrew the instruction cache: rocprofv3 SQ_WAIT_INST_ANY was 43% of
// the G1 accumulation's wave cycles.  Same values as fp_mul (tests/test_gpu_parity.py).
// ---------------------------------------------------------------------------
#include "fp_mul_asm.h"

ZK_DEV Fq fq_mul_compact(const Fq& a, const Fq& b) {
  uint32_t u[8];
  ZK_FP_MUL_ASM(u, a.v, b.v, FqP::P, FqP::INV);
  Fq r;
  fp_reduce_once<FqP>(r.v, u);
  return r;
}

// a*b + c*d and sum_{k<4} x_k*y_k over Fq (one Montgomery reduction, one conditional
// subtraction).  The C forms (fp_mul_sum2 / fp_mul_sum4) compile to one asm statement per
// product, and the compiler pads every statement boundary with an s_nop (G2 accumulation: ~2,500
// s_nop of ~12,000 instructions); ZK_ASM_MULSUM selects one whole-asm statement per sum
// (tools/gen_fp_mul_asm.py) instead.  Measured on MI355X: G2 accumulation 0.961 (C) vs 0.981 ms
// (asm) per proof, bench flat — the other waves issue during the nops, and the compiler's
// interleaving of independent products in the C form is worth more (profiles/r02_s4_ab_asm_mul.log).
ZK_DEV Fq fq_mulsum2(const Fq& a, const Fq& b, const Fq& c, const Fq& d) {
#ifndef ZK_ASM_MULSUM
  return fp_mul_sum2(a, b, c, d);
#else
  uint32_t u[8];
  ZK_FP_MULSUM2_ASM(u, a.v, b.v, c.v, d.v, FqP::P, FqP::INV);
  Fq r;
  fp_reduce_once<FqP>(r.v, u);
  return r;
#endif
}

ZK_DEV Fq fq_mulsum4(const Fq* x, const Fq* y) {
#ifndef ZK_ASM_MULSUM
  return fp_mul_sum4(x, y);
#else
  uint32_t u[8];
  ZK_FP_MULSUM4_ASM(u, x[0].v, y[0].v, x[1].v, y[1].v, x[2].v, y[2].v, x[3].v, y[3].v, FqP::P, FqP::INV);
  Fq r;
  fp_reduce_once<FqP>(r.v, u);
  return r;
#endif
}

struct FqOpsCompact : FqOps {
  static ZK_DEV T mul(const T& a, const T& b) { return fq_mul_compact(a, b); }
  static ZK_DEV T sqr(const T& a) { return fq_mul_compact(a, a); }
};

// Redundant representation [0, 2p) for the G1 MSM kernels: 4p < 2^256, so a Montgomery product
// of two values < 2p is < 2p without the final conditional subtraction (~24 of ~320 instructions
// per product).  Additions / subtractions reduce modulo 2p, zero tests accept 0 and p, and the
// MSM result is brought back to [0, p) (canon) before it leaves the MSM kernels.
struct FqOpsLazy : FqOps {
  static constexpr uint32_t P2[8] = {0xb0f9fa8eu, 0x7841182du, 0xd0e3951au, 0x2f02d522u,
                                     0x0302b0bbu, 0x70a08b6du, 0xc2634053u, 0x60c89ce5u};  // 2q
  static ZK_DEV bool is_zero(const T& a) {
    uint32_t z = 0, e = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      z |= a.v[i];
      e |= a.v[i] ^ FqP::P[i];
    }
    return z == 0 || e == 0;
  }
  static ZK_DEV T add(const T& a, const T& b) {  // a + b < 4p -> [0, 2p)
    uint32_t s[8], t[8];
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      c += (uint64_t)a.v[i] + b.v[i];
      s[i] = (uint32_t)c;
      c >>= 32;
    }
    uint32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint64_t d = (uint64_t)s[i] - P2[i] - borrow;
      t[i] = (uint32_t)d;
      borrow = (uint32_t)(d >> 63);
    }
    T r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = borrow ? s[i] : t[i];
    return r;
  }
  static ZK_DEV T sub(const T& a, const T& b) {  // a - b in (-2p, 2p) -> [0, 2p)
    uint32_t d[8];
    uint32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint64_t t = (uint64_t)a.v[i] - b.v[i] - borrow;
      d[i] = (uint32_t)t;
      borrow = (uint32_t)(t >> 63);
    }
    const uint32_t mask = 0u - borrow;
    uint64_t c = 0;
    T r;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      c += (uint64_t)d[i] + (P2[i] & mask);
      r.v[i] = (uint32_t)c;
      c >>= 32;
    }
    return r;
  }
  static ZK_DEV T neg(const T& a) { return sub(fp_zero<FqP>(), a); }
  static ZK_DEV T dbl(const T& a) { return add(a, a); }
  static ZK_DEV T mul(const T& a, const T& b) {
    T r;
    ZK_FP_MUL_ASM(r.v, a.v, b.v, FqP::P, FqP::INV);
    return r;
  }
  static ZK_DEV T sqr(const T& a) { return mul(a, a); }
  // inputs < 2p: a*b + c*d < 8p^2, the product-sum is < 2.52p and its one subtraction of p leaves
  // it < 2p
  static ZK_DEV T mul_sub(const T& a, const T& b, const T& c, const T& d) {
    return fp_mul_sum2(a, b, neg(c), d);  // (the one-statement form needs 4 more VGPRs: spills at 128)
  }
  static ZK_DEV T canon(const T& a) {
    T r;
    fp_reduce_once<FqP>(r.v, a.v);
    return r;
  }
};

// ---------------------------------------------------------------------------
// Fq2 split across a lane pair (G2 MSM kernels).  Lanes 2k and 2k+1 hold components c0 and c1
// of the same Fq2 value; each lane keeps 8 registers per Fq2 instead of 16, so the G2 point
// kernels fit the register budget of 3-4 waves/SIMD instead of one wave owning the whole SIMD.
// A product costs each lane one sum of two Fq products with a single reduction (fp_mul_sum2),
// exchanging the partner's component through DPP (quad_perm [1,0,3,2]).
// Callers keep control flow pair-uniform (both lanes of a pair always active together).
// ---------------------------------------------------------------------------
ZK_DEV uint32_t pair_half() { return __lane_id() & 1u; }

ZK_DEV uint32_t pair_swap_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}

// the even / odd lane of each pair to both lanes: DPP quad_perm [0,0,2,2] / [1,1,3,3]
ZK_DEV uint32_t pair_even_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xA0, 0xF, 0xF, false);
}
ZK_DEV uint32_t pair_odd_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xF5, 0xF, 0xF, false);
}

ZK_DEV Fq pair_swap(const Fq& a) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = pair_swap_u32(a.v[i]);
  return r;
}

ZK_DEV Fq fq_sel(bool c, const Fq& a, const Fq& b) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}

struct Fq2PairOps {
  using T = Fq;  // this lane's component
  static ZK_DEV T zero() { return fp_zero<FqP>(); }
  static ZK_DEV T one() { return pair_half() ? fp_zero<FqP>() : fp_one<FqP>(); }
  static ZK_DEV bool is_zero(const T& a) {
    const uint32_t z = fp_is_zero(a) ? 1u : 0u;
    return (z & pair_swap_u32(z)) != 0;
  }
  static ZK_DEV bool eq(const T& a, const T& b) {
    const uint32_t e = fp_eq(a, b) ? 1u : 0u;
    return (e & pair_swap_u32(e)) != 0;
  }
  static ZK_DEV T add(const T& a, const T& b) { return fp_add(a, b); }
  static ZK_DEV T sub(const T& a, const T& b) { return fp_sub(a, b); }
  static ZK_DEV T neg(const T& a) { return fp_neg(a); }
  static ZK_DEV T dbl(const T& a) { return fp_dbl(a); }
  // c0 = a0 b0 + (-a1) b1 (lane 0), c1 = a1 b0 + a0 b1 (lane 1): one sum of two products with
  // a single Montgomery reduction per lane
  static ZK_DEV T mul(const T& a, const T& b) {
    const bool h = pair_half();
    const Fq pa = pair_swap(a), pb = pair_swap(b);
    return fq_mulsum2(a, fq_sel(h, pb, b), fq_sel(h, pa, fp_neg(pa)), fq_sel(h, b, pb));
  }
  // a*b - c*d over Fq2 as one four-product sum per lane:
  //   lane 0: a0 b0 + (-a1) b1 + (-c0) d0 + c1 d1,  lane 1: a1 b0 + a0 b1 + (-c1) d0 + (-c0) d1
  static ZK_DEV T mul_sub(const T& a, const T& b, const T& c, const T& d) {
    const bool h = pair_half();
    const Fq pa = pair_swap(a), pb = pair_swap(b), pc = pair_swap(c), pd = pair_swap(d);
    const Fq npc = fp_neg(pc);
    const Fq x[4] = {a, fq_sel(h, pa, fp_neg(pa)), fp_neg(c), fq_sel(h, npc, pc)};
    const Fq y[4] = {fq_sel(h, pb, b), fq_sel(h, b, pb), fq_sel(h, pd, d), fq_sel(h, d, pd)};
    return fq_mulsum4(x, y);
  }
  static ZK_DEV T canon(const T& a) { return a; }
  // c0 = (a0 + a1)(a0 - a1) (lane 0), c1 = 2 a0 a1 (lane 1)
  static ZK_DEV T sqr(const T& a) {
    const bool h = pair_half();
    const Fq pa = pair_swap(a);
#ifndef ZK_ASM_MULSUM
    const Fq t = fp_mul(fq_sel(h, a, fp_add(a, pa)), fq_sel(h, pa, fp_sub(a, pa)));
#else
    const Fq t = fq_mul_compact(fq_sel(h, a, fp_add(a, pa)), fq_sel(h, pa, fp_sub(a, pa)));
#endif
    return h ? fp_dbl(t) : t;
  }
};

}  // namespace zkfl
