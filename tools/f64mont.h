// BN254 Fq Montgomery multiplication over five 52-bit limbs held in FP64 registers (R = 2^260):
// the FP64-FMA representation measured against the 29-bit integer engine (csrc/field29.h) by
// tools/fp_microbench.hip (round 6).  Not part of the product.
//
// A limb product x y (x, y < 2^52 exact integers in doubles, x y < 2^104) is split EXACTLY into
// column halves by two FMAs around a fixed exponent, with the FP64 rounding mode set to round
// toward zero (f64m::set_rz, once per kernel; every other FP64 operation here is exact):
//   h = fma(x, y, 2^104)            = 2^104 + H 2^52,  H = floor(x y / 2^52)    (binade ulp 2^52)
//   s = (2^104 + 2^52) - h          = (1 - H) 2^52                            (exact)
//   l = fma(x, y, s)                = L + 2^52,       L = x y - H 2^52 in [0, 2^52)
// (Round to nearest would leave L in [-2^51, 2^51]; the bias 3 2^51 that keeps l in one binade
// is not representable next to 2^104, so the split would need a fourth FP64 operation.)
// l lies in [2^52, 2^53), so the IEEE bit patterns are bits(h) = bits(2^104) + H and
// bits(l) = bits(2^52) + L: both halves are
// added to 64-bit integer column accumulators as raw bit patterns, and every column's exponent
// bias (a compile-time count of the products that landed in it) is subtracted once, modulo 2^64.
// Per limb product: 3 v_fma_f64 (the middle one is the exact subtraction) + 2 64-bit integer adds.
//
// Montgomery reduction is product-scanning (as f29_mont): column k < 5 yields m_k = t_k (-p^-1)
// mod 2^52 from its exact integer value t_k, m_k is turned into a double by the exponent trick
// (or 2^52's pattern into it, subtract 2^52), and m_k p_j is split like any other product.
// Output normalized (limbs < 2^52, limb 4 holds the rest); a product of a, b is < p + a b / 2^260,
// so inputs < 9p give < 1.96p, like the 29-bit engine's lazy bounds.
#pragma once
#include <cstdint>
#include <cstring>
#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define F64_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#define F64_HD inline
#endif

namespace f64m {

struct D52 {
  double v[5];
};

constexpr uint64_t M52 = (1ull << 52) - 1;
constexpr uint64_t P52[5] = {0x8c16d87cfd47ull, 0x916871ca8d3c2ull, 0x181585d97816aull, 0xa029b85045b68ull,
                             0x30644e72e131ull};
constexpr uint64_t PINV52 = 0x20782e4866389ull;  // -p^-1 mod 2^52
constexpr uint64_t BITS_C1 = 0x4670000000000000ull;  // bits(2^104)
constexpr uint64_t BITS_2P52 = 0x4330000000000000ull;  // bits(2^52)
constexpr uint64_t BITS_L = BITS_2P52;

F64_HD uint64_t dbits(double d) {
#ifdef __HIP_DEVICE_COMPILE__
  return (uint64_t)__double_as_longlong(d);
#else
  uint64_t u;
  memcpy(&u, &d, 8);
  return u;
#endif
}
F64_HD double bitsd(uint64_t u) {
#ifdef __HIP_DEVICE_COMPILE__
  return __longlong_as_double((long long)u);
#else
  double d;
  memcpy(&d, &u, 8);
  return d;
#endif
}
// v_fma_f64 as inline asm on the device: the compiler's mode-register pass marks every FP64
// instruction IT emits as needing round-to-nearest and writes MODE back to it in front of them,
// which would silently undo set_rz; it does not look inside asm statements.
F64_HD double ffma(double a, double b, double c) {
#ifdef __HIP_DEVICE_COMPILE__
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
#else
  return std::fma(a, b, c);
#endif
}
// FP64 rounding toward zero for the rest of the wave (MODE.FP_ROUND bits 3:2 = 3); every FP64
// operation of this file is an asm v_fma_f64 (ffma)
#ifdef __HIPCC__
__device__ __forceinline__ void set_rz() { __builtin_amdgcn_s_setreg(1 | (2 << 6) | (1 << 11), 3); }
#endif
// 0 <= u < 2^52 -> (double)u, exactly: 2^52 + u has u as its mantissa field
F64_HD double u52d(uint64_t u) { return ffma(bitsd(u | BITS_2P52), 1.0, -0x1p52); }

// x y split into its column halves' bit patterns: lo += bits(l), hi += bits(h)
F64_HD void prod(double x, double y, uint64_t& lo, uint64_t& hi) {
  const double h = ffma(x, y, 0x1p104);
  const double s = ffma(h, -1.0, 0x1p104 + 0x1p52);
  const double l = ffma(x, y, s);
  hi += dbits(h);
  lo += dbits(l);
}

// exponent bias of column k (mod 2^64): BITS_L per product whose low half lands in k, BITS_C1 per
// product whose high half does.  For k < 5 the m_k p_0 product is left out (it is added to t_k
// after m_k is known).
struct Bias {
  uint64_t b[10];
  constexpr Bias() : b{} {
    for (int k = 0; k < 10; k++) {
      uint64_t nl = 0, nh = 0;
      for (int i = 0; i < 5; i++)
        for (int j = 0; j < 5; j++) {
          const int c = i + j;
          if (c == k) nl += (k < 5 && j == 0) ? 1 : 2;  // x_i y_j and m_i p_j (m_k p_0 excluded)
          if (c + 1 == k) nh += 2;
        }
      b[k] = nl * BITS_L + nh * BITS_C1;
    }
  }
};

F64_HD D52 mul(const D52& a, const D52& b) {
  constexpr Bias B;
  uint64_t col[10];
#pragma unroll
  for (int k = 0; k < 10; k++) col[k] = 0;
  double md[5];
  int64_t carry = 0;
  D52 r;
#pragma unroll
  for (int k = 0; k < 10; k++) {
#pragma unroll
    for (int i = 0; i < 5; i++) {
      const int j = k - i;
      if (j < 0 || j > 4) continue;
      prod(a.v[i], b.v[j], col[k], col[k + 1 < 10 ? k + 1 : 9]);
      if (i < k) prod(md[i], (double)P52[j], col[k], col[k + 1 < 10 ? k + 1 : 9]);
    }
    const int64_t t = (int64_t)(col[k] - B.b[k]) + carry;
    if (k < 5) {
      const uint64_t m = ((uint64_t)t * PINV52) & M52;
      md[k] = u52d(m);
      uint64_t lo = 0;
      prod(md[k], (double)P52[0], lo, col[k + 1]);
      carry = (t + (int64_t)(lo - BITS_L)) >> 52;  // exact: t + m_k p_0 = 0 mod 2^52
    } else if (k < 9) {
      r.v[k - 5] = u52d((uint64_t)t & M52);
      carry = t >> 52;
    } else {
      r.v[4] = u52d((uint64_t)t);
    }
  }
  return r;
}

// 8 x 32-bit (value < 2^256) <-> 5 x 52-bit
F64_HD D52 pack(const uint32_t (&a)[8]) {
  uint64_t w[4];
  for (int i = 0; i < 4; i++) w[i] = (uint64_t)a[2 * i] | ((uint64_t)a[2 * i + 1] << 32);
  D52 r;
  for (int i = 0; i < 5; i++) {
    const int bit = 52 * i, q = bit >> 6, s = bit & 63;
    uint64_t x = w[q] >> s;
    if (s > 12 && q + 1 < 4) x |= w[q + 1] << (64 - s);
    r.v[i] = u52d(x & M52);
  }
  return r;
}
F64_HD void unpack(uint32_t (&r)[8], const D52& a) {  // normalized, value < 2^256
  uint64_t l[5];
  for (int i = 0; i < 5; i++) l[i] = dbits(ffma(a.v[i], 1.0, 0x1p52)) & M52;
  uint64_t w[4] = {0, 0, 0, 0};
  for (int i = 0; i < 5; i++) {
    const int bit = 52 * i, q = bit >> 6, s = bit & 63;
    if (q < 4) w[q] |= l[i] << s;
    if (s > 12 && q + 1 < 4) w[q + 1] |= l[i] >> (64 - s);
  }
  for (int i = 0; i < 4; i++) {
    r[2 * i] = (uint32_t)w[i];
    r[2 * i + 1] = (uint32_t)(w[i] >> 32);
  }
}

}  // namespace f64m
