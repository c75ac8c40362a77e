// BN254 Fq in nine 29-bit limbs (Montgomery R = 2^261) for the G1 MSM kernels.
//
// Why: the G1 accumulation is bound by the issue rate of the Fq multiply.  With
// 32-bit limbs every 32x32 product costs a v_mad_u64_u32 plus a v_addc_co_u32 for the third
// accumulator word.  With 29-bit limbs a product is < 2^58, so a whole column (up to 27 products
// of the operand kinds used here, plus the carry) fits one 64-bit accumulator: one
// v_mad_u64_u32 per product and no carry word.  tools/limb29_bench.hip: 171.8 vs 136.6 G
// Fq-mul/s on MI355X (9x9 + 9x9 products against 8x8 + 8x8 mad/addc pairs).
//
// Representation and bounds (p ~ 2^253.6, 2^256 ~ 5.29p, 2^261 ~ 169.3p):
//  * "normalized": limbs 0..7 < 2^29, limb 8 holds the rest (< 2^29).  "lazy": limbs 0..7 may
//    reach 3 * 2^29 (a sum or a borrowed difference, never fed to carry-sensitive code).
//  * A Montgomery product of values a, b is < p + a b / 2^261, normalized, no final subtraction:
//    for the operand ranges below always < 2p.
//  * Point coordinates between operations: X, Y < 6p, ZZ, ZZZ < 2p, all normalized; stored
//    points (buckets, items: 8 x 32-bit limbs) < 2^256 (below256 folds X, Y once).
//  * A difference a - b is a + K - b with K a multiple of p written "borrowed" (every lower
//    limb raised by d * 2^29, the next limb lowered by d), so no limb goes negative for up to d
//    normalized subtrahends; the per-call choice of K in f29_madd / f29_add / f29_dbl comes
//    from the bound analysis in their comments (checked by tests/test_field29.py).
//  * Column bound of the product sums: per product (limb_a * limb_b) <= 3 * 2^58 (one operand
//    normalized, the other lazy), so 9 + 9 products plus 9 reduction products stay
//    <= 54 * 2^58 < 2^64.
// The MSM stores data in this Montgomery domain (x 2^261); bases are converted at key load
// (k_msm_to_m29) and the MSM result is converted back to the 2^256 domain by canon.
#pragma once
#include "curve.h"

namespace zkfl {

#define ZK_HD __host__ __device__ __forceinline__

struct F29 {
  uint32_t v[9];
};

struct P29 {
  static constexpr uint32_t MASK = (1u << 29) - 1;
  static constexpr uint32_t NINV = 0x4866389u;  // -p^-1 mod 2^29
  static constexpr uint32_t P[9] = {0x187cfd47u, 0x010460b6u, 0x1c72a34fu, 0x02d522d0u, 0x1585d978u,
                                    0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
  static constexpr uint32_t P2[9] = {0x10f9fa8eu, 0x0208c16du, 0x18e5469eu, 0x05aa45a1u, 0x0b0bb2f0u,
                                     0x05b68181u, 0x014dc282u, 0x1cb84c68u, 0x0060c89cu};  // 2p
  static constexpr uint32_t ONE[9] = {0x157ccc21u, 0x141c2758u, 0x185230d3u, 0x014c0419u, 0x0aa36fb9u,
                                      0x1d4240ceu, 0x11d54c07u, 0x052ac7a8u, 0x000dc836u};  // 2^261 mod p
  static constexpr uint32_t C261[8] = {0x157ccc21u, 0x4e8384ebu, 0x0ce148c3u, 0xfb90a602u,
                                       0x819caa36u, 0x5301fa84u, 0x563d4475u, 0x0dc83629u};  // 2^261 mod p, 8 x 32
  // k p borrowed by d (name K<k>_<d>)
  static constexpr uint32_t K1_1[9] = {0x387cfd47u, 0x210460b5u, 0x3c72a34eu, 0x22d522cfu, 0x3585d977u,
                                       0x22db40bfu, 0x20a6e140u, 0x2e5c2633u, 0x0030644du};
  static constexpr uint32_t K2_1[9] = {0x30f9fa8eu, 0x2208c16cu, 0x38e5469du, 0x25aa45a0u, 0x2b0bb2efu,
                                       0x25b68180u, 0x214dc281u, 0x3cb84c67u, 0x0060c89bu};
  static constexpr uint32_t K3_2[9] = {0x4976f7d5u, 0x430d2222u, 0x5557e9ebu, 0x487f6870u, 0x40918c66u,
                                       0x4891c240u, 0x41f4a3c1u, 0x4b14729au, 0x00912ce9u};
  static constexpr uint32_t K4_3[9] = {0x61f3f51cu, 0x641182d8u, 0x71ca8d39u, 0x6b548b40u, 0x761765ddu,
                                       0x6b6d02ffu, 0x629b8501u, 0x797098cdu, 0x00c19136u};
  static constexpr uint32_t K5_1[9] = {0x3a70f263u, 0x2515e390u, 0x2e3d308au, 0x2e29ae13u, 0x2b9d3f57u,
                                       0x2e4843c2u, 0x23426644u, 0x27ccbf03u, 0x00f1f587u};
  static constexpr uint32_t K6_1[9] = {0x32edefaau, 0x261a4447u, 0x2aafd3d9u, 0x30fed0e4u, 0x212318cfu,
                                       0x31238483u, 0x23e94785u, 0x3628e537u, 0x012259d5u};
  static constexpr uint32_t K7_1[9] = {0x2b6aecf1u, 0x271ea4feu, 0x27227728u, 0x33d3f3b5u, 0x36a8f247u,
                                       0x33fec543u, 0x249028c6u, 0x24850b6bu, 0x0152be24u};
};

ZK_HD F29 f29_const(const uint32_t (&c)[9]) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = c[i];
  return r;
}

ZK_HD F29 f29_zero() {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = 0;
  return r;
}

// 8 x 32-bit (value < 2^256) <-> normalized 9 x 29-bit
ZK_HD F29 f29_pack(const uint32_t (&a)[8]) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int b = 29 * i, w = b >> 5, s = b & 31;
    uint32_t x = a[w] >> s;
    if (s > 3 && w + 1 < 8) x |= a[w + 1] << (32 - s);
    r.v[i] = x & P29::MASK;
  }
  return r;
}

ZK_HD void f29_unpack(uint32_t (&r)[8], const F29& a) {  // normalized, value < 2^256
#pragma unroll
  for (int w = 0; w < 8; w++) {
    const int b = 32 * w, i = b / 29, s = b % 29;
    uint32_t x = a.v[i] >> s;
    if (i + 1 < 9) x |= a.v[i + 1] << (29 - s);
    if (s > 26 && i + 2 < 9) x |= a.v[i + 2] << (58 - s);
    r[w] = x;
  }
}

// carry propagation; lower limbs non-negative (< 2^32), limb 8 wraps modulo 2^32 (the value is
// non-negative, so it comes out right)
ZK_HD void f29_norm(F29& a) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a.v[i + 1] += a.v[i] >> 29;
    a.v[i] &= P29::MASK;
  }
}

// a + K - b, lazy (no carries)
ZK_HD F29 f29_ksub(const uint32_t (&k)[9], const F29& a, const F29& b) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + k[i] - b.v[i];
  return r;
}

// a + K - b - c - d, lazy
ZK_HD F29 f29_ksub3(const uint32_t (&k)[9], const F29& a, const F29& b, const F29& c, const F29& d) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + k[i] - b.v[i] - c.v[i] - d.v[i];
  return r;
}

ZK_HD F29 f29_add_lazy(const F29& a, const F29& b) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + b.v[i];
  return r;
}

// normalized a < 2p: a == 0 mod p
ZK_HD bool f29_is_zero(const F29& a) {
  uint32_t z = 0, e = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    z |= a.v[i];
    e |= a.v[i] ^ P29::P[i];
  }
  return z == 0 || e == 0;
}

// normalized a < 6p -> normalized, < 2^256 (one conditional subtraction of 2p when a >= 2^256)
ZK_HD F29 f29_below256(const F29& a) {
  F29 t;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int32_t x = (int32_t)a.v[i] - (int32_t)P29::P2[i] + c;
    t.v[i] = (uint32_t)x & P29::MASK;
    c = x >> 29;
  }
  t.v[8] = a.v[8] - P29::P2[8] + (uint32_t)c;
  const bool big = (a.v[8] >> 24) != 0;
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = big ? t.v[i] : a.v[i];
  return r;
}

// Montgomery product a b 2^-261 (product scanning, one 64-bit column accumulator)
ZK_HD F29 f29_mul(const F29& a, const F29& b) {
  uint32_t m[9];
  F29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
#pragma unroll
    for (int i = 0; i < k; i++) {
      acc += (uint64_t)a.v[i] * b.v[k - i];
      acc += (uint64_t)m[i] * P29::P[k - i];
    }
    acc += (uint64_t)a.v[k] * b.v[0];
    m[k] = ((uint32_t)acc * P29::NINV) & P29::MASK;
    acc += (uint64_t)m[k] * P29::P[0];
    acc >>= 29;
  }
#pragma unroll
  for (int k = 9; k < 17; k++) {
#pragma unroll
    for (int i = k - 8; i < 9; i++) {
      acc += (uint64_t)a.v[i] * b.v[k - i];
      acc += (uint64_t)m[i] * P29::P[k - i];
    }
    r.v[k - 9] = (uint32_t)acc & P29::MASK;
    acc >>= 29;
  }
  r.v[8] = (uint32_t)acc;
  return r;
}

// (a b + c d) 2^-261 with one reduction
ZK_HD F29 f29_mulsum2(const F29& a, const F29& b, const F29& c, const F29& d) {
  uint32_t m[9];
  F29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
#pragma unroll
    for (int i = 0; i < k; i++) {
      acc += (uint64_t)a.v[i] * b.v[k - i];
      acc += (uint64_t)c.v[i] * d.v[k - i];
      acc += (uint64_t)m[i] * P29::P[k - i];
    }
    acc += (uint64_t)a.v[k] * b.v[0];
    acc += (uint64_t)c.v[k] * d.v[0];
    m[k] = ((uint32_t)acc * P29::NINV) & P29::MASK;
    acc += (uint64_t)m[k] * P29::P[0];
    acc >>= 29;
  }
#pragma unroll
  for (int k = 9; k < 17; k++) {
#pragma unroll
    for (int i = k - 8; i < 9; i++) {
      acc += (uint64_t)a.v[i] * b.v[k - i];
      acc += (uint64_t)c.v[i] * d.v[k - i];
      acc += (uint64_t)m[i] * P29::P[k - i];
    }
    r.v[k - 9] = (uint32_t)acc & P29::MASK;
    acc >>= 29;
  }
  r.v[8] = (uint32_t)acc;
  return r;
}

// Compute type of the G1 MSM kernels over this representation (storage: Affine/XYZZ<FqOps>).
struct FqOps29 {
  using T = F29;
  static ZK_DEV T zero() { return f29_zero(); }
  static ZK_DEV T one() { return f29_const(P29::ONE); }
  static ZK_DEV bool is_zero(const T& a) { return f29_is_zero(a); }
  static ZK_DEV T mul(const T& a, const T& b) { return f29_mul(a, b); }
  static ZK_DEV T sqr(const T& a) { return f29_mul(a, a); }
  static ZK_DEV T neg(const T& a) {  // a < p -> p - a in (0, p]
    T r = f29_ksub(P29::K1_1, f29_zero(), a);
    f29_norm(r);
    return r;
  }
  // MSM result: 2^261 domain -> canonical 2^256-domain value (x 2^261 * 2^251 * 2^-256)
  static ZK_DEV T canon(const T& a) {
    Fq u, c = fp_zero<FqP>();
    f29_unpack(u.v, f29_below256(a));
    c.v[7] = 1u << 27;
    return f29_pack(fp_mul(u, c).v);
  }
};

ZK_HD XYZZ<FqOps29> f29_inf() {
  return {f29_const(P29::ONE), f29_const(P29::ONE), f29_zero(), f29_zero()};
}

// dbl-2008-s-1.  In: X, Y < 6p, ZZ, ZZZ < 2p.
//   U = 2Y < 12p (lazy, limbs < 2^30); V = U^2 < 1.86p; W = U V < 1.14p; S = X V < 1.07p;
//   X^2 < 1.22p; M = 3 X^2 < 3.64p (normalized: it is squared); M^2 < 1.08p;
//   X3 = M^2 + 3p - 2S < 4.08p; SX = S + 5p - X3 < 6.07p (lazy); nY = 7p - Y (lazy);
//   Y3 = M SX + nY W < p + (3.64 * 6.07 + 7 * 1.14) p / 169 < 1.18p; ZZ3, ZZZ3 < 1.03p.
ZK_HD XYZZ<FqOps29> f29_dbl(const XYZZ<FqOps29>& p) {
  if (f29_is_zero(p.ZZ)) return p;
  const F29 U = f29_add_lazy(p.Y, p.Y);
  const F29 V = f29_mul(U, U);
  const F29 W = f29_mul(U, V);
  const F29 S = f29_mul(p.X, V);
  const F29 X2 = f29_mul(p.X, p.X);
  F29 M = f29_add_lazy(f29_add_lazy(X2, X2), X2);
  f29_norm(M);
  XYZZ<FqOps29> r;
  r.X = f29_ksub3(P29::K3_2, f29_mul(M, M), S, S, f29_zero());
  f29_norm(r.X);
  const F29 SX = f29_ksub(P29::K5_1, S, r.X);
  const F29 nY = f29_ksub(P29::K7_1, f29_zero(), p.Y);
  r.Y = f29_mulsum2(M, SX, nY, W);
  r.ZZ = f29_mul(V, p.ZZ);
  r.ZZZ = f29_mul(W, p.ZZZ);
  return r;
}

// madd-2008-s.  In: X1, Y1 < 6p, ZZ1, ZZZ1 < 2p; x < p, y <= p (canonical base, y possibly
// negated).  U2 = x ZZ1 < 1.02p, S2 = y ZZZ1 < 1.03p; P = U2 + 7p - X1 < 8.02p, R < 8.03p
// (normalized: squared); PP < 1.39p; PPP < 1.07p; Q = X1 PP < 1.05p; R^2 < 1.39p;
// X3 = R^2 + 4p - PPP - 2Q < 5.39p; QX = Q + 6p - X3 < 7.05p (lazy); nY = 7p - Y1 (lazy);
// Y3 = R QX + nY PPP < p + (8.03 * 7.05 + 7 * 1.07) p / 169 < 1.38p; ZZ3, ZZZ3 < 1.02p.
// P == 0 (mod p) is tested on PP (< 2p: 0 or p), R == 0 on R^2.
ZK_HD XYZZ<FqOps29> f29_madd(const XYZZ<FqOps29>& p, const Affine<FqOps29>& a) {
  if (f29_is_zero(a.x) && f29_is_zero(a.y)) return p;
  if (f29_is_zero(p.ZZ)) return {a.x, a.y, f29_const(P29::ONE), f29_const(P29::ONE)};
  const F29 U2 = f29_mul(a.x, p.ZZ);
  const F29 S2 = f29_mul(a.y, p.ZZZ);
  F29 P = f29_ksub(P29::K7_1, U2, p.X);
  F29 R = f29_ksub(P29::K7_1, S2, p.Y);
  f29_norm(P);
  f29_norm(R);
  const F29 PP = f29_mul(P, P);
  if (f29_is_zero(PP)) {
    if (f29_is_zero(f29_mul(R, R))) return f29_dbl({a.x, a.y, f29_const(P29::ONE), f29_const(P29::ONE)});
    return f29_inf();
  }
  const F29 PPP = f29_mul(P, PP);
  const F29 Q = f29_mul(p.X, PP);
  const F29 RR = f29_mul(R, R);
  XYZZ<FqOps29> r;
  r.X = f29_ksub3(P29::K4_3, RR, PPP, Q, Q);
  f29_norm(r.X);
  const F29 QX = f29_ksub(P29::K6_1, Q, r.X);
  const F29 nY = f29_ksub(P29::K7_1, f29_zero(), p.Y);
  r.Y = f29_mulsum2(R, QX, nY, PPP);
  r.ZZ = f29_mul(p.ZZ, PP);
  r.ZZZ = f29_mul(p.ZZZ, PPP);
  return r;
}

// add-2008-s.  In: X, Y < 6p, ZZ, ZZZ < 2p (both).  U1, U2, S1, S2 < 1.08p; P = U2 + 2p - U1,
// R < 3.08p (normalized); PP < 1.06p; PPP < 1.02p; Q = U1 PP < 1.01p; R^2 < 1.06p;
// X3 = R^2 + 4p - PPP - 2Q < 5.06p; QX = Q + 6p - X3 < 7.01p (lazy); nS1 = 2p - S1 (lazy);
// Y3 < p + (3.08 * 7.01 + 2 * 1.02) p / 169 < 1.14p; ZZ3, ZZZ3 < 1.01p.
ZK_HD XYZZ<FqOps29> f29_add(const XYZZ<FqOps29>& p, const XYZZ<FqOps29>& q) {
  if (f29_is_zero(q.ZZ)) return p;
  if (f29_is_zero(p.ZZ)) return q;
  const F29 U1 = f29_mul(p.X, q.ZZ);
  const F29 U2 = f29_mul(q.X, p.ZZ);
  const F29 S1 = f29_mul(p.Y, q.ZZZ);
  const F29 S2 = f29_mul(q.Y, p.ZZZ);
  F29 P = f29_ksub(P29::K2_1, U2, U1);
  F29 R = f29_ksub(P29::K2_1, S2, S1);
  f29_norm(P);
  f29_norm(R);
  const F29 PP = f29_mul(P, P);
  const F29 RR = f29_mul(R, R);
  if (f29_is_zero(PP)) {
    if (f29_is_zero(RR)) return f29_dbl(p);
    return f29_inf();
  }
  const F29 PPP = f29_mul(P, PP);
  const F29 Q = f29_mul(U1, PP);
  XYZZ<FqOps29> r;
  r.X = f29_ksub3(P29::K4_3, RR, PPP, Q, Q);
  f29_norm(r.X);
  const F29 QX = f29_ksub(P29::K6_1, Q, r.X);
  const F29 nS1 = f29_ksub(P29::K2_1, f29_zero(), S1);
  r.Y = f29_mulsum2(R, QX, nS1, PPP);
  r.ZZ = f29_mul(f29_mul(p.ZZ, q.ZZ), PP);
  r.ZZZ = f29_mul(f29_mul(p.ZZZ, q.ZZZ), PPP);
  return r;
}

// the generic point templates (curve.h) for this representation
template <>
ZK_DEV Affine<FqOps29> aff_neg<FqOps29>(const Affine<FqOps29>& a) {
  return {a.x, FqOps29::neg(a.y)};
}
template <>
ZK_DEV XYZZ<FqOps29> xyzz_madd<FqOps29>(const XYZZ<FqOps29>& p, const Affine<FqOps29>& a) {
  return f29_madd(p, a);
}
template <>
ZK_DEV XYZZ<FqOps29> xyzz_add<FqOps29>(const XYZZ<FqOps29>& p, const XYZZ<FqOps29>& q) {
  return f29_add(p, q);
}
template <>
ZK_DEV XYZZ<FqOps29> xyzz_dbl<FqOps29>(const XYZZ<FqOps29>& p) {
  return f29_dbl(p);
}

}  // namespace zkfl
