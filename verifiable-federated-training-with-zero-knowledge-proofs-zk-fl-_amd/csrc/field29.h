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
  static constexpr uint32_t K3_1[9] = {0x2976f7d5u, 0x230d2223u, 0x3557e9ecu, 0x287f6871u, 0x20918c67u,
                                       0x2891c241u, 0x21f4a3c2u, 0x2b14729bu, 0x00912ceau};
  static constexpr uint32_t K4_1[9] = {0x21f3f51cu, 0x241182dau, 0x31ca8d3bu, 0x2b548b42u, 0x361765dfu,
                                       0x2b6d0301u, 0x229b8503u, 0x397098cfu, 0x00c19138u};
  static constexpr uint32_t K9_1[9] = {0x3c64e77fu, 0x2927666bu, 0x2007bdc6u, 0x397e3957u, 0x21b4a537u,
                                       0x39b546c5u, 0x25ddeb48u, 0x213d57d3u, 0x01b386c1u};
  static constexpr uint32_t K13_1[9] = {0x3e58dc9bu, 0x2d38e946u, 0x31d24b02u, 0x24d2c49au, 0x37cc0b18u,
                                        0x252249c7u, 0x2879704du, 0x3aadf0a3u, 0x027517fau};
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

// normalized a < 3p: a == 0 mod p (0, p or 2p)
ZK_HD bool f29_is_zero3(const F29& a) {
  uint32_t z = 0, e = 0, e2 = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    z |= a.v[i];
    e |= a.v[i] ^ P29::P[i];
    e2 |= a.v[i] ^ P29::P2[i];
  }
  return z == 0 || e == 0 || e2 == 0;
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

// Product-scanning Montgomery engine over NP operand pairs: (sum_j x_j y_j) 2^-261, one
// reduction.  Each column's products are dealt to two 64-bit accumulators in turn, kept apart by
// an empty asm barrier so the compiler cannot re-associate them into one chain: a lone column
// chain of dependent v_mad_u64_u32 made one product ~3,700 cycles of latency, two chains ~1,400
// (tools/limb29_bench.hip: 1537 -> 578 ns single-lane; 172 -> 166 G/s at full occupancy).
#ifndef F29_SPLIT
#define F29_SPLIT 1
#endif
// 1: the point formulas take their independent products two at a time (f29_mont2); 0: one at a
// time, each column split over two accumulators (A/B builds).  G1 madd: 2,345 -> 2,211 VALU
// instructions per entry (the 17 column joins of each paired product gone); +2.0% proofs/s,
// 4 same-box alternations (profiles/r05_ab_paired2.log)
#ifndef F29_PAIRED
#define F29_PAIRED 1
#endif
// 1 (default): the madd's last products as a triple and a pair (f29_mont3), so no product of the
// G1 madd joins split columns: formula 2,211 -> 2,194 VALU per entry (tools/isa_check.py census);
// the G1 accumulation 1.5807 vs 1.5901 ms per proof alone (2 traced runs each), 429 vs 427 proofs/s
// (4 same-box alternations, profiles/r05_ab_triple.log)
#ifndef F29_TRIPLE
#define F29_TRIPLE 1
#endif
ZK_HD void f29_keep(uint64_t& a) {
#ifdef __HIP_DEVICE_COMPILE__
  asm volatile("" : "+v"(a));
#else
  (void)a;
#endif
}

// NACC: accumulators per column (chains a lone wave can issue from; every extra chain costs one
// 64-bit join per column: the throughput kernels take 2, and so do k_assemble's quad additions,
// where 4 measured no better, profiles/r05_ab_q29_acc.log).  M: the modulus (P29 = Fq; R29 = Fr, fr29.h) -- MASK, NINV, P[9].
template <int NP, int NACC = (F29_SPLIT ? 2 : 1), class M = P29>
ZK_HD F29 f29_mont(const F29 (&x)[NP], const F29 (&y)[NP]) {
  static_assert(NACC == 1 || NACC == 2 || NACC == 4, "accumulators per column");
  uint32_t m[9];
  F29 r;
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
    uint64_t acc[NACC];
    acc[0] = carry;
#pragma unroll
    for (int q = 1; q < NACC; q++) acc[q] = 0;
    int t = 0;
    const int lo = k < 9 ? 0 : k - 8, hi = k < 9 ? k : 8;
#pragma unroll
    for (int i = lo; i <= hi; i++) {
#pragma unroll
      for (int j = 0; j < NP; j++) acc[(t++) % NACC] += (uint64_t)x[j].v[i] * y[j].v[k - i];
      if (i < k) acc[(t++) % NACC] += (uint64_t)m[i] * M::P[k - i];  // m_k is not known yet
    }
#pragma unroll
    for (int q = 0; q < NACC; q++) f29_keep(acc[q]);
    uint64_t c = acc[0];
    if (NACC == 4) c = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    else if (NACC == 2) c = acc[0] + acc[1];
    if (k < 9) {
      m[k] = ((uint32_t)c * M::NINV) & M::MASK;
      c += (uint64_t)m[k] * M::P[0];
    } else {
      r.v[k - 9] = (uint32_t)c & M::MASK;
    }
    carry = c >> 29;
  }
  r.v[8] = (uint32_t)carry;
  return r;
}

// Montgomery product a b 2^-261
template <class M = P29>
ZK_HD F29 f29_mul(const F29& a, const F29& b) {
  const F29 x[1] = {a}, y[1] = {b};
  return f29_mont<1, (F29_SPLIT ? 2 : 1), M>(x, y);
}

// The same product with ACC accumulators per column (latency-bound single-wave kernels)
template <int ACC>
ZK_HD F29 f29_mul_acc(const F29& a, const F29& b) {
  const F29 x[1] = {a}, y[1] = {b};
  return f29_mont<1, ACC>(x, y);
}

// Montgomery square a^2 2^-261 of a NORMALIZED a (every limb < 2^29): the cross products
// a_i a_j (i < j) are taken once against the doubled limb 2 a_i < 2^30, so 45 limb products
// instead of 81 (+ the 81 of the reduction).  Column bound: <= 4 cross products < 2^59 and one
// square < 2^58, plus 9 reduction products < 2^58: 18 x 2^58 < 2^63.  Same value, same
// Montgomery bound (< p + a^2 / 2^261) as f29_mul(a, a).
template <class M = P29>
ZK_HD F29 f29_sqr(const F29& a) {
  uint32_t a2[9];
#pragma unroll
  for (int i = 0; i < 9; i++) a2[i] = a.v[i] << 1;
  uint32_t m[9];
  F29 r;
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
    uint64_t acc[2] = {carry, 0};
    int t = 0;
    const int lo = k < 9 ? 0 : k - 8, hi = k < 9 ? k : 8;
#pragma unroll
    for (int i = lo; i <= hi; i++) {
      const int j = k - i;
      if (i < j) acc[F29_SPLIT ? (t++ & 1) : 0] += (uint64_t)a2[i] * a.v[j];
      else if (i == j) acc[F29_SPLIT ? (t++ & 1) : 0] += (uint64_t)a.v[i] * a.v[i];
      if (i < k) acc[F29_SPLIT ? (t++ & 1) : 0] += (uint64_t)m[i] * M::P[k - i];
    }
    f29_keep(acc[0]);
    f29_keep(acc[1]);
    uint64_t c = acc[0] + acc[1];
    if (k < 9) {
      m[k] = ((uint32_t)c * M::NINV) & M::MASK;
      c += (uint64_t)m[k] * M::P[0];
    } else {
      r.v[k - 9] = (uint32_t)c & M::MASK;
    }
    carry = c >> 29;
  }
  r.v[8] = (uint32_t)carry;
  return r;
}

// Two INDEPENDENT Montgomery products side by side: A = (sum_j xa_j ya_j) 2^-261 and B likewise,
// their columns interleaved with ONE 64-bit accumulator per product per column.  f29_mont splits
// each column over two accumulators so that a product has two dependency chains to issue from,
// and pays one 64-bit addition per column (17 per product) to join them; here the second chain is
// the other product, so the joins are gone and a wave still has two chains per column (and the
// carry of one column no longer waits for the other accumulator's join).  SQA / SQB: that
// product is the square of xa[0] / xb[0] (normalized), taking each cross product a_i a_j (i < j)
// once against the doubled limb, as f29_sqr.  Same values and bounds as f29_mont / f29_sqr.
// Both results come back by value and every loop runs over constant bounds (the inner loop over all
// nine limbs, its terms guarded by constant conditions): with output references and k-dependent
// inner bounds the first version kept a product's limbs in scratch memory (76 B of stack per lane).
struct F29x2 {
  F29 a, b;
};
template <int NA, int NB, bool SQA, bool SQB>
ZK_HD F29x2 f29_mont2(const F29 (&xa)[NA], const F29 (&ya)[NA], const F29 (&xb)[NB], const F29 (&yb)[NB]) {
  uint32_t da[9], db[9];  // doubled limbs of the squared operands (unused otherwise)
#pragma unroll
  for (int i = 0; i < 9; i++) {
    da[i] = SQA ? xa[0].v[i] << 1 : 0u;
    db[i] = SQB ? xb[0].v[i] << 1 : 0u;
  }
  uint32_t ma[9], mb[9];
  F29x2 r;
  uint64_t ca = 0, cb = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
    uint64_t a = ca, b = cb;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j < 0 || j > 8) continue;
      if (SQA) {
        if (i < j) a += (uint64_t)da[i] * xa[0].v[j];
        else if (i == j) a += (uint64_t)xa[0].v[i] * xa[0].v[i];
      } else {
#pragma unroll
        for (int q = 0; q < NA; q++) a += (uint64_t)xa[q].v[i] * ya[q].v[j];
      }
      if (SQB) {
        if (i < j) b += (uint64_t)db[i] * xb[0].v[j];
        else if (i == j) b += (uint64_t)xb[0].v[i] * xb[0].v[i];
      } else {
#pragma unroll
        for (int q = 0; q < NB; q++) b += (uint64_t)xb[q].v[i] * yb[q].v[j];
      }
      if (i < k && i < 9) {
        a += (uint64_t)ma[i] * P29::P[j];
        b += (uint64_t)mb[i] * P29::P[j];
      }
    }
    f29_keep(a);
    f29_keep(b);
    if (k < 9) {
      ma[k] = ((uint32_t)a * P29::NINV) & P29::MASK;
      mb[k] = ((uint32_t)b * P29::NINV) & P29::MASK;
      a += (uint64_t)ma[k] * P29::P[0];
      b += (uint64_t)mb[k] * P29::P[0];
    } else {
      r.a.v[k - 9] = (uint32_t)a & P29::MASK;
      r.b.v[k - 9] = (uint32_t)b & P29::MASK;
    }
    ca = a >> 29;
    cb = b >> 29;
  }
  r.a.v[8] = (uint32_t)ca;
  r.b.v[8] = (uint32_t)cb;
  return r;
}

// Three independent product sums side by side (as f29_mont2, no squares): one accumulator each per
// column, so three chains and no joins.  Used by the madd for PPP | Q | ZZ3 (F29_TRIPLE).
struct F29x3 {
  F29 a, b, c;
};
template <int NA, int NB, int NC>
ZK_HD F29x3 f29_mont3(const F29 (&xa)[NA], const F29 (&ya)[NA], const F29 (&xb)[NB], const F29 (&yb)[NB],
                      const F29 (&xc)[NC], const F29 (&yc)[NC]) {
  uint32_t ma[9], mb[9], mc[9];
  F29x3 r;
  uint64_t ca = 0, cb = 0, cc = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
    uint64_t a = ca, b = cb, c = cc;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j < 0 || j > 8) continue;
#pragma unroll
      for (int q = 0; q < NA; q++) a += (uint64_t)xa[q].v[i] * ya[q].v[j];
#pragma unroll
      for (int q = 0; q < NB; q++) b += (uint64_t)xb[q].v[i] * yb[q].v[j];
#pragma unroll
      for (int q = 0; q < NC; q++) c += (uint64_t)xc[q].v[i] * yc[q].v[j];
      if (i < k) {
        a += (uint64_t)ma[i] * P29::P[j];
        b += (uint64_t)mb[i] * P29::P[j];
        c += (uint64_t)mc[i] * P29::P[j];
      }
    }
    f29_keep(a);
    f29_keep(b);
    f29_keep(c);
    if (k < 9) {
      ma[k] = ((uint32_t)a * P29::NINV) & P29::MASK;
      mb[k] = ((uint32_t)b * P29::NINV) & P29::MASK;
      mc[k] = ((uint32_t)c * P29::NINV) & P29::MASK;
      a += (uint64_t)ma[k] * P29::P[0];
      b += (uint64_t)mb[k] * P29::P[0];
      c += (uint64_t)mc[k] * P29::P[0];
    } else {
      r.a.v[k - 9] = (uint32_t)a & P29::MASK;
      r.b.v[k - 9] = (uint32_t)b & P29::MASK;
      r.c.v[k - 9] = (uint32_t)c & P29::MASK;
    }
    ca = a >> 29;
    cb = b >> 29;
    cc = c >> 29;
  }
  r.a.v[8] = (uint32_t)ca;
  r.b.v[8] = (uint32_t)cb;
  r.c.v[8] = (uint32_t)cc;
  return r;
}

// {a b, c d} (two independent products, f29_mont2)
ZK_HD F29x2 f29_mul2(const F29& a, const F29& b, const F29& c, const F29& d) {
  const F29 xa[1] = {a}, ya[1] = {b}, xb[1] = {c}, yb[1] = {d};
  return f29_mont2<1, 1, false, false>(xa, ya, xb, yb);
}

// {a^2, c^2} of NORMALIZED a, c (two independent squares, f29_mont2)
ZK_HD F29x2 f29_sqr2(const F29& a, const F29& c) {
  const F29 xa[1] = {a}, xb[1] = {c};
  return f29_mont2<1, 1, true, true>(xa, xa, xb, xb);
}

// (a b + c d) 2^-261 with one reduction
ZK_HD F29 f29_mulsum2(const F29& a, const F29& b, const F29& c, const F29& d) {
  const F29 x[2] = {a, c}, y[2] = {b, d};
  return f29_mont<2>(x, y);
}

// (sum_{j<4} x_j y_j) 2^-261 with one reduction (the G2 y-coordinate product pair)
ZK_HD F29 f29_mulsum4(const F29 (&x)[4], const F29 (&y)[4]) { return f29_mont<4>(x, y); }

// Compute type of the G1 MSM kernels over this representation (storage: Affine/XYZZ<FqOps>).
struct FqOps29 {
  using T = F29;
  static ZK_DEV T zero() { return f29_zero(); }
  static ZK_DEV T one() { return f29_const(P29::ONE); }
  static ZK_DEV bool is_zero(const T& a) { return f29_is_zero(a); }
  static ZK_DEV T mul(const T& a, const T& b) { return f29_mul(a, b); }
  static ZK_DEV T sqr(const T& a) { return f29_mul(a, a); }  // a may be lazy here: not f29_sqr
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
  F29 U = f29_add_lazy(p.Y, p.Y);
  f29_norm(U);  // squared below (f29_sqr takes normalized limbs)
  const F29 V = f29_sqr(U);
  const F29 W = f29_mul(U, V);
  const F29 S = f29_mul(p.X, V);
  const F29 X2 = f29_sqr(p.X);
  F29 M = f29_add_lazy(f29_add_lazy(X2, X2), X2);
  f29_norm(M);
  XYZZ<FqOps29> r;
  r.X = f29_ksub3(P29::K3_2, f29_sqr(M), S, S, f29_zero());
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
  const F29 PP = f29_sqr(P);
  if (f29_is_zero(PP)) {
    if (f29_is_zero(f29_sqr(R))) return f29_dbl({a.x, a.y, f29_const(P29::ONE), f29_const(P29::ONE)});
    return f29_inf();
  }
  const F29 PPP = f29_mul(P, PP);
  const F29 Q = f29_mul(p.X, PP);
  const F29 RR = f29_sqr(R);
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

// madd of the base (x, y) or, for neg, of (x, -y) -- the MSM accumulation's signed digit.
// Instead of negating y (a subtraction, a carry pass and a select per limb) the sign is applied
// to S2 = y ZZZ1 < 1.03p: t = 2p - S2 for neg (borrowed 2p, lazy, limbs < 2^30), else S2, and
// R = t + 7p - Y1 < 9.03p (normalized: squared); RR < p + 9.03^2 p / 169 = 1.49p;
// X3 = RR + 4p - PPP - 2Q < 5.49p; Y3 < p + (9.03 * 7.05 + 7 * 1.07) p / 169 < 1.43p; the rest as
// f29_madd.  A base at infinity is stored as (0, 0); a canonical base is never p, and y = 0 is
// no point of the prime-order group, so a plain all-limbs-zero test suffices for it.
ZK_HD XYZZ<FqOps29> f29_madd_signed(const XYZZ<FqOps29>& p, const Affine<FqOps29>& a, bool neg) {
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) z |= a.x.v[i] | a.y.v[i];
  if (z == 0) return p;
  if (f29_is_zero(p.ZZ)) {
    F29 y = a.y;
    if (neg) {
      y = f29_ksub(P29::K1_1, f29_zero(), a.y);
      f29_norm(y);
    }
    return {a.x, y, f29_const(P29::ONE), f29_const(P29::ONE)};
  }
#if F29_PAIRED
  // the same products as below, two independent ones at a time (f29_mont2): U2 | S2, PP | RR,
  // PPP | Q, ZZ3 | ZZZ3, then Y3 (a two-product sum: its own two chains)
  const F29x2 us = f29_mul2(a.x, p.ZZ, a.y, p.ZZZ);
  const F29 U2 = us.a, S2 = us.b;
  F29 t;
#pragma unroll
  for (int i = 0; i < 9; i++) t.v[i] = neg ? P29::K2_1[i] - S2.v[i] : S2.v[i];
  F29 P = f29_ksub(P29::K7_1, U2, p.X);
  F29 R = f29_ksub(P29::K7_1, t, p.Y);
  f29_norm(P);
  f29_norm(R);
  const F29x2 sq = f29_sqr2(P, R);
  const F29 PP = sq.a, RR = sq.b;
  if (f29_is_zero(PP)) {
    if (f29_is_zero(RR)) {
      F29 y = a.y;
      if (neg) {
        y = f29_ksub(P29::K1_1, f29_zero(), a.y);
        f29_norm(y);
      }
      return f29_dbl({a.x, y, f29_const(P29::ONE), f29_const(P29::ONE)});
    }
    return f29_inf();
  }
#if F29_TRIPLE
  // PPP | Q | ZZ3 as three chains, then ZZZ3 | Y3 (Y3's two products in one accumulator): no
  // column joins at all
  const F29 x3a[1] = {P}, x3b[1] = {p.X}, x3c[1] = {p.ZZ}, y3[1] = {PP};
  const F29x3 t3 = f29_mont3<1, 1, 1>(x3a, y3, x3b, y3, x3c, y3);
  const F29 PPP = t3.a, Q = t3.b;
  F29 X3 = f29_ksub3(P29::K4_3, RR, PPP, Q, Q);
  f29_norm(X3);
  const F29 QX = f29_ksub(P29::K6_1, Q, X3);
  const F29 nY = f29_ksub(P29::K7_1, f29_zero(), p.Y);
  const F29 xz[1] = {p.ZZZ}, yz[1] = {PPP}, xy[2] = {R, nY}, yy[2] = {QX, PPP};
  const F29x2 zy = f29_mont2<1, 2, false, false>(xz, yz, xy, yy);
  return {X3, zy.b, t3.c, zy.a};
#else
  const F29x2 pq = f29_mul2(P, PP, p.X, PP);
  const F29 PPP = pq.a, Q = pq.b;
  const F29x2 zz = f29_mul2(p.ZZ, PP, p.ZZZ, PPP);
  F29 X3 = f29_ksub3(P29::K4_3, RR, PPP, Q, Q);
  f29_norm(X3);
  const F29 QX = f29_ksub(P29::K6_1, Q, X3);
  const F29 nY = f29_ksub(P29::K7_1, f29_zero(), p.Y);
  // the result as one aggregate: a named XYZZ filled member by member here kept two coordinates in
  // scratch memory (its slot merged with the early returns' through a pointer phi)
  return {X3, f29_mulsum2(R, QX, nY, PPP), zz.a, zz.b};
#endif
#else
  const F29 U2 = f29_mul(a.x, p.ZZ);
  const F29 S2 = f29_mul(a.y, p.ZZZ);
  F29 t;
#pragma unroll
  for (int i = 0; i < 9; i++) t.v[i] = neg ? P29::K2_1[i] - S2.v[i] : S2.v[i];
  F29 P = f29_ksub(P29::K7_1, U2, p.X);
  F29 R = f29_ksub(P29::K7_1, t, p.Y);
  f29_norm(P);
  f29_norm(R);
  const F29 PP = f29_sqr(P);
  if (f29_is_zero(PP)) {
    if (f29_is_zero(f29_sqr(R))) {
      F29 y = a.y;
      if (neg) {
        y = f29_ksub(P29::K1_1, f29_zero(), a.y);
        f29_norm(y);
      }
      return f29_dbl({a.x, y, f29_const(P29::ONE), f29_const(P29::ONE)});
    }
    return f29_inf();
  }
  const F29 PPP = f29_mul(P, PP);
  const F29 Q = f29_mul(p.X, PP);
  const F29 RR = f29_sqr(R);
  XYZZ<FqOps29> r;
  r.X = f29_ksub3(P29::K4_3, RR, PPP, Q, Q);
  f29_norm(r.X);
  const F29 QX = f29_ksub(P29::K6_1, Q, r.X);
  const F29 nY = f29_ksub(P29::K7_1, f29_zero(), p.Y);
  r.Y = f29_mulsum2(R, QX, nY, PPP);
  r.ZZ = f29_mul(p.ZZ, PP);
  r.ZZZ = f29_mul(p.ZZZ, PPP);
  return r;
#endif
}

// ---------------------------------------------------------------------------
// Canonicalization and inversion (the assembly's affine conversions, k_assemble)
// ---------------------------------------------------------------------------
// normalized a < (k + 1) p -> canonical (< p): k conditional subtractions of p (M: the modulus)
template <int K, class M = P29>
ZK_HD F29 f29_canon_sub(F29 a) {
#pragma unroll
  for (int t = 0; t < K; t++) {
    F29 s;
    int32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int32_t x = (int32_t)a.v[i] - (int32_t)M::P[i] + c;
      s.v[i] = (uint32_t)x & M::MASK;
      c = x >> 29;
    }
    const int32_t top = (int32_t)a.v[8] - (int32_t)M::P[8] + c;
    s.v[8] = (uint32_t)top;
    const bool ge = top >= 0;
#pragma unroll
    for (int i = 0; i < 9; i++) a.v[i] = ge ? s.v[i] : a.v[i];
  }
  return a;
}

struct P29Inv {
  // R^3 mod p (R = 2^261): a plain inverse x = (aR)^-1 times R^3 through a Montgomery product is
  // a^-1 R (the Montgomery form of the inverse)
  static constexpr uint32_t R3[9] = {0x0e2312b2u, 0x16c05ca2u, 0x0bc84389u, 0x1cdf310bu, 0x11adafddu,
                                     0x032e568eu, 0x1d6ae48cu, 0x10d4cd1fu, 0x0026c2d2u};
};

// a^-1 (the assembly's inversions, one lane each): in normalized a < 2p (Montgomery form a R), out
// a^-1 R < p; a = 0 mod p gives 0 (as the Fermat inverse 0^(p-2)).  Bernstein-Yang divsteps ("Fast
// constant-time gcd computation and modular inversion", 2019) in the 30-bit-limb form of
// libsecp256k1's modinv32: 20 batches of 30 divsteps,
// each batch run on the low 30 bits of f and g alone (a 2 x 2 transition matrix scaled by 2^30),
// then applied to the full f, g and to the Bezout coefficients d, e -- the latter mod p, plus the
// multiple of p that makes them divisible by 2^30.  600 >= 590 divsteps settle any input below
// 2^256 (f = +-1, d = +-(aR)^-1).  A fixed sequence of ~13 k 32/64-bit integer instructions on one
// lane: the binary extended Euclid it replaced (~500 data-dependent rounds of 9-limb shifts and
// subtractions) took 248 against 123 us in k_assemble_c (profiles/r06_ab_divsteps.log), Fermat's
// chain of ~316 dependent products ~5x the Euclid.
struct S30 {
  int32_t v[9];  // signed 30-bit limbs: 0..7 in [0, 2^30), limb 8 signed
};
constexpr int32_t S30_M = (1 << 30) - 1;
// normalized 29-bit limbs (value < 2^261) -> 30-bit limbs
ZK_HD constexpr S30 s30_from29(const uint32_t (&a)[9]) {
  S30 r{};
  uint64_t acc = 0;
  int bits = 0, k = 0;
  for (int i = 0; i < 9; i++) {
    acc |= (uint64_t)a[i] << bits;
    bits += 29;
    if (bits >= 30) {
      r.v[k++] = (int32_t)(acc & S30_M);
      acc >>= 30;
      bits -= 30;
    }
  }
  r.v[8] = (int32_t)acc;
  return r;
}
// 30-bit limbs of a value in [0, 2^261) -> normalized 29-bit limbs
ZK_HD F29 f29_from30(const S30& a) {
  F29 r;
  uint64_t acc = 0;
  int bits = 0, k = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    acc |= (uint64_t)(uint32_t)a.v[i] << bits;
    bits += 30;
    while (bits >= 29 && k < 8) {
      r.v[k++] = (uint32_t)acc & P29::MASK;
      acc >>= 29;
      bits -= 29;
    }
  }
  r.v[8] = (uint32_t)acc;
  return r;
}
ZK_HD constexpr uint32_t inv_mod2_30(uint32_t a) {  // a^-1 mod 2^30, a odd (Newton doubles the good bits)
  uint32_t x = a;
  for (int i = 0; i < 5; i++) x *= 2u - a * x;
  return x & (uint32_t)S30_M;
}
struct P30 {
  static constexpr S30 P = s30_from29(P29::P);
  static constexpr uint32_t INV = inv_mod2_30((uint32_t)s30_from29(P29::P).v[0]);  // p^-1 mod 2^30
};
struct DivTrans {
  int32_t u, v, q, r;
};
// 30 divsteps on the low bits of f (odd) and g; zeta = -(delta + 1/2).  Branch-free: masks pick
// g +- f, and the swap when delta > 0 and g is odd.
ZK_HD int32_t divsteps30(int32_t zeta, uint32_t f, uint32_t g, DivTrans& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll
  for (int i = 0; i < 30; i++) {
    uint32_t c1 = (uint32_t)(zeta >> 31);  // delta > 0
    const uint32_t c2 = 0u - (g & 1u);     // g odd
    const uint32_t x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
    g += x & c2;
    q += y & c2;
    r += z & c2;
    c1 &= c2;  // swap
    zeta = (zeta ^ (int32_t)c1) - 1;
    f += g & c1;
    u += q & c1;
    v += r & c1;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  t = {(int32_t)u, (int32_t)v, (int32_t)q, (int32_t)r};
  return zeta;
}
// (f, g) <- t (f, g) / 2^30 (exact)
ZK_HD void update_fg30(S30& f, S30& g, const DivTrans& t) {
  int64_t cf = (int64_t)t.u * f.v[0] + (int64_t)t.v * g.v[0];
  int64_t cg = (int64_t)t.q * f.v[0] + (int64_t)t.r * g.v[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    cf += (int64_t)t.u * f.v[i] + (int64_t)t.v * g.v[i];
    cg += (int64_t)t.q * f.v[i] + (int64_t)t.r * g.v[i];
    f.v[i - 1] = (int32_t)cf & S30_M;
    g.v[i - 1] = (int32_t)cg & S30_M;
    cf >>= 30;
    cg >>= 30;
  }
  f.v[8] = (int32_t)cf;
  g.v[8] = (int32_t)cg;
}
// (d, e) <- (t (d, e) + p (md, me)) / 2^30, md, me chosen so the division is exact; d, e stay in
// (-2p, p)
ZK_HD void update_de30(S30& d, S30& e, const DivTrans& t) {
  const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
  int32_t md = (t.u & sd) + (t.v & se), me = (t.q & sd) + (t.r & se);
  int64_t cd = (int64_t)t.u * d.v[0] + (int64_t)t.v * e.v[0];
  int64_t ce = (int64_t)t.q * d.v[0] + (int64_t)t.r * e.v[0];
  md -= (int32_t)((P30::INV * (uint32_t)cd + (uint32_t)md) & (uint32_t)S30_M);
  me -= (int32_t)((P30::INV * (uint32_t)ce + (uint32_t)me) & (uint32_t)S30_M);
  cd += (int64_t)P30::P.v[0] * md;
  ce += (int64_t)P30::P.v[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    cd += (int64_t)t.u * d.v[i] + (int64_t)t.v * e.v[i] + (int64_t)P30::P.v[i] * md;
    ce += (int64_t)t.q * d.v[i] + (int64_t)t.r * e.v[i] + (int64_t)P30::P.v[i] * me;
    d.v[i - 1] = (int32_t)cd & S30_M;
    e.v[i - 1] = (int32_t)ce & S30_M;
    cd >>= 30;
    ce >>= 30;
  }
  d.v[8] = (int32_t)cd;
  e.v[8] = (int32_t)ce;
}
// x + s p (s = 0 or +-1) with the limbs carried: 0..7 in [0, 2^30), limb 8 signed
ZK_HD S30 s30_addp(const S30& x, int32_t s) {
  S30 r;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    c += (int64_t)x.v[i] + (int64_t)s * P30::P.v[i];
    r.v[i] = i < 8 ? (int32_t)c & S30_M : (int32_t)c;
    c >>= 30;
  }
  return r;
}
ZK_HD F29 f29_inv_divsteps(const F29& a_in) {
  const F29 a = f29_canon_sub<1>(a_in);
  {
    uint32_t z = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) z |= a.v[i];
    if (z == 0) return f29_zero();
  }
  S30 f = P30::P, g = s30_from29(a.v), d{}, e{};
  e.v[0] = 1;
  int32_t zeta = -1;
#pragma unroll 1
  for (int i = 0; i < 20; i++) {
    DivTrans t;
    zeta = divsteps30(zeta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    update_de30(d, e, t);
    update_fg30(f, g, t);
  }
  // f = +-1: d (in (-2p, p)) times its sign is (aR)^-1 mod p; carry it, then bring it into [0, p)
  const int32_t neg = f.v[8] >> 31;
  S30 x;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    c += (int64_t)((d.v[i] ^ neg) - neg);
    x.v[i] = i < 8 ? (int32_t)c & S30_M : (int32_t)c;
    c >>= 30;
  }
#pragma unroll
  for (int k = 0; k < 2; k++) x = s30_addp(x, x.v[8] < 0 ? 1 : 0);  // (-2p, 2p) -> [0, 2p)
  const S30 y = s30_addp(x, -1);
  if (y.v[8] >= 0) x = y;  // [0, p)
  return f29_canon_sub<1>(f29_mul(f29_from30(x), f29_const(P29Inv::R3)));
}

// add-2008-s.  In: X, Y < 6p, ZZ, ZZZ < 2p (both).  U1, U2, S1, S2 < 1.08p; P = U2 + 2p - U1,
// R < 3.08p (normalized); PP < 1.06p; PPP < 1.02p; Q = U1 PP < 1.01p; R^2 < 1.06p;
// X3 = R^2 + 4p - PPP - 2Q < 5.06p; QX = Q + 6p - X3 < 7.01p (lazy); nS1 = 2p - S1 (lazy);
// Y3 < p + (3.08 * 7.01 + 2 * 1.02) p / 169 < 1.14p; ZZ3, ZZZ3 < 1.01p.
ZK_HD XYZZ<FqOps29> f29_add(const XYZZ<FqOps29>& p, const XYZZ<FqOps29>& q) {
  if (f29_is_zero(q.ZZ)) return p;
  if (f29_is_zero(p.ZZ)) return q;
#if F29_PAIRED
  // two independent products at a time (f29_mont2), the same values as below
  const F29x2 u = f29_mul2(p.X, q.ZZ, q.X, p.ZZ), sv = f29_mul2(p.Y, q.ZZZ, q.Y, p.ZZZ);
  const F29 U1 = u.a, U2 = u.b, S1 = sv.a, S2 = sv.b;
  F29 P = f29_ksub(P29::K2_1, U2, U1);
  F29 R = f29_ksub(P29::K2_1, S2, S1);
  f29_norm(P);
  f29_norm(R);
  const F29x2 sq = f29_sqr2(P, R);
  const F29 PP = sq.a, RR = sq.b;
  if (f29_is_zero(PP)) {
    if (f29_is_zero(RR)) return f29_dbl(p);
    return f29_inf();
  }
  const F29x2 pq = f29_mul2(P, PP, U1, PP), z = f29_mul2(p.ZZ, q.ZZ, p.ZZZ, q.ZZZ);
  const F29 PPP = pq.a, Q = pq.b;
  const F29x2 zz = f29_mul2(z.a, PP, z.b, PPP);
  F29 X3 = f29_ksub3(P29::K4_3, RR, PPP, Q, Q);
  f29_norm(X3);
  const F29 QX = f29_ksub(P29::K6_1, Q, X3);
  const F29 nS1 = f29_ksub(P29::K2_1, f29_zero(), S1);
  return {X3, f29_mulsum2(R, QX, nS1, PPP), zz.a, zz.b};  // no named result: see f29_madd_signed
#else
  const F29 U1 = f29_mul(p.X, q.ZZ);
  const F29 U2 = f29_mul(q.X, p.ZZ);
  const F29 S1 = f29_mul(p.Y, q.ZZZ);
  const F29 S2 = f29_mul(q.Y, p.ZZZ);
  F29 P = f29_ksub(P29::K2_1, U2, U1);
  F29 R = f29_ksub(P29::K2_1, S2, S1);
  f29_norm(P);
  f29_norm(R);
  const F29 PP = f29_sqr(P);
  const F29 RR = f29_sqr(R);
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
#endif
}

// ---------------------------------------------------------------------------
// G2: Fq2 on lane pairs (lane 2k + h holds component h of every value, as Fq2PairOps), each
// component in 29-bit limbs.  The formulas are written against a lane policy L (the device one
// exchanges partner components through DPP; the host one in tools/f29_check.cpp runs both lanes
// of a pair side by side), so tests/test_field29.py checks the same code on the CPU.
//   L::V  one lane's component;  swap: the partner's;  sel(v1, v0): v1 in lane 1, v0 in lane 0;
//   is_zero: both components == 0 mod p (each normalized, < 2p).
// An Fq2 product is one sum of two Fq products per lane with one reduction:
//   lane 0: a0 b0 + (K - a1) b1,  lane 1: a1 b0 + a0 b1     (f2_mul; a normalized, K > a)
// so a product of a < A p and b < B p is < p + (A + K) B p / 169 per component; the column bound
// needs a normalized and b normalized or lazy with limbs < 2^30.  A square is ONE product per lane
// (f2_sqr: (a0 + a1)(a0 + K - a1) and (2 a0) a1) instead of a sum of two, at the price of a looser
// bound, < p + 2 A (A + K) p / 169.  Bounds per formula below, in units of p, for each component;
// invariant between operations: X < 6.7p, Y < 6p, ZZ, ZZZ < 2p, normalized (X is looser than
// G1's 6p: the squares' bound carries into X3).
// ---------------------------------------------------------------------------
template <class L>
struct G2P29 {
  typename L::V X, Y, ZZ, ZZZ;
};

template <class L>
ZK_HD typename L::V f2_mul(const typename L::V& a, const typename L::V& b, const uint32_t (&k)[9]) {
  using V = typename L::V;
  const V pa = L::swap(a);
  const V zero = L::zero();
  // b0 and b1 to both lanes by one broadcast each (was: swap(b) and two selects)
  return L::mulsum2(a, L::even(b), L::sel(pa, L::ksub(k, zero, pa)), L::odd(b));
}

// a^2 over Fq2 (a normalized, a < A p, K >= A p): one Montgomery product per lane
//   lane 0: (a0 + a1) (a0 + K - a1) = a0^2 - a1^2,   lane 1: (a0 + a0) a1 = 2 a0 a1
// x = the sum, normalized (limbs < 2^29); y lazy (lane 0: limbs < 2^29 + 2^30) or normalized, so a
// column holds <= 9 products < 3 x 2^58 + 9 reduction products: < 36 x 2^58.
// Bound: lane 0 < p + 2 A (A + K) p / 169, lane 1 < p + 2 A^2 p / 169.
template <class L>
ZK_HD typename L::V f2_sqr(const typename L::V& a, const uint32_t (&k)[9]) {
  using V = typename L::V;
  const V pa = L::swap(a);
  V x = L::add(pa, L::sel(pa, a));  // lane 0: a1 + a0, lane 1: a0 + a0
  L::norm(x);
  return L::mul(x, L::sel(a, L::ksub(k, a, pa)));  // lane 1: a1, lane 0: a0 + K - a1
}

// Two independent Fq2 products a b (k_a) and c d (k_c) side by side (L::mulsum2x2, F29_PAIRED)
template <class L>
ZK_HD typename L::V2 f2_mul2(const typename L::V& a, const typename L::V& b, const uint32_t (&ka)[9],
                             const typename L::V& c, const typename L::V& d, const uint32_t (&kc)[9]) {
  using V = typename L::V;
  const V pa = L::swap(a), pc = L::swap(c);
  const V zero = L::zero();
  return L::mulsum2x2(a, L::even(b), L::sel(pa, L::ksub(ka, zero, pa)), L::odd(b), c, L::even(d),
                      L::sel(pc, L::ksub(kc, zero, pc)), L::odd(d));
}

// Two independent Fq2 squares (f2_sqr each) side by side (L::mul2, F29_PAIRED)
template <class L>
ZK_HD typename L::V2 f2_sqr2(const typename L::V& a, const uint32_t (&ka)[9], const typename L::V& c,
                             const uint32_t (&kc)[9]) {
  using V = typename L::V;
  const V pa = L::swap(a), pc = L::swap(c);
  V x = L::add(pa, L::sel(pa, a)), z = L::add(pc, L::sel(pc, c));
  L::norm(x);
  L::norm(z);
  return L::mul2(x, L::sel(a, L::ksub(ka, a, pa)), z, L::sel(c, L::ksub(kc, c, pc)));
}

// A B - Y D over Fq2 (a normalized A < kA, Y < kY; B, D normalized): four products per lane
//   lane 0: A0 B0 + (kA - A1) B1 + (kY - Y0) D0 + Y1 D1
//   lane 1: A1 B0 + A0 B1 + (kY - Y1) D0 + (kY - Y0) D1
template <class L>
ZK_HD typename L::V f2_mulsub(const typename L::V& A, const typename L::V& B, const uint32_t (&kA)[9],
                              const typename L::V& Y, const typename L::V& D, const uint32_t (&kY)[9]) {
  using V = typename L::V;
  const V pA = L::swap(A), pY = L::swap(Y);
  const V zero = L::zero();
  const V x[4] = {A, L::sel(pA, L::ksub(kA, zero, pA)), L::ksub(kY, zero, Y), L::sel(L::ksub(kY, zero, pY), pY)};
  const V y[4] = {L::even(B), L::odd(B), L::even(D), L::odd(D)};
  return L::mulsum4(x, y);
}

template <class L>
ZK_HD G2P29<L> f2_inf() {
  return {L::one(), L::one(), L::zero(), L::zero()};
}

// dbl-2008-s-1.  U = 2Y < 12p (normalized); V = U^2 < p + (12 + 13) 12/169 p = 2.78p;
// W = V U < 1.48p; S = V X < p + (2.78 + 4) 6.7/169 p = 1.27p; X^2 < p + (6.7 + 7) 6.7/169 p = 1.55p;
// M = 3 X^2 < 4.65p (normalized); M^2 < 1.27p; X3 = M^2 + 3p - 2S < 4.27p; SX = S + 5p - X3
// < 6.27p (normalized); Y3 = M SX - Y W < p + ((4.65 + 5) 6.27 + (7 + 6) 1.48)/169 p < 1.47p;
// ZZ3, ZZZ3 < 1.07p.
template <class L>
ZK_HD G2P29<L> f2_dbl(const G2P29<L>& p) {
  using V = typename L::V;
  if (L::is_zero(p.ZZ)) return p;
  V U = L::add(p.Y, p.Y);
  L::norm(U);
  const V Vv = f2_mul<L>(U, U, P29::K13_1);
  const V W = f2_mul<L>(Vv, U, P29::K4_1);
  const V S = f2_mul<L>(Vv, p.X, P29::K4_1);
  const V X2 = f2_mul<L>(p.X, p.X, P29::K7_1);
  V M = L::add(L::add(X2, X2), X2);
  L::norm(M);
  G2P29<L> r;
  r.X = L::ksub3(P29::K3_2, f2_mul<L>(M, M, P29::K5_1), S, S, L::zero());
  L::norm(r.X);
  V SX = L::ksub(P29::K5_1, S, r.X);
  L::norm(SX);
  r.Y = f2_mulsub<L>(M, SX, P29::K5_1, p.Y, W, P29::K7_1);
  r.ZZ = f2_mul<L>(Vv, p.ZZ, P29::K4_1);
  r.ZZZ = f2_mul<L>(W, p.ZZZ, P29::K2_1);
  return r;
}

// madd-2008-s.  x, y <= p (canonical base, y possibly negated); U2, S2 < 1.04p;
// P = U2 + 7p - X1, R < 8.04p (normalized); PP, R^2 (f2_sqr, K = 9p) < p + 2 8.04 17.04/169 p
// = 2.62p -- a multiple of p below 3p when P == 0, so the zero tests take 0, p and 2p;
// PPP = PP P < p + (2.62 + 3) 8.04/169 p = 1.27p; Q = PP X1 < p + 5.62 6.7/169 p = 1.23p;
// X3 = R^2 + 4p - PPP - 2Q < 6.62p (4p > PPP + 2Q = 3.73p); QX = Q + 7p - X3 < 8.23p (normalized);
// Y3 = R QX - Y1 PPP < p + ((8.04 + 9) 8.23 + (7 + 6) 1.27)/169 p < 1.93p;
// ZZ3 < p + (2 + 3) 2.62/169 p = 1.08p, ZZZ3 < 1.04p.
template <class L>
ZK_HD G2P29<L> f2_madd(const G2P29<L>& p, const typename L::V& ax, const typename L::V& ay) {
  using V = typename L::V;
  if (L::is_zero(ax) && L::is_zero(ay)) return p;
  if (L::is_zero(p.ZZ)) return {ax, ay, L::one(), L::one()};
#if F29_PAIRED
  // the same products, two independent ones at a time: U2 | S2, PP | RR, PPP | Q, ZZ3 | ZZZ3; the
  // result returned as one aggregate (see f29_madd_signed)
  const typename L::V2 us = f2_mul2<L>(ax, p.ZZ, P29::K2_1, ay, p.ZZZ, P29::K2_1);
  V P = L::ksub(P29::K7_1, us.a, p.X);
  V R = L::ksub(P29::K7_1, us.b, p.Y);
  L::norm(P);
  L::norm(R);
  const typename L::V2 sq = f2_sqr2<L>(P, P29::K9_1, R, P29::K9_1);
  if (L::is_zero3(sq.a)) {
    if (L::is_zero3(sq.b)) return f2_dbl<L>({ax, ay, L::one(), L::one()});
    return f2_inf<L>();
  }
  const V PP = sq.a, RR = sq.b;
  const typename L::V2 pq = f2_mul2<L>(PP, P, P29::K3_1, PP, p.X, P29::K3_1);
  const V PPP = pq.a, Q = pq.b;
  const typename L::V2 zz = f2_mul2<L>(p.ZZ, PP, P29::K3_1, p.ZZZ, PPP, P29::K3_1);
  V X3 = L::ksub3(P29::K4_3, RR, PPP, Q, Q);
  L::norm(X3);
  V QX = L::ksub(P29::K7_1, Q, X3);
  L::norm(QX);
  return {X3, f2_mulsub<L>(R, QX, P29::K9_1, p.Y, PPP, P29::K7_1), zz.a, zz.b};
#else
  const V U2 = f2_mul<L>(ax, p.ZZ, P29::K2_1);
  const V S2 = f2_mul<L>(ay, p.ZZZ, P29::K2_1);
  V P = L::ksub(P29::K7_1, U2, p.X);
  V R = L::ksub(P29::K7_1, S2, p.Y);
  L::norm(P);
  L::norm(R);
  const V PP = f2_sqr<L>(P, P29::K9_1);
  if (L::is_zero3(PP)) {
    if (L::is_zero3(f2_sqr<L>(R, P29::K9_1))) return f2_dbl<L>({ax, ay, L::one(), L::one()});
    return f2_inf<L>();
  }
  const V PPP = f2_mul<L>(PP, P, P29::K3_1);
  const V Q = f2_mul<L>(PP, p.X, P29::K3_1);
  const V RR = f2_sqr<L>(R, P29::K9_1);
  G2P29<L> r;
  r.X = L::ksub3(P29::K4_3, RR, PPP, Q, Q);
  L::norm(r.X);
  V QX = L::ksub(P29::K7_1, Q, r.X);
  L::norm(QX);
  r.Y = f2_mulsub<L>(R, QX, P29::K9_1, p.Y, PPP, P29::K7_1);
  r.ZZ = f2_mul<L>(p.ZZ, PP, P29::K3_1);
  r.ZZZ = f2_mul<L>(p.ZZZ, PPP, P29::K3_1);
  return r;
#endif
}

// add-2008-s.  U1, U2, S1, S2 = (ZZ or ZZZ) (X or Y) < p + (2 + 3) 6.7/169 p = 1.2p;
// P = U2 + 2p - U1, R < 3.2p (normalized); PP, R^2 (f2_sqr, K = 4p) < p + 2 3.2 7.2/169 p
// = 1.28p; PPP < p + 3.28 3.2/169 p = 1.07p; Q < 1.03p; X3 = R^2 + 4p - PPP - 2Q < 5.28p;
// QX < 7.03p (normalized); Y3 = R QX - S1 PPP < p + ((3.2 + 4) 7.03 + (2 + 1.2) 1.07)/169 p < 1.32p;
// ZZ1 ZZ2 < 1.06p, ZZ3 = (ZZ1 ZZ2) PP < 1.03p (ZZZ likewise).
template <class L>
ZK_HD G2P29<L> f2_add(const G2P29<L>& p, const G2P29<L>& q) {
  using V = typename L::V;
  if (L::is_zero(q.ZZ)) return p;
  if (L::is_zero(p.ZZ)) return q;
  const V U1 = f2_mul<L>(q.ZZ, p.X, P29::K3_1);
  const V U2 = f2_mul<L>(p.ZZ, q.X, P29::K3_1);
  const V S1 = f2_mul<L>(q.ZZZ, p.Y, P29::K3_1);
  const V S2 = f2_mul<L>(p.ZZZ, q.Y, P29::K3_1);
  V P = L::ksub(P29::K2_1, U2, U1);
  V R = L::ksub(P29::K2_1, S2, S1);
  L::norm(P);
  L::norm(R);
  const V PP = f2_sqr<L>(P, P29::K4_1);
  if (L::is_zero(PP)) {
    if (L::is_zero(f2_sqr<L>(R, P29::K4_1))) return f2_dbl<L>(p);
    return f2_inf<L>();
  }
  const V PPP = f2_mul<L>(PP, P, P29::K2_1);
  const V Q = f2_mul<L>(PP, U1, P29::K2_1);
  const V RR = f2_sqr<L>(R, P29::K4_1);
  G2P29<L> r;
  r.X = L::ksub3(P29::K4_3, RR, PPP, Q, Q);
  L::norm(r.X);
  V QX = L::ksub(P29::K6_1, Q, r.X);
  L::norm(QX);
  r.Y = f2_mulsub<L>(R, QX, P29::K4_1, S1, PPP, P29::K2_1);
  r.ZZ = f2_mul<L>(f2_mul<L>(p.ZZ, q.ZZ, P29::K3_1), PP, P29::K2_1);
  r.ZZZ = f2_mul<L>(f2_mul<L>(p.ZZZ, q.ZZZ, P29::K3_1), PPP, P29::K2_1);
  return r;
}

// Device lane policy for the G2 formulas: this lane's component, the partner's through DPP
struct Pair29Dev {
  using V = F29;
  static ZK_DEV V zero() { return f29_zero(); }
  static ZK_DEV V one() { return pair_half() ? f29_zero() : f29_const(P29::ONE); }
  static ZK_DEV V swap(const V& a) {
    V r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] = pair_swap_u32(a.v[i]);
    return r;
  }
  static ZK_DEV V sel(const V& v1, const V& v0) {
    const bool h = pair_half() != 0;
    V r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] = h ? v1.v[i] : v0.v[i];
    return r;
  }
  static ZK_DEV V even(const V& a) {  // component 0 of the pair in both lanes
    V r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] = pair_even_u32(a.v[i]);
    return r;
  }
  static ZK_DEV V odd(const V& a) {  // component 1 of the pair in both lanes
    V r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] = pair_odd_u32(a.v[i]);
    return r;
  }
  static ZK_DEV bool is_zero(const V& a) {
    const uint32_t z = f29_is_zero(a) ? 1u : 0u;
    return (z & pair_swap_u32(z)) != 0;
  }
  static ZK_DEV bool is_zero3(const V& a) {
    const uint32_t z = f29_is_zero3(a) ? 1u : 0u;
    return (z & pair_swap_u32(z)) != 0;
  }
  static ZK_DEV V mul(const V& a, const V& b) { return f29_mul(a, b); }
  static ZK_DEV V add(const V& a, const V& b) { return f29_add_lazy(a, b); }
  static ZK_DEV void norm(V& a) { f29_norm(a); }
  static ZK_DEV V ksub(const uint32_t (&k)[9], const V& a, const V& b) { return f29_ksub(k, a, b); }
  static ZK_DEV V ksub3(const uint32_t (&k)[9], const V& a, const V& b, const V& c, const V& d) {
    return f29_ksub3(k, a, b, c, d);
  }
  static ZK_DEV V mulsum2(const V& a, const V& b, const V& c, const V& d) { return f29_mulsum2(a, b, c, d); }
  static ZK_DEV V mulsum4(const V (&x)[4], const V (&y)[4]) { return f29_mulsum4(x, y); }
  using V2 = F29x2;
  // two independent products / product sums side by side (f29_mont2: one accumulator each, no joins)
  static ZK_DEV V2 mul2(const V& a, const V& b, const V& c, const V& d) { return f29_mul2(a, b, c, d); }
  static ZK_DEV V2 mulsum2x2(const V& a, const V& b, const V& c, const V& d, const V& e, const V& f, const V& g,
                             const V& h) {
    const F29 xa[2] = {a, c}, ya[2] = {b, d}, xb[2] = {e, g}, yb[2] = {f, h};
    return f29_mont2<2, 2, false, false>(xa, ya, xb, yb);
  }
};

// Compute type of the G2 MSM kernels: Fq2 on lane pairs, 29-bit limbs (storage Affine/XYZZ<Fq2Ops>)
struct Fq2Pair29 {
  using T = F29;  // this lane's component
  static ZK_DEV T zero() { return f29_zero(); }
  static ZK_DEV T one() { return Pair29Dev::one(); }
  static ZK_DEV bool is_zero(const T& a) { return Pair29Dev::is_zero(a); }
  static ZK_DEV T canon(const T& a) { return FqOps29::canon(a); }
};

// the generic point templates (curve.h) for this representation
template <>
ZK_DEV Affine<FqOps29> aff_neg<FqOps29>(const Affine<FqOps29>& a) {
  return {a.x, FqOps29::neg(a.y)};
}
template <>
ZK_DEV XYZZ<FqOps29> xyzz_madd<FqOps29>(const XYZZ<FqOps29>& p, const Affine<FqOps29>& a) {
  return f29_madd(p, a);
}
// F29_SIGNED_MADD 0: negate the base and use f29_madd (A/B of the sign folding)
#ifndef F29_SIGNED_MADD
#define F29_SIGNED_MADD 1
#endif
#if F29_SIGNED_MADD
template <>
ZK_DEV XYZZ<FqOps29> xyzz_madd_signed<FqOps29>(const XYZZ<FqOps29>& p, const Affine<FqOps29>& a, bool neg) {
  return f29_madd_signed(p, a, neg);
}
#endif
template <>
ZK_DEV XYZZ<FqOps29> xyzz_add<FqOps29>(const XYZZ<FqOps29>& p, const XYZZ<FqOps29>& q) {
  return f29_add(p, q);
}
template <>
ZK_DEV XYZZ<FqOps29> xyzz_dbl<FqOps29>(const XYZZ<FqOps29>& p) {
  return f29_dbl(p);
}

template <>
ZK_DEV Affine<Fq2Pair29> aff_neg<Fq2Pair29>(const Affine<Fq2Pair29>& a) {
  return {a.x, FqOps29::neg(a.y)};  // both components: p - y
}
template <>
ZK_DEV XYZZ<Fq2Pair29> xyzz_madd<Fq2Pair29>(const XYZZ<Fq2Pair29>& p, const Affine<Fq2Pair29>& a) {
  const G2P29<Pair29Dev> r = f2_madd<Pair29Dev>({p.X, p.Y, p.ZZ, p.ZZZ}, a.x, a.y);
  return {r.X, r.Y, r.ZZ, r.ZZZ};
}
template <>
ZK_DEV XYZZ<Fq2Pair29> xyzz_add<Fq2Pair29>(const XYZZ<Fq2Pair29>& p, const XYZZ<Fq2Pair29>& q) {
  const G2P29<Pair29Dev> r = f2_add<Pair29Dev>({p.X, p.Y, p.ZZ, p.ZZZ}, {q.X, q.Y, q.ZZ, q.ZZZ});
  return {r.X, r.Y, r.ZZ, r.ZZZ};
}
template <>
ZK_DEV XYZZ<Fq2Pair29> xyzz_dbl<Fq2Pair29>(const XYZZ<Fq2Pair29>& p) {
  const G2P29<Pair29Dev> r = f2_dbl<Pair29Dev>({p.X, p.Y, p.ZZ, p.ZZZ});
  return {r.X, r.Y, r.ZZ, r.ZZZ};
}

}  // namespace zkfl
