// BN254 Fr in nine 29-bit limbs (Montgomery R = 2^261): the witness engine's arithmetic.
//
// The witness program is a chain of dependent levels with few lanes each (config 5: 8 witnesses
// per key and round), so the Poseidon permutations of k_wit_lvl run one wave per SIMD and pay the
// full latency -- issue and dependency -- of every product.  The 29-bit engine (field29.h, the
// product-scanning f29_mont over modulus R29) takes one v_mad_u64_u32 per limb product and no
// carry words: ~2.5x less single-wave latency than the 32-bit fp_mul (field29.h header).
//
// Representation: every value the witness kernels keep (the wire vector W, the program's
// coefficients and Poseidon constants) is CANONICAL x 2^261 mod r, stored as 8 x 32-bit words
// (f29_pack / f29_unpack move it into registers).  Products and sums are brought back below r
// at once (one conditional subtraction), so no bound bookkeeping is needed:
//   a, b < r -> f29_mul < r + r^2 / 2^261 < 2r;  a + b < 2r.
// Column bound of f29_mont<NP> over normalized operands: (9 NP + 9) 2^58 < 2^64 for NP <= 6.
#pragma once
#include "field29.h"

namespace zkfl {

struct R29 {
  static constexpr uint32_t MASK = (1u << 29) - 1;
  static constexpr uint32_t NINV = 0x0fffffffu;  // -r^-1 mod 2^29
  // r
  static constexpr uint32_t P[9] = {0x10000001u, 0x1f0fac9fu, 0x0e5c2450u, 0x07d090f3u, 0x1585d283u,
                                    0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
  // 2^261 mod r: one
  static constexpr uint32_t ONE[9] = {0x0fffff57u, 0x1ea70ab4u, 0x052c068bu, 0x17504f49u, 0x0aa8075bu,
                                      0x1d4240ceu, 0x11d54c07u, 0x052ac7a8u, 0x000dc836u};
  // 2^522 mod r: plain x -> x 2^261 (one Montgomery product)
  static constexpr uint32_t R2[9] = {0x05b69bd4u, 0x06170a5au, 0x020cddceu, 0x1db6310bu, 0x0e54d0ffu,
                                     0x1cf855e3u, 0x1c15e103u, 0x07d09161u, 0x000a054au};
  // 2^266 mod r: x 2^256 (the 32-bit engine's Montgomery form) -> x 2^261
  static constexpr uint32_t K266[9] = {0x0fffead7u, 0x1d5444f4u, 0x04438aa5u, 0x03b4d096u, 0x134c84dau,
                                       0x0e92d304u, 0x14cb95b3u, 0x041b9d3du, 0x00058003u};
  // 2^256 mod r: x 2^261 -> x 2^256
  static constexpr uint32_t K256[9] = {0x0ffffffbu, 0x04b1a0e2u, 0x18334a6bu, 0x18ed2b3eu, 0x1462e36fu,
                                       0x11b7bc3cu, 0x1cbd99bau, 0x183340fbu, 0x000e0a77u};
};

using Fr29 = F29;

ZK_HD Fr29 fr29_ld(const Fr& x) { return f29_pack(x.v); }
ZK_HD Fr fr29_st(const Fr29& a) {
  Fr r;
  f29_unpack(r.v, a);
  return r;
}
ZK_HD Fr29 fr29_mul(const Fr29& a, const Fr29& b) { return f29_canon_sub<1, R29>(f29_mul<R29>(a, b)); }
ZK_HD Fr29 fr29_sqr(const Fr29& a) { return f29_canon_sub<1, R29>(f29_sqr<R29>(a)); }
ZK_HD Fr29 fr29_add(const Fr29& a, const Fr29& b) {
  Fr29 r = f29_add_lazy(a, b);
  f29_norm(r);
  return f29_canon_sub<1, R29>(r);
}
// sum_j x_j y_j with one reduction (NP <= 6)
template <int NP>
ZK_HD Fr29 fr29_mulsum(const Fr29 (&x)[NP], const Fr29 (&y)[NP]) {
  static_assert(NP >= 1 && NP <= 6, "column bound");
  // < r + NP r^2 / 2^261 < 2r
  return f29_canon_sub<1, R29>(f29_mont<NP, (F29_SPLIT ? 2 : 1), R29>(x, y));
}
ZK_HD bool fr29_eq(const Fr29& a, const Fr29& b) {
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) d |= a.v[i] ^ b.v[i];
  return d == 0;
}
ZK_HD bool fr29_is_zero(const Fr29& a) {
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) z |= a.v[i];
  return z == 0;
}
// x 2^261 <-> the 32-bit engine's x 2^256 (the inverse of the rare K_INV ops runs there)
ZK_HD Fr29 fr29_from_m256(const Fr& x) { return fr29_mul(fr29_ld(x), f29_const(R29::K266)); }
ZK_HD Fr fr29_to_m256(const Fr29& a) { return fr29_st(fr29_mul(a, f29_const(R29::K256))); }
// plain (standard form, < r) <-> x 2^261
ZK_HD Fr29 fr29_from_plain(const Fr& x) { return fr29_mul(fr29_ld(x), f29_const(R29::R2)); }
ZK_HD Fr fr29_to_plain(const Fr29& a) {
  Fr29 one = f29_zero();
  one.v[0] = 1;
  return fr29_st(fr29_mul(a, one));
}

}  // namespace zkfl
