// GLV decomposition for the proof assembly T = s*pi_A + r*B1 (BN254 G1).
//
// Replaces the scalar multiplications of snarkjs groth16_prove's final step (proof.pi_c =
// C + H + s*A + r*B1 - rs*delta [ext]; call site tests/full_system_simulation.mjs:773-776).
// phi(x, y) = (beta x, y) acts on G1 as [lambda] (lambda^2 + lambda + 1 = 0 mod r), so
// k*P = k1*P + k2*phi(P) with |k1|, |k2| < 2^128: four 128-bit scalar multiplications on four
// lanes instead of one 254-bit double-scalar chain on one lane (half the doublings in the
// critical path).  Constants from tools/gen_glv_consts.py (checked there against the oracle).
// The split runs on the host: r and s are known when the proof is enqueued.
#pragma once
#include <stdint.h>
#include <string.h>

namespace zkfl {

// beta, standard form (the kernel converts it to Montgomery form)
static constexpr uint32_t GLV_BETA[8] = {0x77fffffeu, 0x57634731u, 0xacdb5c4fu, 0xd4f263f1u,
                                         0xa0d48bacu, 0x59e26bceu, 0x00000000u, 0x00000000u};

struct GlvScalar {   // one 128-bit signed half-scalar, as uploaded to the device
  uint32_t mag[4];   // |k|, little-endian
  uint32_t neg;      // 1 if k < 0
  uint32_t pad[3];
};

namespace glv_detail {
using u128 = unsigned __int128;
// out[0..na+nb) = a * b (u64 limbs, little-endian)
inline void mul(const uint64_t* a, int na, const uint64_t* b, int nb, uint64_t* out) {
  memset(out, 0, sizeof(uint64_t) * (na + nb));
  for (int i = 0; i < na; i++) {
    uint64_t carry = 0;
    for (int j = 0; j < nb; j++) {
      u128 t = (u128)a[i] * b[j] + out[i + j] + carry;
      out[i + j] = (uint64_t)t;
      carry = (uint64_t)(t >> 64);
    }
    out[i + nb] = carry;
  }
}
// x -= y over n limbs (two's complement)
inline void sub(uint64_t* x, const uint64_t* y, int n) {
  uint64_t borrow = 0;
  for (int i = 0; i < n; i++) {
    u128 t = (u128)x[i] - y[i] - borrow;
    x[i] = (uint64_t)t;
    borrow = (uint64_t)(t >> 64) & 1;
  }
}
inline void add(uint64_t* x, const uint64_t* y, int n) {
  uint64_t carry = 0;
  for (int i = 0; i < n; i++) {
    u128 t = (u128)x[i] + y[i] + carry;
    x[i] = (uint64_t)t;
    carry = (uint64_t)(t >> 64);
  }
}
inline void to_scalar(const uint64_t* v, int n, GlvScalar& out) {  // n-limb two's complement, |v| < 2^128
  uint64_t m[8];
  memcpy(m, v, sizeof(uint64_t) * n);
  out.neg = (m[n - 1] >> 63) ? 1u : 0u;
  if (out.neg) {  // negate
    uint64_t zero[8] = {0};
    sub(zero, m, n);
    memcpy(m, zero, sizeof(uint64_t) * n);
  }
  out.mag[0] = (uint32_t)m[0];
  out.mag[1] = (uint32_t)(m[0] >> 32);
  out.mag[2] = (uint32_t)m[1];
  out.mag[3] = (uint32_t)(m[1] >> 32);
  out.pad[0] = out.pad[1] = out.pad[2] = 0;
}
}  // namespace glv_detail

// k (8 x u32 standard form, < r) -> k1, k2 with k = k1 + k2 * lambda (mod r):
//   c1 = (k g1) >> 384, c2 = (k g2) >> 384,  k1 = k - c1 a1 - c2 a2,  k2 = c1 (-b1) - c2 b2
inline void glv_split(const uint32_t k32[8], GlvScalar& k1, GlvScalar& k2) {
  using namespace glv_detail;
  static const uint64_t a1[1] = {0x89d3256894d213e3ull};
  static const uint64_t b1n[2] = {0x8211bbeb7d4f1128ull, 0x6f4d8248eeb859fcull};  // -b1 (b1 < 0)
  static const uint64_t a2[2] = {0x0be4e1541221250bull, 0x6f4d8248eeb859fdull};
  static const uint64_t b2[1] = {0x89d3256894d213e3ull};
  static const uint64_t g1[4] = {0x8fa7d32d2fafba64ull, 0x6eb9c714773a6ef2ull, 0xd91d232ec7e0b3d7ull,
                                 0x0000000000000002ull};  // round(2^384 b2 / r)
  static const uint64_t g2[5] = {0x869375169b9bdffaull, 0xa5e38cfb5eaa26d9ull, 0x7a7bd9d4391eb18dull,
                                 0x4ccef014a773d2cfull, 0x0000000000000002ull};  // round(2^384 (-b1) / r)
  uint64_t k[4];
  for (int i = 0; i < 4; i++) k[i] = (uint64_t)k32[2 * i] | ((uint64_t)k32[2 * i + 1] << 32);
  uint64_t p1[8], p2[9];
  mul(k, 4, g1, 4, p1);  // < 2^448
  mul(k, 4, g2, 5, p2);  // < 2^512
  const uint64_t c1[1] = {p1[6]};         // bits 384..447
  const uint64_t c2[2] = {p2[6], p2[7]};  // bits 384..511
  uint64_t x[5] = {k[0], k[1], k[2], k[3], 0}, t[5];
  uint64_t m[4];
  mul(c1, 1, a1, 1, m);
  memset(t, 0, sizeof t);
  memcpy(t, m, 2 * sizeof(uint64_t));
  sub(x, t, 5);
  mul(c2, 2, a2, 2, m);
  memset(t, 0, sizeof t);
  memcpy(t, m, 4 * sizeof(uint64_t));
  sub(x, t, 5);
  to_scalar(x, 5, k1);
  uint64_t y[5] = {0, 0, 0, 0, 0};
  mul(c1, 1, b1n, 2, m);
  memcpy(y, m, 3 * sizeof(uint64_t));
  mul(c2, 2, b2, 1, m);
  memset(t, 0, sizeof t);
  memcpy(t, m, 3 * sizeof(uint64_t));
  sub(y, t, 5);
  to_scalar(y, 5, k2);
}

}  // namespace zkfl
