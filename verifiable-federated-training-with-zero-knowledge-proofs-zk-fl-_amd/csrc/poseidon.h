// circomlib Poseidon over BN254 Fr for gfx950, one lane per hash, state in registers.
//
// Replaces circomlibjs `poseidon(inputs)` as the reference's server/data side calls it
// (tests/full_system_simulation.mjs:139-238: vectorHash, the commitments, buildMerkleTree) and the
// semantics of src/circuits/lib/poseidon.circom:35-96 (circomlib ^2.0.5 [ext]): state = [0, in...],
// R_F = 8 full rounds (4 + 4) around R_P partial rounds, ARK -> x^5 -> MDS, output state[0].
//
// gfx950 shape: round constants and the MDS matrix are uniform across the wave, so they are read
// with scalar loads into SGPRs and every constant product is a v_mad_u64_u32 with an SGPR operand
// (ZK_MAC_VS).  An MDS row is ONE sum of up to 5 products with a single Montgomery reduction
// (5 p^2 < 2^256 p keeps the result below 2p: one final subtraction), so a t = 3 row costs
// 3 x 64 + 64 multiply-adds instead of 3 x 128.
#pragma once
#include "field.h"

namespace zkfl {

// sum_{k<N} x_k * c_k * 2^-256 mod r, N <= 5, x in VGPRs (< r), c uniform (< r).
template <int N>
ZK_DEV Fr fr_dot_c(const Fr* x, const Fr* __restrict__ c) {
  static_assert(N >= 1 && N <= 5, "one reduction holds at most 5 products");
  uint32_t m[8], u[9];
  uint64_t lo = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
#pragma unroll
      for (int k = 0; k < N; k++) ZK_MAC_VS(lo, hi, x[k].v[j], c[k].v[i - j]);
      ZK_MAC_VS(lo, hi, m[j], FrP::P[i - j]);
    }
#pragma unroll
    for (int k = 0; k < N; k++) ZK_MAC_VS(lo, hi, x[k].v[i], c[k].v[0]);
    m[i] = (uint32_t)lo * FrP::INV;
    ZK_MAC_VS(lo, hi, m[i], FrP::P[0]);
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
#pragma unroll
  for (int i = 8; i < 16; i++) {
#pragma unroll
    for (int j = i - 7; j < 8; j++) {
#pragma unroll
      for (int k = 0; k < N; k++) ZK_MAC_VS(lo, hi, x[k].v[j], c[k].v[i - j]);
      ZK_MAC_VS(lo, hi, m[j], FrP::P[i - j]);
    }
    u[i - 8] = (uint32_t)lo;
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  u[8] = (uint32_t)lo;
  Fr r;
  fp_reduce_once<FrP>(r.v, u);
  return r;
}

// sum_{k<T} x_k * row_k for any T: groups of at most 5 products, one reduction each.
template <int T>
ZK_DEV Fr fr_row(const Fr* x, const Fr* __restrict__ row) {
  if constexpr (T <= 5) {
    return fr_dot_c<T>(x, row);
  } else {
    return fp_add(fr_dot_c<5>(x, row), fr_row<T - 5>(x + 5, row + 5));
  }
}

ZK_DEV Fr fr_pow5(const Fr& x) {
  const Fr x2 = fp_sqr(x);
  return fp_mul(fp_sqr(x2), x);
}

// Constants of one width in Montgomery form: C[(8 + rp) * T] then M[T][T] (row-major).
struct PosConsts {
  const Fr* C;
  const Fr* M;
  uint32_t rp;
};

// Permutation of a Montgomery-form state; returns the new state[0] (circomlib's output).
template <int T>
ZK_DEV Fr poseidon_perm0(Fr st[T], const PosConsts& K) {
  const Fr* __restrict__ C = K.C;
  const Fr* __restrict__ M = K.M;
  Fr ns[T];
  auto mds = [&]() {
#pragma unroll
    for (int i = 0; i < T; i++) ns[i] = fr_row<T>(st, M + i * T);
#pragma unroll
    for (int i = 0; i < T; i++) st[i] = ns[i];
  };
  uint32_t r = 0;
  for (; r < 4; r++) {  // first half of the full rounds
#pragma unroll
    for (int i = 0; i < T; i++) st[i] = fr_pow5(fp_add(st[i], C[r * T + i]));
    mds();
  }
  const uint32_t pend = 4 + K.rp;
  for (; r < pend; r++) {  // partial rounds: S-box on lane 0 only
#pragma unroll
    for (int i = 0; i < T; i++) st[i] = fp_add(st[i], C[r * T + i]);
    st[0] = fr_pow5(st[0]);
    mds();
  }
  for (; r < pend + 3; r++) {
#pragma unroll
    for (int i = 0; i < T; i++) st[i] = fr_pow5(fp_add(st[i], C[r * T + i]));
    mds();
  }
#pragma unroll
  for (int i = 0; i < T; i++) st[i] = fr_pow5(fp_add(st[i], C[r * T + i]));
  return fr_row<T>(st, M);  // last round: only row 0 of the MDS is observed
}

}  // namespace zkfl
