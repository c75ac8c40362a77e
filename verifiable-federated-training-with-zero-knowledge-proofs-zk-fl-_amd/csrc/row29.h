// Row-distributed 29-bit Montgomery arithmetic: one value per 16-lane row of a wave, lane j of the
// row holding limb j of the nine 29-bit limbs (lanes 9..15 zero), over a modulus M of the 29-bit
// engine (P29 = Fq: the assembly's GLV chains, zkfl.hip glv_row_mul; R29 = Fr: the witness engine's
// Poseidon rounds, witness.hip), in its Montgomery domain (2^261) and with the same integer results
// as its one-lane products (f29_mont: the same reduction digit by digit).
//
// A product is spread over its row: limb i of a is broadcast by DPP row_newbcast (or is already
// replicated in every lane: row_mont's operand a), each lane accumulates column i + j in 64 bits,
// and the row shifts down one lane per reduction step (DPP row_shl, lane 0's carry kept): 18
// v_mad_u64_u32 per lane instead of 162, so a latency-bound chain evaluates four products (one
// per row) per wave at a fraction of a one-lane product's latency.  Values cross rows by the gfx950
// row swaps (bcast<K>).  Limbs are lazy: lanes 0..7 below 2^29 + 2^7 (one or two carry-save steps
// per operation), lane 8 the exact top; the integer bounds are those of the one-lane formulas.
#pragma once
#include "field29.h"

namespace zkfl {

// k M (k < 64) in nine 29-bit limbs: normalized, or borrowed by one for a + k M - b (every lower
// limb raised by 2^29, the next lowered by one, so no limb goes negative for a normalized b)
struct Limbs9 {
  uint32_t v[9];
};
template <class M>
__host__ __device__ constexpr Limbs9 m29_times(uint32_t k, bool borrowed) {
  Limbs9 r{};
  uint64_t c = 0;
  for (int i = 0; i < 9; i++) {
    c += (uint64_t)k * M::P[i];
    r.v[i] = i < 8 ? (uint32_t)(c & M::MASK) : (uint32_t)c;
    c >>= 29;
  }
  if (borrowed) {
    for (int i = 0; i < 8; i++) r.v[i] += (1u << 29) - (i ? 1u : 0u);
    r.v[8] -= 1u;
  }
  return r;
}
__host__ __device__ constexpr Limbs9 p29_times(uint32_t k, bool borrowed) { return m29_times<P29>(k, borrowed); }
template <class M>
__host__ __device__ constexpr Limbs9 m29_one() {
  return Limbs9{{M::ONE[0], M::ONE[1], M::ONE[2], M::ONE[3], M::ONE[4], M::ONE[5], M::ONE[6], M::ONE[7], M::ONE[8]}};
}
// k M + 2^31 (limbs 0..7) - 4 (limbs 1..8): a + this - b keeps every lane in [0, 2^32) for lazy b
// (limbs < 2^29 + 2^7); the top limb may wrap below zero and is made whole by the carries
template <class M>
__host__ __device__ constexpr Limbs9 row_kp(uint32_t k) {
  Limbs9 r = m29_times<M>(k, false);
  for (int i = 0; i < 9; i++) r.v[i] += (i < 8 ? 0x80000000u : 0u) - (i > 0 ? 4u : 0u);
  return r;
}

ZK_DEV uint32_t row_j() { return __lane_id() & 15u; }
template <int CTRL, bool BOUND>
ZK_DEV uint32_t row_dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, BOUND);
}
template <int I>
ZK_DEV uint32_t row_limb(uint32_t v) { return row_dpp<0x150 + I, false>(v); }  // row_newbcast:I
ZK_DEV uint32_t row_up(uint32_t v) { return row_dpp<0x101, true>(v); }         // row_shl:1, lane 15 <- 0
ZK_DEV uint32_t row_down(uint32_t v) { return row_dpp<0x111, true>(v); }       // row_shr:1, lane 0 <- 0
ZK_DEV uint32_t limb_at(const Limbs9& c, uint32_t j) {  // c.v[j] (0 for j > 8)
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) r = j == (uint32_t)i ? c.v[i] : r;
  return r;
}

template <class M>
struct RowF {
  struct T {
    uint32_t v;
  };
  // one carry-save step: lanes 0..7 keep 29 bits and pass the rest up one lane
  static ZK_DEV uint32_t carry(uint32_t x) {
    const bool top = row_j() >= 8;
    const uint32_t h = top ? 0u : x >> 29;
    return (top ? x : x & M::MASK) + row_down(h);
  }
  // sum_k a_k b_k 2^-261: a_k's limbs replicated in every lane of the row (a[k][i] = limb i),
  // b_k row-distributed; K <= 4 keeps a column below (9 K + 9) 2^58.02 < 2^64
  template <int K>
  static ZK_DEV T mont(const uint32_t (&a)[K][9], const uint32_t (&b)[K]) {
    static_assert(K >= 1 && K <= 4, "column bound");
    const uint32_t j = row_j();
    const uint32_t pj = limb_at(m29_times<M>(1, false), j);
    uint64_t t = 0;  // lane j: column i + j
#pragma unroll
    for (int i = 0; i < 9; i++) {
#pragma unroll
      for (int k = 0; k < K; k++) t += (uint64_t)a[k][i] * b[k];
      const uint32_t m = (row_limb<0>((uint32_t)t) * M::NINV) & M::MASK;
      t += (uint64_t)m * pj;  // lane 0: column i is now 0 mod 2^29
      // shift down one lane; lane 0 adds its own carry (t >> 29), as 32-bit add / add-with-carry
      const uint32_t lo = (uint32_t)t, hi = (uint32_t)(t >> 32);
      const uint32_t clo = j == 0 ? __builtin_amdgcn_alignbit(hi, lo, 29) : 0u, chi = j == 0 ? hi >> 29 : 0u;
      const uint32_t nlo = row_up(lo) + clo;
      const uint32_t nhi = row_up(hi) + chi + (nlo < clo ? 1u : 0u);
      t = ((uint64_t)nhi << 32) | nlo;
    }
    // lanes 0..8: columns 9..17 (< 2^64); two carry-save steps -> limbs < 2^29 + 2^7
    const bool top = j >= 8;
    const uint64_t h = top ? 0 : t >> 29;
    const uint64_t x = (top ? t : t & M::MASK) + (((uint64_t)row_down((uint32_t)(h >> 32)) << 32) | row_down((uint32_t)h));
    const uint32_t h2 = top ? 0u : (uint32_t)(x >> 29);
    return {(top ? (uint32_t)x : (uint32_t)x & M::MASK) + row_down(h2)};
  }
  static ZK_DEV T mul(const T& a, const T& b) {
    const uint32_t ai[1][9] = {{row_limb<0>(a.v), row_limb<1>(a.v), row_limb<2>(a.v), row_limb<3>(a.v), row_limb<4>(a.v),
                                row_limb<5>(a.v), row_limb<6>(a.v), row_limb<7>(a.v), row_limb<8>(a.v)}};
    const uint32_t bi[1] = {b.v};
    return mont<1>(ai, bi);
  }
  static ZK_DEV T add(const T& a, const T& b) { return {carry(a.v + b.v)}; }
  template <int K>
  static ZK_DEV T sub(const T& a, const T& b) {
    constexpr Limbs9 k = row_kp<M>(K);
    return {carry(a.v + limb_at(k, row_j()) - b.v)};
  }
  static ZK_DEV T dbl(const T& a) { return add(a, a); }
  static ZK_DEV T zero() { return {0u}; }
  static ZK_DEV T one() {
    constexpr Limbs9 o = m29_one<M>();
    return {limb_at(o, row_j())};
  }
  // row K's value to every row: v_permlane16_swap of v with itself gives rows (0, 0, 2, 2) and
  // (1, 1, 3, 3), v_permlane32_swap of either with itself rows (k, k, k, k) and (k + 2, ...): three
  // VALU swaps serve all four K (the formulas' bcast<K> of one product share them)
  template <int K>
  static ZK_DEV T bcast(const T& v) {
    const auto s = __builtin_amdgcn_permlane16_swap(v.v, v.v, false, false);
    const uint32_t e = (K & 1) ? s[1] : s[0];
    const auto u = __builtin_amdgcn_permlane32_swap(e, e, false, false);
    return {(K & 2) ? u[1] : u[0]};
  }
  static ZK_DEV T pick4(int q, T a, T b, T c, T d) { return {(q & 2) ? ((q & 1) ? d.v : c.v) : ((q & 1) ? b.v : a.v)}; }
  // a full value (every lane) -> its row form, and back (row 0, normalized limbs)
  static ZK_DEV T from(const F29& x) {
    const uint32_t j = row_j();
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) r = j == (uint32_t)i ? x.v[i] : r;
    return {r};
  }
  static ZK_DEV F29 to(const T& x) {
    F29 r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] = (uint32_t)__builtin_amdgcn_readlane((int)x.v, i);
    f29_norm(r);
    return r;
  }
};

}  // namespace zkfl
