// BN254 G1 (over Fq) and G2 (over Fq2, D-type twist) point arithmetic for gfx950.
//
// Replaces the wasmcurves G1/G2 kernels behind snarkjs `multiExpAffine` and the proof
// assembly `G1.add/timesFr` (snarkjs groth16_prove [ext]; call site
// tests/full_system_simulation.mjs:773-776).  Both curves have a = 0.
//
// Coordinates:
//   Affine  (x, y), Montgomery form, infinity encoded as (0, 0) exactly as in the zkey
//           sections 5-9 (ffjavascript toRprLEM of the zero point).
//   XYZZ    (X, Y, ZZ, ZZZ) with x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2; ZZ = 0 is infinity.
//           madd-2008-s / add-2008-s / dbl-2008-s-1 (10M, 14M, 9M for G1).
#pragma once
#include "field.h"

namespace zkfl {

template <class F>
struct Affine {
  typename F::T x, y;
};

template <class F>
struct XYZZ {
  typename F::T X, Y, ZZ, ZZZ;
};

template <class F>
ZK_DEV bool aff_is_inf(const Affine<F>& p) {
  return F::is_zero(p.x) && F::is_zero(p.y);
}

template <class F>
ZK_DEV Affine<F> aff_neg(const Affine<F>& p) {
  Affine<F> r;
  r.x = p.x;
  r.y = F::neg(p.y);
  return r;
}

template <class F>
ZK_DEV XYZZ<F> xyzz_inf() {
  XYZZ<F> r;
  r.X = F::one();
  r.Y = F::one();
  r.ZZ = F::zero();
  r.ZZZ = F::zero();
  return r;
}

template <class F>
ZK_DEV bool xyzz_is_inf(const XYZZ<F>& p) {
  return F::is_zero(p.ZZ);
}

template <class F>
ZK_DEV XYZZ<F> xyzz_from_affine(const Affine<F>& a) {
  if (aff_is_inf(a)) return xyzz_inf<F>();
  XYZZ<F> r;
  r.X = a.x;
  r.Y = a.y;
  r.ZZ = F::one();
  r.ZZZ = F::one();
  return r;
}

template <class F>
ZK_DEV XYZZ<F> xyzz_neg(const XYZZ<F>& p) {
  XYZZ<F> r = p;
  r.Y = F::neg(p.Y);
  return r;
}

// dbl-2008-s-1
template <class F>
ZK_DEV XYZZ<F> xyzz_dbl(const XYZZ<F>& p) {
  if (xyzz_is_inf(p)) return p;
  using T = typename F::T;
  T U = F::dbl(p.Y);
  T V = F::sqr(U);
  T W = F::mul(U, V);
  T S = F::mul(p.X, V);
  T X2 = F::sqr(p.X);
  T M = F::add(F::dbl(X2), X2);
  XYZZ<F> r;
  r.X = F::sub(F::sqr(M), F::dbl(S));
  r.Y = F::mul_sub(M, F::sub(S, r.X), W, p.Y);
  r.ZZ = F::mul(V, p.ZZ);
  r.ZZZ = F::mul(W, p.ZZZ);
  return r;
}

// doubling of an affine point into XYZZ (mdbl-2008-s-1)
template <class F>
ZK_DEV XYZZ<F> xyzz_dbl_affine(const Affine<F>& a) {
  using T = typename F::T;
  T U = F::dbl(a.y);
  T V = F::sqr(U);
  T W = F::mul(U, V);
  T S = F::mul(a.x, V);
  T X2 = F::sqr(a.x);
  T M = F::add(F::dbl(X2), X2);
  XYZZ<F> r;
  r.X = F::sub(F::sqr(M), F::dbl(S));
  r.Y = F::mul_sub(M, F::sub(S, r.X), W, a.y);
  r.ZZ = V;
  r.ZZZ = W;
  return r;
}

template <class F>
ZK_DEV XYZZ<F> xyzz_madd(const XYZZ<F>& p, const Affine<F>& a);

// p + a or p - a (the MSM accumulation's signed digit); representations may fold the sign into
// the formula instead of negating the base (field29.h)
template <class F>
ZK_DEV XYZZ<F> xyzz_madd_signed(const XYZZ<F>& p, const Affine<F>& a, bool neg) {
  return xyzz_madd<F>(p, neg ? aff_neg<F>(a) : a);
}

// p + a (a affine), madd-2008-s
template <class F>
ZK_DEV XYZZ<F> xyzz_madd(const XYZZ<F>& p, const Affine<F>& a) {
  if (aff_is_inf(a)) return p;
  if (xyzz_is_inf(p)) return xyzz_from_affine<F>(a);
  using T = typename F::T;
  T U2 = F::mul(a.x, p.ZZ);
  T S2 = F::mul(a.y, p.ZZZ);
  T P = F::sub(U2, p.X);
  T R = F::sub(S2, p.Y);
  if (F::is_zero(P)) {
    if (F::is_zero(R)) return xyzz_dbl_affine<F>(a);
    return xyzz_inf<F>();
  }
  T PP = F::sqr(P);
  T PPP = F::mul(P, PP);
  T Q = F::mul(p.X, PP);
  XYZZ<F> r;
  r.X = F::sub(F::sub(F::sqr(R), PPP), F::dbl(Q));
  r.Y = F::mul_sub(R, F::sub(Q, r.X), p.Y, PPP);
  r.ZZ = F::mul(p.ZZ, PP);
  r.ZZZ = F::mul(p.ZZZ, PPP);
  return r;
}

// p + q, add-2008-s
template <class F>
ZK_DEV XYZZ<F> xyzz_add(const XYZZ<F>& p, const XYZZ<F>& q) {
  if (xyzz_is_inf(q)) return p;
  if (xyzz_is_inf(p)) return q;
  using T = typename F::T;
  T U1 = F::mul(p.X, q.ZZ);
  T U2 = F::mul(q.X, p.ZZ);
  T S1 = F::mul(p.Y, q.ZZZ);
  T S2 = F::mul(q.Y, p.ZZZ);
  T P = F::sub(U2, U1);
  T R = F::sub(S2, S1);
  if (F::is_zero(P)) {
    if (F::is_zero(R)) return xyzz_dbl<F>(p);
    return xyzz_inf<F>();
  }
  T PP = F::sqr(P);
  T PPP = F::mul(P, PP);
  T Q = F::mul(U1, PP);
  XYZZ<F> r;
  r.X = F::sub(F::sub(F::sqr(R), PPP), F::dbl(Q));
  r.Y = F::mul_sub(R, F::sub(Q, r.X), S1, PPP);
  r.ZZ = F::mul(F::mul(p.ZZ, q.ZZ), PP);
  r.ZZZ = F::mul(F::mul(p.ZZZ, q.ZZZ), PPP);
  return r;
}

// Coordinates back to the canonical range (identity unless F keeps a redundant representation).
template <class F>
ZK_DEV XYZZ<F> xyzz_canon(const XYZZ<F>& p) {
  return {F::canon(p.X), F::canon(p.Y), F::canon(p.ZZ), F::canon(p.ZZZ)};
}

// XYZZ -> affine (Montgomery), one field inversion.  Infinity -> (0, 0).
template <class F>
ZK_DEV Affine<F> xyzz_to_affine(const XYZZ<F>& p) {
  Affine<F> r;
  if (xyzz_is_inf(p)) {
    r.x = F::zero();
    r.y = F::zero();
    return r;
  }
  auto iZZZ = F::inv(p.ZZZ);
  auto iZ = F::mul(p.ZZ, iZZZ);  // ZZ/ZZZ = 1/Z
  auto iZZ = F::sqr(iZ);
  r.x = F::mul(p.X, iZZ);
  r.y = F::mul(p.Y, iZZZ);
  return r;
}

// k * p for a standard-form scalar (8 x u32 limbs), left-to-right double-and-add.
template <class F>
ZK_DEV XYZZ<F> xyzz_scalar_mul(const XYZZ<F>& p, const uint32_t k[8]) {
  XYZZ<F> acc = xyzz_inf<F>();
  for (int i = 7; i >= 0; i--) {
    for (int b = 31; b >= 0; b--) {
      acc = xyzz_dbl<F>(acc);
      if ((k[i] >> b) & 1u) acc = xyzz_add<F>(acc, p);
    }
  }
  return acc;
}

using G1Aff = Affine<FqOps>;
using G1P = XYZZ<FqOps>;
using G2Aff = Affine<Fq2Ops>;
using G2P = XYZZ<Fq2Ops>;

}  // namespace zkfl
