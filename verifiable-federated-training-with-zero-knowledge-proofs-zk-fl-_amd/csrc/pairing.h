// BN254 optimal-ate pairing on gfx950: Fq6/Fq12 tower, prepared G2 lines, multi-Miller loop,
// final exponentiation.
//
// Replaces ffjavascript's bn128 `pairingEq` behind `snarkjs groth16 verify` [ext] (reference
// call site tests/full_system_simulation.mjs:865-868).  Every step is restated in
// oracle/pairing_tower.py (same formulas, same order), which tests/test_pairing_tower.py checks
// against the independent oracle pairing in oracle/bn254.py; the GPU is compared bit-exactly
// with it (Miller-loop values and GT elements).
//
// Tower (the ffjavascript one): Fq2 = Fq[u]/(u^2+1), Fq6 = Fq2[v]/(v^3 - xi), xi = 9+u,
// Fq12 = Fq6[w]/(w^2 - v).  G2 lives on the D-type twist y^2 = x^3 + 3/xi.
// One lane evaluates one pairing product (latency-bound, batched across lanes); the big
// routines are __noinline__ so the kernel stays compact enough to keep its registers.
#pragma once
#include "field.h"
#include "pairing_consts.h"

namespace zkfl {

#define ZK_NOINLINE __device__ __attribute__((noinline))

struct Fq6 {
  Fq2 c0, c1, c2;
};
struct Fq12 {
  Fq6 c0, c1;
};
struct LineCoef {  // line = c0*yP + c3*xP*w + c4*v*w  (sparse "034" element)
  Fq2 c0, c3, c4;
};
struct G2Proj {  // homogeneous projective on the twist: x = X/Z, y = Y/Z
  Fq2 X, Y, Z;
};

ZK_DEV Fq load_fq(const uint32_t* s) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = s[i];
  return r;
}
ZK_DEV Fq2 load_fq2(const uint32_t s[2][8]) { return {load_fq(s[0]), load_fq(s[1])}; }

ZK_DEV Fq2 f2_mul_fq(const Fq2& a, const Fq& s) { return {fp_mul(a.c0, s), fp_mul(a.c1, s)}; }
ZK_DEV Fq2 f2_conj(const Fq2& a) { return {a.c0, fp_neg(a.c1)}; }
ZK_DEV Fq2 f2_mul_xi(const Fq2& a) {  // a * (9 + u) = (9 a0 - a1) + (a0 + 9 a1) u
  Fq a0_8 = fp_dbl(fp_dbl(fp_dbl(a.c0)));
  Fq a1_8 = fp_dbl(fp_dbl(fp_dbl(a.c1)));
  return {fp_sub(fp_add(a0_8, a.c0), a.c1), fp_add(fp_add(a1_8, a.c1), a.c0)};
}

// ---------------------------------------------------------------- Fq6
ZK_DEV Fq6 f6_zero() { return {f2_zero(), f2_zero(), f2_zero()}; }
ZK_DEV Fq6 f6_one() { return {f2_one(), f2_zero(), f2_zero()}; }
ZK_DEV Fq6 f6_add(const Fq6& a, const Fq6& b) { return {f2_add(a.c0, b.c0), f2_add(a.c1, b.c1), f2_add(a.c2, b.c2)}; }
ZK_DEV Fq6 f6_sub(const Fq6& a, const Fq6& b) { return {f2_sub(a.c0, b.c0), f2_sub(a.c1, b.c1), f2_sub(a.c2, b.c2)}; }
ZK_DEV Fq6 f6_neg(const Fq6& a) { return {f2_neg(a.c0), f2_neg(a.c1), f2_neg(a.c2)}; }
ZK_DEV Fq6 f6_mul_v(const Fq6& a) { return {f2_mul_xi(a.c2), a.c0, a.c1}; }
ZK_DEV bool f6_eq(const Fq6& a, const Fq6& b) { return f2_eq(a.c0, b.c0) && f2_eq(a.c1, b.c1) && f2_eq(a.c2, b.c2); }

// Karatsuba-style (6 Fq2 multiplications), same grouping as oracle/pairing_tower.py::f6_mul
ZK_NOINLINE Fq6 f6_mul(const Fq6& a, const Fq6& b) {
  Fq2 t0 = f2_mul(a.c0, b.c0), t1 = f2_mul(a.c1, b.c1), t2 = f2_mul(a.c2, b.c2);
  Fq6 r;
  r.c0 = f2_add(t0, f2_mul_xi(f2_sub(f2_sub(f2_mul(f2_add(a.c1, a.c2), f2_add(b.c1, b.c2)), t1), t2)));
  r.c1 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c1), f2_add(b.c0, b.c1)), t0), t1), f2_mul_xi(t2));
  r.c2 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c2), f2_add(b.c0, b.c2)), t0), t2), t1);
  return r;
}

// a * (b0 + b1 v)  (b2 = 0): 5 Fq2 multiplications
ZK_NOINLINE Fq6 f6_mul_01(const Fq6& a, const Fq2& b0, const Fq2& b1) {
  Fq2 t0 = f2_mul(a.c0, b0), t1 = f2_mul(a.c1, b1);
  Fq6 r;
  r.c0 = f2_add(t0, f2_mul_xi(f2_mul(a.c2, b1)));
  r.c1 = f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c1), f2_add(b0, b1)), t0), t1);
  r.c2 = f2_add(f2_mul(a.c2, b0), t1);
  return r;
}

ZK_NOINLINE Fq6 f6_inv(const Fq6& a) {
  Fq2 t0 = f2_sub(f2_sqr(a.c0), f2_mul_xi(f2_mul(a.c1, a.c2)));
  Fq2 t1 = f2_sub(f2_mul_xi(f2_sqr(a.c2)), f2_mul(a.c0, a.c1));
  Fq2 t2 = f2_sub(f2_sqr(a.c1), f2_mul(a.c0, a.c2));
  Fq2 d = f2_add(f2_mul(a.c0, t0), f2_mul_xi(f2_add(f2_mul(a.c2, t1), f2_mul(a.c1, t2))));
  Fq2 di = f2_inv(d);
  return {f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di)};
}

// ---------------------------------------------------------------- Fq12
ZK_DEV Fq12 f12_one() { return {f6_one(), f6_zero()}; }
ZK_DEV bool f12_is_one(const Fq12& a) { return f6_eq(a.c0, f6_one()) && f6_eq(a.c1, f6_zero()); }
ZK_DEV Fq12 f12_conj(const Fq12& a) { return {a.c0, f6_neg(a.c1)}; }

ZK_NOINLINE Fq12 f12_mul(const Fq12& a, const Fq12& b) {
  Fq6 t0 = f6_mul(a.c0, b.c0), t1 = f6_mul(a.c1, b.c1);
  Fq6 c1 = f6_sub(f6_sub(f6_mul(f6_add(a.c0, a.c1), f6_add(b.c0, b.c1)), t0), t1);
  return {f6_add(t0, f6_mul_v(t1)), c1};
}

// complex squaring: (a + b w)^2 = ((a+b)(a+vb) - ab - v ab) + 2ab w
ZK_NOINLINE Fq12 f12_sqr(const Fq12& x) {
  Fq6 ab = f6_mul(x.c0, x.c1);
  Fq6 t = f6_mul(f6_add(x.c0, x.c1), f6_add(x.c0, f6_mul_v(x.c1)));
  return {f6_sub(f6_sub(t, ab), f6_mul_v(ab)), f6_add(ab, ab)};
}

ZK_NOINLINE Fq12 f12_inv(const Fq12& x) {
  Fq6 d = f6_inv(f6_sub(f6_mul(x.c0, x.c0), f6_mul_v(f6_mul(x.c1, x.c1))));
  return {f6_mul(x.c0, d), f6_neg(f6_mul(x.c1, d))};
}

// f * (c0 + (c3 + c4 v) w)
ZK_NOINLINE Fq12 f12_mul_034(const Fq12& f, const Fq2& c0, const Fq2& c3, const Fq2& c4) {
  Fq6 a0 = {f2_mul(f.c0.c0, c0), f2_mul(f.c0.c1, c0), f2_mul(f.c0.c2, c0)};
  Fq6 bb = f6_mul_01(f.c1, c3, c4);
  Fq6 c1 = f6_sub(f6_sub(f6_mul_01(f6_add(f.c0, f.c1), f2_add(c0, c3), c4), a0), bb);
  return {f6_add(a0, f6_mul_v(bb)), c1};
}

// Frobenius: coefficient of w^k (k = 2i + j for c_j.c_i) -> conj(c) * gamma1[k]
ZK_NOINLINE Fq12 f12_frob(const Fq12& x) {
  Fq12 r;
  r.c0.c0 = f2_conj(x.c0.c0);
  r.c1.c0 = f2_mul(f2_conj(x.c1.c0), load_fq2(GAMMA1[1]));
  r.c0.c1 = f2_mul(f2_conj(x.c0.c1), load_fq2(GAMMA1[2]));
  r.c1.c1 = f2_mul(f2_conj(x.c1.c1), load_fq2(GAMMA1[3]));
  r.c0.c2 = f2_mul(f2_conj(x.c0.c2), load_fq2(GAMMA1[4]));
  r.c1.c2 = f2_mul(f2_conj(x.c1.c2), load_fq2(GAMMA1[5]));
  return r;
}

ZK_NOINLINE Fq12 f12_frob2(const Fq12& x) {
  Fq12 r;
  r.c0.c0 = x.c0.c0;
  r.c1.c0 = f2_mul_fq(x.c1.c0, load_fq(GAMMA2[1]));
  r.c0.c1 = f2_mul_fq(x.c0.c1, load_fq(GAMMA2[2]));
  r.c1.c1 = f2_mul_fq(x.c1.c1, load_fq(GAMMA2[3]));
  r.c0.c2 = f2_mul_fq(x.c0.c2, load_fq(GAMMA2[4]));
  r.c1.c2 = f2_mul_fq(x.c1.c2, load_fq(GAMMA2[5]));
  return r;
}

ZK_NOINLINE Fq12 f12_pow_u(const Fq12& x) {
  Fq12 r = x;  // top bit of u
  for (int b = 61; b >= 0; b--) {
    r = f12_sqr(r);
    if ((BN_U >> b) & 1ull) r = f12_mul(r, x);
  }
  return r;
}

// ---------------------------------------------------------------- lines (prepared G2)
// Doubling step in homogeneous projective coordinates (oracle/pairing_tower.py::dbl_step)
ZK_NOINLINE LineCoef g2_dbl_step(G2Proj& R) {
  Fq2 a = f2_mul_fq(f2_mul(R.X, R.Y), load_fq(FQ_TWO_INV));
  Fq2 b = f2_sqr(R.Y);
  Fq2 c = f2_sqr(R.Z);
  Fq2 e = f2_mul(load_fq2(TWIST_B), f2_add(f2_dbl(c), c));
  Fq2 f = f2_add(f2_dbl(e), e);
  Fq2 g = f2_mul_fq(f2_add(b, f), load_fq(FQ_TWO_INV));
  Fq2 h = f2_sub(f2_sqr(f2_add(R.Y, R.Z)), f2_add(b, c));
  Fq2 i = f2_sub(e, b);
  Fq2 j = f2_sqr(R.X);
  Fq2 e2 = f2_sqr(e);
  R.X = f2_mul(a, f2_sub(b, f));
  R.Y = f2_sub(f2_sqr(g), f2_add(f2_dbl(e2), e2));
  R.Z = f2_mul(b, h);
  return {f2_neg(h), f2_add(f2_dbl(j), j), i};
}

// Mixed addition R + Q, Q affine (oracle/pairing_tower.py::add_step)
ZK_NOINLINE LineCoef g2_add_step(G2Proj& R, const Fq2& qx, const Fq2& qy) {
  Fq2 theta = f2_sub(R.Y, f2_mul(qy, R.Z));
  Fq2 lam = f2_sub(R.X, f2_mul(qx, R.Z));
  Fq2 c = f2_sqr(theta);
  Fq2 d = f2_sqr(lam);
  Fq2 e = f2_mul(lam, d);
  Fq2 f = f2_mul(R.Z, c);
  Fq2 g = f2_mul(R.X, d);
  Fq2 h = f2_sub(f2_add(e, f), f2_dbl(g));
  Fq2 j = f2_sub(f2_mul(theta, qx), f2_mul(lam, qy));
  R.Y = f2_sub(f2_mul(theta, f2_sub(g, h)), f2_mul(e, R.Y));
  R.X = f2_mul(lam, h);
  R.Z = f2_mul(R.Z, e);
  return {lam, f2_neg(theta), j};
}

// All ATE_NLINES line coefficients of the Miller loop for a fixed affine Q (not infinity).
ZK_DEV void g2_prepare_lines(const Fq2& qx, const Fq2& qy, LineCoef* out) {
  G2Proj R = {qx, qy, f2_one()};
  int k = 0;
  for (int b = 63; b >= 0; b--) {
    out[k++] = g2_dbl_step(R);
    if ((ATE_LOW >> b) & 1ull) out[k++] = g2_add_step(R, qx, qy);
  }
  // Q1 = pi(Q), -Q2 = -pi^2(Q)
  Fq2 q1x = f2_mul(f2_conj(qx), load_fq2(TWIST_FROB_X));
  Fq2 q1y = f2_mul(f2_conj(qy), load_fq2(TWIST_FROB_Y));
  Fq2 q2x = f2_mul(f2_conj(q1x), load_fq2(TWIST_FROB_X));
  Fq2 q2y = f2_mul(f2_conj(q1y), load_fq2(TWIST_FROB_Y));
  out[k++] = g2_add_step(R, q1x, q1y);
  out[k++] = g2_add_step(R, q2x, f2_neg(q2y));
}

ZK_DEV Fq12 ell(const Fq12& f, const LineCoef& l, const Fq& px, const Fq& py) {
  return f12_mul_034(f, f2_mul_fq(l.c0, py), f2_mul_fq(l.c3, px), l.c4);
}

// Multi-Miller loop over up to 4 pairs with prepared lines.  Pairs with skip[i] contribute 1.
ZK_DEV Fq12 miller_prepared(int npairs, const Fq* px, const Fq* py, const LineCoef* const* lines,
                            const bool* skip) {
  Fq12 f = f12_one();
  int k = 0;
  for (int b = 63; b >= -1; b--) {
    // b == -1: the two Frobenius lines (no squaring)
    if (b >= 0 && b < 63) f = f12_sqr(f);
    int nl = (b < 0) ? 2 : (((ATE_LOW >> b) & 1ull) ? 2 : 1);
    for (int t = 0; t < nl; t++, k++)
      for (int i = 0; i < npairs; i++)
        if (!skip[i]) f = ell(f, lines[i][k], px[i], py[i]);
  }
  return f;
}

// f^((p^12-1)/r): easy part, then the Devegili-Scott-Dahab hard part (exact exponent).
ZK_NOINLINE Fq12 final_exp(const Fq12& f) {
  Fq12 t = f12_mul(f12_conj(f), f12_inv(f));
  t = f12_mul(f12_frob2(t), t);
  Fq12 fp = f12_frob(t);
  Fq12 fp2 = f12_frob2(t);
  Fq12 fp3 = f12_frob(fp2);
  Fq12 fu = f12_pow_u(t);
  Fq12 fu2 = f12_pow_u(fu);
  Fq12 fu3 = f12_pow_u(fu2);
  Fq12 y3 = f12_conj(f12_frob(fu));
  Fq12 fu2p = f12_frob(fu2);
  Fq12 fu3p = f12_frob(fu3);
  Fq12 y2 = f12_frob2(fu2);
  Fq12 y0 = f12_mul(f12_mul(fp, fp2), fp3);
  Fq12 y1 = f12_conj(t);
  Fq12 y5 = f12_conj(fu2);
  Fq12 y4 = f12_conj(f12_mul(fu, fu2p));
  Fq12 y6 = f12_conj(f12_mul(fu3, fu3p));
  Fq12 t0 = f12_mul(f12_mul(f12_sqr(y6), y4), y5);
  Fq12 t1 = f12_mul(f12_mul(y3, y5), t0);
  t0 = f12_mul(t0, y2);
  t1 = f12_sqr(f12_mul(f12_sqr(t1), t0));
  t0 = f12_mul(t1, y1);
  t1 = f12_mul(t1, y0);
  t0 = f12_sqr(t0);
  return f12_mul(t0, t1);
}

}  // namespace zkfl
