// Host-side driver for the 29-bit-limb field and point formulas (csrc/field29.h), used by
// tests/test_field29.py: the formulas are __host__ __device__, so their bound analysis is
// checked on the CPU against Python big integers.  One operation per stdin line:
//   mul a b | sqr a | invb a | canon a | mulsum2 a b c d | below256 a | dbl P | madd P x y | madds P x y neg | add P Q
//   g2dbl P | g2madd P x y | g2add P Q   (Fq2 values as two elements: c0 c1)
//   rmul a b | rsqr a | radd a b | rmulsum4 x0 x1 x2 x3 y0 y1 y2 y3 | rfromplain a | rtoplain a |
//   rfrom256 a | rto256 a   (Fr in the witness engine's 29-bit form, csrc/fr29.h)
// field elements as 9 comma-separated decimal limbs, points as X Y ZZ ZZZ; the result is
// printed the same way.
// Build: hipcc --offload-arch=gfx950 -O1 -std=c++17 -I<pkg>/csrc -o f29_check f29_check.cpp
#include <cstdio>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>

#include "field29.h"
#include "fr29.h"
using namespace zkfl;

static Fr as_fr(const F29& a) {
  Fr r;
  f29_unpack(r.v, a);
  return r;
}

static F29 rd(std::istringstream& in) {
  std::string t;
  in >> t;
  F29 r;
  std::istringstream ls(t);
  for (int i = 0; i < 9; i++) {
    std::string x;
    std::getline(ls, x, ',');
    r.v[i] = (uint32_t)std::stoul(x);
  }
  return r;
}

static void wr(const F29& a) {
  for (int i = 0; i < 9; i++) printf("%u%c", a.v[i], i < 8 ? ',' : ' ');
}

static XYZZ<FqOps29> rdp(std::istringstream& in) {
  XYZZ<FqOps29> p;
  p.X = rd(in);
  p.Y = rd(in);
  p.ZZ = rd(in);
  p.ZZZ = rd(in);
  return p;
}

static void wrp(const XYZZ<FqOps29>& p) {
  wr(p.X);
  wr(p.Y);
  wr(p.ZZ);
  wr(p.ZZZ);
}

// both lanes of a pair side by side (the device policy is Pair29Dev)
struct PairHost {
  struct V {
    F29 l[2];
  };
  static V zero() { return {f29_zero(), f29_zero()}; }
  static V one() { return {f29_const(P29::ONE), f29_zero()}; }
  static V swap(const V& a) { return {a.l[1], a.l[0]}; }
  static V sel(const V& v1, const V& v0) { return {v0.l[0], v1.l[1]}; }
  static V even(const V& a) { return {a.l[0], a.l[0]}; }
  static V odd(const V& a) { return {a.l[1], a.l[1]}; }
  static bool is_zero(const V& a) { return f29_is_zero(a.l[0]) && f29_is_zero(a.l[1]); }
  static bool is_zero3(const V& a) { return f29_is_zero3(a.l[0]) && f29_is_zero3(a.l[1]); }
  static V mul(const V& a, const V& b) { return {f29_mul(a.l[0], b.l[0]), f29_mul(a.l[1], b.l[1])}; }
  static V add(const V& a, const V& b) { return {f29_add_lazy(a.l[0], b.l[0]), f29_add_lazy(a.l[1], b.l[1])}; }
  static void norm(V& a) {
    f29_norm(a.l[0]);
    f29_norm(a.l[1]);
  }
  static V ksub(const uint32_t (&k)[9], const V& a, const V& b) {
    return {f29_ksub(k, a.l[0], b.l[0]), f29_ksub(k, a.l[1], b.l[1])};
  }
  static V ksub3(const uint32_t (&k)[9], const V& a, const V& b, const V& c, const V& d) {
    return {f29_ksub3(k, a.l[0], b.l[0], c.l[0], d.l[0]), f29_ksub3(k, a.l[1], b.l[1], c.l[1], d.l[1])};
  }
  static V mulsum2(const V& a, const V& b, const V& c, const V& d) {
    return {f29_mulsum2(a.l[0], b.l[0], c.l[0], d.l[0]), f29_mulsum2(a.l[1], b.l[1], c.l[1], d.l[1])};
  }
  struct V2 {
    V a, b;
  };
  // two independent products / product sums (the device policy runs them through f29_mont2)
  static V2 mul2(const V& a, const V& b, const V& c, const V& d) {
    V2 r;
    for (int l = 0; l < 2; l++) {
      const F29x2 t = f29_mul2(a.l[l], b.l[l], c.l[l], d.l[l]);
      r.a.l[l] = t.a;
      r.b.l[l] = t.b;
    }
    return r;
  }
  static V2 mulsum2x2(const V& a, const V& b, const V& c, const V& d, const V& e, const V& f, const V& g,
                      const V& h) {
    V2 r;
    for (int l = 0; l < 2; l++) {
      const F29 xa[2] = {a.l[l], c.l[l]}, ya[2] = {b.l[l], d.l[l]}, xb[2] = {e.l[l], g.l[l]}, yb[2] = {f.l[l], h.l[l]};
      const F29x2 t = f29_mont2<2, 2, false, false>(xa, ya, xb, yb);
      r.a.l[l] = t.a;
      r.b.l[l] = t.b;
    }
    return r;
  }
  static V mulsum4(const V (&x)[4], const V (&y)[4]) {
    V r;
    for (int h = 0; h < 2; h++) {
      const F29 xs[4] = {x[0].l[h], x[1].l[h], x[2].l[h], x[3].l[h]};
      const F29 ys[4] = {y[0].l[h], y[1].l[h], y[2].l[h], y[3].l[h]};
      r.l[h] = f29_mulsum4(xs, ys);
    }
    return r;
  }
};

static PairHost::V rd2(std::istringstream& in) {
  PairHost::V v;
  v.l[0] = rd(in);
  v.l[1] = rd(in);
  return v;
}

static G2P29<PairHost> rdp2(std::istringstream& in) {
  G2P29<PairHost> p;
  p.X = rd2(in);
  p.Y = rd2(in);
  p.ZZ = rd2(in);
  p.ZZZ = rd2(in);
  return p;
}

static void wrp2(const G2P29<PairHost>& p) {
  for (const PairHost::V* v : {&p.X, &p.Y, &p.ZZ, &p.ZZZ}) {
    wr(v->l[0]);
    wr(v->l[1]);
  }
}

int main() {
  std::string line;
  while (std::getline(std::cin, line)) {
    std::istringstream in(line);
    std::string op;
    in >> op;
    if (op == "mul") {
      F29 a = rd(in), b = rd(in);
      wr(f29_mul(a, b));
    } else if (op == "rmul") {
      F29 a = rd(in), b = rd(in);
      wr(fr29_mul(a, b));
    } else if (op == "rsqr") {
      wr(fr29_sqr(rd(in)));
    } else if (op == "radd") {
      F29 a = rd(in), b = rd(in);
      wr(fr29_add(a, b));
    } else if (op == "rmulsum4") {
      F29 x[4], y[4];
      for (auto& v : x) v = rd(in);
      for (auto& v : y) v = rd(in);
      wr(fr29_mulsum<4>(x, y));
    } else if (op == "rfromplain") {
      wr(fr29_from_plain(as_fr(rd(in))));
    } else if (op == "rtoplain") {
      wr(f29_pack(fr29_to_plain(rd(in)).v));
    } else if (op == "rfrom256") {
      wr(fr29_from_m256(as_fr(rd(in))));
    } else if (op == "rto256") {
      wr(f29_pack(fr29_to_m256(rd(in)).v));
    } else if (op == "sqr") {
      wr(f29_sqr(rd(in)));
    } else if (op == "invd") {
      wr(f29_inv_divsteps(rd(in)));
    } else if (op == "canon") {  // normalized a < 4p -> canonical
      wr(f29_canon_sub<3>(rd(in)));
    } else if (op == "mulsum2") {
      F29 a = rd(in), b = rd(in), c = rd(in), d = rd(in);
      wr(f29_mulsum2(a, b, c, d));
    } else if (op == "below256") {
      wr(f29_below256(rd(in)));
    } else if (op == "dbl") {
      wrp(f29_dbl(rdp(in)));
    } else if (op == "madd") {
      XYZZ<FqOps29> p = rdp(in);
      Affine<FqOps29> a;
      a.x = rd(in);
      a.y = rd(in);
      wrp(f29_madd(p, a));
    } else if (op == "madds") {  // signed madd: base (x, y), minus it when neg != 0
      XYZZ<FqOps29> p = rdp(in);
      Affine<FqOps29> a;
      a.x = rd(in);
      a.y = rd(in);
      int neg = 0;
      in >> neg;
      wrp(f29_madd_signed(p, a, neg != 0));
    } else if (op == "add") {
      XYZZ<FqOps29> p = rdp(in), q = rdp(in);
      wrp(f29_add(p, q));
    } else if (op == "g2dbl") {
      wrp2(f2_dbl<PairHost>(rdp2(in)));
    } else if (op == "g2madd") {
      G2P29<PairHost> p = rdp2(in);
      PairHost::V x = rd2(in), y = rd2(in);
      wrp2(f2_madd<PairHost>(p, x, y));
    } else if (op == "g2add") {
      G2P29<PairHost> p = rdp2(in), q = rdp2(in);
      wrp2(f2_add<PairHost>(p, q));
    } else {
      printf("?");
    }
    printf("\n");
  }
  return 0;
}
