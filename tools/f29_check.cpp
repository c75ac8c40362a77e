// Host-side driver for the 29-bit-limb field and point formulas (csrc/field29.h), used by
// tests/test_field29.py: the formulas are __host__ __device__, so their bound analysis is
// checked on the CPU against Python big integers.  One operation per stdin line:
//   mul a b | mulsum2 a b c d | below256 a | dbl P | madd P x y | add P Q
// field elements as 9 comma-separated decimal limbs, points as X Y ZZ ZZZ; the result is
// printed the same way.
// Build: hipcc --offload-arch=gfx950 -O1 -std=c++17 -I<pkg>/csrc -o f29_check f29_check.cpp
#include <cstdio>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>

#include "field29.h"
using namespace zkfl;

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

int main() {
  std::string line;
  while (std::getline(std::cin, line)) {
    std::istringstream in(line);
    std::string op;
    in >> op;
    if (op == "mul") {
      F29 a = rd(in), b = rd(in);
      wr(f29_mul(a, b));
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
    } else if (op == "add") {
      XYZZ<FqOps29> p = rdp(in), q = rdp(in);
      wrp(f29_add(p, q));
    } else {
      printf("?");
    }
    printf("\n");
  }
  return 0;
}
