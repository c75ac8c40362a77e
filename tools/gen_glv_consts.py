#!/usr/bin/env python3
"""BN254 G1 GLV constants for the proof-assembly kernel (csrc/glv.h).

phi(x, y) = (beta x, y) is the endomorphism of y^2 = x^3 + 3 with beta a primitive cube root of
unity mod q; on the order-r group it acts as [lambda] for the matching cube root lambda mod r.
The short basis of the lattice {(a, b) : a + b lambda = 0 mod r} comes from the extended
Euclidean algorithm on (r, lambda) (Gallant-Lambert-Vanstone 2001, Sec. 4); k is split as
k = k1 + k2 lambda with c1 = round(b2 k / r), c2 = round(-b1 k / r),
k1 = k - c1 a1 - c2 a2, k2 = -c1 b1 - c2 b2, |k1|, |k2| < 2^128, the roundings done as
(k g) >> 384 with g = round(2^384 b / r).  Checked here against the oracle's scalar multiplication.
"""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import bn254 as bn  # noqa: E402

Q, R = bn.Q, bn.R


def cube_roots(p):
    for g in range(2, 100):
        w = pow(g, (p - 1) // 3, p)
        if w != 1:
            return w, w * w % p
    raise ValueError


def basis(lam):
    # extended Euclid on (r, lam): remainders r_i = s_i r + t_i lam
    r0, r1, t0, t1 = R, lam, 0, 1
    seq = []
    while r1 != 0:
        q = r0 // r1
        r0, r1 = r1, r0 - q * r1
        t0, t1 = t1, t0 - q * t1
        seq.append((r0, t0))
    # first remainder below sqrt(r)
    import math
    sq = math.isqrt(R)
    for i, (ri, ti) in enumerate(seq):
        if ri < sq:
            l = i
            break
    a1, b1 = seq[l][0], -seq[l][1]
    c = [seq[l - 1], seq[l + 1]]
    (a2, b2) = min(((x, -t) for x, t in c), key=lambda v: v[0] ** 2 + v[1] ** 2)
    return a1, b1, a2, b2


def split(k, c):
    a1, b1, a2, b2, g1, g2 = c
    c1 = (k * g1) >> 384
    c2 = (k * g2) >> 384
    k1 = k - c1 * a1 - c2 * a2
    k2 = -c1 * b1 - c2 * b2
    return k1, k2


def main():
    G = bn.G1_GEN
    bq = cube_roots(Q)
    lr = cube_roots(R)
    beta = lam = None
    for b_ in bq:
        for l_ in lr:
            if bn.mul(G, l_) == (b_ * G[0] % Q, G[1]):
                beta, lam = b_, l_
    assert beta is not None
    a1, b1, a2, b2 = basis(lam)
    assert (a1 + b1 * lam) % R == 0 and (a2 + b2 * lam) % R == 0
    g1 = ((b2 << 384) + R // 2) // R
    g2 = ((-b1 << 384) + R // 2) // R
    c = (a1, b1, a2, b2, g1, g2)
    rnd = random.Random(7)
    mx = 0
    for _ in range(2000):
        k = rnd.randrange(R)
        k1, k2 = split(k, c)
        assert (k1 + k2 * lam - k) % R == 0
        mx = max(mx, abs(k1).bit_length(), abs(k2).bit_length())
    for k in (0, 1, R - 1, R // 2):
        k1, k2 = split(k, c)
        assert (k1 + k2 * lam - k) % R == 0
        mx = max(mx, abs(k1).bit_length(), abs(k2).bit_length())
    P = bn.mul(G, 12345)
    k = rnd.randrange(R)
    k1, k2 = split(k, c)
    phiP = (beta * P[0] % Q, P[1])
    lhs = bn.add(bn.mul(P, k1 % R), bn.mul(phiP, k2 % R))
    assert lhs == bn.mul(P, k)
    print(f"// max |k1|,|k2| bits over the samples: {mx}")
    for name, v in (("beta", beta), ("lambda", lam), ("a1", a1), ("b1", b1), ("a2", a2), ("b2", b2),
                    ("g1", g1), ("g2", g2)):
        print(f"{name} = {v:#x}  ({'neg' if v < 0 else 'pos'}, {abs(v).bit_length()} bits)")


if __name__ == "__main__":
    main()
