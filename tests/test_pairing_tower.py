"""CPU: the tower-pairing restatement (oracle/pairing_tower.py — what the GPU verifier runs) is
checked against the independent oracle pairing (oracle/bn254.py) and against the algebra it relies
on.  Pins the verifier's algorithm before the GPU is compared with it bit-exactly."""

import random

from oracle import bn254 as bn
from oracle import pairing_tower as T
from oracle.bn254 import Q, R


def _rnd_g1(rng):
    return bn.mul(bn.G1_GEN, rng.randrange(1, R))


def _rnd_g2(rng):
    return bn.mul(bn.G2_GEN, rng.randrange(1, R))


def test_hard_part_chain_is_exact_exponent():
    """The Devegili-Scott-Dahab chain realises exactly (p^4 - p^2 + 1)/r on the cyclotomic
    subgroup (exponent arithmetic mod Phi12(p); conj = -1, Frobenius = *p)."""
    M = Q ** 4 - Q ** 2 + 1
    u = T.U
    fu, fu2 = u % M, u * u % M
    fu3 = fu2 * u % M
    y0 = (Q + Q * Q + Q ** 3) % M
    y1, y2 = -1 % M, fu2 * Q * Q % M
    y3, y5 = -fu * Q % M, -fu2 % M
    y4 = -(fu + fu2 * Q) % M
    y6 = -(fu3 + fu3 * Q) % M
    t0 = (2 * y6 + y4 + y5) % M
    t1 = (y3 + y5 + t0) % M
    t0 = (t0 + y2) % M
    t1 = 2 * (2 * t1 + t0) % M
    t0 = 2 * (t1 + y1) % M
    assert (t0 + t1 + y0) % M == (M // R) % M
    assert M % R == 0


def test_tower_matches_oracle_pairing():
    rng = random.Random(11)
    for _ in range(2):
        P, Qg = _rnd_g1(rng), _rnd_g2(rng)
        assert T.to_bn254_fq12(T.pairing(P, T.from_bn254_g2(Qg))) == bn.pairing(P, Qg)


def test_bilinearity_and_nondegeneracy():
    rng = random.Random(12)
    a, b = rng.randrange(1, 1 << 64), rng.randrange(1, 1 << 64)
    g = T.pairing(bn.G1_GEN, T.from_bn254_g2(bn.G2_GEN))
    assert g != T.F12_ONE
    lhs = T.pairing(bn.mul(bn.G1_GEN, a), T.from_bn254_g2(bn.mul(bn.G2_GEN, b)))
    rhs = T.pairing(bn.mul(bn.G1_GEN, a * b % R), T.from_bn254_g2(bn.G2_GEN))
    assert lhs == rhs
    # order r: g^r == 1
    x, e, acc = g, R, T.F12_ONE
    while e:
        if e & 1:
            acc = T.f12_mul(acc, x)
        x = T.f12_sqr(x)
        e >>= 1
    assert acc == T.F12_ONE


def test_multi_miller_is_product_of_millers():
    """Exact field equality (not only after the final exponentiation): the GPU multiplies the
    key's precomputed (alpha, beta) Miller value into the 3-pair loop."""
    rng = random.Random(13)
    pairs = [(_rnd_g1(rng), T.from_bn254_g2(_rnd_g2(rng))) for _ in range(2)]
    f = T.miller_loop(pairs)
    g = T.f12_mul(T.miller_loop(pairs[:1]), T.miller_loop(pairs[1:]))
    assert f == g


def test_field_helpers():
    rng = random.Random(14)
    x = T.from_flat([rng.randrange(Q) for _ in range(12)])
    assert T.f12_mul(x, T.f12_inv(x)) == T.F12_ONE
    assert T.f12_sqr(x) == T.f12_mul(x, x)
    # Frobenius = x^p, twice = x^(p^2)
    xb = T.to_bn254_fq12(x)
    assert T.to_bn254_fq12(T.f12_frob(x)) == xb ** Q
    assert T.f12_frob2(x) == T.f12_frob(T.f12_frob(x))
    c0, c3, c4 = [(rng.randrange(Q), rng.randrange(Q)) for _ in range(3)]
    sparse = ((c0, T.F2_ZERO, T.F2_ZERO), (c3, c4, T.F2_ZERO))
    assert T.f12_mul_034(x, c0, c3, c4) == T.f12_mul(x, sparse)
    assert T.from_flat(T.to_flat(x)) == x
    assert T.gt_from_bytes(T.gt_bytes(x)) == x


def test_groth16_verify_equation_with_tower():
    """A dev-ceremony proof passes the 4-pair check in the tower form, a tampered one fails."""
    from oracle import groth16 as og
    rng = random.Random(15)
    # toy instance: the equation only (no circuit): pick A, B, then C so that it holds
    alpha, beta, gamma, delta = (rng.randrange(1, R) for _ in range(4))
    a, b, x = rng.randrange(1, R), rng.randrange(1, R), rng.randrange(1, R)
    # a*b = alpha*beta + x*gamma + c*delta  ->  c
    c = (a * b - alpha * beta - x * gamma) * pow(delta, -1, R) % R
    G1, G2 = bn.G1_GEN, bn.G2_GEN
    A, B, C = bn.mul(G1, a), bn.mul(G2, b), bn.mul(G1, c)
    vkx = bn.mul(G1, x)
    g2 = T.from_bn254_g2
    pairs = [(bn.neg(A), g2(B)), (vkx, g2(bn.mul(G2, gamma))), (C, g2(bn.mul(G2, delta))),
             (bn.mul(G1, alpha), g2(bn.mul(G2, beta)))]
    assert T.f12_is_one(T.pairing_product(pairs))
    pairs[2] = (bn.add(C, G1), pairs[2][1])
    assert not T.f12_is_one(T.pairing_product(pairs))
    assert og is not None
