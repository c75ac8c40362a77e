"""Optimal-ate pairing over the Fq2 -> Fq6 -> Fq12 tower — TEST INFRASTRUCTURE ONLY.

Part of the parity oracle (only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it).  It restates, step by step, the algorithm the GPU verifier
(``csrc/verify.hip``) runs, so that intermediate values (Miller-loop output, final
exponentiation) can be compared bit-exactly; it is itself checked against the independent
formulation in ``oracle/bn254.py`` (``pairing``, Fq[w]/(w^12 - 18 w^6 + 82)) by
``tests/test_pairing_tower.py``.

What the GPU path restates (snarkjs ``groth16 verify`` -> ffjavascript ``pairingEq``,
reference call site ``tests/full_system_simulation.mjs:865-868``):
  * tower: Fq2 = Fq[u]/(u^2+1), Fq6 = Fq2[v]/(v^3 - xi), xi = 9+u, Fq12 = Fq6[w]/(w^2 - v)
    (the ffjavascript bn128 tower, so an Fq12 serialises as [[c0.c0,c0.c1,c0.c2],[c1.c0,...]]);
  * Miller loop over the bits of 6u+2 (MSB first, top bit implicit), G2 point in homogeneous
    projective coordinates on the D-type twist, lines evaluated at the affine G1 point and
    multiplied in sparsely (coefficients at 1, w, v*w), then the two Frobenius lines
    (Q1 = pi(Q), -Q2 = -pi^2(Q));
  * final exponentiation: easy part f^((p^6-1)(p^2+1)), hard part by the
    Devegili-Scott-Dahab chain in u (exactly (p^4-p^2+1)/r; see tests).
"""

from __future__ import annotations

from .bn254 import Q, R

U = 4965661367192848881               # BN parameter: p = 36u^4 + 36u^3 + 24u^2 + 6u + 1
ATE = 6 * U + 2
assert ATE == 29793968203157093288


# ---------------------------------------------------------------- Fq2 (tuples (a, b) = a + b u)
def f2(a, b=0):
    return (a % Q, b % Q)


F2_ZERO, F2_ONE = (0, 0), (1, 0)


def f2_add(x, y):
    return ((x[0] + y[0]) % Q, (x[1] + y[1]) % Q)


def f2_sub(x, y):
    return ((x[0] - y[0]) % Q, (x[1] - y[1]) % Q)


def f2_neg(x):
    return ((-x[0]) % Q, (-x[1]) % Q)


def f2_mul(x, y):
    return ((x[0] * y[0] - x[1] * y[1]) % Q, (x[0] * y[1] + x[1] * y[0]) % Q)


def f2_sqr(x):
    return f2_mul(x, x)


def f2_mul_fq(x, s):
    return (x[0] * s % Q, x[1] * s % Q)


def f2_conj(x):
    return (x[0], (-x[1]) % Q)


def f2_inv(x):
    n = pow(x[0] * x[0] + x[1] * x[1], -1, Q)
    return (x[0] * n % Q, (-x[1]) * n % Q)


def f2_mul_xi(x):
    """x * (9 + u)."""
    return ((9 * x[0] - x[1]) % Q, (x[0] + 9 * x[1]) % Q)


def f2_pow(x, e):
    r_ = F2_ONE
    while e:
        if e & 1:
            r_ = f2_mul(r_, x)
        x = f2_sqr(x)
        e >>= 1
    return r_


XI = (9, 1)
# Frobenius coefficients: gamma1[k] = xi^(k(p-1)/6), gamma2[k] = xi^(k(p^2-1)/6), k = 0..5
GAMMA1 = [f2_pow(XI, k * (Q - 1) // 6) for k in range(6)]
GAMMA2 = [f2_pow(XI, k * (Q * Q - 1) // 6) for k in range(6)]
# twist Frobenius on E'(Fq2): pi(x, y) = (conj(x) * xi^((p-1)/3), conj(y) * xi^((p-1)/2))
TWIST_FROB_X = f2_pow(XI, (Q - 1) // 3)
TWIST_FROB_Y = f2_pow(XI, (Q - 1) // 2)
B_TWIST = f2_mul((3, 0), f2_inv(XI))          # b' = 3 / xi


# ---------------------------------------------------------------- Fq6 (c0, c1, c2) over v
F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)


def f6_add(x, y):
    return tuple(f2_add(a, b) for a, b in zip(x, y))


def f6_sub(x, y):
    return tuple(f2_sub(a, b) for a, b in zip(x, y))


def f6_neg(x):
    return tuple(f2_neg(a) for a in x)


def f6_mul(x, y):
    a0, a1, a2 = x
    b0, b1, b2 = y
    t0, t1, t2 = f2_mul(a0, b0), f2_mul(a1, b1), f2_mul(a2, b2)
    c0 = f2_add(t0, f2_mul_xi(f2_sub(f2_sub(f2_mul(f2_add(a1, a2), f2_add(b1, b2)), t1), t2)))
    c1 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a0, a1), f2_add(b0, b1)), t0), t1), f2_mul_xi(t2))
    c2 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a0, a2), f2_add(b0, b2)), t0), t2), t1)
    return (c0, c1, c2)


def f6_mul_v(x):
    """x * v: (c0, c1, c2) -> (xi c2, c0, c1)."""
    return (f2_mul_xi(x[2]), x[0], x[1])


def f6_inv(x):
    a0, a1, a2 = x
    t0 = f2_sub(f2_sqr(a0), f2_mul_xi(f2_mul(a1, a2)))
    t1 = f2_sub(f2_mul_xi(f2_sqr(a2)), f2_mul(a0, a1))
    t2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    d = f2_add(f2_mul(a0, t0), f2_mul_xi(f2_add(f2_mul(a2, t1), f2_mul(a1, t2))))
    di = f2_inv(d)
    return (f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di))


# ---------------------------------------------------------------- Fq12 (c0, c1) over w
F12_ONE = (F6_ONE, F6_ZERO)


def f12_mul(x, y):
    a0, a1 = x
    b0, b1 = y
    t0, t1 = f6_mul(a0, b0), f6_mul(a1, b1)
    c1 = f6_sub(f6_sub(f6_mul(f6_add(a0, a1), f6_add(b0, b1)), t0), t1)
    return (f6_add(t0, f6_mul_v(t1)), c1)


def f12_sqr(x):
    """Complex squaring: (a + b w)^2 = (a^2 + v b^2) + 2ab w, via (a+b)(a+vb) - ab - v ab."""
    a, b = x
    ab = f6_mul(a, b)
    t = f6_mul(f6_add(a, b), f6_add(a, f6_mul_v(b)))
    c0 = f6_sub(f6_sub(t, ab), f6_mul_v(ab))
    return (c0, f6_add(ab, ab))


def f12_conj(x):
    return (x[0], f6_neg(x[1]))


def f12_inv(x):
    a, b = x
    d = f6_inv(f6_sub(f6_mul(a, a), f6_mul_v(f6_mul(b, b))))
    return (f6_mul(a, d), f6_neg(f6_mul(b, d)))


def _coeffs(x):
    """Fq2 coefficients of x in the basis w^k, k = 0..5 (w^2 = v)."""
    (c00, c01, c02), (c10, c11, c12) = x
    return [c00, c10, c01, c11, c02, c12]


def _from_coeffs(c):
    return ((c[0], c[2], c[4]), (c[1], c[3], c[5]))


def f12_frob(x):
    return _from_coeffs([f2_mul(f2_conj(c), GAMMA1[k]) for k, c in enumerate(_coeffs(x))])


def f12_frob2(x):
    return _from_coeffs([f2_mul(c, GAMMA2[k]) for k, c in enumerate(_coeffs(x))])


def f12_mul_034(f, c0, c3, c4):
    """f * (c0 + (c3 + c4 v) w) with c0, c3, c4 in Fq2 (sparse line)."""
    a, b = f
    # a*c0 (c0 scalar in Fq2)
    a0 = tuple(f2_mul(t, c0) for t in a)
    # b*(c3 + c4 v)
    bb = f6_mul(b, (c3, c4, F2_ZERO))
    c1 = f6_sub(f6_sub(f6_mul(f6_add(a, b), (f2_add(c0, c3), c4, F2_ZERO)), a0), bb)
    return (f6_add(a0, f6_mul_v(bb)), c1)


def f12_pow_u(x):
    r_ = F12_ONE
    for bit in bin(U)[2:]:
        r_ = f12_sqr(r_)
        if bit == "1":
            r_ = f12_mul(r_, x)
    return r_


# ---------------------------------------------------------------- Miller loop
TWO_INV = pow(2, -1, Q)


def dbl_step(Rp):
    """Homogeneous projective doubling on E'; returns (R', (c0, c3, c4)) before scaling by P."""
    X, Y, Z = Rp
    a = f2_mul_fq(f2_mul(X, Y), TWO_INV)
    b = f2_sqr(Y)
    c = f2_sqr(Z)
    e = f2_mul(B_TWIST, f2_add(f2_add(c, c), c))
    f = f2_add(f2_add(e, e), e)
    g = f2_mul_fq(f2_add(b, f), TWO_INV)
    h = f2_sub(f2_sqr(f2_add(Y, Z)), f2_add(b, c))
    i = f2_sub(e, b)
    j = f2_sqr(X)
    e2 = f2_sqr(e)
    X3 = f2_mul(a, f2_sub(b, f))
    Y3 = f2_sub(f2_sqr(g), f2_add(f2_add(e2, e2), e2))
    Z3 = f2_mul(b, h)
    return (X3, Y3, Z3), (f2_neg(h), f2_add(f2_add(j, j), j), i)


def add_step(Rp, Qa):
    """Mixed addition R + Q (Q affine on E'); returns (R', line (c0, c3, c4))."""
    X, Y, Z = Rp
    qx, qy = Qa
    theta = f2_sub(Y, f2_mul(qy, Z))
    lam = f2_sub(X, f2_mul(qx, Z))
    c = f2_sqr(theta)
    d = f2_sqr(lam)
    e = f2_mul(lam, d)
    f = f2_mul(Z, c)
    g = f2_mul(X, d)
    h = f2_sub(f2_add(e, f), f2_add(g, g))
    X3 = f2_mul(lam, h)
    Y3 = f2_sub(f2_mul(theta, f2_sub(g, h)), f2_mul(e, Y))
    Z3 = f2_mul(Z, e)
    j = f2_sub(f2_mul(theta, qx), f2_mul(lam, qy))
    return (X3, Y3, Z3), (lam, f2_neg(theta), j)


def _ell(f, line, P):
    c0, c3, c4 = line
    return f12_mul_034(f, f2_mul_fq(c0, P[1]), f2_mul_fq(c3, P[0]), c4)


def twist_frob(Qa):
    return (f2_mul(f2_conj(Qa[0]), TWIST_FROB_X), f2_mul(f2_conj(Qa[1]), TWIST_FROB_Y))


def miller_loop(pairs):
    """Multi-Miller loop prod f_{6u+2,Q_i}(P_i) * lines(Q1, -Q2); pairs = [(P affine Fq, Q affine Fq2)]
    with infinity (None) pairs skipped."""
    pairs = [(P, Qa) for P, Qa in pairs if P is not None and Qa is not None]
    Rs = [(Qa[0], Qa[1], F2_ONE) for _, Qa in pairs]
    f = F12_ONE
    bits = bin(ATE)[3:]                      # top bit implicit (R starts at Q)
    for k, bit in enumerate(bits):
        if k:
            f = f12_sqr(f)
        for i, (P, Qa) in enumerate(pairs):
            Rs[i], line = dbl_step(Rs[i])
            f = _ell(f, line, P)
        if bit == "1":
            for i, (P, Qa) in enumerate(pairs):
                Rs[i], line = add_step(Rs[i], Qa)
                f = _ell(f, line, P)
    for i, (P, Qa) in enumerate(pairs):
        q1 = twist_frob(Qa)
        q2 = twist_frob(q1)
        nq2 = (q2[0], f2_neg(q2[1]))
        Rs[i], line = add_step(Rs[i], q1)
        f = _ell(f, line, P)
        Rs[i], line = add_step(Rs[i], nq2)
        f = _ell(f, line, P)
    return f


def final_exp(f):
    # easy part: f^(p^6 - 1) then ^(p^2 + 1)
    t = f12_mul(f12_conj(f), f12_inv(f))
    t = f12_mul(f12_frob2(t), t)
    # hard part (Devegili-Scott-Dahab)
    fp = f12_frob(t)
    fp2 = f12_frob2(t)
    fp3 = f12_frob(fp2)
    fu = f12_pow_u(t)
    fu2 = f12_pow_u(fu)
    fu3 = f12_pow_u(fu2)
    y3 = f12_conj(f12_frob(fu))
    fu2p = f12_frob(fu2)
    fu3p = f12_frob(fu3)
    y2 = f12_frob2(fu2)
    y0 = f12_mul(f12_mul(fp, fp2), fp3)
    y1 = f12_conj(t)
    y5 = f12_conj(fu2)
    y4 = f12_conj(f12_mul(fu, fu2p))
    y6 = f12_conj(f12_mul(fu3, fu3p))
    t0 = f12_mul(f12_mul(f12_sqr(y6), y4), y5)
    t1 = f12_mul(f12_mul(y3, y5), t0)
    t0 = f12_mul(t0, y2)
    t1 = f12_sqr(f12_mul(f12_sqr(t1), t0))
    t0 = f12_mul(t1, y1)
    t1 = f12_mul(t1, y0)
    t0 = f12_sqr(t0)
    return f12_mul(t0, t1)


def pairing(P, Qa):
    return final_exp(miller_loop([(P, Qa)]))


def pairing_product(pairs):
    return final_exp(miller_loop(pairs))


def f12_is_one(x):
    return x == F12_ONE


# ---------------------------------------------------------------- conversions / encodings
def from_bn254_g2(Qg):
    """oracle.bn254 G2 affine (Fq2 objects) -> tuples."""
    if Qg is None:
        return None
    return ((Qg[0].c0, Qg[0].c1), (Qg[1].c0, Qg[1].c1))


def to_flat(x):
    """Fq12 -> 12 ints in the ffjavascript toObject order (c0.c0.a, c0.c0.b, c0.c1.a, ...)."""
    return [v for f6 in x for f2_ in f6 for v in f2_]


def from_flat(v):
    return tuple(tuple((v[6 * i + 2 * j], v[6 * i + 2 * j + 1]) for j in range(3)) for i in range(2))


def to_bn254_fq12(x):
    """Tower element -> oracle.bn254.Fq12 coefficients (basis w^0..w^11, u = w^6 - 9)."""
    from .bn254 import Fq12
    coeffs = [0] * 12
    for k, (a, b) in enumerate(_coeffs(x)):
        # (a + b u) w^k = (a - 9 b) w^k + b w^(k+6)
        coeffs[k] += a - 9 * b
        coeffs[k + 6] += b
    return Fq12(coeffs)


def gt_bytes(x) -> bytes:
    return b"".join(int(v).to_bytes(32, "little") for v in to_flat(x))


def gt_from_bytes(b: bytes):
    return from_flat([int.from_bytes(b[32 * i:32 * i + 32], "little") for i in range(12)])


def vk_alphabeta_json(vk_alpha_1, vk_beta_2):
    """snarkjs vkey.json ``vk_alphabeta_12`` layout for e(alpha1, beta2) (decimal strings)."""
    gt = pairing(vk_alpha_1, from_bn254_g2(vk_beta_2))
    return [[[str(v) for v in f2_] for f2_ in f6] for f6 in gt]
