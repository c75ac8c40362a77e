"""BN254 (alt_bn128 / snarkjs "bn128") CPU restatement — TEST INFRASTRUCTURE ONLY.

This module is part of the parity oracle.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it; the product path
(``verifiable-...-_amd``) never does.

What it restates (third-party, not vendored in the reference — SURVEY.md §8c):
  * ffjavascript ^0.2.63 / wasmcurves (``package.json:44-45`` of the reference):
    the bn128 curve object used by snarkjs ``groth16 prove``/``verify``
    (call sites ``tests/full_system_simulation.mjs:773-776, 865-868``).
    Field primes: r at ``tests/full_system_simulation.mjs:65``.
  * Root-of-unity convention: ffjavascript picks nqr = smallest quadratic
    non-residue >= 2 (=5 for Fr), w[s] = nqr^t with r-1 = 2^s * t (s = 28),
    w[i] = w[i+1]^2, and ``shift`` = nqr^2.  snarkjs's prover uses
    ``inc = power == Fr.s ? Fr.shift : Fr.w[power+1]`` for the odd coset.
  * Pairing: optimal-ate on the D-type sextic twist, Fq12 as Fq[w]/(w^12 - 18 w^6 + 82)
    (the classic reference formulation); only used to verify proofs.

Pure-Python big ints; sized for small cases (a few thousand group operations).
"""

from __future__ import annotations

# ----------------------------------------------------------------------------
# Field parameters
# ----------------------------------------------------------------------------
Q = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617

R_MONT = pow(2, 256)          # Montgomery radix used by ffjavascript (n64 = 4 limbs)


def to_mont(x: int, p: int) -> int:
    return (x * R_MONT) % p


def from_mont(x: int, p: int) -> int:
    return (x * pow(R_MONT, -1, p)) % p


# ----------------------------------------------------------------------------
# Fr roots of unity (ffjavascript convention)
# ----------------------------------------------------------------------------
def _fr_two_adicity():
    t, s = R - 1, 0
    while t % 2 == 0:
        t //= 2
        s += 1
    return s, t


FR_S, FR_T = _fr_two_adicity()            # s = 28


def _fr_nqr():
    g = 2
    while pow(g, (R - 1) // 2, R) != R - 1:
        g += 1
    return g


FR_NQR = _fr_nqr()                          # 5
FR_W = [0] * (FR_S + 1)
FR_W[FR_S] = pow(FR_NQR, FR_T, R)
for _i in range(FR_S - 1, -1, -1):
    FR_W[_i] = FR_W[_i + 1] * FR_W[_i + 1] % R
FR_SHIFT = FR_NQR * FR_NQR % R


def coset_inc(power: int) -> int:
    """Multiplier used by snarkjs groth16_prove (``batchApplyKey`` increment)."""
    return FR_SHIFT if power == FR_S else FR_W[power + 1]


# ----------------------------------------------------------------------------
# Fq2
# ----------------------------------------------------------------------------
class Fq2:
    __slots__ = ("c0", "c1")

    def __init__(self, c0, c1=0):
        self.c0 = c0 % Q
        self.c1 = c1 % Q

    def __add__(self, o):
        return Fq2(self.c0 + o.c0, self.c1 + o.c1)

    def __sub__(self, o):
        return Fq2(self.c0 - o.c0, self.c1 - o.c1)

    def __neg__(self):
        return Fq2(-self.c0, -self.c1)

    def __mul__(self, o):
        if isinstance(o, int):
            return Fq2(self.c0 * o, self.c1 * o)
        a, b, c, d = self.c0, self.c1, o.c0, o.c1
        return Fq2(a * c - b * d, a * d + b * c)

    __rmul__ = __mul__

    def __eq__(self, o):
        return self.c0 == o.c0 and self.c1 == o.c1

    def __hash__(self):
        return hash((self.c0, self.c1))

    def is_zero(self):
        return self.c0 == 0 and self.c1 == 0

    def inv(self):
        d = pow(self.c0 * self.c0 + self.c1 * self.c1, -1, Q)
        return Fq2(self.c0 * d, -self.c1 * d)

    def __repr__(self):
        return f"Fq2({self.c0}, {self.c1})"


# ----------------------------------------------------------------------------
# Generic short-Weierstrass arithmetic (y^2 = x^3 + b) over Fq (ints) or Fq2
# Points are affine tuples (x, y) or None for infinity.
# ----------------------------------------------------------------------------
B1 = 3
B2 = Fq2(3) * Fq2(9, 1).inv()               # twist b' = 3/(9+u)

G1_GEN = (1, 2)
G2_GEN = (
    Fq2(10857046999023057135944570762232829481370756359578518086990519993285655852781,
        11559732032986387107991004021392285783925812861821192530917403151452391805634),
    Fq2(8495653923123431417604973247489272438418190587263600148770280649306958101930,
        4082367875863433681332203403145435568316851327593401208105741076214120093531),
)


def _is_fq2(x):
    return isinstance(x, Fq2)


def _inv(x):
    return x.inv() if _is_fq2(x) else pow(x, -1, Q)


def _zero_like(x):
    return Fq2(0) if _is_fq2(x) else 0


def _one_like(x):
    return Fq2(1) if _is_fq2(x) else 1


def _m(a, b):
    return a * b if _is_fq2(a) else a * b % Q


def _ad(a, b):
    return a + b if _is_fq2(a) else (a + b) % Q


def _sb(a, b):
    return a - b if _is_fq2(a) else (a - b) % Q


def on_curve(P) -> bool:
    if P is None:
        return True
    x, y = P
    b = B2 if _is_fq2(x) else B1
    return _sb(_m(y, y), _ad(_m(_m(x, x), x), b)) == _zero_like(x)


def neg(P):
    if P is None:
        return None
    x, y = P
    return (x, -y if _is_fq2(y) else (-y) % Q)


# Jacobian: (X, Y, Z), x = X/Z^2, y = Y/Z^3; Z == 0 -> infinity
def to_jac(P):
    if P is None:
        return None
    return (P[0], P[1], _one_like(P[0]))


def from_jac(J):
    if J is None:
        return None
    X, Y, Z = J
    if (Z.is_zero() if _is_fq2(Z) else Z == 0):
        return None
    zi = _inv(Z)
    zi2 = _m(zi, zi)
    return (_m(X, zi2), _m(Y, _m(zi2, zi)))


def jdouble(J):
    if J is None:
        return None
    X, Y, Z = J
    if (Y.is_zero() if _is_fq2(Y) else Y == 0):
        return None
    A = _m(X, X)
    Bv = _m(Y, Y)
    C = _m(Bv, Bv)
    t = _ad(X, Bv)
    D = _sb(_sb(_m(t, t), A), C)
    D = _ad(D, D)
    E = _ad(_ad(A, A), A)
    F = _m(E, E)
    X3 = _sb(F, _ad(D, D))
    C8 = _ad(C, C)
    C8 = _ad(C8, C8)
    C8 = _ad(C8, C8)
    Y3 = _sb(_m(E, _sb(D, X3)), C8)
    Z3 = _m(Y, Z)
    Z3 = _ad(Z3, Z3)
    return (X3, Y3, Z3)


def jadd(J1, J2):
    if J1 is None:
        return J2
    if J2 is None:
        return J1
    X1, Y1, Z1 = J1
    X2, Y2, Z2 = J2
    Z1Z1 = _m(Z1, Z1)
    Z2Z2 = _m(Z2, Z2)
    U1 = _m(X1, Z2Z2)
    U2 = _m(X2, Z1Z1)
    S1 = _m(_m(Y1, Z2), Z2Z2)
    S2 = _m(_m(Y2, Z1), Z1Z1)
    if U1 == U2:
        if S1 == S2:
            return jdouble(J1)
        return None
    H = _sb(U2, U1)
    Rr = _sb(S2, S1)
    H2 = _m(H, H)
    H3 = _m(H2, H)
    U1H2 = _m(U1, H2)
    X3 = _sb(_sb(_m(Rr, Rr), H3), _ad(U1H2, U1H2))
    Y3 = _sb(_m(Rr, _sb(U1H2, X3)), _m(S1, H3))
    Z3 = _m(_m(Z1, Z2), H)
    return (X3, Y3, Z3)


def add(P1, P2):
    return from_jac(jadd(to_jac(P1), to_jac(P2)))


def mul(P, k: int):
    """Scalar multiplication (k taken mod R; group order is R on both G1 and G2)."""
    k %= R
    acc = None
    base = to_jac(P)
    while k:
        if k & 1:
            acc = jadd(acc, base)
        base = jdouble(base)
        k >>= 1
    return from_jac(acc)


def msm(points, scalars, window: int = 0):
    """Pippenger MSM (unsigned windows) — restates ffjavascript multiExpAffine semantics:
    result = sum_i scalars[i] * points[i], infinity entries and zero scalars skipped."""
    pts = [(to_jac(p), s % R) for p, s in zip(points, scalars) if p is not None and s % R]
    if not pts:
        return None
    n = len(pts)
    if window <= 0:
        window = max(2, min(12, n.bit_length() - 2))
    nwin = (254 + window - 1) // window
    mask = (1 << window) - 1
    total = None
    for w in range(nwin - 1, -1, -1):
        if total is not None:
            for _ in range(window):
                total = jdouble(total)
        buckets = [None] * (1 << window)
        for J, s in pts:
            d = (s >> (w * window)) & mask
            if d:
                buckets[d] = jadd(buckets[d], J)
        run = None
        acc = None
        for d in range(mask, 0, -1):
            run = jadd(run, buckets[d])
            acc = jadd(acc, run)
        total = jadd(total, acc)
    return from_jac(total)


# ----------------------------------------------------------------------------
# Pairing (optimal ate), Fq12 = Fq[w]/(w^12 - 18 w^6 + 82)
# ----------------------------------------------------------------------------
_FQ12_MOD = [82, 0, 0, 0, 0, 0, -18, 0, 0, 0, 0, 0]   # w^12 = 18 w^6 - 82


class Fq12:
    __slots__ = ("c",)

    def __init__(self, coeffs):
        self.c = [x % Q for x in coeffs]

    @staticmethod
    def one():
        return Fq12([1] + [0] * 11)

    def __add__(self, o):
        return Fq12([a + b for a, b in zip(self.c, o.c)])

    def __sub__(self, o):
        return Fq12([a - b for a, b in zip(self.c, o.c)])

    def __mul__(self, o):
        if isinstance(o, int):
            return Fq12([a * o for a in self.c])
        b = [0] * 23
        for i, x in enumerate(self.c):
            if x:
                for j, y in enumerate(o.c):
                    b[i + j] += x * y
        for k in range(22, 11, -1):
            top = b[k]
            if top:
                b[k] = 0
                # w^k = w^(k-12) * (18 w^6 - 82)
                b[k - 6] += 18 * top
                b[k - 12] -= 82 * top
        return Fq12(b[:12])

    def __eq__(self, o):
        return self.c == o.c

    def __pow__(self, e):
        res = Fq12.one()
        base = self
        while e:
            if e & 1:
                res = res * base
            base = base * base
            e >>= 1
        return res

    def inv(self):
        """Extended Euclid over Fq[x] modulo w^12 - 18 w^6 + 82."""
        lm, hm = [1] + [0] * 12, [0] * 13
        low, high = self.c + [0], [82, 0, 0, 0, 0, 0, -18 % Q, 0, 0, 0, 0, 0, 1]
        while _deg(low):
            r = _poly_div(high, low)
            r += [0] * (13 - len(r))
            nm = [x for x in hm]
            new = [x for x in high]
            for i in range(13):
                for j in range(13 - i):
                    nm[i + j] -= lm[i] * r[j]
                    new[i + j] -= low[i] * r[j]
            nm = [x % Q for x in nm]
            new = [x % Q for x in new]
            lm, low, hm, high = nm, new, lm, low
        inv0 = pow(low[0], -1, Q)
        return Fq12([x * inv0 for x in lm[:12]])

    def is_one(self):
        return self.c == [1] + [0] * 11


def _deg(p):
    d = len(p) - 1
    while d and p[d] % Q == 0:
        d -= 1
    return d


def _poly_div(a, b):
    dega, degb = _deg(a), _deg(b)
    temp = [x for x in a]
    o = [0] * len(a)
    ib = pow(b[degb], -1, Q)
    for i in range(dega - degb, -1, -1):
        o[i] = (o[i] + temp[degb + i] * ib) % Q
        for c in range(degb + 1):
            temp[c + i] = (temp[c + i] - o[i] * b[c]) % Q
    return [x % Q for x in o[:_deg(o) + 1]]


ATE_LOOP_COUNT = 29793968203157093288
LOG_ATE_LOOP_COUNT = 63


def _twist(P):
    """Map a G2 point (over Fq2) into Fq12 coordinates (D-type twist)."""
    if P is None:
        return None
    x, y = P
    # Fq2 element a + b*u -> in Fq12: u = w^6 - 9
    xc = [x.c0 - x.c1 * 9, x.c1]
    yc = [y.c0 - y.c1 * 9, y.c1]
    nx = Fq12([xc[0]] + [0] * 5 + [xc[1]] + [0] * 5)
    ny = Fq12([yc[0]] + [0] * 5 + [yc[1]] + [0] * 5)
    w2 = Fq12([0, 0, 1] + [0] * 9)
    w3 = Fq12([0, 0, 0, 1] + [0] * 8)
    return (nx * w2, ny * w3)


def _cast_g1(P):
    return (Fq12([P[0]] + [0] * 11), Fq12([P[1]] + [0] * 11))


def _fq12_div(a, b):
    return a * b.inv()


def _linefunc(P1, P2, T):
    x1, y1 = P1
    x2, y2 = P2
    xt, yt = T
    if x1 != x2:
        m = _fq12_div(y2 - y1, x2 - x1)
        return m * (xt - x1) - (yt - y1)
    elif y1 == y2:
        m = _fq12_div(x1 * x1 * 3, y1 * 2)
        return m * (xt - x1) - (yt - y1)
    else:
        return xt - x1


def _fq12_add_pts(P1, P2):
    x1, y1 = P1
    x2, y2 = P2
    if x1 == x2 and y1 == y2:
        m = _fq12_div(x1 * x1 * 3, y1 * 2)
    elif x1 == x2:
        return None
    else:
        m = _fq12_div(y2 - y1, x2 - x1)
    x3 = m * m - x1 - x2
    y3 = m * (x1 - x3) - y1
    return (x3, y3)


def _frob(P):
    x, y = P
    return (x ** Q, y ** Q)


def miller_loop(Qp, Pp):
    """Qp: G2 point already twisted into Fq12; Pp: G1 point cast into Fq12."""
    if Qp is None or Pp is None:
        return Fq12.one()
    Rp = Qp
    f = Fq12.one()
    for i in range(LOG_ATE_LOOP_COUNT, -1, -1):
        f = f * f * _linefunc(Rp, Rp, Pp)
        Rp = _fq12_add_pts(Rp, Rp)
        if ATE_LOOP_COUNT & (2 ** i):
            f = f * _linefunc(Rp, Qp, Pp)
            Rp = _fq12_add_pts(Rp, Qp)
    Q1 = _frob(Qp)
    nQ2 = _frob(Q1)
    nQ2 = (nQ2[0], Fq12([0] * 12) - nQ2[1])
    f = f * _linefunc(Rp, Q1, Pp)
    Rp = _fq12_add_pts(Rp, Q1)
    f = f * _linefunc(Rp, nQ2, Pp)
    return f


FINAL_EXP = (Q ** 12 - 1) // R


def pairing_product(pairs):
    """prod e(P_i, Q_i) for [(G1 affine, G2 affine)], with one final exponentiation."""
    f = Fq12.one()
    for P, Qg in pairs:
        if P is None or Qg is None:
            continue
        f = f * miller_loop(_twist(Qg), _cast_g1(P))
    return f ** FINAL_EXP


def pairing(P, Qg):
    return pairing_product([(P, Qg)])


# ----------------------------------------------------------------------------
# Byte encodings (snarkjs/ffjavascript conventions)
# ----------------------------------------------------------------------------
def int_to_le(x: int, n: int = 32) -> bytes:
    return int(x).to_bytes(n, "little")


def le_to_int(b: bytes) -> int:
    return int.from_bytes(b, "little")


def g1_to_bytes_mont(P) -> bytes:
    """zkey affine G1 (``toRprLEM``): Montgomery x || y, infinity = 64 zero bytes."""
    if P is None:
        return bytes(64)
    return int_to_le(to_mont(P[0], Q)) + int_to_le(to_mont(P[1], Q))


def g1_from_bytes_mont(b: bytes):
    x = from_mont(le_to_int(b[0:32]), Q)
    y = from_mont(le_to_int(b[32:64]), Q)
    if x == 0 and y == 0:
        return None
    return (x, y)


def g2_to_bytes_mont(P) -> bytes:
    if P is None:
        return bytes(128)
    x, y = P
    return b"".join(int_to_le(to_mont(v, Q)) for v in (x.c0, x.c1, y.c0, y.c1))


def g2_from_bytes_mont(b: bytes):
    v = [from_mont(le_to_int(b[32 * i:32 * i + 32]), Q) for i in range(4)]
    if all(x == 0 for x in v):
        return None
    return (Fq2(v[0], v[1]), Fq2(v[2], v[3]))


def g1_to_bytes_std(P) -> bytes:
    if P is None:
        return bytes(64)
    return int_to_le(P[0]) + int_to_le(P[1])


def g2_to_bytes_std(P) -> bytes:
    if P is None:
        return bytes(128)
    x, y = P
    return b"".join(int_to_le(v) for v in (x.c0, x.c1, y.c0, y.c1))


def g1_from_bytes_std(b: bytes):
    x, y = le_to_int(b[0:32]), le_to_int(b[32:64])
    return None if x == 0 and y == 0 else (x, y)


def g2_from_bytes_std(b: bytes):
    v = [le_to_int(b[32 * i:32 * i + 32]) for i in range(4)]
    return None if all(x == 0 for x in v) else (Fq2(v[0], v[1]), Fq2(v[2], v[3]))
