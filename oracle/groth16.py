"""snarkjs Groth16 restated on the CPU (pure Python) — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.  It is the checker, never the thing measured or shipped.

Restated third-party algorithms (absent from /root/reference):
  * snarkjs ^0.7.5 ``groth16 prove`` (call site ``tests/full_system_simulation.mjs:773-776``):
    buildABC1 -> 3 x (ifft, batchApplyKey(inc), fft) -> joinABC -> 5 multiExpAffine
    -> assembly with blinding r, s.  Parity with snarkjs itself is *unpinned* (snarkjs draws
    r, s at random and the reference commits no proofs); parity here is defined with
    injected (r, s) plus pairing verification.
  * snarkjs ``groth16 verify`` (``tests/full_system_simulation.mjs:865-868``): pairing check
    e(-A, B) e(alpha1, beta2) e(vk_x, gamma2) e(C, delta2) == 1.
  * snarkjs ``zkey new`` + one ``zkey contribute`` (``tests/full_system_simulation.mjs:713-730``)
    as a known-tau dev ceremony: IC/C = (beta*A_i + alpha*B_i + C_i)/gamma|delta, H = odd
    Lagrange points of the 2n domain / delta; public-input rows A[nConstraints+k][k] = 1.
  * iden3 binfile formats (.r1cs v1, .wtns v2, .zkey groth16), SURVEY.md Appendix A.
Sized for small circuits (a few hundred wires).
"""

from __future__ import annotations

import struct

from . import bn254 as bn
from .bn254 import Q, R

# ---------------------------------------------------------------------------
# iden3 binfile
# ---------------------------------------------------------------------------


def read_binfile(buf: bytes, magic: bytes):
    if buf[:4] != magic:
        raise ValueError(f"bad magic {buf[:4]!r}, want {magic!r}")
    version, nsec = struct.unpack_from("<II", buf, 4)
    off = 12
    sections = {}
    for _ in range(nsec):
        typ, size = struct.unpack_from("<IQ", buf, off)
        off += 12
        sections.setdefault(typ, []).append((off, size))
        off += size
    return version, sections


def _sec(buf, sections, typ):
    off, size = sections[typ][0]
    return buf[off:off + size]


def parse_wtns(buf: bytes):
    _, secs = read_binfile(buf, b"wtns")
    h = _sec(buf, secs, 1)
    n8 = struct.unpack_from("<I", h, 0)[0]
    prime = int.from_bytes(h[4:4 + n8], "little")
    nw = struct.unpack_from("<I", h, 4 + n8)[0]
    assert prime == R
    d = _sec(buf, secs, 2)
    return [int.from_bytes(d[i * n8:(i + 1) * n8], "little") for i in range(nw)]


def parse_r1cs(buf: bytes):
    _, secs = read_binfile(buf, b"r1cs")
    h = _sec(buf, secs, 1)
    n8 = struct.unpack_from("<I", h, 0)[0]
    prime = int.from_bytes(h[4:4 + n8], "little")
    assert prime == R
    o = 4 + n8
    nWires, nPubOut, nPubIn, nPrvIn = struct.unpack_from("<IIII", h, o)
    nLabels = struct.unpack_from("<Q", h, o + 16)[0]
    nConstraints = struct.unpack_from("<I", h, o + 24)[0]
    d = _sec(buf, secs, 2)
    p = 0
    cons = []
    for _ in range(nConstraints):
        lcs = []
        for _m in range(3):
            nt = struct.unpack_from("<I", d, p)[0]
            p += 4
            lc = {}
            for _t in range(nt):
                w = struct.unpack_from("<I", d, p)[0]
                c = int.from_bytes(d[p + 4:p + 4 + n8], "little")
                p += 4 + n8
                lc[w] = c
            lcs.append(lc)
        cons.append(tuple(lcs))
    return dict(nWires=nWires, nPubOut=nPubOut, nPubIn=nPubIn, nPrvIn=nPrvIn,
                nLabels=nLabels, nConstraints=nConstraints, constraints=cons)


def parse_zkey(buf: bytes):
    _, secs = read_binfile(buf, b"zkey")
    assert struct.unpack_from("<I", _sec(buf, secs, 1), 0)[0] == 1, "not groth16"
    h = _sec(buf, secs, 2)
    n8q = struct.unpack_from("<I", h, 0)[0]
    q = int.from_bytes(h[4:4 + n8q], "little")
    o = 4 + n8q
    n8r = struct.unpack_from("<I", h, o)[0]
    r = int.from_bytes(h[o + 4:o + 4 + n8r], "little")
    o += 4 + n8r
    assert q == Q and r == R
    nVars, nPublic, domainSize = struct.unpack_from("<III", h, o)
    o += 12
    z = dict(nVars=nVars, nPublic=nPublic, domainSize=domainSize)
    z["alpha1"] = bn.g1_from_bytes_mont(h[o:o + 64]); o += 64
    z["beta1"] = bn.g1_from_bytes_mont(h[o:o + 64]); o += 64
    z["beta2"] = bn.g2_from_bytes_mont(h[o:o + 128]); o += 128
    z["gamma2"] = bn.g2_from_bytes_mont(h[o:o + 128]); o += 128
    z["delta1"] = bn.g1_from_bytes_mont(h[o:o + 64]); o += 64
    z["delta2"] = bn.g2_from_bytes_mont(h[o:o + 128]); o += 128
    ic = _sec(buf, secs, 3)
    z["IC"] = [bn.g1_from_bytes_mont(ic[i * 64:(i + 1) * 64]) for i in range(nPublic + 1)]
    cs = _sec(buf, secs, 4)
    nc = struct.unpack_from("<I", cs, 0)[0]
    coeffs = []
    rinv2 = pow(bn.R_MONT * bn.R_MONT, -1, R)
    for i in range(nc):
        m, c, s = struct.unpack_from("<III", cs, 4 + i * 44)
        raw = int.from_bytes(cs[4 + i * 44 + 12:4 + i * 44 + 44], "little")
        coeffs.append((m, c, s, raw * rinv2 % R))    # stored raw = coef * R^2
    z["coeffs"] = coeffs
    A = _sec(buf, secs, 5)
    z["A"] = [bn.g1_from_bytes_mont(A[i * 64:(i + 1) * 64]) for i in range(nVars)]
    B1 = _sec(buf, secs, 6)
    z["B1"] = [bn.g1_from_bytes_mont(B1[i * 64:(i + 1) * 64]) for i in range(nVars)]
    B2 = _sec(buf, secs, 7)
    z["B2"] = [bn.g2_from_bytes_mont(B2[i * 128:(i + 1) * 128]) for i in range(nVars)]
    C = _sec(buf, secs, 8)
    z["C"] = [bn.g1_from_bytes_mont(C[i * 64:(i + 1) * 64]) for i in range(nVars - nPublic - 1)]
    H = _sec(buf, secs, 9)
    z["H"] = [bn.g1_from_bytes_mont(H[i * 64:(i + 1) * 64]) for i in range(domainSize)]
    return z


# ---------------------------------------------------------------------------
# Fr NTT (natural order in / out), ffjavascript root convention
# ---------------------------------------------------------------------------


def _bitrev(a):
    n = len(a)
    j = 0
    a = list(a)
    for i in range(1, n):
        bit = n >> 1
        while j & bit:
            j ^= bit
            bit >>= 1
        j ^= bit
        if i < j:
            a[i], a[j] = a[j], a[i]
    return a


def fft(a, inverse=False):
    n = len(a)
    power = n.bit_length() - 1
    assert 1 << power == n
    w = bn.FR_W[power]
    if inverse:
        w = pow(w, -1, R)
    a = _bitrev(a)
    m = 1
    while m < n:
        wm = pow(w, n // (2 * m), R)
        for k in range(0, n, 2 * m):
            wk = 1
            for j in range(m):
                t = wk * a[k + j + m] % R
                u = a[k + j]
                a[k + j] = (u + t) % R
                a[k + j + m] = (u - t) % R
                wk = wk * wm % R
        m *= 2
    if inverse:
        ninv = pow(n, -1, R)
        a = [x * ninv % R for x in a]
    return a


# ---------------------------------------------------------------------------
# Prover (snarkjs groth16_prove restated)
# ---------------------------------------------------------------------------


def build_abc(z, w):
    n = z["domainSize"]
    a = [0] * n
    b = [0] * n
    for m, c, s, coef in z["coeffs"]:
        if m == 0:
            a[c] = (a[c] + coef * w[s]) % R
        else:
            b[c] = (b[c] + coef * w[s]) % R
    c = [x * y % R for x, y in zip(a, b)]
    return a, b, c


def coset_evals(vec):
    n = len(vec)
    power = n.bit_length() - 1
    inc = bn.coset_inc(power)
    coef = fft(vec, inverse=True)
    f = 1
    for i in range(n):
        coef[i] = coef[i] * f % R
        f = f * inc % R
    return fft(coef)


def compute_h(z, w):
    a, b, c = build_abc(z, w)
    ao, bo, co = coset_evals(a), coset_evals(b), coset_evals(c)
    return [(x * y - v) % R for x, y, v in zip(ao, bo, co)]


def prove(z, w, r, s):
    """Returns dict(pi_a G1, pi_b G2, pi_c G1, public list, msm partials)."""
    nPub = z["nPublic"]
    assert len(w) == z["nVars"]
    h = compute_h(z, w)
    msmA = bn.msm(z["A"], w)
    msmB1 = bn.msm(z["B1"], w)
    msmB2 = bn.msm(z["B2"], w)
    msmC = bn.msm(z["C"], w[nPub + 1:])
    msmH = bn.msm(z["H"], h)
    pi_a = bn.add(bn.add(msmA, z["alpha1"]), bn.mul(z["delta1"], r))
    pi_b = bn.add(bn.add(msmB2, z["beta2"]), bn.mul(z["delta2"], s))
    pib1 = bn.add(bn.add(msmB1, z["beta1"]), bn.mul(z["delta1"], s))
    pi_c = bn.add(msmC, msmH)
    pi_c = bn.add(pi_c, bn.mul(pi_a, s))
    pi_c = bn.add(pi_c, bn.mul(pib1, r))
    pi_c = bn.add(pi_c, bn.mul(z["delta1"], (-(r * s)) % R))
    return dict(pi_a=pi_a, pi_b=pi_b, pi_c=pi_c, public=w[1:nPub + 1], h=h,
                msm=dict(A=msmA, B1=msmB1, B2=msmB2, C=msmC, H=msmH))


def proof_bytes(p) -> bytes:
    """Layout of the C-ABI proof buffer: pi_a G1 64 B | pi_b G2 128 B | pi_c G1 64 B,
    standard-form little-endian affine coordinates."""
    return bn.g1_to_bytes_std(p["pi_a"]) + bn.g2_to_bytes_std(p["pi_b"]) + bn.g1_to_bytes_std(p["pi_c"])


def verify(vk, public, pi_a, pi_b, pi_c) -> bool:
    if len(public) != len(vk["IC"]) - 1:
        return False
    vk_x = vk["IC"][0]
    for x, P in zip(public, vk["IC"][1:]):
        vk_x = bn.add(vk_x, bn.mul(P, int(x)))
    f = bn.pairing_product([(bn.neg(pi_a), pi_b), (vk["alpha1"], vk["beta2"]),
                            (vk_x, vk["gamma2"]), (pi_c, vk["delta2"])])
    return f.is_one()


# ---------------------------------------------------------------------------
# Known-tau dev ceremony (zkey new + one contribution), for small circuits
# ---------------------------------------------------------------------------


def lagrange_at(tau, n, omega):
    """[L_j(tau)] for the size-n domain generated by omega."""
    tn = pow(tau, n, R)
    num = (tn - 1) * pow(n, -1, R) % R
    out = []
    wj = 1
    for _ in range(n):
        out.append(num * wj % R * pow((tau - wj) % R, -1, R) % R)
        wj = wj * omega % R
    return out


def setup(r1cs, tau, alpha, beta, gamma, delta):
    nPub = r1cs["nPubOut"] + r1cs["nPubIn"]
    nVars = r1cs["nWires"]
    ncons = r1cs["nConstraints"]
    n = 1
    while n < ncons + nPub + 1:
        n *= 2
    power = n.bit_length() - 1
    L = lagrange_at(tau, n, bn.FR_W[power])
    Ai = [0] * nVars
    Bi = [0] * nVars
    Ci = [0] * nVars
    coeffs = []
    for j, (A, B, C) in enumerate(r1cs["constraints"]):
        for wv, c in A.items():
            Ai[wv] = (Ai[wv] + c * L[j]) % R
            coeffs.append((0, j, wv, c % R))
        for wv, c in B.items():
            Bi[wv] = (Bi[wv] + c * L[j]) % R
            coeffs.append((1, j, wv, c % R))
        for wv, c in C.items():
            Ci[wv] = (Ci[wv] + c * L[j]) % R
    for k in range(nPub + 1):
        Ai[k] = (Ai[k] + L[ncons + k]) % R
        coeffs.append((0, ncons + k, k, 1))
    gi = pow(gamma, -1, R)
    di = pow(delta, -1, R)
    G1, G2 = bn.G1_GEN, bn.G2_GEN
    z = dict(nVars=nVars, nPublic=nPub, domainSize=n, coeffs=coeffs)
    z["alpha1"] = bn.mul(G1, alpha)
    z["beta1"] = bn.mul(G1, beta)
    z["beta2"] = bn.mul(G2, beta)
    z["gamma2"] = bn.mul(G2, gamma)
    z["delta1"] = bn.mul(G1, delta)
    z["delta2"] = bn.mul(G2, delta)
    k = [(beta * Ai[i] + alpha * Bi[i] + Ci[i]) % R for i in range(nVars)]
    z["IC"] = [bn.mul(G1, k[i] * gi) for i in range(nPub + 1)]
    z["C"] = [bn.mul(G1, k[i] * di) for i in range(nPub + 1, nVars)]
    z["A"] = [bn.mul(G1, x) for x in Ai]
    z["B1"] = [bn.mul(G1, x) for x in Bi]
    z["B2"] = [bn.mul(G2, x) for x in Bi]
    w2n = bn.FR_W[power + 1]
    L2 = lagrange_at(tau, 2 * n, w2n)
    z["H"] = [bn.mul(G1, L2[2 * i + 1] * di) for i in range(n)]
    return z
