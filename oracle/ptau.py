"""snarkjs Powers-of-Tau ceremony + `groth16 setup` from a .ptau, restated on the CPU — TEST
INFRASTRUCTURE ONLY (see oracle/__init__.py: only tests/ may use it, as the checker).

Restated third-party algorithms (snarkjs ^0.7.5 [ext], absent from /root/reference; call sites
tests/test_secureagg.cjs:25-57 and tests/full_system_simulation.mjs:713-730):
  * powersoftau contribute: tauG1[i] *= tau^i (i < 2^(p+1) - 1), tauG2[i] *= tau^i,
    alphaTauG1[i] *= alpha tau^i, betaTauG1[i] *= beta tau^i, betaG2 *= beta;
  * powersoftau prepare phase2: for each 2^p prefix the group inverse FFT
    L_j = (1/N) sum_i w_N^{-ij} P_i (w = Fr.w[p], nqr = 5), tauG1 also at p = power + 1 with the
    missing last power taken as the point at infinity;
  * groth16 setup (zkey_new): A_i = sum_j a_ij L_j, B1_i / B2_i likewise, IC_i / C_i =
    sum_j (a_ij betaL_j + b_ij alphaL_j + c_ij L_j), public rows A[m + k][k] = 1, H_j = the odd
    Lagrange points of the 2n block, gamma = delta = 1;
  * zkey contribute: delta *= d, C and H *= 1/d.
Points are oracle/bn254.py affine tuples (None = infinity).  Written independently of
zkfl/ptau.py and zkfl/zkey.py (plain loops, no term sorting, no GPU) and sized for tiny circuits.
Parity unpinned against snarkjs itself (absent here; the reference commits no .ptau or .zkey).
"""

from __future__ import annotations

from . import bn254 as bn
from .bn254 import R


def group_ifft(points, logn):
    """(1/N) sum_i w^{-ij} P_i for j < N = 2^logn (recursive radix-2 over the group)."""
    n = 1 << logn
    assert len(points) == n
    w_inv = pow(bn.FR_W[logn], R - 2, R)

    def rec(pts, w):
        m = len(pts)
        if m == 1:
            return list(pts)
        ev = rec(pts[0::2], w * w % R)
        od = rec(pts[1::2], w * w % R)
        out = [None] * m
        t = 1
        for k in range(m // 2):
            x = bn.mul(od[k], t) if od[k] is not None else None
            out[k] = bn.add(ev[k], x)
            out[k + m // 2] = bn.add(ev[k], bn.neg(x) if x is not None else None)
            t = t * w % R
        return out
    ninv = pow(n, R - 2, R)
    return [bn.mul(p, ninv) if p is not None else None for p in rec(list(points), w_inv)]


def contribute(sections, power, tau, alpha, beta):
    """sections: {2: [G1], 3: [G2], 4: [G1], 5: [G1], 6: G2} -> the contributed sections."""
    n = 1 << power
    out = {2: [bn.mul(sections[2][i], pow(tau, i, R)) for i in range(2 * n - 1)],
           3: [bn.mul(sections[3][i], pow(tau, i, R)) for i in range(n)],
           4: [bn.mul(sections[4][i], alpha * pow(tau, i, R)) for i in range(n)],
           5: [bn.mul(sections[5][i], beta * pow(tau, i, R)) for i in range(n)],
           6: bn.mul(sections[6], beta)}
    return out


def prepare_phase2(sections, power):
    """-> {12: [blocks], 13: ..., 14: ..., 15: ...}, block p = list of 2^p points."""
    out = {}
    for src, dst in ((2, 12), (3, 13), (4, 14), (5, 15)):
        top = power + 1 if src == 2 else power
        blocks = []
        for p in range(top + 1):
            if src == 2 and p == power + 1:
                pts = sections[2][:(1 << p) - 1] + [None]
            else:
                pts = sections[src][:1 << p]
            blocks.append(group_ifft(pts, p))
        out[dst] = blocks
    return out


def groth16_setup(r1cs, sections, lagrange):
    """zkey fields (oracle/groth16.py::parse_zkey layout) from a prepared ceremony.
    r1cs: oracle/groth16.py::parse_r1cs dict; sections: contributed {4, 5, 6}; lagrange: prepare_phase2."""
    npub = r1cs["nPubOut"] + r1cs["nPubIn"]
    nv = r1cs["nWires"]
    m = r1cs["nConstraints"]
    n = 1
    while n < m + npub + 1:
        n *= 2
    p = n.bit_length() - 1
    L, L2, La, Lb = lagrange[12][p], lagrange[13][p], lagrange[14][p], lagrange[15][p]
    A = [None] * nv
    B1 = [None] * nv
    B2 = [None] * nv
    K = [None] * nv
    for j, (ca, cb, cc) in enumerate(r1cs["constraints"]):
        for w, c in ca.items():
            A[w] = bn.add(A[w], bn.mul(L[j], c))
            K[w] = bn.add(K[w], bn.mul(Lb[j], c))
        for w, c in cb.items():
            B1[w] = bn.add(B1[w], bn.mul(L[j], c))
            B2[w] = bn.add(B2[w], bn.mul(L2[j], c))
            K[w] = bn.add(K[w], bn.mul(La[j], c))
        for w, c in cc.items():
            K[w] = bn.add(K[w], bn.mul(L[j], c))
    for k in range(npub + 1):
        A[k] = bn.add(A[k], L[m + k])
        K[k] = bn.add(K[k], Lb[m + k])
    H2 = lagrange[12][p + 1]
    return dict(nVars=nv, nPublic=npub, domainSize=n, alpha1=sections[4][0], beta1=sections[5][0],
                beta2=sections[6], gamma2=bn.G2_GEN, delta1=bn.G1_GEN, delta2=bn.G2_GEN,
                IC=K[:npub + 1], C=K[npub + 1:], A=A, B1=B1, B2=B2, H=[H2[2 * j + 1] for j in range(n)])


def zkey_contribute(z, d):
    di = pow(d, R - 2, R)
    out = dict(z)
    out["delta1"] = bn.mul(z["delta1"], d)
    out["delta2"] = bn.mul(z["delta2"], d)
    out["C"] = [bn.mul(P, di) if P is not None else None for P in z["C"]]
    out["H"] = [bn.mul(P, di) if P is not None else None for P in z["H"]]
    return out
