"""iden3 binfile writers (.wtns, .zkey) and the known-tau dev ceremony.

Formats are snarkjs's:
  .wtns v2  : §1 n8, prime, nWitness ; §2 witness values, std form LE
  .zkey     : §1 protocol=1 (groth16) ; §2 header (n8q, q, n8r, r, nVars, nPublic, domainSize,
              alpha1, beta1, beta2, gamma2, delta1, delta2 — affine Montgomery LE) ; §3 IC ;
              §4 coefficients (nCoeffs; matrix, constraint, signal, coef*R^2 mod r) incl. the
              public-input rows A[nConstraints+k][k] = 1 ; §5 A ; §6 B1 ; §7 B2 ; §8 C ; §9 H ;
              §10 contributions.
The ceremony replaces ``snarkjs groth16 setup`` + one ``zkey contribute`` of the reference
harness (tests/full_system_simulation.mjs:713-730): with toxic waste (tau, alpha, beta, gamma,
delta) it computes IC_i = (beta A_i + alpha B_i + C_i)(tau)/gamma, C_i = (...)/delta,
H_i = L^{(2n)}_{2i+1}(tau)/delta (odd Lagrange points of the 2n domain, as snarkjs takes from
ptau section 12).  It is a DEVELOPMENT ceremony (secrets known to the caller), as documented
in DESIGN.md.  The fixed-base multiplications run on the GPU (libzkfl zkfl_setup_*).
"""

from __future__ import annotations

import hashlib
import secrets
import struct

from .field import Q, R

R2_MONT = pow(2, 512, R)          # coefficient scaling: stored raw = coef * R^2 mod r
N8 = 32

# ffjavascript Fr roots of unity: nqr = 5, w[28] = 5^t, w[i] = w[i+1]^2
_FR_S = 28
_FR_T = (R - 1) >> _FR_S
_W = [0] * (_FR_S + 1)
_W[_FR_S] = pow(5, _FR_T, R)
for _i in range(_FR_S - 1, -1, -1):
    _W[_i] = _W[_i + 1] * _W[_i + 1] % R


def root_of_unity(power: int) -> int:
    return _W[power]


def _binfile(magic: bytes, version: int, sections) -> bytes:
    out = [magic, struct.pack("<II", version, len(sections))]
    for typ, data in sections:
        out.append(struct.pack("<IQ", typ, len(data)))
        out.append(data)
    return b"".join(out)


def wtns_bytes(witness) -> bytes:
    hdr = struct.pack("<I", N8) + R.to_bytes(N8, "little") + struct.pack("<I", len(witness))
    data = b"".join(int(v).to_bytes(N8, "little") for v in witness)
    return _binfile(b"wtns", 2, [(1, hdr), (2, data)])


def read_wtns(buf: bytes):
    assert buf[:4] == b"wtns"
    nsec = struct.unpack_from("<I", buf, 8)[0]
    off, secs = 12, {}
    for _ in range(nsec):
        typ, size = struct.unpack_from("<IQ", buf, off)
        secs[typ] = buf[off + 12: off + 12 + size]
        off += 12 + size
    n = struct.unpack_from("<I", secs[1], 4 + N8)[0]
    d = secs[2]
    return [int.from_bytes(d[i * N8:(i + 1) * N8], "little") for i in range(n)]


def _batch_inv(vals):
    n = len(vals)
    pref = [1] * (n + 1)
    for i, v in enumerate(vals):
        pref[i + 1] = pref[i] * v % R
    inv = pow(pref[n], R - 2, R)
    out = [0] * n
    for i in range(n - 1, -1, -1):
        out[i] = inv * pref[i] % R
        inv = inv * vals[i] % R
    return out


def lagrange_at(tau: int, n: int, omega: int, odd_only: bool = False):
    """[L_j(tau)] on the size-n domain of omega (tau must not be a domain point).
    odd_only: return only j = 1, 3, 5, ... (used for the 2n domain H basis)."""
    num = (pow(tau, n, R) - 1) * pow(n, R - 2, R) % R
    step = 2 if odd_only else 1
    wj = omega if odd_only else 1
    w_step = omega * omega % R if odd_only else omega
    pts = []
    dens = []
    for _ in range(0, n, step):
        pts.append(wj)
        dens.append((tau - wj) % R)
        wj = wj * w_step % R
    inv = _batch_inv(dens)
    return [num * p % R * i % R for p, i in zip(pts, inv)]


class Toxic:
    """Ceremony secrets.  Random by default; pass ints for reproducible test keys."""

    def __init__(self, tau=None, alpha=None, beta=None, gamma=None, delta=None):
        rnd = lambda: secrets.randbelow(R - 2) + 2  # noqa: E731
        self.tau = tau if tau is not None else rnd()
        self.alpha = alpha if alpha is not None else rnd()
        self.beta = beta if beta is not None else rnd()
        self.gamma = gamma if gamma is not None else rnd()
        self.delta = delta if delta is not None else rnd()


def _coef_table(builder):
    """snarkjs zkey section 4 rows: A and B entries per constraint, then A public rows."""
    rows = []
    for j, (A, B, _C) in enumerate(builder.cons):
        for w, c in A.items():
            rows.append((0, j, w, c))
        for w, c in B.items():
            rows.append((1, j, w, c))
    n_cons = len(builder.cons)
    for k in range(builder.n_public + 1):
        rows.append((0, n_cons + k, k, 1))
    return rows


def qap_at_tau(builder, tau: int, n: int):
    """A_i(tau), B_i(tau), C_i(tau) for every wire (incl. public-input rows)."""
    power = n.bit_length() - 1
    L = lagrange_at(tau, n, root_of_unity(power))
    nv = builder.n_wires
    Ai, Bi, Ci = [0] * nv, [0] * nv, [0] * nv
    for j, (A, B, Cc) in enumerate(builder.cons):
        lj = L[j]
        for w, c in A.items():
            Ai[w] += c * lj
        for w, c in B.items():
            Bi[w] += c * lj
        for w, c in Cc.items():
            Ci[w] += c * lj
    n_cons = len(builder.cons)
    for k in range(builder.n_public + 1):
        Ai[k] += L[n_cons + k]
    return [x % R for x in Ai], [x % R for x in Bi], [x % R for x in Ci]


def domain_size_for(builder) -> int:
    n = 1
    while n < builder.n_constraints + builder.n_public + 1:
        n *= 2
    return n


def _scalars(vals) -> bytes:
    return b"".join(int(v).to_bytes(32, "little") for v in vals)


def groth16_setup(builder, ctx, toxic: Toxic | None = None) -> bytes:
    """Dev ceremony -> snarkjs-layout .zkey bytes (fixed-base work on the GPU via ctx)."""
    tx = toxic or Toxic()
    n = domain_size_for(builder)
    power = n.bit_length() - 1
    if power + 1 > _FR_S:
        raise ValueError("circuit too large for the BN254 2-adic domain")
    nv, npub = builder.n_wires, builder.n_public
    Ai, Bi, Ci = qap_at_tau(builder, tx.tau, n)
    gi = pow(tx.gamma, R - 2, R)
    di = pow(tx.delta, R - 2, R)
    K = [(tx.beta * a + tx.alpha * b + c) % R for a, b, c in zip(Ai, Bi, Ci)]
    Hs = lagrange_at(tx.tau, 2 * n, root_of_unity(power + 1), odd_only=True)

    g1 = ctx.g1_gen_mul
    g2 = ctx.g2_gen_mul
    hdr_pts_g1 = g1(_scalars([tx.alpha, tx.beta, tx.delta]))
    hdr_pts_g2 = g2(_scalars([tx.beta, tx.gamma, tx.delta]))
    alpha1, beta1, delta1 = hdr_pts_g1[0:64], hdr_pts_g1[64:128], hdr_pts_g1[128:192]
    beta2, gamma2, delta2 = hdr_pts_g2[0:128], hdr_pts_g2[128:256], hdr_pts_g2[256:384]
    ic = g1(_scalars([K[i] * gi % R for i in range(npub + 1)]))
    sec_c = g1(_scalars([K[i] * di % R for i in range(npub + 1, nv)]))
    sec_a = g1(_scalars(Ai))
    sec_b1 = g1(_scalars(Bi))
    sec_b2 = g2(_scalars(Bi))
    sec_h = g1(_scalars([h * di % R for h in Hs]))

    hdr = struct.pack("<I", 32) + Q.to_bytes(32, "little") + struct.pack("<I", 32) + R.to_bytes(32, "little")
    hdr += struct.pack("<III", nv, npub, n)
    hdr += alpha1 + beta1 + beta2 + gamma2 + delta1 + delta2
    sections = [(1, struct.pack("<I", 1)), (2, hdr), (3, ic), (4, _coef_bytes(builder)), (5, sec_a), (6, sec_b1),
                (7, sec_b2), (8, sec_c), (9, sec_h)]
    return _binfile(b"zkey", 1, sections + [(10, _cs_hash(sections) + struct.pack("<I", 0))])


def _coef_bytes(builder) -> bytes:
    rows = _coef_table(builder)
    cache = {}
    parts = [struct.pack("<I", len(rows))]
    for m, c, s, v in rows:
        vb = cache.get(v)
        if vb is None:
            vb = (v * R2_MONT % R).to_bytes(32, "little")
            cache[v] = vb
        parts.append(struct.pack("<III", m, c, s) + vb)
    return b"".join(parts)


def _cs_hash(sections) -> bytes:
    """zkey section 10's circuit hash: Blake2b-512 over the delta-independent part of the key (the
    header up to gamma2, IC, A, B1, B2), so a contribution carries it unchanged.  snarkjs hashes the
    uncompressed points of the initial key in its own order [ext]; this hash is the framework's (no
    tool here reads it), computed the same way by every setup path."""
    h = hashlib.blake2b(digest_size=64)
    for typ, data in sections:
        if typ == 2:
            h.update(data[:468])
        elif typ in (3, 5, 6, 7):
            h.update(data)
    return h.digest()


def _sorted_terms(rows_of, n_rows):
    """[(row, base, coef)] -> (rowptr u64[n_rows + 1], idx u32[nnz], coefs 32 B std each), rows ascending."""
    import numpy as np
    rows = np.fromiter((t[0] for t in rows_of), dtype=np.int64, count=len(rows_of))
    order = np.argsort(rows, kind="stable")
    rowptr = np.zeros(n_rows + 1, dtype=np.uint64)
    np.cumsum(np.bincount(rows, minlength=n_rows), out=rowptr[1:])
    idx = np.fromiter((rows_of[i][1] for i in order), dtype=np.uint32, count=len(rows_of))
    cache = {}

    def cb(v):
        b = cache.get(v)
        if b is None:
            b = cache[v] = int(v).to_bytes(32, "little")
        return b
    coefs = b"".join(cb(rows_of[i][2]) for i in order)
    return rowptr, idx, coefs


def setup_from_ptau(cs, ptau_buf, ctx) -> bytes:
    """snarkjs `groth16 setup <c>.r1cs <pot>.ptau <c>_0000.zkey` (zkey_new [ext]; the harness's
    tests/full_system_simulation.mjs:713-716 and tests/test_secureagg.cjs:48-57).  cs: a
    zkfl.r1cs.Builder or a circom .r1cs read by zkfl.r1cs_file.  Every query point is a sparse
    combination of the ptau's Lagrange points, computed on the GPU (zkfl_setup_*_lincomb):
        A_i  = sum_j a_ij L_j(tau) G1 (+ L_{m+k} for public k)     <- section 12
        B1_i = sum_j b_ij L_j(tau) G1,  B2_i = ... G2               <- sections 12, 13
        IC_i / C_i = sum_j (a_ij beta + b_ij alpha + c_ij) L_j(tau) G1   <- sections 15, 14, 12
        H_j  = L^{2n}_{2j+1}(tau) G1                                <- section 12, block 2n
    with gamma = delta = 1 (the header's gamma2 / delta1 / delta2 are the generators) until a
    `zkey contribute` rescales delta.  alpha1 / beta1 / beta2 are the ptau's alphaTauG1[0],
    betaTauG1[0], betaG2."""
    from . import ptau as pt_mod
    pt = pt_mod.Ptau(ptau_buf)
    if not pt.prepared:
        raise ValueError("Powers of tau is not prepared.")
    n = domain_size_for(cs)
    power = n.bit_length() - 1
    if power > pt.power:
        raise ValueError(f"circuit too big for this power of tau ceremony. {cs.n_constraints}*2 > 2**{pt.power}")
    nv, npub, ncons = cs.n_wires, cs.n_public, cs.n_constraints
    L = pt.lagrange(12, power)
    L2 = pt.lagrange(13, power)
    k_bases = L + pt.lagrange(14, power) + pt.lagrange(15, power)   # tau | alpha tau | beta tau
    h2 = pt.lagrange(12, power + 1)
    sec_h = b"".join(h2[64 * (2 * j + 1):64 * (2 * j + 2)] for j in range(n))
    a_terms, b_terms, k_terms = [], [], []
    for j, (A, B, C) in enumerate(cs.cons):
        for w, c in A.items():
            a_terms.append((w, j, c))
            k_terms.append((w, 2 * n + j, c))          # beta * a_ij
        for w, c in B.items():
            b_terms.append((w, j, c))
            k_terms.append((w, n + j, c))              # alpha * b_ij
        for w, c in C.items():
            k_terms.append((w, j, c))
    for s in range(npub + 1):                          # public-input rows
        a_terms.append((s, ncons + s, 1))
        k_terms.append((s, 2 * n + ncons + s, 1))
    ta, tb, tk = _sorted_terms(a_terms, nv), _sorted_terms(b_terms, nv), _sorted_terms(k_terms, nv)
    sec_a = ctx.g1_lincomb(L, *ta)
    sec_b1 = ctx.g1_lincomb(L, *tb)
    sec_b2 = ctx.g2_lincomb(L2, *tb)
    k = ctx.g1_lincomb(k_bases, *tk)
    ic, sec_c = k[:64 * (npub + 1)], k[64 * (npub + 1):]
    hdr = struct.pack("<I", 32) + Q.to_bytes(32, "little") + struct.pack("<I", 32) + R.to_bytes(32, "little")
    hdr += struct.pack("<III", nv, npub, n)
    hdr += (pt.points(4, 0, 1) + pt.points(5, 0, 1) + pt.section(6) + pt_mod.G2_ONE + pt_mod.G1_ONE
            + pt_mod.G2_ONE)
    sections = [(1, struct.pack("<I", 1)), (2, hdr), (3, ic), (4, _coef_bytes(cs)), (5, sec_a), (6, sec_b1),
                (7, sec_b2), (8, sec_c), (9, sec_h)]
    return _binfile(b"zkey", 1, sections + [(10, _cs_hash(sections) + struct.pack("<I", 0))])


def zkey_contribute(buf, ctx, d: int, name: str = "") -> bytes:
    """snarkjs `zkey contribute <old> <new> --name=<name> -e=<entropy>` with the secret d given
    (tests/full_system_simulation.mjs:723-726): delta1, delta2 *= d; C and H (sections 8, 9) *= 1/d
    on the GPU; a contribution record (deltaAfter, the (g1_s, g1_sx, g2_spx) key, transcript, type,
    params) is appended to section 10 — a dev record, as in zkfl/ptau.py."""
    from . import ptau as pt_mod
    d %= R
    if d == 0:
        raise ValueError("zkey contribute: zero secret")
    secs = pt_mod.read_sections(buf, b"zkey")
    for t in range(1, 11):
        if t not in secs:
            raise ValueError(f"zkey: missing section {t}")
    order = sorted(secs, key=lambda t: secs[t][0])
    data = {t: bytes(buf[secs[t][0]:secs[t][0] + secs[t][1]]) for t in order}
    hdr = bytearray(data[2])
    if len(hdr) < 660:
        raise ValueError("zkey: header")
    dinv = pow(d, R - 2, R)
    hdr[468:532] = ctx.g1_scale(bytes(hdr[468:532]), _scalars([d]))
    hdr[532:660] = ctx.g2_scale(bytes(hdr[532:660]), _scalars([d]))
    data[2] = bytes(hdr)
    for t in (8, 9):
        npts = len(data[t]) // 64
        data[t] = ctx.g1_scale(data[t], _scalars([dinv]) * npts) if npts else data[t]
    mpc = data[10]
    if len(mpc) < 68:
        raise ValueError("zkey: section 10")
    cs_hash, count = mpc[:64], struct.unpack_from("<I", mpc, 64)[0]
    s = pt_mod.derive_secret(str(d), "s")
    sp = pt_mod.derive_secret(str(d), "sp")
    g1 = ctx.g1_gen_mul(_scalars([s, s * d % R]))
    g2spx = ctx.g2_gen_mul(_scalars([sp * d % R]))
    transcript = hashlib.blake2b(mpc + hdr[468:532], digest_size=64).digest()
    record = bytes(hdr[468:532]) + g1 + g2spx + transcript + struct.pack("<I", 0) + pt_mod._params_bytes(name)
    data[10] = cs_hash + struct.pack("<I", count + 1) + mpc[68:] + record
    return _binfile(b"zkey", 1, [(t, data[t]) for t in order])


def zkey_header(buf: bytes) -> dict:
    """Header fields of a groth16 zkey (for vkey export / info)."""
    assert buf[:4] == b"zkey"
    nsec = struct.unpack_from("<I", buf, 8)[0]
    off, secs = 12, {}
    for _ in range(nsec):
        typ, size = struct.unpack_from("<IQ", buf, off)
        secs.setdefault(typ, (off + 12, size))
        off += 12 + size
    o, _ = secs[2]
    nv, npub, dom = struct.unpack_from("<III", buf, o + 72)
    p = o + 84
    pts = dict(alpha1=buf[p:p + 64], beta1=buf[p + 64:p + 128], beta2=buf[p + 128:p + 256],
               gamma2=buf[p + 256:p + 384], delta1=buf[p + 384:p + 448], delta2=buf[p + 448:p + 576])
    io, isz = secs[3]
    ic = [buf[io + 64 * i: io + 64 * i + 64] for i in range(isz // 64)]
    return dict(nVars=nv, nPublic=npub, domainSize=dom, IC=ic, **pts)
