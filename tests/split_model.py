"""Test-only CPU model of a split proof (zkfl_zkey_load_shard / zkfl_groth16_prove_part_batch /
zkfl_groth16_assemble, include/zkfl.h), built from the oracle's own prover pieces
(oracle/groth16.py::prove, which restates snarkjs groth16_prove).

Shard k of G holds element i of every query when i % G == k; shard 0 also carries the
alpha/beta/delta augmentation terms.  A part is A' | B1' | B2' | C'+H | H(infinity) as XYZZ points
with std-form coordinates (the device layout, include/zkfl.h); the model writes each point with
ZZ = ZZZ = 1 (infinity: all zero), the device with whatever ZZ its accumulation ended on, so parts
compare through `affine`.  Summing the parts of all shards and assembling must give exactly the
unsplit proof for the same (r, s)."""
from oracle import bn254 as bn
from oracle import groth16 as og

R = bn.R


def part(z, w, h, r, s, shard, n_shards) -> bytes:
    nPub = z["nPublic"]

    def msm(points, scalars):
        idx = [i for i in range(len(points)) if i % n_shards == shard]
        return bn.msm([points[i] for i in idx], [scalars[i] for i in idx])

    A = msm(z["A"], w)
    B1 = msm(z["B1"], w)
    B2 = msm(z["B2"], w)
    C = bn.add(msm(z["C"], w[nPub + 1:]), msm(z["H"], h))
    if shard == 0:
        A = bn.add(bn.add(A, z["alpha1"]), bn.mul(z["delta1"], r))
        B1 = bn.add(bn.add(B1, z["beta1"]), bn.mul(z["delta1"], s))
        B2 = bn.add(bn.add(B2, z["beta2"]), bn.mul(z["delta2"], s))
        C = bn.add(C, bn.mul(z["delta1"], (-(r * s)) % R))
    return _g1(A) + _g1(B1) + _g2(B2) + _g1(C) + bytes(128)


def _le(v):
    return int(v).to_bytes(32, "little")


def _g1(P) -> bytes:  # affine -> XYZZ (ZZ = ZZZ = 1), std coordinates
    return bytes(128) if P is None else _le(P[0]) + _le(P[1]) + _le(1) + _le(1)


def _g2(P) -> bytes:
    if P is None:
        return bytes(256)
    x, y = P
    return _le(x.c0) + _le(x.c1) + _le(y.c0) + _le(y.c1) + _le(1) + _le(0) + _le(1) + _le(0)


def _ints(b):
    return [int.from_bytes(b[32 * i:32 * i + 32], "little") for i in range(len(b) // 32)]


def affine(part: bytes) -> dict:
    """A part's five points as oracle affine points (None = infinity): x = X / ZZ, y = Y / ZZZ."""
    Q = bn.Q
    out = {}
    for name, (a, b) in (("A", (0, 128)), ("B1", (128, 256)), ("C", (512, 640)), ("H", (640, 768))):
        X, Y, ZZ, ZZZ = _ints(part[a:b])
        out[name] = None if ZZ == 0 else (X * pow(ZZ, -1, Q) % Q, Y * pow(ZZZ, -1, Q) % Q)
    v = _ints(part[256:512])
    X, Y, ZZ, ZZZ = bn.Fq2(v[0], v[1]), bn.Fq2(v[2], v[3]), bn.Fq2(v[4], v[5]), bn.Fq2(v[6], v[7])
    out["B2"] = None if (v[4] == 0 and v[5] == 0) else (X * ZZ.inv(), Y * ZZZ.inv())
    return out


def assemble(parts: bytes, n_parts: int, rs: bytes) -> list:
    n = len(rs) // 64
    out = []
    for i in range(n):
        r = int.from_bytes(rs[64 * i:64 * i + 32], "little")
        s = int.from_bytes(rs[64 * i + 32:64 * i + 64], "little")
        A = B1 = B2 = C = None
        for j in range(n_parts):
            p = affine(parts[768 * (i * n_parts + j):768 * (i * n_parts + j + 1)])
            A = bn.add(A, p["A"])
            B1 = bn.add(B1, p["B1"])
            B2 = bn.add(B2, p["B2"])
            C = bn.add(C, bn.add(p["C"], p["H"]))
        pi_c = bn.add(bn.add(C, bn.mul(A, s)), bn.mul(B1, r))
        out.append(og.proof_bytes(dict(pi_a=A, pi_b=B2, pi_c=pi_c)))
    return out
