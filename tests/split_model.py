"""Test-only CPU model of a split proof (zkfl_zkey_load_shard / zkfl_groth16_prove_part_batch /
zkfl_groth16_assemble, include/zkfl.h), built from the oracle's own prover pieces
(oracle/groth16.py::prove, which restates snarkjs groth16_prove).

Shard k of G holds element i of every query when i % G == k; shard 0 also carries the
alpha/beta/delta augmentation terms.  A part is A' | B1' | B2' | C'+H | H(infinity), std affine,
the device layout.  Summing the parts of all shards and assembling must give exactly the unsplit
proof for the same (r, s)."""
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
    return (bn.g1_to_bytes_std(A) + bn.g1_to_bytes_std(B1) + bn.g2_to_bytes_std(B2) + bn.g1_to_bytes_std(C)
            + bytes(64))


def assemble(parts: bytes, n_parts: int, rs: bytes) -> list:
    n = len(rs) // 64
    out = []
    for i in range(n):
        r = int.from_bytes(rs[64 * i:64 * i + 32], "little")
        s = int.from_bytes(rs[64 * i + 32:64 * i + 64], "little")
        A = B1 = B2 = C = None
        for j in range(n_parts):
            p = parts[384 * (i * n_parts + j):384 * (i * n_parts + j + 1)]
            A = bn.add(A, bn.g1_from_bytes_std(p[0:64]))
            B1 = bn.add(B1, bn.g1_from_bytes_std(p[64:128]))
            B2 = bn.add(B2, bn.g2_from_bytes_std(p[128:256]))
            C = bn.add(C, bn.add(bn.g1_from_bytes_std(p[256:320]), bn.g1_from_bytes_std(p[320:384])))
        pi_c = bn.add(bn.add(C, bn.mul(A, s)), bn.mul(B1, r))
        out.append(og.proof_bytes(dict(pi_a=A, pi_b=B2, pi_c=pi_c)))
    return out
