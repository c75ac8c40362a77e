"""Test-only point backend: the oracle's scalar multiplication behind the ctx interface the
product dev ceremony expects (g1_gen_mul / g2_gen_mul -> Montgomery affine bytes)."""
from oracle import bn254 as bn


class OraclePoints:
    def g1_gen_mul(self, scalars: bytes) -> bytes:
        ks = [int.from_bytes(scalars[i:i + 32], "little") for i in range(0, len(scalars), 32)]
        return b"".join(bn.g1_to_bytes_mont(bn.mul(bn.G1_GEN, k)) for k in ks)

    def g2_gen_mul(self, scalars: bytes) -> bytes:
        ks = [int.from_bytes(scalars[i:i + 32], "little") for i in range(0, len(scalars), 32)]
        return b"".join(bn.g2_to_bytes_mont(bn.mul(bn.G2_GEN, k)) for k in ks)
