"""Test-only point backend: the oracle's scalar multiplication behind the ctx interface the
product dev ceremony expects (g1_gen_mul / g2_gen_mul -> Montgomery affine bytes)."""
from oracle import bn254 as bn


class OraclePoints:
    """Pure-Python scalar multiplication (slow; small circuits)."""

    def g1_gen_mul(self, scalars: bytes) -> bytes:
        ks = [int.from_bytes(scalars[i:i + 32], "little") for i in range(0, len(scalars), 32)]
        return b"".join(bn.g1_to_bytes_mont(bn.mul(bn.G1_GEN, k)) for k in ks)

    def g2_gen_mul(self, scalars: bytes) -> bytes:
        ks = [int.from_bytes(scalars[i:i + 32], "little") for i in range(0, len(scalars), 32)]
        return b"".join(bn.g2_to_bytes_mont(bn.mul(bn.G2_GEN, k)) for k in ks)


class COraclePoints:
    """The C oracle's fixed-base multiplication (fast; used for larger CPU-side test keys)."""

    def __init__(self):
        import os
        import subprocess
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        subprocess.run(["make", "-s"], cwd=os.path.join(root, "oracle"), check=True)
        from oracle import cbaseline
        self.cb = cbaseline

    def g1_gen_mul(self, scalars: bytes) -> bytes:
        return self.cb.g1_gen_mul(scalars)

    def g2_gen_mul(self, scalars: bytes) -> bytes:
        return self.cb.g2_gen_mul(scalars)
