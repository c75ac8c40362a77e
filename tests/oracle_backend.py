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

    # ceremony primitives (the zkfl_setup_* contract of include/zkfl.h)
    @staticmethod
    def _pts(b: bytes, g2: bool):
        size = 128 if g2 else 64
        dec = bn.g2_from_bytes_mont if g2 else bn.g1_from_bytes_mont
        return [dec(b[i:i + size]) for i in range(0, len(b), size)]

    @staticmethod
    def _enc(pts, g2: bool) -> bytes:
        enc = bn.g2_to_bytes_mont if g2 else bn.g1_to_bytes_mont
        return b"".join(enc(p) for p in pts)

    def _scale(self, points, scalars, g2):
        ks = [int.from_bytes(scalars[i:i + 32], "little") for i in range(0, len(scalars), 32)]
        return self._enc([bn.mul(p, k) for p, k in zip(self._pts(points, g2), ks)], g2)

    def g1_scale(self, points, scalars):
        return self._scale(points, scalars, False)

    def g2_scale(self, points, scalars):
        return self._scale(points, scalars, True)

    def g1_lagrange(self, points, logn):
        from oracle import ptau as op
        return self._enc(op.group_ifft(self._pts(points, False), logn), False)

    def g2_lagrange(self, points, logn):
        from oracle import ptau as op
        return self._enc(op.group_ifft(self._pts(points, True), logn), True)

    def _lincomb(self, bases, rowptr, idx, coefs, g2):
        b = self._pts(bases, g2)
        out = []
        for r in range(len(rowptr) - 1):
            acc = None
            for t in range(int(rowptr[r]), int(rowptr[r + 1])):
                acc = bn.add(acc, bn.mul(b[int(idx[t])], int.from_bytes(coefs[32 * t:32 * t + 32], "little")))
            out.append(acc)
        return self._enc(out, g2)

    def g1_lincomb(self, bases, rowptr, idx, coefs):
        return self._lincomb(bases, rowptr, idx, coefs, False)

    def g2_lincomb(self, bases, rowptr, idx, coefs):
        return self._lincomb(bases, rowptr, idx, coefs, True)


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
