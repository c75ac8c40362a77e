"""Powers of Tau (.ptau) files and the snarkjs ceremony commands, with the group work on the GPU.

The reference runs the whole ceremony through snarkjs [ext] before it can prove:
  npx snarkjs powersoftau new bn128 12 pot12_0000.ptau -v              tests/test_secureagg.cjs:25-31
  npx snarkjs powersoftau contribute pot12_0000.ptau pot12_0001.ptau -v -e="..."       :32-38
  npx snarkjs powersoftau prepare phase2 pot12_0001.ptau pot12_final.ptau              :41-47
  npx snarkjs groth16 setup <c>.r1cs pot12_final.ptau <c>_0000.zkey                    :48-57
and `Client._runZKProof` refuses to go on without `pot17_final.ptau` / `pot14_final.ptau`
(tests/full_system_simulation.mjs:677-695), then runs `groth16 setup` + `zkey contribute`
(:713-730).  This module restates those commands (snarkjs 0.7 powersoftau_new / _contribute /
_preparephase2, zkey_new, zkey_contribute): the file layout and the algebra are snarkjs's, the
group arithmetic runs through libzkfl (`zkfl_setup_*`, csrc/setup.hip):

.ptau (iden3 binfile "ptau", version 1; points affine little-endian Montgomery, infinity = 0):
  1  header        n8 u32 | q (n8 B) | power u32 | ceremonyPower u32
  2  tauG1         tau^i G1,            i < 2^(power+1) - 1
  3  tauG2         tau^i G2,            i < 2^power
  4  alphaTauG1    alpha tau^i G1,      i < 2^power
  5  betaTauG1     beta tau^i G1,       i < 2^power
  6  betaG2        beta G2
  7  contributions u32 count, then one record per contribution
  12..15 (after `prepare phase2`): for p = 0..power the 2^p Lagrange evaluations L_j(tau) of
     sections 2..5 (section 12 also p = power + 1, computed with its missing last power set to
     the point at infinity, exactly as snarkjs does), block p at offset (2^p - 1) points.

Contribution records follow snarkjs's layout (new tauG1[1], tauG2[1], alphaG1, betaG1, betaG2, the
three (g1_s, g1_sx, g2_spx) keys, partial hash, next challenge, type, params) but are this
framework's dev records: the keys are fresh random multiples, the 216-byte Blake2b partial state
is zero and the challenge is Blake2b-512 of the new points, so snarkjs's `powersoftau verify` would
not accept the transcript.  The points themselves are exactly what snarkjs computes for the same
secrets.  Secrets come from Blake2b(entropy || 64 OS-random bytes); ZKFL_DETERMINISTIC_SETUP=1
drops the OS randomness (tests only: the secrets are then a function of the entropy string).
"""

from __future__ import annotations

import hashlib
import os
import struct

from .field import Q, R

N8 = 32
G1_SIZE = 64
G2_SIZE = 128
MAX_POWER = 28
# prepare phase2 needs a 2^(power + 1) Lagrange block of tauG1 and the GPU group iFFT stops at 2^28
# (zkfl_setup_g1_lagrange): a power-28 file is a valid phase-1 transcript but cannot be prepared
MAX_PHASE2_POWER = 27

# generators, standard form (ffjavascript bn128 G1.g / G2.g)
G1_GEN = (1, 2)
G2_GEN = ((0x1800DEEF121F1E76426A00665E5C4479674322D4F75EDADD46DEBD5CD992F6ED,
           0x198E9393920D483A7260BFB731FB5D25F1AA493335A9E71297E485B7AEF312C2),
          (0x12C85EA5DB8C6DEB4AAB71808DCB408FE3D1E7690C43D37B4CE6CC0166FA7DAA,
           0x090689D0585FF075EC9E99AD690C3395BC4B313370B38EF355ACDADCD122975B))


def _mont(v: int) -> bytes:
    return (v * (1 << 256) % Q).to_bytes(32, "little")


G1_ONE = _mont(G1_GEN[0]) + _mont(G1_GEN[1])
G2_ONE = _mont(G2_GEN[0][0]) + _mont(G2_GEN[0][1]) + _mont(G2_GEN[1][0]) + _mont(G2_GEN[1][1])
G1_ZERO = bytes(G1_SIZE)


def binfile(magic: bytes, version: int, sections) -> bytes:
    out = [magic, struct.pack("<II", version, len(sections))]
    for typ, data in sections:
        out.append(struct.pack("<IQ", typ, len(data)))
        out.append(data)
    return b"".join(out)


def read_sections(buf, magic: bytes) -> dict:
    """iden3 binfile -> {type: (offset, size)} (first occurrence), bounds-checked."""
    if len(buf) < 12 or bytes(buf[:4]) != magic:
        raise ValueError(f"not a {magic.decode()} file")
    nsec = struct.unpack_from("<I", buf, 8)[0]
    off, secs = 12, {}
    for _ in range(nsec):
        if off + 12 > len(buf):
            raise ValueError(f"{magic.decode()}: truncated section header")
        typ, size = struct.unpack_from("<IQ", buf, off)
        off += 12
        if size > len(buf) - off:
            raise ValueError(f"{magic.decode()}: truncated section {typ}")
        secs.setdefault(typ, (off, size))
        off += size
    return secs


def derive_secret(entropy: str, label: str) -> int:
    """A ceremony secret in [1, r): Blake2b-512(entropy || label || 64 OS-random bytes) mod r
    (snarkjs: getRandomRng(entropy) [ext]).  ZKFL_DETERMINISTIC_SETUP=1 omits the OS bytes."""
    h = hashlib.blake2b(digest_size=64)
    h.update((entropy or "").encode())
    h.update(b"\x00" + label.encode())
    if os.environ.get("ZKFL_DETERMINISTIC_SETUP") != "1":
        h.update(os.urandom(64))
    return int.from_bytes(h.digest(), "little") % (R - 1) + 1


def _scalars(vals) -> bytes:
    return b"".join(int(v).to_bytes(32, "little") for v in vals)


def _powers(base: int, n: int, first: int = 1) -> bytes:
    out, v = [], first % R
    for _ in range(n):
        out.append(v.to_bytes(32, "little"))
        v = v * base % R
    return b"".join(out)


def _params_bytes(name: str) -> bytes:
    if not name:
        return struct.pack("<I", 0)
    nb = name[:64].encode()
    p = bytes([1, len(nb)]) + nb
    return struct.pack("<I", len(p)) + p


class Ptau:
    """A parsed .ptau image (the caller keeps the buffer)."""

    def __init__(self, buf):
        self.buf = buf
        self.secs = read_sections(buf, b"ptau")
        if struct.unpack_from("<I", buf, 4)[0] != 1:
            raise ValueError("ptau: unsupported version")
        for t in range(1, 8):
            if t not in self.secs:
                raise ValueError(f"ptau: missing section {t}")
        o, sz = self.secs[1]
        if sz < 4 + N8 + 8:
            raise ValueError("ptau: header")
        n8 = struct.unpack_from("<I", buf, o)[0]
        if n8 != N8 or int.from_bytes(buf[o + 4:o + 4 + N8], "little") != Q:
            raise ValueError("ptau: curve is not bn128 (BN254)")
        self.power, self.ceremony_power = struct.unpack_from("<II", buf, o + 4 + N8)
        if not 1 <= self.power <= MAX_POWER:
            raise ValueError(f"ptau: power {self.power} out of range")
        n = 1 << self.power
        self.counts = {2: 2 * n - 1, 3: n, 4: n, 5: n, 6: 1}
        for t, cnt in self.counts.items():
            size = G2_SIZE if t in (3, 6) else G1_SIZE
            if self.secs[t][1] != cnt * size:
                raise ValueError(f"ptau: section {t} holds {self.secs[t][1]} bytes, expected {cnt * size}")
        self.prepared = all(t in self.secs for t in (12, 13, 14, 15))
        if self.prepared:
            for t in (12, 13, 14, 15):
                size = G2_SIZE if t == 13 else G1_SIZE
                nblk = (2 * (2 * n) - 1) if t == 12 else (2 * n - 1)
                if self.secs[t][1] != nblk * size:
                    raise ValueError(f"ptau: section {t} is not a prepared Lagrange section")

    def section(self, t: int) -> bytes:
        o, sz = self.secs[t]
        return bytes(self.buf[o:o + sz])

    def points(self, t: int, start: int, count: int) -> bytes:
        size = G2_SIZE if t in (3, 6, 13) else G1_SIZE
        o, sz = self.secs[t]
        if (start + count) * size > sz:
            raise ValueError(f"ptau: section {t} too short")
        return bytes(self.buf[o + start * size:o + (start + count) * size])

    def lagrange(self, t: int, p: int) -> bytes:
        """The 2^p Lagrange points of prepared section t (12..15)."""
        if not self.prepared:
            raise ValueError("Powers of tau is not prepared.")
        return self.points(t, (1 << p) - 1, 1 << p)

    def contributions(self):
        o, sz = self.secs[7]
        if sz < 4:
            raise ValueError("ptau: contributions section")
        return struct.unpack_from("<I", self.buf, o)[0], bytes(self.buf[o + 4:o + sz])


def header_bytes(power: int, ceremony_power: int | None = None) -> bytes:
    return struct.pack("<I", N8) + Q.to_bytes(N8, "little") + struct.pack("<II", power, ceremony_power or power)


def new(power: int) -> bytes:
    """snarkjs `powersoftau new bn128 <power>`: every point the generator (tau = alpha = beta = 1)."""
    if not 1 <= power <= MAX_POWER:
        raise ValueError(f"power must be in 1..{MAX_POWER}")
    n = 1 << power
    return binfile(b"ptau", 1, [(1, header_bytes(power)), (2, G1_ONE * (2 * n - 1)), (3, G2_ONE * n),
                                (4, G1_ONE * n), (5, G1_ONE * n), (6, G2_ONE), (7, struct.pack("<I", 0))])


def _key(ctx, x: int):
    """One (g1_s, g1_sx, g2_spx) proof-of-knowledge triple for secret x (dev record)."""
    s = derive_secret(str(x), "s")
    sp = derive_secret(str(x), "sp")
    g1 = ctx.g1_gen_mul(_scalars([s, s * x % R]))
    return g1[:G1_SIZE], g1[G1_SIZE:], ctx.g2_gen_mul(_scalars([sp * x % R]))


def contribute(buf, ctx, tau: int, alpha: int, beta: int, name: str = "") -> bytes:
    """snarkjs `powersoftau contribute <old> <new> -e=<entropy> --name=<name>` with the secrets given:
    tauG1[i] *= tau^i, tauG2[i] *= tau^i, alphaTauG1[i] *= alpha tau^i, betaTauG1[i] *= beta tau^i,
    betaG2 *= beta (a prepared input loses its Lagrange sections, as in snarkjs)."""
    pt = Ptau(buf)
    n = 1 << pt.power
    tau_g1 = ctx.g1_scale(pt.section(2), _powers(tau, 2 * n - 1))
    tau_g2 = ctx.g2_scale(pt.section(3), _powers(tau, n))
    alpha_g1 = ctx.g1_scale(pt.section(4), _powers(tau, n, alpha))
    beta_g1 = ctx.g1_scale(pt.section(5), _powers(tau, n, beta))
    beta_g2 = ctx.g2_scale(pt.section(6), _scalars([beta]))
    h = hashlib.blake2b(digest_size=64)
    for part in (tau_g1, tau_g2, alpha_g1, beta_g1, beta_g2):
        h.update(part)
    keys = [_key(ctx, x) for x in (tau, alpha, beta)]
    record = (tau_g1[G1_SIZE:2 * G1_SIZE] + tau_g2[G2_SIZE:2 * G2_SIZE] + alpha_g1[:G1_SIZE] + beta_g1[:G1_SIZE]
              + beta_g2 + b"".join(k[0] + k[1] for k in keys) + b"".join(k[2] for k in keys)
              + bytes(216) + h.digest() + struct.pack("<I", 0) + _params_bytes(name))
    count, old = pt.contributions()
    return binfile(b"ptau", 1, [(1, header_bytes(pt.power, pt.ceremony_power)), (2, tau_g1), (3, tau_g2),
                                (4, alpha_g1), (5, beta_g1), (6, beta_g2),
                                (7, struct.pack("<I", count + 1) + old + record)])


def prepare_phase2(buf, ctx) -> bytes:
    """snarkjs `powersoftau prepare phase2 <old> <new>`: sections 12..15 = the Lagrange evaluations
    of every 2^p prefix of sections 2..5 (p = 0..power, and p = power + 1 for tauG1 with its last,
    absent power replaced by the point at infinity)."""
    pt = Ptau(buf)
    if pt.power > MAX_PHASE2_POWER:  # before any GPU work
        raise ValueError(f"prepare phase2: power {pt.power} > {MAX_PHASE2_POWER}: its 2^{pt.power + 1} tauG1 "
                         f"Lagrange block exceeds the GPU group FFT's 2^28")
    secs = [(t, pt.section(t)) for t in range(1, 8)]
    for src, dst, g2 in ((2, 12, False), (3, 13, True), (4, 14, False), (5, 15, False)):
        lag = ctx.g2_lagrange if g2 else ctx.g1_lagrange
        blocks = []
        top = pt.power + 1 if src == 2 else pt.power
        for p in range(top + 1):
            if src == 2 and p == pt.power + 1:
                pts = pt.points(2, 0, (1 << p) - 1) + G1_ZERO
            else:
                pts = pt.points(src, 0, 1 << p)
            blocks.append(lag(pts, p))
        secs.append((dst, b"".join(blocks)))
    return binfile(b"ptau", 1, secs)
