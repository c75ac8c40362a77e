"""circom artifact ingest: iden3 ``.r1cs`` (binary constraint system) and ``.sym`` (signal map).

The reference compiles its circuits with ``circom <c>.circom --r1cs --wasm --sym``
(tests/full_system_simulation.mjs:700-708) and hands the ``.r1cs`` to ``snarkjs groth16 setup``
(:713-716) and ``snarkjs r1cs info`` (tests/test_verified_gradient.mjs:351-356).  An
:class:`R1csFile` read here stands wherever a :class:`zkfl.r1cs.Builder` is used for the key
side — ``zkey.groth16_setup``, ``groth16.r1cs_info`` — so a circom-compiled circuit gets a
proving key from this framework, and a witness for it (``.wtns`` from circom's own witness
calculator) proves through ``zkfl_groth16_prove``.  What an ``.r1cs`` does not carry is the
witness *program* (circom's hints: Num2Bits, IsZero's inverse, ...), so GPU witness generation
stays with circuits built by ``zkfl.circuits``.

Format (iden3 binfile "r1cs", version 1; snarkjs/r1csfile): sections of (type u32, size u64):
  1 header : n8 u32 | prime (n8 B LE) | nWires u32 | nPubOut u32 | nPubIn u32 | nPrvIn u32 |
             nLabels u64 | mConstraints u32
  2 constraints : per constraint, A, B, C each: nTerms u32, then nTerms x (wire u32, coef n8 B LE)
  3 wire2label : nWires x u64
  (other section types, e.g. circom 2.1's custom gates, are skipped)
Wire 0 is the constant 1, then outputs, public inputs, private inputs (the same order as
``zkfl.r1cs.Builder``, whose ``r1cs_bytes`` writes this format).  Every read is bounds-checked;
a malformed file raises ``ValueError``.
"""

from __future__ import annotations

import struct

from .field import R


class R1csFile:
    """A parsed .r1cs: the attributes ``zkey.groth16_setup`` and ``groth16.r1cs_info`` read."""

    def __init__(self, n_wires, n_pub_out, n_pub_in, n_prv_in, n_labels, cons, wire2label):
        self.n_wires = n_wires
        self.n_pub_out = n_pub_out
        self.n_pub_in = n_pub_in
        self.n_prv_in = n_prv_in
        self.n_labels = n_labels
        self.cons = cons                  # [(A, B, C)] of {wire: coef (std form, < r)}
        self.wire2label = wire2label

    @property
    def n_public(self) -> int:
        return self.n_pub_out + self.n_pub_in

    @property
    def n_constraints(self) -> int:
        return len(self.cons)

    def check(self, w) -> bool:
        """Every constraint <A,w> * <B,w> == <C,w> over Fr (a witness vector of n_wires values)."""
        def ev(lc):
            return sum(c * w[k] for k, c in lc.items()) % R
        return all(ev(A) * ev(B) % R == ev(C) for A, B, C in self.cons)


class _Reader:
    def __init__(self, buf: bytes, off: int, end: int):
        self.buf, self.off, self.end = buf, off, end

    def take(self, n: int) -> bytes:
        if n < 0 or self.off + n > self.end:
            raise ValueError("r1cs: truncated section")
        b = self.buf[self.off:self.off + n]
        self.off += n
        return b

    def u32(self) -> int:
        return struct.unpack("<I", self.take(4))[0]

    def u64(self) -> int:
        return struct.unpack("<Q", self.take(8))[0]


def _sections(buf: bytes):
    if len(buf) < 12 or buf[:4] != b"r1cs":
        raise ValueError("r1cs: bad magic")
    version, nsec = struct.unpack_from("<II", buf, 4)
    if version != 1:
        raise ValueError(f"r1cs: unsupported version {version}")
    off, secs = 12, {}
    for _ in range(nsec):
        if off + 12 > len(buf):
            raise ValueError("r1cs: truncated section header")
        typ, size = struct.unpack_from("<IQ", buf, off)
        off += 12
        if size > len(buf) - off:
            raise ValueError("r1cs: truncated section")
        secs.setdefault(typ, (off, off + size))
        off += size
    return secs


def read_r1cs(buf: bytes) -> R1csFile:
    secs = _sections(buf)
    for t in (1, 2):
        if t not in secs:
            raise ValueError(f"r1cs: missing section {t}")
    h = _Reader(buf, *secs[1])
    n8 = h.u32()
    if n8 != 32 or int.from_bytes(h.take(32), "little") != R:
        raise ValueError("r1cs: field is not BN254 Fr (bn128)")
    n_wires, n_pub_out, n_pub_in, n_prv_in = h.u32(), h.u32(), h.u32(), h.u32()
    n_labels, m = h.u64(), h.u32()
    if 1 + n_pub_out + n_pub_in + n_prv_in > n_wires:
        raise ValueError("r1cs: signal counts exceed nWires")
    c = _Reader(buf, *secs[2])
    cons = []
    for _ in range(m):
        lcs = []
        for _ in range(3):
            nt = c.u32()
            if nt * 36 > c.end - c.off:
                raise ValueError("r1cs: truncated constraint")
            lc = {}
            for _ in range(nt):
                w = c.u32()
                v = int.from_bytes(c.take(32), "little")
                if w >= n_wires or v >= R:
                    raise ValueError("r1cs: wire index or coefficient out of range")
                if v:
                    lc[w] = (lc.get(w, 0) + v) % R
            lcs.append(lc)
        cons.append(tuple(lcs))
    if c.off != c.end:
        raise ValueError("r1cs: trailing bytes in the constraints section")
    wire2label = list(range(n_wires))
    if 3 in secs:
        lr = _Reader(buf, *secs[3])
        if lr.end - lr.off != 8 * n_wires:
            raise ValueError("r1cs: wire2label size mismatch")
        wire2label = [lr.u64() for _ in range(n_wires)]
    return R1csFile(n_wires, n_pub_out, n_pub_in, n_prv_in, n_labels, cons, wire2label)


def read_sym(text: str) -> dict:
    """circom .sym lines ``labelIdx,varIdx,componentIdx,name`` -> {name: wire} (varIdx -1:
    a signal the optimizer removed, omitted)."""
    out = {}
    for ln, line in enumerate(text.splitlines(), 1):
        if not line.strip():
            continue
        parts = line.split(",", 3)
        if len(parts) != 4:
            raise ValueError(f"sym line {ln}: expected 4 fields")
        var = int(parts[1])
        if var >= 0:
            out[parts[3].strip()] = var
    return out
