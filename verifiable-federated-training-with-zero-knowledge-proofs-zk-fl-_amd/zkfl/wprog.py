"""Witness program compiler: Builder ops -> the flat, level-scheduled image libzkfl executes on the
GPU (``zkfl_wprog_load`` / ``zkfl_witness_compute``, csrc/witness.hip).

This is the replacement of circom's WASM witness calculator (reference:
``node <c>_js/generate_witness.cjs <c>.wasm input.json out.wtns``,
tests/full_system_simulation.mjs:758-767; ``snarkjs wtns calculate``, tests/test_secureagg.cjs:108-118):
the circuit's witness program (recorded by ``zkfl.r1cs.Builder`` while the circuit is built) is
compiled once per circuit, uploaded once, and evaluated for many inputs at a time.

Scheduling: every op gets the level 1 + max(level of the ops producing the wires its linear
combinations read); inputs and the constant wire are level 0.  Ops of one level are
independent, so the GPU runs one launch per level with one lane per (witness, op).  The M
circuit (sgd_verified(128,4,7)) has 3,857 ops in 15 levels.

Image layout (all little-endian u32 unless noted; Fr values 32 B Montgomery form, R = 2^256):
  "zkwp" | version=2 | n_wires | n_pub_out | n_pub_in | n_prv_in | in_first
  | n_ops | n_levels | n_lcs | n_terms | n_asserts | n_templates | n_widths
  | level_ptr[n_levels+1]                       (op index ranges, ops stored level by level)
  | ops[n_ops] x 4 u32: kind | out | lc0 | aux   (kind: 0 LC, 1 MUL, 2 INV, 3 BITS, 4 POS;
                                                 aux: BITS -> n, POS -> t | template << 8)
  | lc_ptr[n_lcs+1]                             (term index ranges)
  | term_wire[n_terms]                          (bit 31 set: coefficient is 1, no multiply)
  | term_coef[n_terms] (Fr)
  | asserts[n_asserts]                          (lc0 of A; B = lc0+1, C = lc0+2)
  | templates[n_templates] x 8 u32: n_sbox | live bitmap words[7]   (204 S-boxes max)
  | widths[n_widths]: t | rp | C[(8+rp)*t] (Fr) | M[t*t] (Fr)
  | n_signals | signals[n_signals]: name_len | name (padded to 4 B) | ndims | dims[ndims] | first_wire | public
                                                 (the circuit's input signals in declaration order:
                                                  what input.json is mapped through, zkfl_witness_compute_json)
"""

from __future__ import annotations

import struct

from .field import POSEIDON_RF, POSEIDON_RP, R, poseidon_params

MAGIC = b"zkwp"
VERSION = 2
K_LC, K_MUL, K_INV, K_BITS, K_POS = 0, 1, 2, 3, 4
_MONT = 1 << 256
_ONE_MONT = _MONT % R


def _mont(x: int) -> bytes:
    return (x * _MONT % R).to_bytes(32, "little")


class _Lcs:
    def __init__(self):
        self.ptr = [0]
        self.wires = []
        self.coefs = []

    def add(self, lc: dict) -> int:
        idx = len(self.ptr) - 1
        for w, c in sorted(lc.items()):
            c %= R
            if not c:
                continue
            self.wires.append(w | (0x80000000 if c == 1 else 0))
            self.coefs.append(c)
        self.ptr.append(len(self.wires))
        return idx


def compile_program(b) -> bytes:
    """Builder -> witness program image."""
    lcs = _Lcs()
    lvl = {}                      # wire -> level (absent: input / constant = 0)
    templates, tmpl_index = [], {}
    widths = []
    recs = []                     # (level, kind, out, lc0, aux)

    def dep(lc):
        return max((lvl.get(k, 0) for k in lc), default=0)

    for op in b.ops:
        kind = op[0]
        if kind == "m":
            _, w, a, c = op
            L = max(dep(a), dep(c)) + 1
            lc0 = lcs.add(a)
            lcs.add(c)
            recs.append((L, K_MUL, w, lc0, 0))
            lvl[w] = L
        elif kind == "lc":
            _, w, a = op
            L = dep(a) + 1
            recs.append((L, K_LC, w, lcs.add(a), 0))
            lvl[w] = L
        elif kind == "inv":
            _, w, a = op
            L = dep(a) + 1
            recs.append((L, K_INV, w, lcs.add(a), 0))
            lvl[w] = L
        elif kind == "bits":
            _, w0, n, a = op
            if not 1 <= n <= 254:
                raise ValueError("Num2Bits width out of range")
            L = dep(a) + 1
            recs.append((L, K_BITS, w0, lcs.add(a), n))
            for i in range(n):
                lvl[w0 + i] = L
        elif kind == "pos":
            _, w0, t, ins, tp = op
            L = max((dep(a) for a in ins), default=0) + 1
            lc0 = lcs.add(ins[0])
            for a in ins[1:]:
                lcs.add(a)
            live = tuple(tp.live)
            key = (t, live)
            if key not in tmpl_index:
                tmpl_index[key] = len(templates)
                n_sbox = POSEIDON_RF * t + POSEIDON_RP[t - 2]
                words = [0] * 7
                for s in live:
                    words[s >> 5] |= 1 << (s & 31)
                templates.append([n_sbox] + words)
                if t not in widths:
                    widths.append(t)
            recs.append((L, K_POS, w0, lc0, t | (tmpl_index[key] << 8)))
            for i in range(3 * len(live)):
                lvl[w0 + i] = L
        else:  # pragma: no cover
            raise ValueError(kind)

    recs.sort(key=lambda r: r[0])   # stable: program order within a level
    n_levels = recs[-1][0] if recs else 0
    level_ptr = [0] * (n_levels + 1)
    for r in recs:
        level_ptr[r[0]] += 1
    for i in range(1, n_levels + 1):
        level_ptr[i] += level_ptr[i - 1]
    level_ptr = [0] + level_ptr[1:]

    asserts = []
    for ci in b.asserts:
        A, B, C = b.cons[ci]
        a0 = lcs.add(A)
        lcs.add(B)
        lcs.add(C)
        asserts.append(a0)

    in_first = 1 + b.n_pub_out
    head = struct.pack("<4s13I", MAGIC, VERSION, b.n_wires, b.n_pub_out, b.n_pub_in, b.n_prv_in, in_first,
                       len(recs), n_levels, len(lcs.ptr) - 1, len(lcs.wires), len(asserts), len(templates),
                       len(widths))
    parts = [head, struct.pack(f"<{n_levels + 1}I", *level_ptr)]
    parts.append(b"".join(struct.pack("<4I", k, out, lc0, aux) for _, k, out, lc0, aux in recs))
    parts.append(struct.pack(f"<{len(lcs.ptr)}I", *lcs.ptr))
    parts.append(struct.pack(f"<{len(lcs.wires)}I", *lcs.wires))
    parts.append(b"".join(_mont(c) for c in lcs.coefs))
    parts.append(struct.pack(f"<{len(asserts)}I", *asserts))
    parts.append(b"".join(struct.pack("<8I", *t) for t in templates))
    for t in widths:
        C, M = poseidon_params(t)
        rp = POSEIDON_RP[t - 2]
        parts.append(struct.pack("<2I", t, rp))
        parts.append(b"".join(_mont(c) for c in C))
        parts.append(b"".join(_mont(M[i][j]) for i in range(t) for j in range(t)))
    parts.append(struct.pack("<I", len(b.inputs)))
    for name, shape, first, public in b.inputs:
        nb = name.encode()
        parts.append(struct.pack("<I", len(nb)) + nb + b"\0" * (-len(nb) % 4))
        parts.append(struct.pack(f"<I{len(shape)}I", len(shape), *shape) + struct.pack("<2I", first, int(public)))
    return b"".join(parts)


def input_bytes(b, values: dict) -> bytes:
    """input.json-style dict -> the flattened input signals (declaration order), 32 B std each."""
    flat = b.flatten_inputs(values)
    first = 1 + b.n_pub_out
    n = b.n_pub_in + b.n_prv_in
    return b"".join(flat[first + i].to_bytes(32, "little") for i in range(n))


def levels(image: bytes):
    """(n_ops, n_levels) of an image (diagnostics)."""
    f = struct.unpack_from("<4s13I", image, 0)
    return f[7], f[8]
