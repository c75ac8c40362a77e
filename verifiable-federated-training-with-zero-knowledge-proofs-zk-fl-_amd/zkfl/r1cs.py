"""R1CS builder + witness program — the in-repo replacement for the circom compiler and its
WASM witness calculator (circom is absent from this image).

Semantics follow circom 2 with full linear simplification (``--O2``):
  * wire 0 is the constant ONE, then public outputs, public inputs, private inputs, then
    internal signals — the order snarkjs relies on for ``public.json`` (witness[1..nPublic]);
  * ``<==`` of a linear expression allocates no wire: linear combinations (LCs) are carried
    symbolically and substituted into the nonlinear constraints (dicts {wire: coef mod r});
  * every product of two non-constant LCs allocates one wire and one constraint A*B = C;
  * products with a compile-time constant fold to a scaled LC (``x * 0`` vanishes);
  * ``===`` becomes an explicit (assert) constraint; the witness evaluator checks every assert
    and raises ``ConstraintError`` the way circom's witness calculator aborts on a failed
    ``assert`` (SURVEY.md §5 failure detection: invalid inputs fail at witness generation).

The witness is produced by a *program* recorded at build time (``Builder.ops``): one op per
allocated wire group ('m' product, 'lc' bound output, 'bits' Num2Bits hint, 'inv' IsZero hint,
'pos' Poseidon permutation).  The structure never depends on input values, so one build serves
all inputs.  zkfl/wprog.py compiles it into the image the GPU witness engine executes
(csrc/witness.hip); oracle/witness.py is the CPU evaluator the tests check the GPU against.
"""

from __future__ import annotations

import struct
from functools import lru_cache

from .field import POSEIDON_RF, POSEIDON_RP, R, fr, poseidon_params


class ConstraintError(ValueError):
    """Witness does not satisfy the circuit (circom: 'Assert Failed')."""


# ---------------------------------------------------------------------------
# LC helpers (dict {wire: coef}); wire 0 = ONE
# ---------------------------------------------------------------------------
def const(c) -> dict:
    c = int(c) % R
    return {0: c} if c else {}


def is_const(a: dict) -> bool:
    return all(k == 0 for k in a)


def const_val(a: dict) -> int:
    return a.get(0, 0)


def add(a: dict, b: dict) -> dict:
    if len(a) < len(b):
        a, b = b, a
    out = dict(a)
    for k, v in b.items():
        nv = (out.get(k, 0) + v) % R
        if nv:
            out[k] = nv
        else:
            out.pop(k, None)
    return out


def scale(a: dict, k) -> dict:
    k = int(k) % R
    if k == 0:
        return {}
    if k == 1:
        return dict(a)
    return {w: v * k % R for w, v in a.items()}


def sub(a: dict, b: dict) -> dict:
    return add(a, scale(b, R - 1))


def add_const(a: dict, c) -> dict:
    return add(a, const(c))


def lc_sum(lcs) -> dict:
    out = {}
    for a in lcs:
        out = add(out, a)
    return out


def evaluate(a: dict, w) -> int:
    return sum(w[k] * v for k, v in a.items()) % R


# ---------------------------------------------------------------------------
# Poseidon constraint template (built once per width, instantiated per hash)
# ---------------------------------------------------------------------------
class _PoseidonTemplate:
    """Constraints of one circomlib Poseidon permutation over local wire ids.

    Local ids: 0 = ONE, 1..3*S = the x2/x4/x5 wires of the S live S-boxes; input slot i is
    referenced by key ('in', i).  Round-0 lane-0 (capacity, constant) is folded."""

    def __init__(self, t: int, const_lanes=None):
        C, M = poseidon_params(t)
        rp = POSEIDON_RP[t - 2]
        half = POSEIDON_RF // 2
        self.t = t
        self.cons = []          # (A, B, C) with local ids / input keys
        self.live = []          # trace indices of live S-boxes
        nw = 0
        const_lanes = const_lanes or (None,) * (t - 1)
        state = [const(0)] + [const(c) if c is not None else {("in", i): 1}
                              for i, c in enumerate(const_lanes)]
        sbox_idx = 0
        for rnd in range(POSEIDON_RF + rp):
            state = [add_const(state[i], C[rnd * t + i]) for i in range(t)]
            full = rnd < half or rnd >= half + rp
            for i in (range(t) if full else range(1)):
                x = state[i]
                if is_const(x):
                    state[i] = const(pow(const_val(x), 5, R))
                else:
                    x2, x4, x5 = nw + 1, nw + 2, nw + 3
                    nw += 3
                    self.cons.append((x, x, {x2: 1}))
                    self.cons.append(({x2: 1}, {x2: 1}, {x4: 1}))
                    self.cons.append(({x4: 1}, x, {x5: 1}))
                    self.live.append(sbox_idx)
                    state[i] = {x5: 1}
                sbox_idx += 1
            state = [lc_sum(scale(state[j], M[i][j]) for j in range(t)) for i in range(t)]
        self.n_local = nw
        self.out = state[0]


@lru_cache(maxsize=None)
def _template(t: int, const_lanes=None) -> _PoseidonTemplate:
    return _PoseidonTemplate(t, const_lanes)


# ---------------------------------------------------------------------------
# Builder
# ---------------------------------------------------------------------------
class Builder:
    def __init__(self, name: str = "circuit"):
        self.name = name
        self.n_wires = 1
        self.cons = []            # (A, B, C)
        self.asserts = []         # indices of assert constraints (checked at witness time)
        self.ops = []             # witness program
        self.inputs = []          # (name, shape, first_wire, public)
        self.n_pub_in = 0
        self.n_prv_in = 0
        self.n_pub_out = 0
        self.outputs = []         # (name, wire)
        self._private_started = False
        self._inputs_started = False

    # -- signals -----------------------------------------------------------
    def output(self, name: str) -> int:
        """Declare a public output of main (wires 1..nOut come first); bind it later."""
        if self._inputs_started:
            raise ValueError("outputs must be declared before inputs")
        w = self._new_wires(1)
        self.outputs.append((name, w))
        self.n_pub_out += 1
        return w

    def bind_output(self, wire: int, value: dict):
        """out <== value (linear): computed by the witness program, checked as an assert."""
        self.ops.append(("lc", wire, value))
        self.assert_eq({wire: 1}, value)

    def input(self, name: str, shape=(), public: bool = False):
        """Declare an input signal (scalar or nested array); returns LC(s) of the same shape."""
        self._inputs_started = True
        if public and self._private_started:
            raise ValueError("public inputs must be declared before private inputs")
        if not public:
            self._private_started = True
        count = 1
        for d in shape:
            count *= d
        first = self.n_wires
        self.n_wires += count
        self.inputs.append((name, tuple(shape), first, public))
        if public:
            self.n_pub_in += count
        else:
            self.n_prv_in += count
        flat = [{first + i: 1} for i in range(count)]

        def nest(items, dims):
            if not dims:
                return items[0]
            step = len(items) // dims[0]
            return [nest(items[i * step:(i + 1) * step], dims[1:]) for i in range(dims[0])]

        return nest(flat, list(shape))

    @property
    def n_public(self) -> int:
        return self.n_pub_out + self.n_pub_in

    @property
    def n_constraints(self) -> int:
        return len(self.cons)

    def _new_wires(self, k: int) -> int:
        w = self.n_wires
        self.n_wires += k
        return w

    # -- constraint primitives ---------------------------------------------
    def mul(self, a: dict, b: dict) -> dict:
        """a * b (circom ``s <== a * b``): folds constants, otherwise one wire + constraint."""
        if is_const(a):
            return scale(b, const_val(a))
        if is_const(b):
            return scale(a, const_val(b))
        w = self._new_wires(1)
        self.cons.append((a, b, {w: 1}))
        self.ops.append(("m", w, a, b))
        return {w: 1}

    def assert_mul(self, a: dict, b: dict, c: dict):
        """a * b === c."""
        if is_const(a) and is_const(b) and is_const(c):
            if const_val(a) * const_val(b) % R != const_val(c):
                raise ConstraintError("constant constraint violated")
            return
        self.asserts.append(len(self.cons))
        self.cons.append((a, b, c))

    def assert_eq(self, a: dict, b: dict):
        """a === b (linear)."""
        d = sub(a, b)
        if is_const(d):
            if const_val(d):
                raise ConstraintError("constant equality violated")
            return
        self.asserts.append(len(self.cons))
        self.cons.append((d, const(1), {}))

    def num2bits(self, x: dict, n: int):
        """circomlib Num2Bits(n): n boolean wires, sum 2^i b_i === x."""
        w0 = self._new_wires(n)
        self.ops.append(("bits", w0, n, x))
        bits = []
        acc = {}
        e = 1
        for i in range(n):
            b = {w0 + i: 1}
            self.assert_mul(b, add_const(b, R - 1), {})
            acc = add(acc, scale(b, e))
            e = e * 2 % R
            bits.append(b)
        self.assert_eq(acc, x)
        return bits

    def is_zero(self, x: dict) -> dict:
        """circomlib IsZero: out = 1 - x * inv, x * out === 0."""
        if is_const(x):
            return const(1 if const_val(x) == 0 else 0)
        w = self._new_wires(1)
        self.ops.append(("inv", w, x))
        inv = {w: 1}
        xi = self.mul(x, inv)
        out = sub(const(1), xi)
        self.assert_mul(x, out, {})
        return out

    def poseidon(self, inputs) -> dict:
        """circomlib Poseidon(len(inputs)) (t = n + 1); returns the output LC (state[0])."""
        ins = [dict(a) for a in inputs]
        t = len(ins) + 1
        if not 2 <= t <= 17:
            raise ValueError("Poseidon supports 1..16 inputs")
        cl = tuple(const_val(a) if is_const(a) else None for a in ins)
        tp = _template(t, cl if any(c is not None for c in cl) else None)
        base = self._new_wires(tp.n_local) - 1   # local id k -> base + k
        ins_c = ins

        def inst(lc):
            out = {}
            for k, v in lc.items():
                if type(k) is tuple:
                    for w2, v2 in ins_c[k[1]].items():
                        nv = (out.get(w2, 0) + v * v2) % R
                        if nv:
                            out[w2] = nv
                        else:
                            out.pop(w2, None)
                elif k == 0:
                    nv = (out.get(0, 0) + v) % R
                    if nv:
                        out[0] = nv
                    else:
                        out.pop(0, None)
                else:
                    out[base + k] = v
            return out

        memo = {}

        def inst_memo(lc):
            key = id(lc)
            r = memo.get(key)
            if r is None:
                r = inst(lc)
                memo[key] = r
            return r

        for A, B, C in tp.cons:
            self.cons.append((inst_memo(A), inst_memo(B), inst_memo(C)))
        self.ops.append(("pos", base + 1, t, ins_c, tp))
        return inst(tp.out)

    # -- witness --------------------------------------------------------------
    def flatten_inputs(self, values: dict):
        """Map an input.json-style dict (decimal strings / ints, nested lists, negatives
        allowed) to {wire: value}.  Missing or mis-shaped signals raise ValueError."""
        out = {}
        for name, shape, first, _pub in self.inputs:
            if name not in values:
                raise ValueError(f"missing input signal '{name}'")
            v = values[name]
            flat = []

            def walk(x, dims):
                if not dims:
                    if isinstance(x, (list, tuple)):
                        raise ValueError(f"input '{name}' has too many dimensions")
                    flat.append(fr(x))
                    return
                if not isinstance(x, (list, tuple)) or len(x) != dims[0]:
                    raise ValueError(f"input '{name}' has wrong shape, expected {shape}")
                for y in x:
                    walk(y, dims[1:])

            walk(v, list(shape))
            for i, x in enumerate(flat):
                out[first + i] = x
        return out

    def check_all(self, w) -> bool:
        """Full R1CS satisfaction check (every constraint)."""
        for A, B, C in self.cons:
            if evaluate(A, w) * evaluate(B, w) % R != evaluate(C, w):
                return False
        return True

    # -- export ---------------------------------------------------------------
    def r1cs_bytes(self) -> bytes:
        """iden3 .r1cs v1 (header, constraints, wire2label), coefficients std form LE."""
        hdr = struct.pack("<I", 32) + R.to_bytes(32, "little")
        hdr += struct.pack("<IIIIQI", self.n_wires, self.n_pub_out, self.n_pub_in, self.n_prv_in, self.n_wires,
                           len(self.cons))
        parts = []
        for A, B, C in self.cons:
            for lc in (A, B, C):
                items = sorted(lc.items())
                parts.append(struct.pack("<I", len(items)))
                parts.append(b"".join(struct.pack("<I", k) + v.to_bytes(32, "little") for k, v in items))
        cons = b"".join(parts)
        labels = b"".join(struct.pack("<Q", i) for i in range(self.n_wires))
        out = [b"r1cs", struct.pack("<II", 1, 3)]
        for typ, data in ((1, hdr), (2, cons), (3, labels)):
            out.append(struct.pack("<IQ", typ, len(data)))
            out.append(data)
        return b"".join(out)
