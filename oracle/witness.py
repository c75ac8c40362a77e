"""CPU witness evaluation (circom witness-calculator semantics) — TEST INFRASTRUCTURE ONLY.

Part of the parity oracle: only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it.  The product computes witnesses on the GPU
(csrc/witness.hip via zkfl/wprog.py); this module is what that engine is checked against.

Restates what circom's generated WASM does for the reference circuits
(``node <c>_js/generate_witness.cjs``, tests/full_system_simulation.mjs:758-767) over the
circuit description recorded by zkfl.r1cs.Builder: inputs placed at their wires, every
intermediate signal computed in program order ('m' a*b, 'lc' bound outputs, 'bits' Num2Bits
hints, 'inv' IsZero hints, 'pos' Poseidon S-box trace x^2, x^4, x^5), then every ``===``
checked (circom: "Assert Failed").  Poseidon uses this oracle's own restatement of circomlib
(oracle/poseidon.py, pinned by the reference fixture), not the product's.
"""

from __future__ import annotations

from . import poseidon as op

R = op.R


class AssertFailed(ValueError):
    pass


def _ev(lc, w):
    return sum(w[k] * v for k, v in lc.items()) % R


def poseidon_trace(state):
    """circomlib permutation; -> (final state, [(x^2, x^4, x^5)] per S-box in circuit order)."""
    t = len(state)
    C, M = op.constants(t)
    rp = op.N_ROUNDS_P[t - 2]
    half = op.N_ROUNDS_F // 2
    st = [x % R for x in state]
    trace = []
    for r in range(op.N_ROUNDS_F + rp):
        st = [(st[i] + C[r * t + i]) % R for i in range(t)]
        for i in (range(t) if (r < half or r >= half + rp) else range(1)):
            x2 = st[i] * st[i] % R
            x4 = x2 * x2 % R
            x5 = x4 * st[i] % R
            trace.append((x2, x4, x5))
            st[i] = x5
        st = [sum(M[i][j] * st[j] for j in range(t)) % R for i in range(t)]
    return st, trace


def evaluate(b, values: dict, check: bool = True):
    """Full witness (list of ints, wire order) of circuit `b` for an input.json-style dict."""
    w = [0] * b.n_wires
    w[0] = 1
    for k, v in b.flatten_inputs(values).items():
        w[k] = v
    for opr in b.ops:
        kind = opr[0]
        if kind == "m":
            _, wi, a, c = opr
            w[wi] = _ev(a, w) * _ev(c, w) % R
        elif kind == "pos":
            _, w0, t, ins, tp = opr
            _, trace = poseidon_trace([0] + [_ev(a, w) for a in ins])
            k = w0
            for idx in tp.live:
                w[k:k + 3] = trace[idx]
                k += 3
        elif kind == "bits":
            _, w0, n, x = opr
            v = _ev(x, w)
            for i in range(n):
                w[w0 + i] = (v >> i) & 1
        elif kind == "lc":
            _, wi, x = opr
            w[wi] = _ev(x, w)
        elif kind == "inv":
            _, wi, x = opr
            v = _ev(x, w)
            w[wi] = pow(v, R - 2, R) if v else 0
        else:  # pragma: no cover
            raise RuntimeError(kind)
    if check:
        for ci in b.asserts:
            A, B, C = b.cons[ci]
            if _ev(A, w) * _ev(B, w) % R != _ev(C, w):
                raise AssertFailed(f"{b.name}: assert constraint {ci} failed")
    return w
