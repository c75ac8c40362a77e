"""CPU: the witness-program compiler (zkfl/wprog.py) — the image's semantics, interpreted here
exactly as csrc/witness.hip executes it (level by level, Montgomery-free integers), reproduce the
oracle's circom-semantics evaluation (oracle/witness.py) on the reference circuits and inputs,
including the fixture data/test_input_v5.json.  The GPU executor itself is compared with the
oracle in tests/test_gpu_witness.py."""
import json
import os
import struct

import pytest

from oracle import poseidon as op
from oracle import witness as ow
from zkfl import circuits, clients, wprog

R = op.R
RINV = pow(1 << 256, -1, R)
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def interpret(img: bytes, inputs: bytes):
    """Run a program image on one input vector (pure Python; mirrors csrc/witness.hip)."""
    f = struct.unpack_from("<4s13I", img, 0)
    _, ver, nw, npo, npi, npv, in_first, n_ops, n_lv, n_lcs, n_terms, n_as, n_tm, n_wd = f
    assert ver == 2
    o = struct.calcsize("<4s13I")

    def u32s(n):
        nonlocal o
        v = struct.unpack_from(f"<{n}I", img, o)
        o += 4 * n
        return v

    def frs(n):
        nonlocal o
        v = [int.from_bytes(img[o + 32 * i:o + 32 * i + 32], "little") * RINV % R for i in range(n)]
        o += 32 * n
        return v

    lvp = u32s(n_lv + 1)
    ops = [u32s(4) for _ in range(n_ops)]
    lcp = u32s(n_lcs + 1)
    tw = u32s(n_terms)
    tc = frs(n_terms)
    asrt = u32s(n_as)
    tmpl = [u32s(8) for _ in range(n_tm)]
    widths = {}
    for _ in range(n_wd):
        t, rp = u32s(2)
        C = frs((8 + rp) * t)
        M = frs(t * t)
        widths[t] = (rp, C, M)
    (n_sig,) = u32s(1)
    for _ in range(n_sig):
        (ln,) = u32s(1)
        o += (ln + 3) // 4 * 4
        (nd,) = u32s(1)
        u32s(nd + 2)
    assert o == len(img)

    w = [0] * nw
    w[0] = 1
    n_in = npi + npv
    for i in range(n_in):
        w[in_first + i] = int.from_bytes(inputs[32 * i:32 * i + 32], "little")

    def ev(lc):
        acc = 0
        for t in range(lcp[lc], lcp[lc + 1]):
            x = tw[t]
            v = w[x & 0x7FFFFFFF]
            acc += v if x >> 31 else v * tc[t]
        return acc % R

    for L in range(n_lv):
        for kind, out, lc0, aux in ops[lvp[L]:lvp[L + 1]]:
            if kind == 0:
                w[out] = ev(lc0)
            elif kind == 1:
                w[out] = ev(lc0) * ev(lc0 + 1) % R
            elif kind == 2:
                v = ev(lc0)
                w[out] = pow(v, R - 2, R) if v else 0
            elif kind == 3:
                v = ev(lc0)
                for i in range(aux):
                    w[out + i] = (v >> i) & 1
            else:
                t, tid = aux & 0xFF, aux >> 8
                rp, C, M = widths[t]
                live = tmpl[tid][1:]
                st = [0] + [ev(lc0 + i) for i in range(t - 1)]
                k, sb = out, 0
                for r in range(8 + rp):
                    st = [(st[i] + C[r * t + i]) % R for i in range(t)]
                    for i in range(t if (r < 4 or r >= 4 + rp) else 1):
                        x2 = st[i] * st[i] % R
                        x4 = x2 * x2 % R
                        x5 = x4 * st[i] % R
                        if (live[sb >> 5] >> (sb & 31)) & 1:
                            w[k:k + 3] = [x2, x4, x5]
                            k += 3
                        st[i] = x5
                        sb += 1
                    st = [sum(M[i * t + j] * st[j] for j in range(t)) % R for i in range(t)]
    ok = all(ev(a) * ev(a + 1) % R == ev(a + 2) for a in asrt)
    return w, ok


def _cases():
    c = clients.Client(1, 8, 4, 3, clients.JsLcg(12345))
    yield "poseidon_hash2", (), {"left": 1, "right": 2}
    yield "sgd_verified", (8, 4, 3, 1000), c.training_input(8, 1000, 100000000)[0]
    yield "balance_unified", (8, 3, 4), c.balance_input()
    _, grad = c.training_input(8, 1000, 100000000)
    yield "secure_masked_update", (4, 2), clients.secagg_input(1, [2, 3], grad, 1, 100000000, c.root_D, 0)
    yield "sgd_step_v5", (8, 16, 7), json.load(open(os.path.join(GOLDEN, "test_input_v5.json")))


@pytest.mark.parametrize("name,params,inp", list(_cases()), ids=lambda x: x if isinstance(x, str) else "")
def test_image_semantics_match_oracle(name, params, inp):
    b = circuits.build(name, *params)
    img = wprog.compile_program(b)
    w, ok = interpret(img, wprog.input_bytes(b, inp))
    assert ok
    assert w == ow.evaluate(b, inp)


def test_levels_respect_dependencies():
    b = circuits.build("sgd_verified", 8, 4, 3, 1000)
    img = wprog.compile_program(b)
    n_ops, n_lv = wprog.levels(img)
    assert n_ops == len(b.ops) and 1 <= n_lv <= n_ops


def test_failed_assert_detected():
    b = circuits.build("poseidon_hash2")
    img = wprog.compile_program(b)
    inp = bytearray(wprog.input_bytes(b, {"left": 1, "right": 2}))
    _, ok = interpret(img, bytes(inp))
    assert ok
    # PoseidonHash2 binds out <== Poseidon(...): tampering with nothing the program writes keeps
    # the asserts true; an unsatisfiable circuit input is exercised on sgd_verified instead
    c = clients.Client(1, 8, 4, 3, clients.JsLcg(12345))
    bb = circuits.build("sgd_verified", 8, 4, 3, 1000)
    bad, _ = c.training_input(8, 1000, 100000000)
    bad["remainder"][0] = str(int(bad["remainder"][0]) + 1)
    _, ok = interpret(wprog.compile_program(bb), wprog.input_bytes(bb, bad))
    assert not ok


# ---------------------------------------------------------------------------
# input.json parsing in libzkfl (host-only C ABI: no GPU needed)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name,params,inp", list(_cases()), ids=lambda x: x if isinstance(x, str) else "")
def test_c_input_json_parser_matches_python(name, params, inp):
    from zkfl import native
    b = circuits.build(name, *params)
    img = wprog.compile_program(b)
    assert native.parse_inputs(img, json.dumps(inp)) == wprog.input_bytes(b, inp)


def test_c_input_json_parser_values_and_errors():
    from zkfl import native
    b = circuits.build("poseidon_hash2")
    img = wprog.compile_program(b)
    enc = lambda *v: b"".join((x % R).to_bytes(32, "little") for x in v)  # noqa: E731
    cases = [('{"left": 1, "right": 2}', enc(1, 2)),
             ('{"right": "-5", "left": "0x10"}', enc(16, -5)),
             (' {"left":%d,"right":%d,"extra":[1,2]} ' % (R + 3, -R), enc(3, 0)),
             ('{"left": "%d", "right": "-%d"}' % (2 ** 300, 2 ** 300), enc(2 ** 300, -2 ** 300))]
    for text, want in cases:
        assert native.parse_inputs(img, text) == want, text
    for bad in ('{"left": 1}', '{"left": [1], "right": 2}', '{"left": 1.5, "right": 2}', '[1, 2]',
                '{"left": 1, "right": 2', '{"left": "a", "right": 2}'):
        with pytest.raises(native.ZkflError) as e:
            native.parse_inputs(img, bad)
        assert e.value.code == -1, bad
    with pytest.raises(native.ZkflError) as e:
        native.parse_inputs(img[:-8], '{"left": 1, "right": 2}')
    assert e.value.code == -2


def test_c_input_json_parser_literal_sweep():
    """Chunked literal reduction (host_parse.cc literal_to_fr): every digit count from 1 to 200,
    decimal and hex, both signs, values around multiples of r and powers of two, == Python mod r."""
    import random
    from zkfl import native
    b = circuits.build("poseidon_hash2")
    img = wprog.compile_program(b)
    rnd = random.Random(7)
    vals = [0, 1, R - 1, R, R + 1, 2 * R - 1, 5 * R + 7, 2 ** 256 - 1, 2 ** 254, 10 ** 18 - 1, 10 ** 18,
            10 ** 36, 16 ** 15 - 1, 16 ** 15, 2 ** 320 + 3, 2 ** 640 - 1, (2 ** 256 // R) * R, (2 ** 320 // R) * R - 1]
    vals += [rnd.randrange(10 ** (d - 1), 10 ** d) for d in range(1, 201)]
    vals += [rnd.randrange(16 ** (d - 1), 16 ** d) for d in range(1, 120, 3)]
    for i in range(0, len(vals), 2):
        x, y = vals[i], vals[(i + 1) % len(vals)]
        for lx, ly in ((str(x), "-" + str(y)), (hex(x), "-" + hex(y)), ("-" + str(x), "+" + hex(y).upper().replace("0X", "0x"))):
            text = '{"left": "%s", "right": "%s"}' % (lx, ly)
            want = b"".join((int(v, 0) % R).to_bytes(32, "little") for v in (lx, ly))
            assert native.parse_inputs(img, text) == want, text
