"""GPU witness engine (zkfl_wprog_load / zkfl_witness_compute[_resident]) vs the oracle — MI355X.

Bar: bit-exact witnesses (every wire) against oracle/witness.py (circom semantics, Poseidon from
oracle/poseidon.py pinned by the reference fixture), on every reference circuit incl. the fixture
data/test_input_v5.json and the metric circuit M; unsatisfiable inputs fail with
ZKFL_E_CONSTRAINT like circom's "Assert Failed"; resident witnesses prove identically.
"""
import json
import os

import pytest

from oracle import groth16 as og
from oracle import witness as ow

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _client(cid=1, n=8, depth=3):
    from zkfl import clients
    return clients.Client(cid, n, 4, depth, clients.JsLcg(12344 + cid))


def _prog(gpu_ctx, b):
    from zkfl import native, wprog
    return native.WitnessProgram(gpu_ctx, wprog.compile_program(b))


def test_reference_circuits_bit_exact(gpu_ctx):
    from zkfl import circuits, clients, wprog, zkey
    c = _client()
    _, grad = c.training_input(8, 1000, 100000000)
    cases = [
        ("poseidon_hash2", (), [{"left": 1, "right": 2}, {"left": 0, "right": -5}]),
        ("sgd_verified", (8, 4, 3, 1000), [_client(i).training_input(8, 1000, 100000000)[0] for i in (1, 2, 3)]),
        ("balance_unified", (8, 3, 4), [c.balance_input()]),
        ("secure_masked_update", (4, 2), [clients.secagg_input(1, [2, 3], grad, 1, 100000000, c.root_D, 0)]),
        ("sgd_step_v5", (8, 16, 7), [json.load(open(os.path.join(GOLDEN, "test_input_v5.json")))]),
    ]
    for name, params, inputs in cases:
        b = circuits.build(name, *params)
        wp = _prog(gpu_ctx, b)
        got = wp.compute([wprog.input_bytes(b, x) for x in inputs])
        for x, wt in zip(inputs, got):
            assert zkey.read_wtns(wt) == ow.evaluate(b, x), name
        wp.close()
    # the fixture's public signals come out of the GPU witness
    d = cases[-1][2][0]
    b = circuits.build("sgd_step_v5", 8, 16, 7)
    wp = _prog(gpu_ctx, b)
    w = zkey.read_wtns(wp.compute([wprog.input_bytes(b, d)])[0])
    assert [str(x) for x in w[1:6]] == [d["client_id"], d["round"], d["root_D"], d["root_G"], d["tauSquared"]]
    wp.close()


def test_metric_circuit_batch(gpu_ctx):
    """M = sgd_verified(128,4,7): a batch of 3 witnesses in one call; one compared wire by wire,
    all satisfy the full R1CS."""
    from zkfl import circuits, wprog, zkey
    b = circuits.build("sgd_verified", 128, 4, 7, 1000)
    inputs = [_client(i, 128, 7).training_input(128, 1000, 100000000)[0] for i in (1, 2, 3)]
    wp = _prog(gpu_ctx, b)
    got = [zkey.read_wtns(x) for x in wp.compute([wprog.input_bytes(b, x) for x in inputs])]
    assert got[0] == ow.evaluate(b, inputs[0])
    for w in got:
        assert b.check_all(w)
    assert got[1] != got[2]
    wp.close()


def test_errors(gpu_ctx):
    from zkfl import circuits, native, wprog
    b = circuits.build("sgd_verified", 8, 4, 3, 1000)
    wp = _prog(gpu_ctx, b)
    bad, _ = _client().training_input(8, 1000, 100000000)
    bad["remainder"][0] = str(int(bad["remainder"][0]) + 1)
    good = wprog.input_bytes(b, _client().training_input(8, 1000, 100000000)[0])
    with pytest.raises(native.ZkflError) as e:          # circom: Assert Failed
        wp.compute([good, wprog.input_bytes(b, bad)])
    assert e.value.code == -7 and "witness 1" in str(e.value)
    with pytest.raises(native.ZkflError) as e:          # input >= r
        wp.compute([b"\xff" * 32 + good[32:]])
    assert e.value.code == -1
    with pytest.raises(native.ZkflError) as e:          # wrong number of inputs
        wp.compute([good[:-32]])
    assert e.value.code == -1
    with pytest.raises(native.ZkflError) as e:          # malformed image
        native.WitnessProgram(gpu_ctx, wprog.compile_program(b)[:-100])
    assert e.value.code == -2
    wp.close()


def test_resident_witness_proves_identically(gpu_ctx):
    from zkfl import circuits, native, wprog, zkey
    b = circuits.build("sgd_verified", 8, 4, 3, 1000)
    zk = zkey.groth16_setup(b, gpu_ctx, zkey.Toxic(tau=99, alpha=2, beta=3, gamma=4, delta=5))
    key = native.ProvingKey(gpu_ctx, zk)
    wp = _prog(gpu_ctx, b)
    inputs = [wprog.input_bytes(b, _client(i).training_input(8, 1000, 100000000)[0]) for i in (1, 2)]
    res = wp.compute_resident(key, inputs)
    wts = wp.compute(inputs)
    rs = (7).to_bytes(32, "little") + (9).to_bytes(32, "little")
    for r_, wt in zip(res, wts):
        assert key.prove_resident(r_, rs) == key.prove(wt, rs)[0]
    ref = og.prove(og.parse_zkey(zk), zkey.read_wtns(wts[0]), r=7, s=9)
    assert key.prove_resident(res[0], rs) == og.proof_bytes(ref)
    # a program of another circuit does not fit this key
    other = _prog(gpu_ctx, circuits.build("poseidon_hash2"))
    with pytest.raises(native.ZkflError) as e:
        other.compute_resident(key, [(1).to_bytes(32, "little") * 2])
    assert e.value.code == -4
    for r_ in res:
        r_.close()
    other.close()
    wp.close()
    key.close()


def test_fullprove_api(gpu_ctx):
    """snarkjs-shaped groth16.fullProve(input, circuit, zkey): GPU witness + GPU proof + GPU verify."""
    from zkfl import circuits, groth16, zkey
    b = circuits.build("poseidon_hash2")
    zk = zkey.groth16_setup(b, gpu_ctx, zkey.Toxic(tau=5, alpha=6, beta=7, gamma=8, delta=9))
    p = groth16.Prover.__new__(groth16.Prover)
    p.ctx, p._keys, p._progs = gpu_ctx, {}, {}
    proof, public = p.full_prove({"left": 1, "right": 2}, b, zk)
    assert public == ["7853200120776062878684798364095072458815029376092732009249414926327459813530"]
    assert p.verify(groth16.export_verification_key(zk, ctx=gpu_ctx), public, proof)
    for k in p._keys.values():
        k.close()
    for _, w in p._progs.values():
        w.close()
