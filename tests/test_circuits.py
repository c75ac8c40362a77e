"""Product circuit builder + witness program vs the oracle and the reference fixture (CPU)."""
import json
import os
import random

import pytest

from oracle import witness as ow

from oracle import groth16 as og
from oracle import poseidon as op
from zkfl import circuits, clients
from zkfl.field import R, poseidon_hash

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("t", range(2, 18))
def test_poseidon_all_widths_match_oracle(t):
    rnd = random.Random(t)
    ins = [rnd.randrange(R) for _ in range(t - 1)]
    assert poseidon_hash(ins) == op.poseidon(ins)


@pytest.mark.parametrize("n", [1, 2, 5, 16])
def test_poseidon_gadget_witness(n):
    from zkfl.r1cs import Builder
    b = Builder("p")
    out = b.output("h")
    xs = b.input("x", (n,))
    b.bind_output(out, b.poseidon(xs))
    vals = [random.Random(n).randrange(R) for _ in range(n)]
    w = ow.evaluate(b, {"x": vals})
    assert w[1] == op.poseidon(vals)
    assert b.check_all(w)


def test_fixture_v5_satisfies_circuit():
    d = json.load(open(os.path.join(GOLDEN, "test_input_v5.json")))
    b = circuits.build("sgd_step_v5", 8, 16, 7)
    w = ow.evaluate(b, d)
    assert b.check_all(w)
    # public.json order = [client_id, round, root_D, root_G, tauSquared]
    assert [str(x) for x in w[1:6]] == [d["client_id"], d["round"], d["root_D"], d["root_G"], d["tauSquared"]]


@pytest.mark.parametrize("field,val", [("root_G", "5"), ("root_D", "7"), ("tauSquared", "1")])
def test_fixture_tampered_rejected(field, val):
    d = json.load(open(os.path.join(GOLDEN, "test_input_v5.json")))
    d[field] = val
    with pytest.raises(ow.AssertFailed):
        ow.evaluate(circuits.build("sgd_step_v5", 8, 16, 7), d)


def test_fixture_non_boolean_path_rejected():
    d = json.load(open(os.path.join(GOLDEN, "test_input_v5.json")))
    d["pathIndices"][0][0] = "2"
    with pytest.raises(ow.AssertFailed):
        ow.evaluate(circuits.build("sgd_step_v5", 8, 16, 7), d)


def test_input_shape_errors():
    b = circuits.build("sgd_step_v5", 8, 16, 7)
    d = json.load(open(os.path.join(GOLDEN, "test_input_v5.json")))
    del d["labels"]
    with pytest.raises(ValueError):
        ow.evaluate(b, d)


def _client(n=8, dim=4, depth=3, cid=1):
    return clients.Client(cid, n, dim, depth, clients.JsLcg(12345))


def test_client_generator_matches_oracle_merkle():
    c = _client()
    leaves = [op.vector_hash(c.features[i] + [c.labels[i]]) for i in range(c.n)]
    assert op.build_merkle_tree(leaves, 3)[-1][0] == c.root_D
    # features are randomInt(0,100): all in range, labels alternate (i + id) % 2
    assert all(0 <= x <= 100 for row in c.features for x in row)
    assert c.labels == [(i + 1) % 2 for i in range(8)]


def test_sgd_verified_reference_instance():
    """sgd_verified(8,4,3,1000) with the harness inputs (weights = 0, tau^2 = 1e8)."""
    b = circuits.build("sgd_verified", 8, 4, 3, 1000)
    c = _client()
    inp, grad = c.training_input(8, 1000, 100000000)
    w = ow.evaluate(b, inp)
    assert b.check_all(w)
    assert b.n_public == 6
    pub = [str(x) for x in w[1:7]]
    assert pub == [inp[k] for k in ("client_id", "round", "root_D", "root_G", "root_W", "tauSquared")]
    assert int(inp["root_G"]) == op.gradient_commitment([g % R for g in grad], 1, 1)


def test_sgd_verified_wrong_gradient_rejected():
    b = circuits.build("sgd_verified", 8, 4, 3, 1000)
    inp, _ = _client().training_input(8, 1000, 100000000)
    inp["remainder"][0] = str(int(inp["remainder"][0]) + 1)
    with pytest.raises(ow.AssertFailed):
        ow.evaluate(b, inp)


def test_sgd_verified_clipping_bound_enforced():
    b = circuits.build("sgd_verified", 8, 4, 3, 1000)
    inp, grad = _client().training_input(8, 1000, 100000000)
    inp["tauSquared"] = str(sum(g * g for g in grad) - 1)
    with pytest.raises(ow.AssertFailed):
        ow.evaluate(b, inp)


def test_balance_and_secagg():
    c = _client()
    bb = circuits.build("balance_unified", 8, 3, 4)
    assert bb.check_all(ow.evaluate(bb, c.balance_input()))
    bad = c.balance_input()
    bad["c1"] = str(int(bad["c1"]) + 1)
    with pytest.raises(ow.AssertFailed):
        ow.evaluate(bb, bad)
    _, grad = c.training_input(8, 1000, 100000000)
    sa = circuits.build("secure_masked_update", 4, 2)
    inp = clients.secagg_input(1, [2, 3], grad, 1, 100000000, c.root_D, 0)
    w = ow.evaluate(sa, inp)
    assert sa.check_all(w) and sa.n_public == 13


def test_secagg_masks_cancel():
    """3-client pairwise masks cancel in the sum (tests/test_secure_aggregation.mjs:215-238)."""
    grads = {1: [3, -4, 5, 0], 2: [-1, 2, 7, 9], 3: [10, 0, -2, 1]}
    ids = [1, 2, 3]
    total = [0, 0, 0, 0]
    for i in ids:
        inp = clients.secagg_input(i, [j for j in ids if j != i], grads[i], 1, 10**8, 0, 0)
        total = [(a + int(m)) % R for a, m in zip(total, inp["masked_update"])]
    want = [sum(grads[i][k] for i in ids) % R for k in range(4)]
    assert total == want


def test_r1cs_bytes_parse_with_oracle():
    b = circuits.build("poseidon_hash2")
    r = og.parse_r1cs(b.r1cs_bytes())
    assert r["nWires"] == b.n_wires and r["nConstraints"] == b.n_constraints
    assert r["nPubOut"] == 1 and r["nPrvIn"] == 2
    assert r["constraints"][0][0] == b.cons[0][0]


def test_metric_circuit_size():
    """M = TrainingStepVerified(128,4,7,1000): ~2^18 constraints, domain 2^18."""
    from zkfl.zkey import domain_size_for
    b = circuits.build("sgd_verified", 128, 4, 7, 1000)
    assert 2 ** 17 < b.n_constraints < 2 ** 18
    assert domain_size_for(b) == 2 ** 18


def test_sparse_merkle_tree_equals_padded_tree():
    """clients.MerkleTree keeps the Poseidon([0]) padding implicit; every node and proof equals the
    reference's fully padded tree (oracle build_merkle_tree, tests/full_system_simulation.mjs:198-238)."""
    leaves = [op.vector_hash([i, 2 * i, 3, 4, i % 2]) for i in range(11)]
    for depth in (4, 5):
        full = op.build_merkle_tree(leaves, depth)
        t = clients.merkle_tree(leaves, depth)
        assert t.root == full[-1][0]
        for lvl in range(depth + 1):
            assert [t.node(lvl, j) for j in range(len(full[lvl]))] == full[lvl]
        for idx in (0, 5, 10):
            assert clients.merkle_proof(t, idx, depth) == op.merkle_proof(full, idx, depth)


def test_federated_round_inputs_satisfy_circuits():
    """BASELINE config 5 inputs: 8 clients' training and SecureMaskedUpdate(4,7) inputs satisfy their
    circuits and the 8-way pairwise masks cancel (tests/full_system_simulation.mjs:1278-1343)."""
    rnd = clients.federated_round(8)
    sa = circuits.build("secure_masked_update", 4, 7)
    tr = circuits.build("sgd_verified", 8, 4, 3, 1000)
    total = [0] * 4
    for k, (t, s, g) in enumerate(rnd):
        if k in (0, 7):
            assert tr.check_all(ow.evaluate(tr, t))
            assert sa.check_all(ow.evaluate(sa, s))
        assert s["root_G"] == t["root_G"] and len(s["peer_ids"]) == 7
        total = [(a + int(m)) % R for a, m in zip(total, s["masked_update"])]
    assert total == [sum(g[k] for _, _, g in rnd) % R for k in range(4)]
