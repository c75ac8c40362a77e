"""The metric circuit M = sgd_verified(128, 4, 7, 1000) proven on the GPU and checked against the
C oracle (oracle/c/groth16_ref.c) at full size — MI355X (-m gpu).

Bar: bit-exact.  With fixed (r, s) the 256 proof bytes, the H-MSM scalars h (2^18 coset
evaluations) and the five plain MSM results (A, B1, B2, C, H) equal the oracle's.  The same key
is then driven the way bench.py drives it — 20 proof slots in flight over 28 hardware queues
(conftest.py sets GPU_MAX_HW_QUEUES before HIP initialises) — and every concurrent proof must
equal the same proof made alone on one slot, with a subset checked against the oracle again.
Reference call site: `npx snarkjs groth16 prove` (tests/full_system_simulation.mjs:773-776) on the
Report's N=128 training circuit (Report.pdf p.6 Table 5).
"""
import os
import secrets

import pytest

from oracle import bn254 as bn

pytestmark = pytest.mark.gpu

R = bn.R
PARAMS = (128, 4, 7, 1000)


def _le(x):
    return int(x).to_bytes(32, "little")


@pytest.fixture(scope="module")
def metric(gpu_ctx):
    from zkfl import circuits, clients, native, wprog, zkey
    b = circuits.build("sgd_verified", *PARAMS)
    zk = zkey.groth16_setup(b, gpu_ctx, zkey.Toxic(tau=0x5EED, alpha=0xA1, beta=0xB2, gamma=0xC3, delta=0xD4))
    key = native.ProvingKey(gpu_ctx, zk)
    wp = native.WitnessProgram(gpu_ctx, wprog.compile_program(b))
    inputs = []
    for cid in (1, 2, 3, 4):
        c = clients.Client(cid, 128, 4, 7, clients.JsLcg(12345 + cid))
        inputs.append(wprog.input_bytes(b, c.training_input(128, 1000, 100000000)[0]))
    wts = wp.compute(inputs)            # GPU witnesses (checked wire by wire in test_gpu_witness.py)
    yield b, zk, key, wp, wts
    wp.close()
    key.close()


def _threads():
    from oracle import cbaseline
    return cbaseline.default_threads()


def test_metric_proof_and_parts_bit_exact_vs_c_oracle(metric):
    from oracle import cbaseline
    b, zk, key, _, wts = metric
    assert key.domain_size == 1 << 18 and key.n_vars == b.n_wires
    for i, (r, s) in enumerate([(0x1234567, 0x7654321), (R - 1, R - 2)]):
        rs = _le(r) + _le(s)
        proof, pub = key.prove(wts[i], rs)
        ref, ref_h, ref_parts = cbaseline.prove_parts(zk, wts[i], rs, key.domain_size, _threads())
        assert proof == ref, f"client {i + 1}: proof bytes differ from the C oracle"
        hs, parts = key.debug_parts(wts[i])
        assert hs == ref_h, "h (coset evaluations a*b - c) differ"
        for name in ("A", "B1", "B2", "C", "H"):
            assert parts[name] == ref_parts[name], f"MSM {name} differs"
        assert len(pub) == 6 and pub[0] == i + 1


def test_metric_key_by_path_equals_key_by_bytes(metric, gpu_ctx, tmp_path):
    """zkfl_zkey_file_open + zkfl_zkey_load_file (the CLI's path: the key file mapped and parsed
    on host threads) make the same key as zkfl_zkey_load on its bytes: same proofs."""
    from zkfl import native
    _, zk, key, _, wts = metric
    p = tmp_path / "m_final.zkey"
    p.write_bytes(zk)
    k2 = native.ProvingKey(gpu_ctx, str(p))
    try:
        assert (k2.n_vars, k2.n_public, k2.domain_size) == (key.n_vars, key.n_public, key.domain_size)
        rs = _le(0xABCDEF) + _le(0x123457)
        assert k2.prove(wts[0], rs) == key.prove(wts[0], rs)
    finally:
        k2.close()


def test_metric_latency_schedule_equals_batch(metric):
    """A batch of one takes the latency schedule (enqueue_proof_lowlat: three streams, A / B1 and
    B2 beside ABC / NTT / C + H, k_assemble_t + k_assemble_c).  Repeated latency-schedule proofs
    of one resident witness equal the one-stream batch proof of the same (witness, r, s) -- which
    test_metric_proof_and_parts_bit_exact_vs_c_oracle pins to the C oracle."""
    _, _, key, _, wts = metric
    w = key.upload(wts[1])
    try:
        rs = _le(0x1111) + _le(0x2222)
        singles = [key.prove_batch([w], rs)[0] for _ in range(4)]
        pair = key.prove_batch([w, w], rs + rs)
        assert all(p == pair[0] for p in singles) and pair[0] == pair[1]
    finally:
        w.close()


def test_metric_concurrent_slots_equal_single_slot(metric):
    """bench.py's concurrency (20 slots x 1 stream each over 28 HW queues): 40 proofs with
    distinct fixed (r, s) from the batch prover equal one-at-a-time proofs; 2 vs the oracle."""
    from oracle import cbaseline
    _, zk, key, wp, wts = metric
    assert os.environ.get("GPU_MAX_HW_QUEUES") == "28"
    res = [key.upload(w) for w in wts]
    n = 40
    rs_list = [_le(secrets.randbelow(R)) + _le(secrets.randbelow(R)) for _ in range(n)]
    ws = [res[i % len(res)] for i in range(n)]
    key.set_slots(20)
    batch = key.prove_batch(ws, b"".join(rs_list))
    batch2 = key.prove_batch(ws[::-1], b"".join(rs_list[::-1]))   # slots re-used in another order
    key.set_slots(1)
    for i in range(n):
        single = key.prove_resident(ws[i], rs_list[i])
        assert batch[i] == single, f"proof {i}: 20-slot batch differs from the single-slot proof"
        assert batch2[n - 1 - i] == single
    for i in (0, 37):
        assert batch[i] == cbaseline.prove(zk, wts[i % len(wts)], rs_list[i], _threads())
    key.set_slots(3)
    for r_ in res:
        r_.close()


def test_metric_batch_verifies_on_gpu(metric, gpu_ctx):
    """CSPRNG blinding at 20 slots: every proof passes the GPU batch verifier; a tampered public
    signal and a swapped proof fail."""
    from zkfl import groth16, zkey
    _, zk, key, _, wts = metric
    res = [key.upload(w) for w in wts]
    key.set_slots(20)
    proofs = key.prove_batch([res[i % 4] for i in range(24)])
    key.set_slots(3)
    pubs = [zkey.read_wtns(w)[1:7] for w in wts]
    vk = groth16.vk_bytes(groth16.export_verification_key(zk, alphabeta=False))
    pub_b = b"".join(_le(x) for i in range(24) for x in pubs[i % 4])
    assert all(gpu_ctx.verify_batch(vk, pub_b, b"".join(proofs), 6))
    bad = list(proofs)
    bad[3], bad[4] = proofs[4], proofs[3]      # witnesses 3 and 0 have different publics
    ok = gpu_ctx.verify_batch(vk, pub_b, b"".join(bad), 6)
    assert ok[3] is False and ok[4] is False and all(ok[:3]) and all(ok[5:])
    for r_ in res:
        r_.close()


def test_metric_full_prove_pipeline(metric):
    """zkfl_groth16_full_prove_batch: input vectors -> witness on each slot's stream -> proof, at
    20 slots; equals witness-then-prove proof by proof (same r, s), public signals included."""
    from zkfl import circuits, clients, native, wprog
    _, _, key, wp, wts = metric
    b = circuits.build("sgd_verified", *PARAMS)
    objs = [clients.Client(cid, 128, 4, 7, clients.JsLcg(12345 + cid)).training_input(128, 1000, 100000000)[0]
            for cid in (1, 2, 3, 4)]
    import json
    image = wprog.compile_program(b)
    parsed = [native.parse_inputs(image, json.dumps(o)) for o in objs]
    assert parsed == [wprog.input_bytes(b, o) for o in objs]
    n = 24
    rs = [_le(secrets.randbelow(R)) + _le(secrets.randbelow(R)) for _ in range(n)]
    key.set_slots(20)
    out = key.full_prove_batch(wp, [parsed[i % 4] for i in range(n)], b"".join(rs))
    key.set_slots(3)
    res = [key.upload(w) for w in wts]
    for i, (proof, pub) in enumerate(out):
        assert proof == key.prove_resident(res[i % 4], rs[i])
        assert [str(x) for x in pub] == [objs[i % 4][k] for k in ("client_id", "round", "root_D", "root_G",
                                                                    "root_W", "tauSquared")]
    for r_ in res:
        r_.close()


def test_metric_full_prove_json_batch(metric):
    """zkfl_groth16_full_prove_json_batch: input.json texts parsed by host threads while earlier
    proofs run; 44 proofs at 20 slots equal the vector pipeline's (same r, s) proof by proof."""
    import json
    from zkfl import circuits, clients, wprog
    _, _, key, wp, _ = metric
    b = circuits.build("sgd_verified", *PARAMS)
    objs = [clients.Client(cid, 128, 4, 7, clients.JsLcg(12345 + cid)).training_input(128, 1000, 100000000)[0]
            for cid in (1, 2, 3, 4)]
    texts = [json.dumps(o) for o in objs]
    n = 44
    rs = [_le(secrets.randbelow(R)) + _le(secrets.randbelow(R)) for _ in range(n)]
    key.set_slots(20)
    got = key.full_prove_json_batch(wp, [texts[i % 4] for i in range(n)], b"".join(rs))
    want = key.full_prove_batch(wp, [wprog.input_bytes(b, objs[i % 4]) for i in range(n)], b"".join(rs))
    key.set_slots(3)
    assert got == want


def test_metric_full_prove_json_batch_reuses_witness_sets(metric):
    """4 slots x 20 texts = 5 slot-groups: the pipeline's three device witness sets are each taken
    again (groups 3 and 4) while earlier groups' proofs may still read theirs.  Every proof equals
    the one-at-a-time proof of the same witness and (r, s)."""
    import json
    from zkfl import clients
    _, _, key, wp, wts = metric
    objs = [clients.Client(cid, 128, 4, 7, clients.JsLcg(12345 + cid)).training_input(128, 1000, 100000000)[0]
            for cid in (1, 2, 3, 4)]
    order = [0, 1, 2, 3, 1, 0, 3, 2, 2, 2, 0, 1, 3, 3, 1, 0, 0, 3, 1, 2]
    rs = [_le(secrets.randbelow(R)) + _le(secrets.randbelow(R)) for _ in order]
    key.set_slots(4)
    got = key.full_prove_json_batch(wp, [json.dumps(objs[i]) for i in order], b"".join(rs))
    key.set_slots(1)
    res = [key.upload(w) for w in wts]
    for j, (i, (proof, pub)) in enumerate(zip(order, got)):
        assert proof == key.prove_resident(res[i], rs[j]), f"job {j} (client {i + 1})"
        assert pub[0] == i + 1
    key.set_slots(3)
    for r_ in res:
        r_.close()


def test_domain_2_19_proof_bit_exact_vs_c_oracle(gpu_ctx):
    """sgd_verified(124, 4, 8, 1000): 283,407 constraints (the Report's ~283 K circom count for
    N=128), domain 2^19 -- the 2x NTT / H-MSM size -- proof and all five MSMs equal the C oracle."""
    from oracle import cbaseline
    from zkfl import circuits, clients, native, wprog, zkey
    b = circuits.build("sgd_verified", 124, 4, 8, 1000)
    assert b.n_constraints > (1 << 18)
    zk = zkey.groth16_setup(b, gpu_ctx, zkey.Toxic(tau=0x19, alpha=0xA1, beta=0xB2, gamma=0xC3, delta=0xD4))
    key = native.ProvingKey(gpu_ctx, zk)
    wp = native.WitnessProgram(gpu_ctx, wprog.compile_program(b))
    c = clients.Client(5, 124, 4, 8, clients.JsLcg(12350))
    wt = wp.compute([wprog.input_bytes(b, c.training_input(124, 1000, 100000000)[0])])[0]
    assert key.domain_size == 1 << 19
    rs = _le(0xABCDEF) + _le(0xFEDCBA)
    proof, pub = key.prove(wt, rs)
    ref, ref_h, ref_parts = cbaseline.prove_parts(zk, wt, rs, key.domain_size, _threads())
    assert proof == ref
    hs, parts = key.debug_parts(wt)
    assert hs == ref_h
    for name in ("A", "B1", "B2", "C", "H"):
        assert parts[name] == ref_parts[name], name
    assert pub[0] == 5
    wp.close()
    key.close()


def test_full_prove_json_batch_errors(gpu_ctx):
    """A malformed / incomplete text at index k: ZKFL_E_ARG naming input k; the key keeps working."""
    import json
    from zkfl import circuits, clients, native, wprog, zkey
    b = circuits.build("sgd_verified", 8, 4, 3, 1000)
    zk = zkey.groth16_setup(b, gpu_ctx, zkey.Toxic(tau=98, alpha=2, beta=3, gamma=4, delta=5))
    key = native.ProvingKey(gpu_ctx, zk)
    wp = native.WitnessProgram(gpu_ctx, wprog.compile_program(b))
    good = [json.dumps(clients.Client(c, 8, 4, 3, clients.JsLcg(12345 + c)).training_input(8, 1000, 100000000)[0])
            for c in (1, 2)]
    missing = json.loads(good[0])
    del missing["remainder"]
    key.set_slots(4)
    for bad in ('{"client_id": 1', json.dumps(missing)):
        with pytest.raises(native.ZkflError) as e:
            key.full_prove_json_batch(wp, [good[0], good[1], good[0], bad, good[1]])
        assert e.value.code == -1 and "input 3" in str(e.value)
    rs = _le(5) + _le(6)
    (p, pub), = key.full_prove_json_batch(wp, [good[1]], rs)
    assert (p, pub) == key.full_prove_batch(wp, [native.parse_inputs(wprog.compile_program(b), good[1])], rs)[0]
    wp.close()
    key.close()


def test_full_prove_constraint_failure_and_recovery(gpu_ctx):
    """One unsatisfiable witness in a batch: ZKFL_E_CONSTRAINT names it; the key keeps working."""
    from zkfl import circuits, clients, native, wprog, zkey
    b = circuits.build("sgd_verified", 8, 4, 3, 1000)
    zk = zkey.groth16_setup(b, gpu_ctx, zkey.Toxic(tau=99, alpha=2, beta=3, gamma=4, delta=5))
    key = native.ProvingKey(gpu_ctx, zk)
    wp = native.WitnessProgram(gpu_ctx, wprog.compile_program(b))
    good = [clients.Client(c, 8, 4, 3, clients.JsLcg(12345 + c)).training_input(8, 1000, 100000000)[0]
            for c in (1, 2, 3)]
    bad = dict(good[1])
    bad["remainder"] = list(bad["remainder"])
    bad["remainder"][0] = str(int(bad["remainder"][0]) + 1)
    key.set_slots(4)
    with pytest.raises(native.ZkflError) as e:
        key.full_prove_batch(wp, [wprog.input_bytes(b, x) for x in (good[0], good[2], bad, good[1], good[0])])
    assert e.value.code == -7 and "witness 2" in str(e.value)
    with pytest.raises(native.ZkflError) as e:          # input >= r: rejected before any work
        key.full_prove_batch(wp, [b"\xff" * 32 + wprog.input_bytes(b, good[0])[32:]])
    assert e.value.code == -1
    rs = _le(5) + _le(6)
    (p, pub), = key.full_prove_batch(wp, [wprog.input_bytes(b, good[0])], rs)
    assert p == key.prove(wp.compute([wprog.input_bytes(b, good[0])])[0], rs)[0]
    assert [str(x) for x in pub][:2] == [good[0]["client_id"], good[0]["round"]]
    wp.close()
    key.close()
