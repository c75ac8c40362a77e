"""BASELINE configs 3, 4 and 5 proven on the GPU and checked against the oracles — MI355X (-m gpu).

Bar: bit-exact.  Witnesses equal oracle/witness.py wire by wire; with fixed (r, s) every proof equals
the C oracle's (oracle/c/groth16_ref.c) over the same zkey and witness; every proof passes the GPU
verifier and the public signals carry what the reference's server checks.

* Config 3 — BalanceProofUnified(32, 16, 4) (src/circuits/balance/balance_unified.circom:74-180): a
  Poseidon Merkle inclusion proof of depth 16 for each of 32 samples, 134,755 constraints, domain 2^18
  (SURVEY.md §8d C3).  Leaves padded with Poseidon([0]) (tests/full_system_simulation.mjs:198-223);
  the server's checks of the balance publics [client_id, root, N_public, c0, c1] (:340-366).
* Config 4 — three SecureMaskedUpdate(4, 2) proofs (secure_masked_update.circom:231-343), mask
  cancellation checked on the masked_update public signals the GPU proofs carry
  (tests/test_secure_aggregation.mjs:215-238; publics per tests/full_system_simulation.mjs:1040-1107).
* Config 5 — one federated round of 8 clients x {training sgd_verified(8,4,3), secure aggregation
  SecureMaskedUpdate(4,7)} (tests/full_system_simulation.mjs:1298-1343): both keys resident, the 16
  proofs interleaved on one GPU through zkfl_groth16_full_prove_multi (input vectors -> witness ->
  proof per slot).  Each equals the single-key single-slot proof of the same witness and (r, s).
"""
import json
import secrets

import pytest

from oracle import bn254 as bn
from oracle import witness as ow

pytestmark = pytest.mark.gpu

R = bn.R
TAU_SQ = 100000000      # CONFIG.TAU_SQUARED (tests/full_system_simulation.mjs:47-51)


def _le(x):
    return int(x).to_bytes(32, "little")


def _threads():
    from oracle import cbaseline
    return cbaseline.default_threads()


def _key(ctx, b, seed):
    from zkfl import native, wprog, zkey
    zk = zkey.groth16_setup(b, ctx, zkey.Toxic(tau=seed, alpha=seed + 1, beta=seed + 2, gamma=seed + 3,
                                               delta=seed + 4))
    return zk, native.ProvingKey(ctx, zk), native.WitnessProgram(ctx, wprog.compile_program(b))


def _vk(zk):
    from zkfl import groth16
    return groth16.vk_bytes(groth16.export_verification_key(zk, alphabeta=False))


# ---------------------------------------------------------------------------
# Config 3: depth-16 balance proof
# ---------------------------------------------------------------------------
def test_config3_balance_depth16_vs_oracle(gpu_ctx):
    from oracle import cbaseline
    from zkfl import circuits, clients, wprog, zkey
    b = circuits.build("balance_unified", 32, 16, 4)
    assert 2 ** 17 <= b.n_constraints < 2 ** 18
    zk, key, wp = _key(gpu_ctx, b, 0xBA1)
    assert key.domain_size == 1 << 18
    cl = [clients.Client(cid, 32, 4, 16, clients.JsLcg(12345 + cid)) for cid in (1, 2)]
    objs = [c.balance_input() for c in cl]
    wts = wp.compute([wprog.input_bytes(b, o) for o in objs])
    assert zkey.read_wtns(wts[0]) == ow.evaluate(b, objs[0])     # GPU witness, every wire
    vk = _vk(zk)
    for c, o, wt, (r, s) in zip(cl, objs, wts, [(0xB0B, 0xCAFE), (R - 3, 17)]):
        rs = _le(r) + _le(s)
        proof, pub = key.prove(wt, rs)
        ref, ref_h, ref_parts = cbaseline.prove_parts(zk, wt, rs, key.domain_size, _threads())
        assert proof == ref, f"client {c.id}: proof differs from the C oracle"
        hs, parts = key.debug_parts(wt)
        assert hs == ref_h and parts == ref_parts
        # the server's balance checks (verifyBalanceProof): publics = [client_id, root, N, c0, c1]
        assert pub == [c.id, c.root_D, 32, c.c0, c.c1] and c.c0 + c.c1 == 32
        pb = b"".join(_le(x) for x in pub)
        assert gpu_ctx.verify(vk, pb, proof)
        bad = b"".join(_le(x) for x in [c.id, c.root_D, 32, c.c0 + 1, c.c1 - 1])
        assert not gpu_ctx.verify(vk, bad, proof)
    # a sample outside the committed dataset: its leaf's path no longer reaches root_D
    forged = dict(objs[0])
    forged["features"] = [list(r) for r in forged["features"]]
    forged["features"][5][2] = str(int(forged["features"][5][2]) + 1)
    from zkfl import native
    with pytest.raises(native.ZkflError) as e:
        wp.compute([wprog.input_bytes(b, forged)])
    assert e.value.code == -7
    wp.close()
    key.close()


# ---------------------------------------------------------------------------
# Config 4: 3-client secure aggregation, masks cancel on the proven publics
# ---------------------------------------------------------------------------
def test_config4_secagg_three_clients_mask_cancel(gpu_ctx):
    from oracle import cbaseline
    from zkfl import circuits, clients, native, wprog, zkey
    b = circuits.build("secure_masked_update", 4, 2)
    zk, key, wp = _key(gpu_ctx, b, 0x5EC)
    image = wprog.compile_program(b)
    ids = [1, 2, 3]
    # negative entries as the reference's clipped gradients have them (wrapped mod r in the input)
    grads = {1: [73, -79, 90, -14], 2: [-98, 74, 61, -71], 3: [98, 95, -48, 53]}
    objs = [clients.secagg_input(i, [j for j in ids if j != i], grads[i], 1, TAU_SQ, 1000 + i, 2000 + i)
            for i in ids]
    inputs = [native.parse_inputs(image, json.dumps(o)) for o in objs]   # the C input.json parser
    assert inputs == [wprog.input_bytes(b, o) for o in objs]
    rs = [_le(secrets.randbelow(R)) + _le(secrets.randbelow(R)) for _ in ids]
    key.set_slots(3)
    out = key.full_prove_batch(wp, inputs, b"".join(rs))
    wts = wp.compute(inputs)
    vk = _vk(zk)
    total = [0] * 4
    for i, o, wt, r_s, (proof, pub) in zip(ids, objs, wts, rs, out):
        assert zkey.read_wtns(wt) == ow.evaluate(b, o)
        assert proof == cbaseline.prove(zk, wt, r_s, _threads()), f"client {i}: differs from the C oracle"
        assert len(pub) == 13 and pub[0] == i and pub[11:13] == [j for j in ids if j != i]
        assert gpu_ctx.verify(vk, b"".join(_le(x) for x in pub), proof)
        total = [(t + m) % R for t, m in zip(total, pub[7:11])]          # masked_update[4]
    assert total == [sum(grads[i][k] for i in ids) % R for k in range(4)], "masks do not cancel"
    # a client lying about its masked update cannot prove it
    bad = dict(objs[0])
    bad["masked_update"] = [str((int(bad["masked_update"][0]) + 1) % R)] + bad["masked_update"][1:]
    with pytest.raises(native.ZkflError) as e:
        key.full_prove_batch(wp, [wprog.input_bytes(b, bad)])
    assert e.value.code == -7
    wp.close()
    key.close()


# ---------------------------------------------------------------------------
# Config 5: one federated round, 8 clients x {training, secagg}, keys interleaved
# ---------------------------------------------------------------------------
def test_config5_round_interleaved_multi_key(gpu_ctx):
    from oracle import cbaseline
    from zkfl import circuits, clients, native, wprog, zkey
    bt = circuits.build("sgd_verified", 8, 4, 3, 1000)
    bs = circuits.build("secure_masked_update", 4, 7)
    zk_t, key_t, wp_t = _key(gpu_ctx, bt, 0x7A1)
    zk_s, key_s, wp_s = _key(gpu_ctx, bs, 0x5A6)
    rnd = clients.federated_round(8)
    jobs, objs = [], []
    for tr, sa, _ in rnd:          # client k: training proof, then its secure-aggregation proof
        jobs.append((key_t, wp_t, wprog.input_bytes(bt, tr)))
        jobs.append((key_s, wp_s, wprog.input_bytes(bs, sa)))
        objs += [tr, sa]
    rs = [_le(secrets.randbelow(R)) + _le(secrets.randbelow(R)) for _ in jobs]
    key_t.set_slots(8)
    key_s.set_slots(8)
    out = gpu_ctx.full_prove_multi(jobs, b"".join(rs))
    assert len(out) == 16
    # every interleaved proof == the same witness proven alone on one slot of its key
    key_t.set_slots(1)
    key_s.set_slots(1)
    vk = {id(key_t): _vk(zk_t), id(key_s): _vk(zk_s)}
    total = [0] * 4
    for i, ((k, wp, inp), o, r_s, (proof, pub)) in enumerate(zip(jobs, objs, rs, out)):
        wt = wp.compute([inp])[0]
        w = k.upload(wt)
        assert proof == k.prove_resident(w, r_s), f"job {i}: interleaved proof differs from the single-slot proof"
        w.close()
        assert pub == zkey.read_wtns(wt)[1:1 + k.n_public]
        assert gpu_ctx.verify(vk[id(k)], b"".join(_le(x) for x in pub), proof)
        if i in (0, 1, 15):
            zk = zk_t if k is key_t else zk_s
            assert proof == cbaseline.prove(zk, wt, r_s, _threads()), f"job {i}: differs from the C oracle"
        if k is key_t:
            assert [str(x) for x in pub] == [o[f] for f in ("client_id", "round", "root_D", "root_G", "root_W",
                                                           "tauSquared")]
        else:
            total = [(t + m) % R for t, m in zip(total, pub[7:11])]
    assert total == [sum(g[k] for _, _, g in rnd) % R for k in range(4)], "8-client masks do not cancel"
    assert ow.evaluate(bs, objs[1]) == zkey.read_wtns(wp_s.compute([jobs[1][2]])[0])

    # the witness pipes at small slot counts: several groups per key, a ragged last group
    key_t.set_slots(3)
    key_s.set_slots(2)
    assert gpu_ctx.full_prove_multi(jobs, b"".join(rs)) == out
    wp_t2 = native.WitnessProgram(gpu_ctx, wprog.compile_program(bt))   # the same key, another program
    with pytest.raises(native.ZkflError) as e:
        gpu_ctx.full_prove_multi([jobs[0], (key_t, wp_t2, jobs[2][2])])
    assert e.value.code == -1
    wp_t2.close()
    bad = dict(objs[4])                                # client 2's training input, made unsatisfiable
    bad["remainder"] = list(bad["remainder"])
    bad["remainder"][0] = str(int(bad["remainder"][0]) + 1)
    with pytest.raises(native.ZkflError) as e:         # job 12 sits in key_t's third group
        gpu_ctx.full_prove_multi(jobs[:12] + [(key_t, wp_t, wprog.input_bytes(bt, bad))] + jobs[13:])
    assert e.value.code == -7 and "witness 12" in str(e.value)
    assert gpu_ctx.full_prove_multi(jobs[:4], b"".join(rs[:4])) == out[:4]   # keys keep working

    # resident-witness form of the same round: zkfl_groth16_prove_multi
    res = [k.upload(wp.compute([inp])[0]) for k, wp, inp in jobs]
    key_t.set_slots(8)
    key_s.set_slots(8)
    proofs = gpu_ctx.prove_multi([(k, w) for (k, _, _), w in zip(jobs, res)], b"".join(rs))
    assert proofs == [p for p, _ in out]
    with pytest.raises(native.ZkflError):           # a witness uploaded for the other key
        gpu_ctx.prove_multi([(key_s, res[0])])
    for w in res:
        w.close()
    for x in (wp_t, wp_s, key_t, key_s):
        x.close()
