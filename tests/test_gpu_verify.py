"""GPU verifier and pairing (zkfl_groth16_verify / _batch, zkfl_pairing) vs the oracle — MI355X.

Bar: GT elements and Miller-loop values bit-identical to oracle/pairing_tower.py (itself pinned
to oracle/bn254.py's independent pairing by tests/test_pairing_tower.py); verification verdicts
equal to oracle/groth16.py::verify on valid, tampered and malformed proofs (snarkjs groth16
verify semantics, tests/full_system_simulation.mjs:865-868).
"""
import json
import os
import random
import shutil
import subprocess

import pytest

from oracle import witness as ow

from oracle import bn254 as bn
from oracle import groth16 as og
from oracle import pairing_tower as T

pytestmark = pytest.mark.gpu

R, Q = bn.R, bn.Q


def _g1b(P):
    return bn.g1_to_bytes_std(P)


def _g2b(Qg):
    return bn.g2_to_bytes_std(Qg)


def _fq2_sqrt(a):
    """sqrt in Fq2 (q = 3 mod 4) or None."""
    a0, a1 = a.c0, a.c1
    n = (a0 * a0 + a1 * a1) % Q
    s = pow(n, (Q + 1) // 4, Q)
    if s * s % Q != n:
        return None
    for t in (s, -s % Q):
        x0sq = (a0 + t) * pow(2, -1, Q) % Q
        x0 = pow(x0sq, (Q + 1) // 4, Q)
        if x0 * x0 % Q == x0sq and x0:
            x1 = a1 * pow(2 * x0, -1, Q) % Q
            r = bn.Fq2(x0, x1)
            if r * r == a:
                return r
    return None


def _twist_point_outside_g2(seed=5):
    """A point on y^2 = x^3 + b' over Fq2 that is not in the order-r subgroup."""
    x = seed
    while True:
        X = bn.Fq2(x, 1)
        Y = _fq2_sqrt(X * X * X + bn.B2)
        if Y is not None:
            P = (X, Y)
            assert bn.on_curve(P)
            acc, base, k = None, bn.to_jac(P), R  # [r]P by hand (bn.mul reduces k mod r)
            while k:
                if k & 1:
                    acc = bn.jadd(acc, base)
                base = bn.jdouble(base)
                k >>= 1
            if bn.from_jac(acc) is not None:
                return P
        x += 1


# ---------------------------------------------------------------------------
# pairing primitive
# ---------------------------------------------------------------------------
def test_pairing_and_miller_bit_exact_vs_tower(gpu_ctx):
    rng = random.Random(7)
    Ps = [bn.G1_GEN] + [bn.mul(bn.G1_GEN, rng.randrange(1, R)) for _ in range(69)]
    Qs = [bn.G2_GEN] + [bn.mul(bn.G2_GEN, rng.randrange(1, R)) for _ in range(69)]
    g1 = b"".join(_g1b(P) for P in Ps)
    g2 = b"".join(_g2b(Qg) for Qg in Qs)
    ml = gpu_ctx.pairing(g1, g2, final_exp=False)
    gt = gpu_ctx.pairing(g1, g2)
    for i in (0, 1, 2, 69):  # the Python tower is slow; a few lanes incl. two wavefronts
        f = T.miller_loop([(Ps[i], T.from_bn254_g2(Qs[i]))])
        assert ml[384 * i:384 * i + 384] == T.gt_bytes(f), i
        assert gt[384 * i:384 * i + 384] == T.gt_bytes(T.final_exp(f)), i
    # the oracle's independent pairing agrees on lane 1
    assert T.to_bn254_fq12(T.gt_from_bytes(gt[384:768])) == bn.pairing(Ps[1], Qs[1])
    # bilinearity across lanes: e(aG, H) == e(G, aH)
    a = rng.randrange(1, R)
    gt2 = gpu_ctx.pairing(_g1b(bn.mul(bn.G1_GEN, a)) + _g1b(bn.G1_GEN),
                          _g2b(bn.G2_GEN) + _g2b(bn.mul(bn.G2_GEN, a)))
    assert gt2[:384] == gt2[384:]


def test_pairing_infinity_and_invalid(gpu_ctx):
    from zkfl import native
    one = T.gt_bytes(T.F12_ONE)
    gt = gpu_ctx.pairing(bytes(64) + _g1b(bn.G1_GEN), _g2b(bn.G2_GEN) + bytes(128))
    assert gt == one + one
    with pytest.raises(native.ZkflError) as e:  # off-curve G1
        gpu_ctx.pairing(_le(1) + _le(3), _g2b(bn.G2_GEN))
    assert e.value.code == -1
    with pytest.raises(native.ZkflError) as e:  # on the twist, outside G2
        gpu_ctx.pairing(_g1b(bn.G1_GEN), _g2b(_twist_point_outside_g2()))
    assert e.value.code == -1


def _le(x):
    return int(x).to_bytes(32, "little")


# ---------------------------------------------------------------------------
# Groth16 verification
# ---------------------------------------------------------------------------
def _setup_and_prove(gpu_ctx, name, *params, inputs, n_proofs=1):
    from zkfl import circuits, native, zkey
    b = circuits.build(name, *params)
    zk = zkey.groth16_setup(b, gpu_ctx, zkey.Toxic(tau=4242, alpha=9, beta=10, gamma=11, delta=12))
    key = native.ProvingKey(gpu_ctx, zk)
    w = ow.evaluate(b, inputs)
    out = [key.prove(zkey.wtns_bytes(w)) for _ in range(n_proofs)]
    key.close()
    return zk, out


def test_verify_valid_and_tampered(gpu_ctx):
    from zkfl import groth16
    zk, [(proof, pub)] = _setup_and_prove(gpu_ctx, "poseidon_hash2", inputs={"left": 3, "right": 4})
    vkj = groth16.export_verification_key(zk, ctx=gpu_ctx)
    vk = groth16.vk_bytes(vkj)
    pubb = b"".join(_le(x) for x in pub)
    z = og.parse_zkey(zk)
    assert gpu_ctx.verify(vk, pubb, proof) is True
    # snarkjs-shaped API
    pj = groth16.proof_to_json(proof)
    p = groth16.Prover.__new__(groth16.Prover)
    p.ctx = gpu_ctx
    assert p.verify(vkj, [str(x) for x in pub], pj)
    # wrong public signal
    assert gpu_ctx.verify(vk, _le(pub[0] + 1), proof) is False
    # public signal >= r (snarkjs publicInputsAreValid)
    assert gpu_ctx.verify(vk, _le(pub[0] + R), proof) is False
    # tampered pi_c (another valid point), pi_a off-curve, coordinate >= q
    pc = bn.add(bn.g1_from_bytes_std(proof[192:256]), bn.G1_GEN)
    bad_c = proof[:192] + _g1b(pc)
    assert gpu_ctx.verify(vk, pubb, bad_c) is False
    assert not og.verify(z, pub, bn.g1_from_bytes_std(proof[:64]), bn.g2_from_bytes_std(proof[64:192]), pc)
    assert gpu_ctx.verify(vk, pubb, _le(1) + _le(5) + proof[64:]) is False
    assert gpu_ctx.verify(vk, pubb, _le(bn.G1_GEN[0] + Q) + proof[32:]) is False
    # pi_b swapped for a twist point outside G2
    assert gpu_ctx.verify(vk, pubb, proof[:64] + _g2b(_twist_point_outside_g2()) + proof[192:]) is False
    # vk_alphabeta_12 = e(alpha1, beta2), ffjavascript layout
    h = og.parse_zkey(zk)
    assert vkj["vk_alphabeta_12"] == T.vk_alphabeta_json(h["alpha1"], h["beta2"])


def test_verify_errors(gpu_ctx):
    from zkfl import groth16, native
    zk, [(proof, pub)] = _setup_and_prove(gpu_ctx, "poseidon_hash2", inputs={"left": 1, "right": 2})
    vk = groth16.vk_bytes(groth16.export_verification_key(zk, alphabeta=False))
    with pytest.raises(native.ZkflError) as e:  # truncated vk
        gpu_ctx.verify(vk[:-10], _le(pub[0]), proof)
    assert e.value.code == -2
    with pytest.raises(native.ZkflError) as e:  # npub != nPublic
        gpu_ctx.verify(vk, _le(pub[0]) + _le(1), proof)
    assert e.value.code == -4
    bad = bytearray(vk)
    bad[4:36] = _le(12345)  # alpha1 off curve
    with pytest.raises(native.ZkflError) as e:
        gpu_ctx.verify(bytes(bad), _le(pub[0]), proof)
    assert e.value.code == -2
    assert gpu_ctx.verify(vk, _le(pub[0]), proof) is True  # the cache recovers after a bad key


def test_verify_batch_matches_oracle(gpu_ctx):
    """sgd_verified(8,4,3): 6 public signals (4-bit-window vk_x over 6 IC tables); a batch of
    100 (two wavefronts) mixing valid proofs, tampered publics and tampered points."""
    from zkfl import clients, groth16
    c = clients.Client(1, 8, 4, 3, clients.JsLcg(12345))
    inp, _ = c.training_input(8, 1000, 100000000)
    zk, proofs = _setup_and_prove(gpu_ctx, "sgd_verified", 8, 4, 3, 1000, inputs=inp, n_proofs=2)
    vk = groth16.vk_bytes(groth16.export_verification_key(zk, alphabeta=False))
    z = og.parse_zkey(zk)
    rng = random.Random(3)
    prs, pubs, want = [], [], []
    for i in range(100):
        proof, pub = proofs[i % 2]
        pub = list(pub)
        kind = rng.randrange(4)
        if kind == 1:
            j = rng.randrange(len(pub))
            pub[j] = (pub[j] + 1) % R
        elif kind == 2:
            proof = _g1b(bn.neg(bn.g1_from_bytes_std(proof[:64]))) + proof[64:]
        prs.append(proof)
        pubs.append(b"".join(_le(x) for x in pub))
        want.append(kind in (0, 3))
    got = gpu_ctx.verify_batch(vk, b"".join(pubs), b"".join(prs), 6)
    assert got == want
    # the oracle agrees on one valid and one invalid entry
    for i in (want.index(True), want.index(False)):
        pub = [int.from_bytes(pubs[i][32 * j:32 * j + 32], "little") for j in range(6)]
        p = prs[i]
        assert og.verify(z, pub, bn.g1_from_bytes_std(p[:64]), bn.g2_from_bytes_std(p[64:192]),
                         bn.g1_from_bytes_std(p[192:])) == want[i]


def test_node_snarkjs_cli_verify(gpu_ctx, tmp_path):
    """`node snarkjs_shim.js groth16 verify vkey.json public.json proof.json` — exit 0 on a valid
    proof, 1 on an invalid one (tests/full_system_simulation.mjs:865-873 checks the exit code)."""
    from zkfl import groth16, native
    node = shutil.which("node")
    shim = os.path.join(os.path.dirname(native.LIB_PATH), "node", "snarkjs_shim.js")
    if not node or not os.path.exists(os.path.join(os.path.dirname(shim), "zkfl.node")):
        pytest.skip("node / addon not available")
    zk, [(proof, pub)] = _setup_and_prove(gpu_ctx, "poseidon_hash2", inputs={"left": 8, "right": 9})
    (tmp_path / "vkey.json").write_text(json.dumps(groth16.export_verification_key(zk, ctx=gpu_ctx)))
    (tmp_path / "proof.json").write_text(json.dumps(groth16.proof_to_json(proof)))
    (tmp_path / "public.json").write_text(json.dumps([str(x) for x in pub]))
    (tmp_path / "bad.json").write_text(json.dumps([str(pub[0] + 1)]))
    ok = subprocess.run([node, shim, "groth16", "verify", "vkey.json", "public.json", "proof.json"],
                        cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert ok.returncode == 0 and "OK!" in ok.stdout, ok.stderr
    bad = subprocess.run([node, shim, "groth16", "verify", "vkey.json", "bad.json", "proof.json"],
                         cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert bad.returncode == 1 and "Invalid proof" in bad.stderr
