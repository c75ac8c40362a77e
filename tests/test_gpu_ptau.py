"""Ceremony on the GPU: zkfl_setup_* primitives vs the oracle, `powersoftau` + `groth16 setup` +
`zkey contribute` vs the CPU path and the known-tau ceremony, proofs from ptau-derived keys — MI355X.

The reference cannot prove without this: `Client._runZKProof` looks for pot17/pot14_final.ptau
(tests/full_system_simulation.mjs:677-695) and sets every circuit up from it (:713-730); the full
ceremony is tests/test_secureagg.cjs:25-64.  The Node strings themselves run in
tests/test_gpu_node_ceremony.py.
"""
import random

import pytest

from oracle import bn254 as bn
from oracle import groth16 as og
from oracle import ptau as op
from oracle_backend import OraclePoints
from zkfl import circuits, native, ptau, wprog, zkey

pytestmark = pytest.mark.gpu

TAU, ALPHA, BETA, DELTA = 0x2468ACE13579, 0x1111, 0x2222, 0x3333


@pytest.fixture(scope="module")
def ctx():
    c = native.Context(0)
    yield c
    c.close()


def _rand_g1(rng, k):
    return [None if i % 7 == 3 else bn.mul(bn.G1_GEN, rng.randrange(1, bn.R)) for i in range(k)]


def _rand_g2(rng, k):
    return [None if i % 5 == 2 else bn.mul(bn.G2_GEN, rng.randrange(1, bn.R)) for i in range(k)]


def _enc1(pts):
    return b"".join(bn.g1_to_bytes_mont(p) for p in pts)


def _enc2(pts):
    return b"".join(bn.g2_to_bytes_mont(p) for p in pts)


def _sc(ks):
    return b"".join(int(k).to_bytes(32, "little") for k in ks)


def test_scale_vs_oracle(ctx):
    rng = random.Random(1)
    p1 = _rand_g1(rng, 40)
    k1 = [0, 1, 2, bn.R - 1, bn.R, (1 << 256) - 1] + [rng.randrange(1 << 256) for _ in range(34)]
    assert ctx.g1_scale(_enc1(p1), _sc(k1)) == _enc1([bn.mul(p, k) for p, k in zip(p1, k1)])
    p2 = _rand_g2(rng, 12)
    k2 = [0, 1, bn.R - 1] + [rng.randrange(bn.R) for _ in range(9)]
    assert ctx.g2_scale(_enc2(p2), _sc(k2)) == _enc2([bn.mul(p, k) for p, k in zip(p2, k2)])
    assert ctx.g1_scale(b"", b"") == b""


@pytest.mark.parametrize("logn", [0, 1, 2, 5])
def test_lagrange_vs_oracle(ctx, logn):
    rng = random.Random(10 + logn)
    pts = _rand_g1(rng, 1 << logn)
    assert ctx.g1_lagrange(_enc1(pts), logn) == _enc1(op.group_ifft(pts, logn))
    if logn <= 2:
        q = _rand_g2(rng, 1 << logn)
        assert ctx.g2_lagrange(_enc2(q), logn) == _enc2(op.group_ifft(q, logn))


def test_lincomb_vs_oracle(ctx):
    """Rows: empty, one term, a 300-term row (three reduction levels), zero and one coefficients,
    repeated bases, infinity bases."""
    rng = random.Random(7)
    bases = _rand_g1(rng, 24)
    lens = [0, 1, 300, 5, 0, 17, 2, 9]
    rowptr, idx, coefs = [0], [], []
    for ln in lens:
        for _ in range(ln):
            idx.append(rng.randrange(len(bases)))
            coefs.append(rng.choice([0, 1, bn.R - 1, rng.randrange(bn.R)]))
        rowptr.append(len(idx))
    got = ctx.g1_lincomb(_enc1(bases), rowptr, idx, _sc(coefs))
    ref = []
    for r in range(len(lens)):
        acc = None
        for t in range(rowptr[r], rowptr[r + 1]):
            acc = bn.add(acc, bn.mul(bases[idx[t]], coefs[t]))
        ref.append(acc)
    assert got == _enc1(ref)
    b2 = _rand_g2(rng, 6)
    rp2, ix2, c2 = [0, 3, 3, 40], [0, 1, 2] + [rng.randrange(6) for _ in range(37)], [rng.randrange(bn.R) for _ in range(40)]
    ref2 = []
    for r in range(3):
        acc = None
        for t in range(rp2[r], rp2[r + 1]):
            acc = bn.add(acc, bn.mul(b2[ix2[t]], c2[t]))
        ref2.append(acc)
    assert ctx.g2_lincomb(_enc2(b2), rp2, ix2, _sc(c2)) == _enc2(ref2)
    with pytest.raises(native.ZkflError):
        ctx.g1_lincomb(_enc1(bases), [0, 1], [24], _sc([1]))      # base index out of range


def test_ceremony_gpu_equals_cpu_path(ctx, monkeypatch):
    """powersoftau new -> contribute -> prepare phase2 -> groth16 setup -> zkey contribute at
    power 3 on the GPU: byte-identical files to the same code over the oracle's points."""
    monkeypatch.setenv("ZKFL_DETERMINISTIC_SETUP", "1")
    from test_ptau_cpu import tiny_circuit
    be = OraclePoints()
    files = {}
    for name, c in (("gpu", ctx), ("cpu", be)):
        p1 = ptau.contribute(ptau.new(3), c, TAU, ALPHA, BETA, name="codex-test")
        p2 = ptau.prepare_phase2(p1, c)
        zk = zkey.zkey_contribute(zkey.setup_from_ptau(tiny_circuit(), p2, c), c, DELTA, name="test")
        files[name] = (p1, p2, zk)
    assert files["gpu"] == files["cpu"]


def test_poseidon_key_from_ptau_equals_known_tau_and_proves(ctx):
    """PoseidonHash2 (domain 2^8) from a power-9 ptau: every Lagrange block exact, so the key is
    byte-identical to the known-tau ceremony (gamma = 1, delta = d after `zkey contribute`); its GPU
    proof equals the oracle's and verifies."""
    b = circuits.build("poseidon_hash2")
    p2 = ptau.prepare_phase2(ptau.contribute(ptau.new(9), ctx, TAU, ALPHA, BETA), ctx)
    zk = zkey.zkey_contribute(zkey.setup_from_ptau(b, p2, ctx), ctx, DELTA)
    known = zkey.groth16_setup(b, ctx, zkey.Toxic(tau=TAU, alpha=ALPHA, beta=BETA, gamma=1, delta=DELTA))
    sz, sk = ptau.read_sections(zk, b"zkey"), ptau.read_sections(known, b"zkey")
    for t in range(1, 10):
        assert zk[sz[t][0]:sz[t][0] + sz[t][1]] == known[sk[t][0]:sk[t][0] + sk[t][1]], t
    _prove_and_check(ctx, b, zk, {"left": 1, "right": 2})


def test_key_from_full_power_ptau_proves(ctx):
    """power 8 == the circuit's: H from snarkjs's truncated top block; proofs still verify."""
    b = circuits.build("poseidon_hash2")
    p2 = ptau.prepare_phase2(ptau.contribute(ptau.new(8), ctx, TAU, ALPHA, BETA), ctx)
    zk = zkey.zkey_contribute(zkey.setup_from_ptau(b, p2, ctx), ctx, DELTA)
    _prove_and_check(ctx, b, zk, {"left": 5, "right": 77})
    with pytest.raises(ValueError, match="too big"):
        zkey.setup_from_ptau(b, ptau.prepare_phase2(ptau.new(7), ctx), ctx)


def _prove_and_check(ctx, b, zk, inp):
    from zkfl import groth16
    from oracle import witness as ow
    wp = native.WitnessProgram(ctx, wprog.compile_program(b))
    wt = wp.compute([wprog.input_bytes(b, inp)])[0]
    wp.close()
    key = native.ProvingKey(ctx, zk)
    r, s = 0x1234, 0x5678
    proof, pub = key.prove(wt, r.to_bytes(32, "little") + s.to_bytes(32, "little"))
    key.close()
    z = og.parse_zkey(zk)
    w = ow.evaluate(b, inp)
    ref = og.prove(z, w, r=r, s=s)
    assert proof == og.proof_bytes(ref)
    assert og.verify(z, ref["public"], ref["pi_a"], ref["pi_b"], ref["pi_c"])
    vk = groth16.vk_bytes(groth16.export_verification_key(zk, alphabeta=False))
    assert ctx.verify(vk, groth16.public_bytes(pub), proof)
    bad = list(pub)
    bad[0] = (bad[0] + 1) % bn.R
    assert not ctx.verify(vk, groth16.public_bytes(bad), proof)
