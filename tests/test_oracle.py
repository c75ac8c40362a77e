"""The oracle pinned against the reference's own fixture and published vectors (CPU)."""
import json
import os

from oracle import bn254 as bn
from oracle import groth16 as og
from oracle import poseidon as op

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_poseidon_circomlibjs_vectors():
    # circomlibjs published vectors
    assert op.poseidon([1, 2]) == 7853200120776062878684798364095072458815029376092732009249414926327459813530
    assert op.poseidon([1]) == 18586133768512220936620570745912940619677854269274689475585506675881198879027
    assert op.poseidon([0]) == 19014214495641488759237505126948346942972912379615652741039992445865937985820


def test_fixture_root_G_leaves_root_D():
    """data/test_input_v5.json: root_G (t=17,t=3), 8 leaves (t=17,t=2,t=3), 8 paths -> root_D."""
    d = json.load(open(os.path.join(GOLDEN, "test_input_v5.json")))
    grad = [int(a) - int(b) for a, b in zip(d["gradPos"], d["gradNeg"])]
    assert op.gradient_commitment([g % op.R for g in grad], 1, 1) == int(d["root_G"])
    for i in range(8):
        leaf = op.vector_hash([int(x) for x in d["features"][i]] + [int(d["labels"][i])])
        assert int(d["siblings"][i ^ 1][0]) == leaf
        assert op.merkle_root_from_path(leaf, [int(s) for s in d["siblings"][i]], d["pathIndices"][i]) == int(d["root_D"])
    # tauSquared = ||g||^2 + 1000 (scripts/generate_test_data_v5.mjs:188)
    assert int(d["tauSquared"]) == sum(g * g for g in grad) + 1000


def test_bn254_group_kats():
    assert bn.on_curve(bn.G1_GEN) and bn.on_curve(bn.G2_GEN)
    # group order r: (r-1)*G == -G
    assert bn.mul(bn.G1_GEN, bn.R - 1) == bn.neg(bn.G1_GEN)
    assert bn.mul(bn.G2_GEN, bn.R - 1) == bn.neg(bn.G2_GEN)
    # ffjavascript root convention
    assert bn.FR_NQR == 5 and bn.FR_S == 28
    assert pow(bn.FR_W[28], 1 << 28, bn.R) == 1 and pow(bn.FR_W[28], 1 << 27, bn.R) != 1


def test_pairing_bilinear():
    P, Q = bn.G1_GEN, bn.G2_GEN
    e = bn.pairing(P, Q)
    assert not e.is_one()
    assert bn.pairing(bn.mul(P, 6), Q) == bn.pairing(bn.mul(P, 2), bn.mul(Q, 3))
    assert bn.pairing_product([(bn.neg(P), Q), (P, Q)]).is_one()


def test_oracle_groth16_tiny_circuit():
    r1cs = dict(nWires=4, nPubOut=0, nPubIn=1, nPrvIn=1, nConstraints=2,
                constraints=[({2: 1}, {2: 1}, {1: 1}), ({2: 1}, {1: 1}, {3: 1})])
    z = og.setup(r1cs, tau=123456789, alpha=11, beta=22, gamma=33, delta=44)
    p = og.prove(z, [1, 9, 3, 27], r=5, s=7)
    assert og.verify(z, p["public"], p["pi_a"], p["pi_b"], p["pi_c"])
    bad = og.prove(z, [1, 9, 3, 28], r=5, s=7)
    assert not og.verify(z, bad["public"], bad["pi_a"], bad["pi_b"], bad["pi_c"])


def test_oracle_fft_roundtrip():
    import random
    rnd = random.Random(1)
    a = [rnd.randrange(bn.R) for _ in range(64)]
    assert og.fft(og.fft(a), inverse=True) == a
    # DFT definition at one point
    w = bn.FR_W[6]
    assert og.fft(a)[5] == sum(x * pow(w, 5 * j, bn.R) for j, x in enumerate(a)) % bn.R
