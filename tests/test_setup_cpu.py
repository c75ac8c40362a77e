from oracle import witness as ow
"""Product dev ceremony + zkey writer, checked by the oracle prover/verifier (CPU).

The fixed-base multiplications are delegated to the oracle (test backend) so the zkey
layout, QAP evaluation, coefficient encoding and public-input rows are checked without a GPU.
"""
from oracle import bn254 as bn
from oracle import groth16 as og
from oracle_backend import OraclePoints
from zkfl import circuits, zkey


def _tiny_zkey():
    b = circuits.build("poseidon_hash2")
    tx = zkey.Toxic(tau=987654321, alpha=111, beta=222, gamma=333, delta=444)
    return b, zkey.groth16_setup(b, OraclePoints(), tx), tx


def test_lagrange_matches_oracle():
    n = 16
    w = zkey.root_of_unity(4)
    assert zkey.lagrange_at(12345, n, w) == og.lagrange_at(12345, n, bn.FR_W[4])
    odd = zkey.lagrange_at(12345, 2 * n, zkey.root_of_unity(5), odd_only=True)
    full = og.lagrange_at(12345, 2 * n, bn.FR_W[5])
    assert odd == full[1::2]


def test_product_zkey_matches_oracle_setup_and_proves():
    b, zk, tx = _tiny_zkey()
    z = og.parse_zkey(zk)
    ref = og.setup(og.parse_r1cs(b.r1cs_bytes()), tx.tau, tx.alpha, tx.beta, tx.gamma, tx.delta)
    for key in ("nVars", "nPublic", "domainSize", "alpha1", "beta1", "beta2", "gamma2", "delta1", "delta2",
                "IC", "A", "B1", "B2", "C", "H"):
        assert z[key] == ref[key], key
    assert sorted(z["coeffs"]) == sorted(ref["coeffs"])
    w = ow.evaluate(b, {"left": 1, "right": 2})
    p = og.prove(z, w, r=3, s=4)
    assert og.verify(z, p["public"], p["pi_a"], p["pi_b"], p["pi_c"])


def test_wtns_roundtrip():
    b = circuits.build("poseidon_hash2")
    w = ow.evaluate(b, {"left": 5, "right": 6})
    buf = zkey.wtns_bytes(w)
    assert og.parse_wtns(buf) == w == zkey.read_wtns(buf)


def test_vkey_export_fields():
    from zkfl import groth16
    _, zk, tx = _tiny_zkey()
    vk = groth16.export_verification_key(zk, alphabeta=False)
    a = bn.mul(bn.G1_GEN, tx.alpha)
    assert vk["vk_alpha_1"][:2] == [str(a[0]), str(a[1])]
    assert vk["nPublic"] == 1 and len(vk["IC"]) == 2
