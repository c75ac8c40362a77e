"""Powers-of-Tau ceremony and `groth16 setup` from a .ptau (zkfl/ptau.py, zkfl/zkey.py) on the CPU.

The product code runs over the oracle's point backend (tests/oracle_backend.py, the zkfl_setup_*
contract in pure Python), so the file layout, the secret schedule, the Lagrange blocks (incl.
snarkjs's truncated top block) and the term assembly of `groth16 setup` are checked without a GPU
against oracle/ptau.py, an independent restatement of the snarkjs commands
(tests/test_secureagg.cjs:25-57, tests/full_system_simulation.mjs:713-730).  The GPU runs the same
code in tests/test_gpu_ptau.py.
"""
import struct

import pytest

from oracle import bn254 as bn
from oracle import groth16 as og
from oracle import ptau as op
from oracle_backend import OraclePoints
from zkfl import ptau, r1cs, zkey
from zkfl.r1cs_file import read_r1cs

TAU, ALPHA, BETA, DELTA = 0x1234567, 0x89ABC, 0xDEF01, 0x5555


def tiny_circuit():
    """y = x^3 + x z + 5 (3 constraints, 1 public output) -> domain 8."""
    b = r1cs.Builder("tiny")
    y = b.output("y")
    x = b.input("x")
    z = b.input("z")
    x2 = b.mul(x, x)
    x3 = b.mul(x2, x)
    xz = b.mul(x, z)
    b.bind_output(y, r1cs.add_const(r1cs.add(x3, xz), 5))
    return b


def _g1s(b):
    return [bn.g1_from_bytes_mont(b[i:i + 64]) for i in range(0, len(b), 64)]


def _g2s(b):
    return [bn.g2_from_bytes_mont(b[i:i + 128]) for i in range(0, len(b), 128)]


@pytest.fixture(scope="module")
def ceremony():
    be = OraclePoints()
    p0 = ptau.new(3)
    p1 = ptau.contribute(p0, be, TAU, ALPHA, BETA, name="codex-test")
    p2 = ptau.prepare_phase2(p1, be)
    return be, p0, p1, p2


def test_new_layout():
    buf = ptau.new(4)
    secs = ptau.read_sections(buf, b"ptau")
    assert sorted(secs) == [1, 2, 3, 4, 5, 6, 7]
    pt = ptau.Ptau(buf)
    assert pt.power == 4 and pt.ceremony_power == 4 and not pt.prepared
    assert _g1s(pt.section(2)) == [bn.G1_GEN] * 31
    assert _g2s(pt.section(3)) == [bn.G2_GEN] * 16
    assert _g2s(pt.section(6)) == [bn.G2_GEN]
    assert pt.contributions() == (0, b"")
    with pytest.raises(ValueError):
        ptau.new(29)


def test_contribute_matches_oracle(ceremony):
    be, p0, p1, _ = ceremony
    pt0, pt1 = ptau.Ptau(p0), ptau.Ptau(p1)
    ref = op.contribute({2: _g1s(pt0.section(2)), 3: _g2s(pt0.section(3)), 4: _g1s(pt0.section(4)),
                         5: _g1s(pt0.section(5)), 6: _g2s(pt0.section(6))[0]}, 3, TAU, ALPHA, BETA)
    assert _g1s(pt1.section(2)) == ref[2]
    assert _g2s(pt1.section(3)) == ref[3]
    assert _g1s(pt1.section(4)) == ref[4]
    assert _g1s(pt1.section(5)) == ref[5]
    assert _g2s(pt1.section(6))[0] == ref[6]
    n, rec = pt1.contributions()
    assert n == 1
    # snarkjs record layout: 5 points (64+128+64+64+128) + 3 G1 pairs + 3 G2 + 216 + 64 + type + params
    fixed = 448 + 6 * 64 + 3 * 128 + 216 + 64 + 4
    assert rec[:64] == pt1.section(2)[64:128]                      # tauG1[1]
    assert struct.unpack_from("<I", rec, fixed)[0] == 2 + len("codex-test")
    assert rec[fixed + 6:fixed + 16] == b"codex-test"


def test_prepare_phase2_blocks(ceremony):
    _, _, p1, p2 = ceremony
    pt = ptau.Ptau(p2)
    assert pt.prepared and sorted(pt.secs) == [1, 2, 3, 4, 5, 6, 7, 12, 13, 14, 15]
    assert pt.section(2) == ptau.Ptau(p1).section(2)
    for p in range(4):   # exact Lagrange evaluations L_j(tau) G for p <= power
        L = og.lagrange_at(TAU, 1 << p, bn.FR_W[p])
        assert _g1s(pt.lagrange(12, p)) == [bn.mul(bn.G1_GEN, x) for x in L]
        assert _g1s(pt.lagrange(14, p)) == [bn.mul(bn.G1_GEN, ALPHA * x) for x in L]
        assert _g1s(pt.lagrange(15, p)) == [bn.mul(bn.G1_GEN, BETA * x) for x in L]
    L = og.lagrange_at(TAU, 8, bn.FR_W[3])
    assert _g2s(pt.lagrange(13, 3)) == [bn.mul(bn.G2_GEN, x) for x in L]
    # the top tauG1 block (p = power + 1): its last power is absent, so
    # L'_j = L_j - (1/N) w^j tau^(N-1) (snarkjs preparePhase2 zeroes that point)
    N = 16
    w = bn.FR_W[4]
    L = og.lagrange_at(TAU, N, w)
    ninv = pow(N, bn.R - 2, bn.R)
    top = [(L[j] - ninv * pow(w, j, bn.R) * pow(TAU, N - 1, bn.R)) % bn.R for j in range(N)]
    assert _g1s(pt.lagrange(12, 4)) == [bn.mul(bn.G1_GEN, x) for x in top]


def test_group_ifft_is_the_dft():
    pts = [bn.mul(bn.G1_GEN, k) for k in (3, 1, 4, 1, 5, 9, 2, 6)]
    got = op.group_ifft(pts, 3)
    winv = pow(bn.FR_W[3], bn.R - 2, bn.R)
    ninv = pow(8, bn.R - 2, bn.R)
    for j in range(8):
        k = sum(c * pow(winv, i * j, bn.R) for i, c in enumerate((3, 1, 4, 1, 5, 9, 2, 6))) * ninv
        assert got[j] == bn.mul(bn.G1_GEN, k)


def _fields(zk):
    z = og.parse_zkey(zk)
    return {k: z[k] for k in ("nVars", "nPublic", "domainSize", "alpha1", "beta1", "beta2", "gamma2", "delta1",
                               "delta2", "IC", "A", "B1", "B2", "C", "H")}


def test_setup_from_ptau_equals_known_tau_setup():
    """power 4 > the circuit's 3: every block exact -> the same key as the known-tau ceremony with
    gamma = delta = 1, byte for byte; after `zkey contribute` d, the ceremony with delta = d."""
    be = OraclePoints()
    b = tiny_circuit()
    p2 = ptau.prepare_phase2(ptau.contribute(ptau.new(4), be, TAU, ALPHA, BETA), be)
    zk = zkey.setup_from_ptau(b, p2, be)
    known = zkey.groth16_setup(b, be, zkey.Toxic(tau=TAU, alpha=ALPHA, beta=BETA, gamma=1, delta=1))
    assert zk == known
    zc = zkey.zkey_contribute(zk, be, DELTA, name="test")
    known_d = zkey.groth16_setup(b, be, zkey.Toxic(tau=TAU, alpha=ALPHA, beta=BETA, gamma=1, delta=DELTA))
    sz, sk = ptau.read_sections(zc, b"zkey"), ptau.read_sections(known_d, b"zkey")
    for t in range(1, 10):
        assert zc[sz[t][0]:sz[t][0] + sz[t][1]] == known_d[sk[t][0]:sk[t][0] + sk[t][1]], t
    o = sz[10][0]
    assert zc[o:o + 64] == known_d[sk[10][0]:sk[10][0] + 64]        # csHash carried
    assert struct.unpack_from("<I", zc, o + 64)[0] == 1              # one contribution
    # the same key through the circom .r1cs reader (section 4 lists the terms in the file's order)
    zr = zkey.setup_from_ptau(read_r1cs(b.r1cs_bytes()), p2, be)
    sr, s0 = ptau.read_sections(zr, b"zkey"), ptau.read_sections(zk, b"zkey")
    for t in (1, 2, 3, 5, 6, 7, 8, 9, 10):
        assert zr[sr[t][0]:sr[t][0] + sr[t][1]] == zk[s0[t][0]:s0[t][0] + s0[t][1]], t
    assert sorted(og.parse_zkey(zr)["coeffs"]) == sorted(og.parse_zkey(zk)["coeffs"])


def test_setup_at_full_power_and_oracle(ceremony):
    """power 3 == the circuit's: H comes from snarkjs's truncated top block.  The key equals
    oracle/ptau.py's restatement and proves and verifies (oracle prover/verifier)."""
    be, _, p1, p2 = ceremony
    b = tiny_circuit()
    zk = zkey.zkey_contribute(zkey.setup_from_ptau(b, p2, be), be, DELTA)
    pt1, ptp = ptau.Ptau(p1), ptau.Ptau(p2)
    secs = {4: _g1s(pt1.section(4)), 5: _g1s(pt1.section(5)), 6: _g2s(pt1.section(6))[0]}
    lag = {12: [_g1s(ptp.lagrange(12, p)) for p in range(5)], 13: [_g2s(ptp.lagrange(13, p)) for p in range(4)],
           14: [_g1s(ptp.lagrange(14, p)) for p in range(4)], 15: [_g1s(ptp.lagrange(15, p)) for p in range(4)]}
    ref = op.zkey_contribute(op.groth16_setup(og.parse_r1cs(b.r1cs_bytes()), secs, lag), DELTA)
    got = _fields(zk)
    for k, v in got.items():
        assert v == ref[k], k
    from oracle import witness as ow
    w = ow.evaluate(b, {"x": 3, "z": 7})
    z = og.parse_zkey(zk)
    pr = og.prove(z, w, r=11, s=13)
    assert pr["public"] == [3 ** 3 + 21 + 5]
    assert og.verify(z, pr["public"], pr["pi_a"], pr["pi_b"], pr["pi_c"])
    bad = list(pr["public"])
    bad[0] += 1
    assert not og.verify(z, bad, pr["pi_a"], pr["pi_b"], pr["pi_c"])


def test_errors(ceremony):
    be, p0, p1, p2 = ceremony
    with pytest.raises(ValueError, match="not prepared"):
        zkey.setup_from_ptau(tiny_circuit(), p1, be)
    from zkfl import circuits
    with pytest.raises(ValueError, match="too big"):
        zkey.setup_from_ptau(circuits.build("poseidon_hash2"), p2, be)
    with pytest.raises(ValueError):
        ptau.Ptau(p0[:-10])
    with pytest.raises(ValueError):
        ptau.Ptau(b"zkey" + p0[4:])


def test_secret_derivation(monkeypatch):
    monkeypatch.setenv("ZKFL_DETERMINISTIC_SETUP", "1")
    a = ptau.derive_secret("entropy", "tau")
    assert a == ptau.derive_secret("entropy", "tau") and 0 < a < bn.R
    assert a != ptau.derive_secret("entropy", "alpha")
    monkeypatch.delenv("ZKFL_DETERMINISTIC_SETUP")
    assert ptau.derive_secret("entropy", "tau") != ptau.derive_secret("entropy", "tau")


def test_prepare_phase2_refuses_too_large_power_before_group_work(monkeypatch):
    """a power-28 transcript (MAX_POWER) is valid phase 1, but its phase-2 tauG1 block
    is 2^29 points, past the GPU group FFT's 2^28: prepare phase2 must refuse it up front, not after
    the earlier blocks' work.  (A real power-28 file is 34 GB; the bound is lowered to test it.)"""
    class NoGroupWork:
        def __getattr__(self, name):
            raise AssertionError(f"group work ({name}) before the power check")
    monkeypatch.setattr(ptau, "MAX_PHASE2_POWER", 3)
    with pytest.raises(ValueError, match="power 4 > 3"):
        ptau.prepare_phase2(ptau.new(4), NoGroupWork())
    assert ptau.MAX_POWER == 28 and ptau.MAX_PHASE2_POWER + 1 <= 28
