"""The C restatement of the oracle agrees with the pure-Python oracle (CPU)."""
import os
import random
import subprocess

import pytest

from oracle import witness as ow

from oracle import bn254 as bn
from oracle import groth16 as og

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def cb():
    subprocess.run(["make", "-s"], cwd=os.path.join(ROOT, "oracle"), check=True)
    from oracle import cbaseline
    return cbaseline


def test_c_msm_matches_python(cb):
    rnd = random.Random(2)
    pts = [bn.mul(bn.G1_GEN, rnd.randrange(bn.R)) for _ in range(50)] + [None]
    ss = [rnd.randrange(bn.R) for _ in range(50)] + [5]
    bases = b"".join(bn.g1_to_bytes_mont(p) for p in pts)
    out = cb.msm_g1(bases, b"".join(s.to_bytes(32, "little") for s in ss), threads=2)
    assert bn.g1_from_bytes_std(out) == bn.msm(pts, ss)


@pytest.mark.parametrize("circ", [("poseidon_hash2",), ("sgd_verified", 8, 4, 3, 1000)])
def test_c_prove_matches_python(cb, circ):
    from oracle_backend import COraclePoints, OraclePoints
    from zkfl import circuits, clients, zkey
    b = circuits.build(*circ)
    if circ[0] == "poseidon_hash2":
        w = ow.evaluate(b, {"left": 3, "right": 4})
    else:
        inp, _ = clients.Client(1, 8, 4, 3, clients.JsLcg(12345)).training_input(8, 1000, 100000000)
        w = ow.evaluate(b, inp)
    backend = OraclePoints() if circ[0] == "poseidon_hash2" else COraclePoints()
    zk = zkey.groth16_setup(b, backend, zkey.Toxic(tau=99, alpha=2, beta=3, gamma=4, delta=5))
    rs = (777).to_bytes(32, "little") + (888).to_bytes(32, "little")
    got = cb.prove(zk, zkey.wtns_bytes(w), rs, threads=4)
    ref = og.prove(og.parse_zkey(zk), w, r=777, s=888)
    assert got == og.proof_bytes(ref)


def test_c_gen_mul_matches_python(cb):
    from oracle_backend import COraclePoints, OraclePoints
    ks = b"".join(k.to_bytes(32, "little") for k in (0, 1, 5, bn.R - 1, 1 << 250, 123456789))
    assert COraclePoints().g1_gen_mul(ks) == OraclePoints().g1_gen_mul(ks)
    assert COraclePoints().g2_gen_mul(ks) == OraclePoints().g2_gen_mul(ks)


def test_cpu_baseline_threads_and_report(cb, monkeypatch, tmp_path):
    """bench.py's cpu_baseline leg: every core the job may use (the allowed CPUs, capped by the
    cgroup quota -- the GPU boxes allow 256 CPUs at a 16-core quota), no fixed cap; the report
    carries the host's core counts and the half-threads scaling point."""
    import builtins
    real_open = builtins.open

    def fake_open(path, *a, **k):
        if path == "/sys/fs/cgroup/cpu.max":
            return real_open(tmp_path / "cpu.max", *a, **k)
        return real_open(path, *a, **k)
    monkeypatch.setattr(builtins, "open", fake_open)
    allowed = len(os.sched_getaffinity(0))
    (tmp_path / "cpu.max").write_text("max 100000\n")
    assert cb._cgroup_quota_cores() is None and cb.default_threads() == allowed
    (tmp_path / "cpu.max").write_text("200000 100000\n")
    assert cb._cgroup_quota_cores() == 2 and cb.default_threads() == min(2, allowed)
    from zkfl import circuits, zkey
    from oracle_backend import OraclePoints
    b = circuits.build("poseidon_hash2")
    w = ow.evaluate(b, {"left": 3, "right": 4})
    zk = zkey.groth16_setup(b, OraclePoints(), zkey.Toxic(tau=99, alpha=2, beta=3, gamma=4, delta=5))
    rep, proof = cb.time_prove(zk, zkey.wtns_bytes(w), seconds_budget=0.5)
    assert rep["cores"] == min(2, allowed) and rep["host"]["cgroup_quota_cores"] == 2
    assert rep["host"]["allowed_cpus"] == allowed and len(proof) == 256
    if rep["cores"] >= 2:
        assert rep["scaling"]["threads"] == [1, 2]
