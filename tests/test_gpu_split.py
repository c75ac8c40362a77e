"""One proof split over G shards (optional row) — MI355X (-m gpu).

zkfl_zkey_load_shard / zkfl_groth16_prove_part_batch / zkfl_groth16_assemble (include/zkfl.h):
  * every shard's 768-byte part (XYZZ points) equals the CPU model's part (tests/split_model.py,
    built from the oracle's prover) point for point, for G = 2 and 3 on config 2's circuit;
  * the assembled proof equals the unsplit GPU proof with the same (r, s), and the oracle's;
  * at the metric size M (2^18 domain) the 2-shard proof equals the unsplit proof;
  * the collective protocol (zkfl/split.py) with 2 real ranks on device 0 over gloo gives the same
    proofs as one GPU (tests/split_worker.py);
  * assemble rejects a coordinate >= q.
Reference call site replaced: `npx snarkjs groth16 prove` (tests/full_system_simulation.mjs:773-776).
"""
import os
import socket
import subprocess
import sys

import pytest

from oracle import bn254 as bn
from oracle import groth16 as og

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R = bn.R
TOXIC = dict(tau=0x5EED, alpha=0xA1, beta=0xB2, gamma=0xC3, delta=0xD4)


def _le(x):
    return int(x).to_bytes(32, "little")


def _setup(ctx, name, *params):
    from zkfl import circuits, clients, native, wprog, zkey
    b = circuits.build(name, *params)
    zk = zkey.groth16_setup(b, ctx, zkey.Toxic(**TOXIC))
    wp = native.WitnessProgram(ctx, wprog.compile_program(b))
    B, D, Dp, P = params
    inputs = [wprog.input_bytes(b, clients.Client(cid, B, D, Dp, clients.JsLcg(777 + cid))
                                .training_input(B, P, 100000000)[0]) for cid in (1, 2)]
    wts = wp.compute(inputs)
    wp.close()
    return b, zk, wts


@pytest.fixture(scope="module")
def small(gpu_ctx):
    return _setup(gpu_ctx, "sgd_verified", 8, 4, 3, 1000)


@pytest.mark.parametrize("world", [2, 3])
def test_parts_equal_model_and_assemble_equals_unsplit(gpu_ctx, small, world):
    from split_model import affine, part
    from zkfl import native
    _, zk, wts = small
    z = og.parse_zkey(zk)
    full = native.ProvingKey(gpu_ctx, zk)
    rss = [_le(0x1234567) + _le(0x7654321), _le(R - 1) + _le(R - 2)]
    rs = b"".join(rss)
    keys = [native.ProvingKey(gpu_ctx, zk, shard=k, n_shards=world) for k in range(world)]
    try:
        parts = []  # [shard][proof]
        for k, key in enumerate(keys):
            ws = [key.upload(w) for w in wts]
            parts.append(key.prove_part_batch(ws, rs))
            for w in ws:
                w.close()
        for i, wt in enumerate(wts):
            w = og.parse_wtns(wt)
            h = og.compute_h(z, w)
            r = int.from_bytes(rss[i][:32], "little")
            s = int.from_bytes(rss[i][32:], "little")
            for k in range(world):
                assert affine(parts[k][i]) == affine(part(z, w, h, r, s, k, world)), f"proof {i}, shard {k}"
        blob = b"".join(parts[k][i] for i in range(len(wts)) for k in range(world))
        proofs = gpu_ctx.assemble(blob, world, rs)
        ws = [full.upload(w) for w in wts]
        unsplit = full.prove_batch(ws, rs)
        for w in ws:
            w.close()
        assert proofs == unsplit
        for i, wt in enumerate(wts):
            r = int.from_bytes(rss[i][:32], "little")
            s = int.from_bytes(rss[i][32:], "little")
            assert proofs[i] == og.proof_bytes(og.prove(z, og.parse_wtns(wt), r, s))
    finally:
        for key in keys:
            key.close()
        full.close()


def test_metric_two_shards_equal_unsplit(gpu_ctx):
    from zkfl import native
    _, zk, wts = _setup(gpu_ctx, "sgd_verified", 128, 4, 7, 1000)
    rs = _le(0xABCDEF) + _le(0x123456) + _le(R - 5) + _le(7)
    full = native.ProvingKey(gpu_ctx, zk)
    assert full.domain_size == 1 << 18
    keys = [native.ProvingKey(gpu_ctx, zk, shard=k, n_shards=2) for k in range(2)]
    try:
        parts = []
        for key in keys:
            ws = [key.upload(w) for w in wts]
            parts.append(key.prove_part_batch(ws, rs))
            for w in ws:
                w.close()
        blob = b"".join(parts[k][i] for i in range(2) for k in range(2))
        proofs = gpu_ctx.assemble(blob, 2, rs)
        ws = [full.upload(w) for w in wts]
        assert proofs == full.prove_batch(ws, rs)
        for w in ws:
            w.close()
    finally:
        for key in keys:
            key.close()
        full.close()


def test_assemble_rejects_bad_coordinates(gpu_ctx):
    from zkfl import native
    bad = bytearray(768)
    bad[0:32] = bn.Q.to_bytes(32, "little")  # X == q: not canonical
    with pytest.raises(native.ZkflError) as e:
        gpu_ctx.assemble(bytes(bad), 1, _le(1) + _le(2))
    assert e.value.code == -1
    # all-infinity parts are legal: pi_a = pi_b = infinity, pi_c = infinity
    out = gpu_ctx.assemble(bytes(768 * 2), 2, _le(1) + _le(2))
    assert out == [bytes(256)]


# word offsets of a part's points (csrc/zkfl.hip PART_OFF): A' 0, B1' 32, B2' 64 (G2), C' 128, H 160;
# a G1 point is X | Y | ZZ | ZZZ, 8 words each, standard form
@pytest.mark.parametrize("case", ["zz_without_zzz", "zzz_without_zz", "off_curve", "zz3_ne_zzz2", "g2_off_curve"])
def test_assemble_rejects_malformed_points(gpu_ctx, case):
    """canonical but malformed parts used to reach the assembly's binary-GCD inversion
    (ZZ = 1, ZZZ = 0 -> inverse of 0, an endless loop).  k_parts_sum now checks every point
    (infinity, or ZZ^3 = ZZZ^2 and Y^2 = X^3 + b ZZ^3) and the call fails with ZKFL_E_ARG."""
    from zkfl import native
    bad = bytearray(768)
    w = lambda word, v: bad.__setitem__(slice(4 * word, 4 * word + 32), _le(v))  # noqa: E731
    if case == "zz_without_zzz":
        w(0 + 16, 1)                                   # A': ZZ = 1, ZZZ = 0
    elif case == "zzz_without_zz":
        w(32 + 24, 1)                                  # B1': ZZ = 0, ZZZ = 1
    elif case == "off_curve":                          # C' = (1, 1, 1, 1): 1 != 1 + 3
        for k in range(4):
            w(128 + 8 * k, 1)
    elif case == "zz3_ne_zzz2":                        # H: the generator (1, 2) with ZZ = 4, ZZZ = 9
        w(160, 4), w(160 + 8, 18), w(160 + 16, 4), w(160 + 24, 9)
    else:                                              # B2': x = 0, y = 1 is no point of the twist
        w(64 + 8, 0), w(64 + 16, 1), w(64 + 32, 1), w(64 + 48, 1)
    with pytest.raises(native.ZkflError) as e:
        gpu_ctx.assemble(bytes(bad), 1, _le(1) + _le(2))
    assert e.value.code == -1
    # the generator as a scaled XYZZ point (X = 4, Y = 16, ZZ = 4, ZZZ = 8: lambda = 2) is accepted
    good = bytearray(768)
    for k, v in enumerate((4, 16, 4, 8)):
        good[4 * (0 + 8 * k):4 * (0 + 8 * k) + 32] = _le(v)
    proof = gpu_ctx.assemble(bytes(good), 1, _le(1) + _le(2))[0]
    assert bn.g1_from_bytes_std(proof[:64]) == bn.G1_GEN


@pytest.mark.parametrize("case", ["double", "cancel"])
def test_assemble_exceptional_sums(gpu_ctx, case):
    """The assembly's quad operations run on lazy values (csrc/zkfl.hip Q29: below small multiples
    of p, is_zero<K> over 0, p, .., (K-1) p): equal points in different XYZZ scalings must still
    take the doubling branch, opposite ones the infinity branch.  double: A' = B1' = P (scalings
    3 and 7), r = s, C' = H = Q (scalings 2 and 11); cancel: B1' = -A', H = -C'."""
    from split_model import assemble
    Q = bn.Q

    def put(buf, word, pt, lam):
        x, y = pt
        for k, v in enumerate((x * lam * lam % Q, y * pow(lam, 3, Q) % Q, lam * lam % Q, pow(lam, 3, Q))):
            buf[4 * (word + 8 * k):4 * (word + 8 * k) + 32] = _le(v)

    P = bn.mul(bn.G1_GEN, 0x1234567)
    Pc = bn.mul(bn.G1_GEN, 0x7654321)
    neg = lambda pt: (pt[0], (Q - pt[1]) % Q)  # noqa: E731
    part = bytearray(768)
    put(part, 0, P, 3)
    put(part, 32, P if case == "double" else neg(P), 7)
    put(part, 128, Pc, 2)
    put(part, 160, Pc if case == "double" else neg(Pc), 11)
    rs = b"".join(_le(v) + _le(v) for v in (5, R - 2, 0x1F2E3D4C5B6A79880))
    out = gpu_ctx.assemble(bytes(part) * 3, 1, rs)
    assert out == assemble(bytes(part) * 3, 1, rs)
    if case == "cancel":
        assert all(p[128:] == bytes(128) for p in out)  # pi_c = infinity


def test_sharded_key_refuses_whole_proofs(gpu_ctx, small):
    """a key loaded as one shard of a split proof holds only its share of every MSM (and
    shards > 0 no alpha/beta/delta terms): proving a whole proof with it is ZKFL_E_ARG, not a
    256-byte proof that does not verify."""
    from zkfl import native
    _, zk, wts = small
    for k in range(2):
        key = native.ProvingKey(gpu_ctx, zk, shard=k, n_shards=2)
        try:
            with pytest.raises(native.ZkflError) as e:
                key.prove(wts[0], _le(3) + _le(4))
            assert e.value.code == -1
            ws = [key.upload(wts[0])]
            with pytest.raises(native.ZkflError):
                key.prove_batch(ws, _le(3) + _le(4))
            assert len(key.prove_part_batch(ws, _le(3) + _le(4))[0]) == 768  # parts still work
            ws[0].close()
        finally:
            key.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_split_prover_two_ranks_one_device(tmp_path, gpu_ctx, small):
    """zkfl.split.SplitProver with 2 real ranks (both on device 0, gloo): rank 0's proofs equal the
    unsplit GPU proofs for the same (r, s)."""
    from zkfl import native
    _, zk, wts = small
    rs = _le(0x51) + _le(0x52) + _le(0x53) + _le(0x54)
    out = tmp_path / "proofs.bin"
    env = dict(os.environ)
    env["ZKFL_HW_QUEUES"] = "8"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "split_worker.py"), "--out", str(out), "--rs", rs.hex()]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    got = out.read_bytes()
    full = native.ProvingKey(gpu_ctx, zk)
    ws = [full.upload(w) for w in wts]
    want = full.prove_batch(ws, rs)
    for w in ws:
        w.close()
    full.close()
    assert got == b"".join(want)


@pytest.mark.parametrize("world", [4, 7])
def test_many_shards_small_circuit(gpu_ctx, world):
    """More shards than some queries have points: shards with few or no bases of a query (empty
    MSMs) still give parts whose sum assembles to the unsplit proof (config 1's PoseidonHash2)."""
    from oracle import witness as ow
    from zkfl import circuits, native, zkey
    b = circuits.build("poseidon_hash2")
    zk = zkey.groth16_setup(b, gpu_ctx, zkey.Toxic(**TOXIC))
    wt = zkey.wtns_bytes(ow.evaluate(b, {"left": 3, "right": 4}))
    rs = _le(0x99) + _le(0x77)
    full = native.ProvingKey(gpu_ctx, zk)
    keys = [native.ProvingKey(gpu_ctx, zk, shard=k, n_shards=world) for k in range(world)]
    try:
        parts = []
        for key in keys:
            w = key.upload(wt)
            parts.append(key.prove_part_batch([w], rs)[0])
            w.close()
        proof = gpu_ctx.assemble(b"".join(parts), world, rs)[0]
        assert proof == full.prove(wt, rs)[0]
    finally:
        for key in keys:
            key.close()
        full.close()
