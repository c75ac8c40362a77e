"""HIP path (through the C ABI) vs the CPU oracle — run on an MI355X (-m gpu).

Bar: bit-exact.  Small sizes compare against the oracle directly; larger sizes use
size-independent identities (MSM over k_i*G equals (sum s_i k_i)*G; the coset NTT is linear
and matches the oracle on a basis) plus pairing verification of every proof.
"""
import json
import os
import random
import zlib

import pytest

from oracle import witness as ow

from oracle import bn254 as bn
from oracle import groth16 as og

pytestmark = pytest.mark.gpu

R = bn.R
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _le(x):
    return int(x).to_bytes(32, "little")


def _scal(vals):
    return b"".join(_le(v) for v in vals)


def _g1_std(b):
    return bn.g1_from_bytes_std(b)


def _g2_std(b):
    return bn.g2_from_bytes_std(b)


# ---------------------------------------------------------------------------
# fixed-base (dev ceremony) multiplications
# ---------------------------------------------------------------------------
def test_gen_mul_g1_g2_match_oracle(gpu_ctx):
    rnd = random.Random(7)
    ks = [0, 1, 2, R - 1, rnd.randrange(R), rnd.randrange(R), 1 << 200, 12345]
    g1 = gpu_ctx.g1_gen_mul(_scal(ks))
    g2 = gpu_ctx.g2_gen_mul(_scal(ks))
    for i, k in enumerate(ks):
        assert bn.g1_from_bytes_mont(g1[64 * i:64 * i + 64]) == bn.mul(bn.G1_GEN, k)
        assert bn.g2_from_bytes_mont(g2[128 * i:128 * i + 128]) == bn.mul(bn.G2_GEN, k)


# ---------------------------------------------------------------------------
# the assembly's scalar multiplications (s pi_A + r B1 in k_assemble): GLV halves as row-distributed
# chains, the parts summed, affine by the divsteps inverse
# ---------------------------------------------------------------------------
def test_assembly_glv_mul_matches_oracle(gpu_ctx):
    """k P through the assembly's own machinery (zkfl_debug_g1_glv_mul) against the oracle's
    double-and-add: edge scalars (0, 1, 2, r - 1, lambda, 2^128 +- 1, digits that carry into the top
    window, scalars whose GLV halves are negative or zero), the point at infinity, P = -G and seeded
    random points and scalars."""
    rnd = random.Random(23)
    lam = 0xb3c4d79d41a917585bfc41088d8daaa78b17ea66b99c90dd
    ks = [0, 1, 2, 3, 8, 9, 16, R - 1, R - 2, lam, R - lam, (1 << 128) - 1, 1 << 128, (1 << 128) + 1,
          int("8" * 32, 16), int("9" * 32, 16) % R, (1 << 253) + 7, R // 2]
    ks += [rnd.randrange(R) for _ in range(46)]
    pts = [bn.mul(bn.G1_GEN, rnd.randrange(1, R)) for _ in ks]
    pts[3] = None                       # infinity
    pts[4] = bn.neg(bn.G1_GEN)          # -G
    pts[5] = bn.G1_GEN
    out = gpu_ctx.g1_glv_mul(b"".join(bn.g1_to_bytes_std(p) for p in pts), _scal(ks))
    for i, (p, k) in enumerate(zip(pts, ks)):
        want = None if p is None else bn.mul(p, k)
        assert _g1_std(out[64 * i:64 * i + 64]) == want, (i, k)


# ---------------------------------------------------------------------------
# NTT (odd-coset shift of snarkjs groth16_prove)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("logn", [1, 2, 5, 10, 11, 13])
def test_ntt_coset_matches_oracle(gpu_ctx, logn):
    rnd = random.Random(logn)
    a = [rnd.randrange(R) for _ in range(1 << logn)]
    out = gpu_ctx.ntt_coset(_scal(a))
    got = [int.from_bytes(out[32 * i:32 * i + 32], "little") for i in range(1 << logn)]
    assert got == og.coset_evals(a)


def test_ntt_coset_large_linearity(gpu_ctx):
    """2^18 (metric domain): coset(e_k) known in closed form: inc^k * w^(i k) / ... checked via
    linearity: coset(a + b) == coset(a) + coset(b) and one sampled output vs direct sum."""
    logn = 18
    n = 1 << logn
    rnd = random.Random(5)
    a = [rnd.randrange(R) for _ in range(n)]
    b = [rnd.randrange(R) for _ in range(n)]
    ca = gpu_ctx.ntt_coset(_scal(a))
    cb = gpu_ctx.ntt_coset(_scal(b))
    cab = gpu_ctx.ntt_coset(_scal([(x + y) % R for x, y in zip(a, b)]))
    for i in rnd.sample(range(n), 64):
        x = int.from_bytes(ca[32 * i:32 * i + 32], "little")
        y = int.from_bytes(cb[32 * i:32 * i + 32], "little")
        z = int.from_bytes(cab[32 * i:32 * i + 32], "little")
        assert (x + y) % R == z
    # delta input e_0: ifft -> all coefficients 1/n, so at coset point x_i = g w^i the value is
    # (1/n)(x_i^n - 1)/(x_i - 1) = (-2/n)/(g w^i - 1)  (g = w_2n, g^n = -1)
    e0 = [1] + [0] * (n - 1)
    c0 = gpu_ctx.ntt_coset(_scal(e0))
    ninv = pow(n, R - 2, R)
    g, w = bn.FR_W[logn + 1], bn.FR_W[logn]
    for i in range(0, n, 4099):
        want = (R - 2) * ninv % R * pow((g * pow(w, i, R) - 1) % R, R - 2, R) % R
        assert int.from_bytes(c0[32 * i:32 * i + 32], "little") == want


# ---------------------------------------------------------------------------
# MSM
# ---------------------------------------------------------------------------
def _bases_g1(ctx, ks):
    return ctx.g1_gen_mul(_scal(ks))


def _bases_g2(ctx, ks):
    return ctx.g2_gen_mul(_scal(ks))


def _expect(ks, ss):
    return sum(k * s for k, s in zip(ks, ss)) % R


@pytest.mark.parametrize("n", [1, 3, 64, 1000, 70000])
def test_msm_g1_identity(gpu_ctx, n):
    rnd = random.Random(n)
    ks = [rnd.randrange(1, R) for _ in range(n)]
    ss = [rnd.randrange(R) for _ in range(n)]
    out = gpu_ctx.msm_g1(_bases_g1(gpu_ctx, ks), _scal(ss))
    assert _g1_std(out) == bn.mul(bn.G1_GEN, _expect(ks, ss))


def test_msm_g1_matches_oracle_pippenger(gpu_ctx):
    rnd = random.Random(11)
    pts = [bn.mul(bn.G1_GEN, rnd.randrange(R)) for _ in range(40)]
    ss = [rnd.randrange(R) for _ in range(40)]
    bases = b"".join(bn.g1_to_bytes_mont(p) for p in pts)
    assert _g1_std(gpu_ctx.msm_g1(bases, _scal(ss))) == bn.msm(pts, ss)


# every case at both window widths a key can take (csrc/msm_api.h msm_pick_c: 14 bits for small
# keys, 16 for large ones; ZKFL_MSM_C forces one)
@pytest.mark.parametrize("width", [14, 16])
@pytest.mark.parametrize("case", ["zeros", "ones", "small", "neg", "dup", "cancel", "inf_base", "max", "binedge",
                                  "binedge17", "binedge14"])
def test_msm_g1_edge_cases(gpu_ctx, monkeypatch, case, width):
    monkeypatch.setenv("ZKFL_MSM_C", str(width))
    rnd = random.Random(zlib.crc32(case.encode()))
    n = 3000
    ks = [rnd.randrange(1, R) for _ in range(n)]
    ss = [rnd.randrange(R) for _ in range(n)]
    if case == "zeros":
        ss = [0] * n
    elif case == "ones":          # every entry in bucket 0: skewed accumulation
        ss = [1] * n
    elif case == "small":         # witness-like bits / small ints
        ss = [rnd.choice([0, 1, 2, 3, 100, 65535, 65536, 1 << 15, (1 << 15) + 1, (1 << 16) + 1, (1 << 17) - 1,
                          1 << 17, (1 << 17) + 1]) for _ in range(n)]
    elif case == "neg":           # digits near the signed boundary
        ss = [(R - rnd.randrange(1, 1 << 20)) for _ in range(n)]
    elif case == "dup":           # same base repeated: P + P inside a bucket
        ks = [ks[0]] * n
        ss = [ss[0]] * n
    elif case == "cancel":        # P and -P with equal scalars
        ks = [ks[i // 2] if i % 2 == 0 else R - ks[i // 2] for i in range(n)]
        ss = [ss[i // 2] for i in range(n)]
    elif case == "max":
        ss = [R - 1] * n
    elif case == "binedge":       # bucket sort (csrc/msm.h k_msm_bin_*): digits on high-bin edges
        edge = [1, 2, 255, 256, 257, 512, 32767, 32768, 32769, 65535]
        ss = [sum(rnd.choice(edge) << (16 * j) for j in range(16)) % R for _ in range(n)]
    elif case == "binedge17":     # the same for 17-bit windows (MSM_WINDOW_BITS=17): bucket 2^16 - 1,
        # the signed-digit boundary 2^16 / 2^16 + 1 and the high-bin edges of 9 low bits
        edge = [1, 2, 511, 512, 513, 65535, 65536, 65537, 131071, 0]
        ss = [sum(rnd.choice(edge) << (17 * j) for j in range(15)) % R for _ in range(n)]
    elif case == "binedge14":     # 14-bit windows: bucket 2^13 - 1, the signed-digit boundary
        # 2^13 / 2^13 + 1 and the high-bin edges of 6 low bits
        edge = [1, 2, 63, 64, 65, 127, 8191, 8192, 8193, 16383, 0]
        ss = [sum(rnd.choice(edge) << (14 * j) for j in range(19)) % R for _ in range(n)]
    bases = bytearray(_bases_g1(gpu_ctx, ks))
    if case == "inf_base":
        for i in range(0, n, 3):
            bases[64 * i:64 * i + 64] = bytes(64)
            ks[i] = 0
    out = gpu_ctx.msm_g1(bytes(bases), _scal(ss))
    want = _expect(ks, ss)
    assert _g1_std(out) == (bn.mul(bn.G1_GEN, want) if want else None)


@pytest.mark.parametrize("n", [1, 5, 500, 20000])
def test_msm_g2_identity(gpu_ctx, n):
    rnd = random.Random(100 + n)
    ks = [rnd.randrange(1, R) for _ in range(n)]
    ss = [rnd.randrange(R) for _ in range(n)]
    out = gpu_ctx.msm_g2(_bases_g2(gpu_ctx, ks), _scal(ss))
    assert _g2_std(out) == bn.mul(bn.G2_GEN, _expect(ks, ss))


@pytest.mark.parametrize("width", [14, 16])
@pytest.mark.parametrize("case", ["zeros", "ones", "dup", "cancel", "neg", "inf_base"])
def test_msm_g2_edge_cases(gpu_ctx, monkeypatch, case, width):
    """G2 runs on lane pairs (csrc/field.h Fq2PairOps): the exceptional additions (P + P inside a
    bucket, P + (-P), infinity bases) and a single-bucket skew must stay pair-uniform."""
    monkeypatch.setenv("ZKFL_MSM_C", str(width))
    rnd = random.Random(zlib.crc32(case.encode()))
    n = 1500
    ks = [rnd.randrange(1, R) for _ in range(n)]
    ss = [rnd.randrange(R) for _ in range(n)]
    if case == "zeros":
        ss = [0] * n
    elif case == "ones":
        ss = [1] * n
    elif case == "dup":
        ks = [ks[0]] * n
        ss = [ss[0]] * n
    elif case == "cancel":
        ks = [ks[i // 2] if i % 2 == 0 else R - ks[i // 2] for i in range(n)]
        ss = [ss[i // 2] for i in range(n)]
    elif case == "neg":
        ss = [(R - rnd.randrange(1, 1 << 20)) for _ in range(n)]
    bases = bytearray(_bases_g2(gpu_ctx, ks))
    if case == "inf_base":
        for i in range(0, n, 3):
            bases[128 * i:128 * i + 128] = bytes(128)
            ks[i] = 0
    out = gpu_ctx.msm_g2(bytes(bases), _scal(ss))
    want = _expect(ks, ss)
    assert _g2_std(out) == (bn.mul(bn.G2_GEN, want) if want else None)


def test_msm_g1_single_bucket_deep_stitch(gpu_ctx):
    """60,000 entries in one bucket: 3,750 chunks, several stitching levels before one lane holds
    the bucket (csrc/msm.h k_msm_stitch)."""
    rnd = random.Random(77)
    n = 60000
    ks = [rnd.randrange(1, R) for _ in range(n)]
    ss = [1] * n
    out = gpu_ctx.msm_g1(_bases_g1(gpu_ctx, ks), _scal(ss))
    assert _g1_std(out) == bn.mul(bn.G1_GEN, _expect(ks, ss))


def test_msm_g2_small_scalars(gpu_ctx):
    rnd = random.Random(3)
    n = 2000
    ks = [rnd.randrange(1, R) for _ in range(n)]
    ss = [rnd.choice([0, 1, 2, 7, 1 << 16]) for _ in range(n)]
    out = gpu_ctx.msm_g2(_bases_g2(gpu_ctx, ks), _scal(ss))
    want = _expect(ks, ss)
    assert _g2_std(out) == bn.mul(bn.G2_GEN, want)


@pytest.mark.parametrize("target", [1, 7, 64, 1000])
@pytest.mark.parametrize("case", ["random", "ones", "small"])
def test_msm_long_chunks(gpu_ctx, monkeypatch, target, case):
    """Adaptive chunk length (csrc/msm_api.h msm_chunk_len): with the resident-lane target forced
    small (ZKFL_MSM_TARGET), small MSMs run chunks of up to all their entries in one lane, with
    chunk edges anywhere in a bucket, and the stitching's liveness flags skip dead levels."""
    monkeypatch.setenv("ZKFL_MSM_TARGET", str(target))
    rnd = random.Random(zlib.crc32(f"{case}{target}".encode()))
    for g2, n in ((False, 2500), (True, 900)):
        ks = [rnd.randrange(1, R) for _ in range(n)]
        if case == "random":
            ss = [rnd.randrange(R) for _ in range(n)]
        elif case == "ones":
            ss = [1] * n
        else:
            ss = [rnd.choice([0, 1, 2, 3, 100, 1 << 15, (1 << 15) + 1, R - 1]) for _ in range(n)]
        want = _expect(ks, ss)
        if g2:
            out = _g2_std(gpu_ctx.msm_g2(_bases_g2(gpu_ctx, ks), _scal(ss)))
            assert out == (bn.mul(bn.G2_GEN, want) if want else None)
        else:
            out = _g1_std(gpu_ctx.msm_g1(_bases_g1(gpu_ctx, ks), _scal(ss)))
            assert out == (bn.mul(bn.G1_GEN, want) if want else None)


# ---------------------------------------------------------------------------
# Full Groth16 proofs
# ---------------------------------------------------------------------------
def _setup(gpu_ctx, name, *params, toxic=None):
    from zkfl import circuits, zkey
    b = circuits.build(name, *params)
    tx = toxic or zkey.Toxic(tau=31337, alpha=5, beta=6, gamma=7, delta=8)
    return b, zkey.groth16_setup(b, gpu_ctx, tx)


RS = _le(0x1234567) + _le(0x7654321)


def test_gpu_setup_zkey_identical_to_oracle_backend(gpu_ctx):
    from oracle_backend import OraclePoints
    from zkfl import circuits, zkey
    b = circuits.build("poseidon_hash2")
    tx = zkey.Toxic(tau=987654321, alpha=111, beta=222, gamma=333, delta=444)
    assert zkey.groth16_setup(b, gpu_ctx, tx) == zkey.groth16_setup(b, OraclePoints(), tx)


def test_proof_poseidon_hash2_bit_exact(gpu_ctx):
    from zkfl import native, zkey
    b, zk = _setup(gpu_ctx, "poseidon_hash2")
    w = ow.evaluate(b, {"left": 1, "right": 2})
    key = native.ProvingKey(gpu_ctx, zk)
    proof, pub = key.prove(zkey.wtns_bytes(w), RS)
    z = og.parse_zkey(zk)
    ref = og.prove(z, w, r=0x1234567, s=0x7654321)
    assert proof == og.proof_bytes(ref)
    assert pub == [7853200120776062878684798364095072458815029376092732009249414926327459813530]
    assert og.verify(z, ref["public"], ref["pi_a"], ref["pi_b"], ref["pi_c"])
    # deterministic core: h and the five plain MSMs
    hs, parts = key.debug_parts(zkey.wtns_bytes(w))
    assert hs == ref["h"]
    assert _g1_std(parts["A"]) == ref["msm"]["A"]
    assert _g1_std(parts["B1"]) == ref["msm"]["B1"]
    assert _g2_std(parts["B2"]) == ref["msm"]["B2"]
    assert _g1_std(parts["C"]) == ref["msm"]["C"]
    assert _g1_std(parts["H"]) == ref["msm"]["H"]
    key.close()


def _verify_bytes(z, proof, pub):
    pa = bn.g1_from_bytes_std(proof[0:64])
    pb = bn.g2_from_bytes_std(proof[64:192])
    pc = bn.g1_from_bytes_std(proof[192:256])
    return og.verify(z, pub, pa, pb, pc)


def test_proof_sgd_verified_reference_instance(gpu_ctx):
    """sgd_verified(8,4,3,1000) with the harness's client-1 inputs: bit-exact vs oracle."""
    from zkfl import clients, native, zkey
    b, zk = _setup(gpu_ctx, "sgd_verified", 8, 4, 3, 1000)
    c = clients.Client(1, 8, 4, 3, clients.JsLcg(12345))
    inp, _ = c.training_input(8, 1000, 100000000)
    w = ow.evaluate(b, inp)
    key = native.ProvingKey(gpu_ctx, zk)
    proof, pub = key.prove(zkey.wtns_bytes(w), RS)
    z = og.parse_zkey(zk)
    ref = og.prove(z, w, r=0x1234567, s=0x7654321)
    assert proof == og.proof_bytes(ref)
    assert [str(x) for x in pub] == [inp[k] for k in ("client_id", "round", "root_D", "root_G", "root_W", "tauSquared")]
    # random blinding (CSPRNG): still verifies; two proofs differ
    p1, _ = key.prove(zkey.wtns_bytes(w))
    p2, _ = key.prove(zkey.wtns_bytes(w))
    assert p1 != p2
    assert _verify_bytes(z, p1, pub) and _verify_bytes(z, p2, pub)
    # tampered public signal does not verify
    assert not _verify_bytes(z, p1, [pub[0] + 1] + pub[1:])
    key.close()


def test_fixture_v5_proof_verifies(gpu_ctx):
    """The reference fixture data/test_input_v5.json through TrainingStepV5(8,16,7)."""
    from zkfl import native, zkey
    d = json.load(open(os.path.join(GOLDEN, "test_input_v5.json")))
    b, zk = _setup(gpu_ctx, "sgd_step_v5", 8, 16, 7)
    key = native.ProvingKey(gpu_ctx, zk)
    proof, pub = key.prove(zkey.wtns_bytes(ow.evaluate(b, d)))
    assert [str(x) for x in pub] == [d["client_id"], d["round"], d["root_D"], d["root_G"], d["tauSquared"]]
    assert _verify_bytes(og.parse_zkey(zk), proof, pub)
    key.close()


def test_resident_batch_and_errors(gpu_ctx):
    from zkfl import clients, native, zkey
    b, zk = _setup(gpu_ctx, "balance_unified", 8, 3, 4)
    key = native.ProvingKey(gpu_ctx, zk)
    wt = []
    for cid in (1, 2, 3):
        c = clients.Client(cid, 8, 4, 3, clients.JsLcg(12345 + cid))
        wt.append(zkey.wtns_bytes(ow.evaluate(b, c.balance_input())))
    ws = [key.upload(x) for x in wt]
    rs = b"".join(_le(11 + i) + _le(22 + i) for i in range(3))
    batch = key.prove_batch(ws, rs)
    for i in range(3):
        assert batch[i] == key.prove_resident(ws[i], rs[64 * i:64 * i + 64])
        assert batch[i] == key.prove(wt[i], rs[64 * i:64 * i + 64])[0]
    z = og.parse_zkey(zk)
    ref = og.prove(z, zkey.read_wtns(wt[0]), r=11, s=22)
    assert batch[0] == og.proof_bytes(ref)
    # wrong witness length -> ZKFL_E_MISMATCH; garbage zkey -> ZKFL_E_FORMAT; r >= r -> ZKFL_E_ARG
    with pytest.raises(native.ZkflError) as e:
        key.prove(zkey.wtns_bytes([1, 2, 3]))
    assert e.value.code == -4
    with pytest.raises(native.ZkflError) as e:
        native.ProvingKey(gpu_ctx, b"zkey" + bytes(40))
    assert e.value.code == -2
    with pytest.raises(native.ZkflError) as e:
        key.prove(wt[0], _le(R) + _le(1))
    assert e.value.code == -1
    for w in ws:
        w.close()
    key.close()


@pytest.mark.parametrize("width", ["14", "16"])
def test_batch_equals_single_proofs(gpu_ctx, monkeypatch, width):
    """A 12-proof batch of a small key over 3 slots (the one-stream chain, every slot's later proofs
    graph-replayed) must equal the same proofs taken alone (the latency schedule, the GLV scalar
    multiplications) byte for byte, and one of them the oracle's -- at the small keys' 14-bit
    windows (the default for this key) and at the large keys' 16."""
    from zkfl import clients, native, zkey
    monkeypatch.setenv("ZKFL_MSM_C", width)
    b, zk = _setup(gpu_ctx, "balance_unified", 8, 3, 4)
    key = native.ProvingKey(gpu_ctx, zk)
    wt = []
    for cid in (1, 2, 3, 4):
        c = clients.Client(cid, 8, 4, 3, clients.JsLcg(777 + cid))
        wt.append(zkey.wtns_bytes(ow.evaluate(b, c.balance_input())))
    ws = [key.upload(x) for x in wt]
    order = [i % 4 for i in range(12)]
    rs = b"".join(_le(1000 + 7 * j) + _le(2000 + 11 * j) for j in range(12))
    batch = key.prove_batch([ws[i] for i in order], rs)
    for j, i in enumerate(order):
        assert batch[j] == key.prove(wt[i], rs[64 * j:64 * j + 64])[0], j
    z = og.parse_zkey(zk)
    assert batch[5] == og.proof_bytes(og.prove(z, zkey.read_wtns(wt[order[5]]), r=1000 + 35, s=2000 + 55))
    for w in ws:
        w.close()
    key.close()


def test_node_snarkjs_cli_prove(gpu_ctx, tmp_path):
    """`node snarkjs_shim.js groth16 prove zkey wtns proof.json public.json` — the reference's
    execSync line (tests/full_system_simulation.mjs:773-776) through N-API -> C ABI -> HIP."""
    import shutil
    import subprocess
    from zkfl import native, zkey
    node = shutil.which("node")
    shim = os.path.join(native._PKG_DIR, "node", "snarkjs_shim.js")
    if not node or not os.path.exists(os.path.join(os.path.dirname(shim), "zkfl.node")):
        pytest.skip("node / addon not available")
    b, zk = _setup(gpu_ctx, "poseidon_hash2")
    w = ow.evaluate(b, {"left": 11, "right": 22})
    (tmp_path / "c_final.zkey").write_bytes(zk)
    (tmp_path / "w.wtns").write_bytes(zkey.wtns_bytes(w))
    out = subprocess.run([node, shim, "groth16", "prove", "c_final.zkey", "w.wtns", "proof.json", "public.json"],
                         cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    proof = json.load(open(tmp_path / "proof.json"))
    pub = json.load(open(tmp_path / "public.json"))
    assert proof["protocol"] == "groth16" and proof["curve"] == "bn128"
    assert pub == [str(w[1])]
    from zkfl.groth16 import proof_from_json
    assert _verify_bytes(og.parse_zkey(zk), proof_from_json(proof), [int(x) for x in pub])
