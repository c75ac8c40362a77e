"""circom .r1cs / .sym ingest (zkfl/r1cs_file.py) — CPU only.

The reference compiles with `circom --r1cs --wasm --sym` (tests/full_system_simulation.mjs:700-708)
and runs `snarkjs groth16 setup <c>.r1cs` (:713-716) / `snarkjs r1cs info` on it.  The reference
commits no .r1cs file and circom is not in this image, so the files here are written by
zkfl.r1cs.Builder.r1cs_bytes in the iden3 layout circom emits: parity is "ingest(write(b)) == b"
(constraints, counts, every section of the zkey the dev ceremony derives from it byte for byte,
its coefficient rows as a set) plus hostile-file rejection; agreement with a circom-written file
is unpinned.  The gpu test proves a .wtns against a key set up from the ingested file.
"""
import os
import struct
import subprocess
import sys

import pytest

from oracle import witness as ow
from zkfl import circuits, groth16, zkey
from zkfl.field import R
from zkfl.r1cs_file import read_r1cs, read_sym

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd")

CASES = [("poseidon_hash2", (), {"left": 1, "right": 2}),
         ("secure_masked_update", (4, 2), None),
         ("sgd_verified", (8, 4, 3, 1000), None)]


def _norm(lc):
    return {k: v % R for k, v in lc.items() if v % R}


@pytest.mark.parametrize("name,params,_inp", CASES, ids=[c[0] for c in CASES])
def test_roundtrip_constraints_and_counts(name, params, _inp):
    b = circuits.build(name, *params)
    rc = read_r1cs(b.r1cs_bytes())
    assert (rc.n_wires, rc.n_pub_out, rc.n_pub_in, rc.n_prv_in) == (b.n_wires, b.n_pub_out, b.n_pub_in, b.n_prv_in)
    assert rc.n_public == b.n_public and rc.n_constraints == b.n_constraints
    assert len(rc.cons) == len(b.cons)
    for (A, B, C), (a, bb, c) in zip(rc.cons, b.cons):
        assert (A, B, C) == (_norm(a), _norm(bb), _norm(c))
    assert groth16.r1cs_info(rc) == groth16.r1cs_info(b)


def test_ingested_witness_satisfies_and_zkey_identical():
    """The dev ceremony over the ingested file gives the builder's .zkey (sections byte for byte,
    coefficient rows in the file's sorted-by-wire order)."""
    from oracle_backend import OraclePoints
    b = circuits.build("poseidon_hash2")
    rc = read_r1cs(b.r1cs_bytes())
    w = ow.evaluate(b, {"left": 1, "right": 2})
    assert rc.check(w)
    bad = list(w)
    bad[1] = (bad[1] + 1) % R
    assert not rc.check(bad)
    toxic = zkey.Toxic(tau=11, alpha=12, beta=13, gamma=14, delta=15)
    got, want = (_zkey_sections(zkey.groth16_setup(x, OraclePoints(), toxic)) for x in (rc, b))
    assert got.keys() == want.keys()
    for t in want:   # section 4 lists the same coefficient rows (the file's terms are sorted by wire)
        assert (sorted(got[t]) if t == 4 else got[t]) == (sorted(want[t]) if t == 4 else want[t]), t


def _zkey_sections(buf):
    nsec = struct.unpack_from("<I", buf, 8)[0]
    off, out = 12, {}
    for _ in range(nsec):
        typ, size = struct.unpack_from("<IQ", buf, off)
        data = buf[off + 12:off + 12 + size]
        if typ == 4:
            n = struct.unpack_from("<I", data, 0)[0]
            data = [data[4 + 44 * i:4 + 44 * (i + 1)] for i in range(n)]
        out[typ] = data
        off += 12 + size
    return out


def test_hostile_files_raise_value_error():
    good = circuits.build("poseidon_hash2").r1cs_bytes()
    read_r1cs(good)
    cases = [good[:k] for k in (0, 3, 11, 12, 20, 60, len(good) // 2, len(good) - 1)]
    cases.append(b"r1cz" + good[4:])
    cases.append(good[:4] + struct.pack("<I", 2) + good[8:])                      # version
    cases.append(good[:12] + struct.pack("<IQ", 1, 2 ** 64 - 16) + good[24:])      # section size
    hdr = bytearray(good)
    hdr[12 + 12 + 4] ^= 1                                                          # prime
    cases.append(bytes(hdr))
    hdr = bytearray(good)
    struct.pack_into("<I", hdr, 12 + 12 + 4 + 32, 2)                               # nWires too small
    cases.append(bytes(hdr))
    for c in cases:
        with pytest.raises(ValueError):
            read_r1cs(c)


def test_read_sym():
    text = "1,1,0,main.out\n2,2,0,main.left\n3,-1,1,main.h.removed\n\n4,3,0,main.right\n"
    assert read_sym(text) == {"main.out": 1, "main.left": 2, "main.right": 3}
    with pytest.raises(ValueError):
        read_sym("1,2,main.x\n")


def test_cli_r1cs_info(tmp_path):
    b = circuits.build("secure_masked_update", 4, 2)
    path = tmp_path / "c.r1cs"
    path.write_bytes(b.r1cs_bytes())
    env = dict(os.environ, PYTHONPATH=PKG + os.pathsep + os.environ.get("PYTHONPATH", ""))
    out = subprocess.run([sys.executable, "-m", "zkfl", "r1cs-info", str(path)], capture_output=True, text=True,
                         env=env, check=True).stdout
    assert f"# of Constraints: {b.n_constraints}" in out and f"# of Wires: {b.n_wires}" in out
    assert f"# of Public Inputs: {b.n_pub_in}" in out and f"# of Private Inputs: {b.n_prv_in}" in out


@pytest.mark.gpu
def test_gpu_setup_from_r1cs_prove_wtns_verify(gpu_ctx):
    """circom flow: .r1cs -> setup (GPU fixed-base) -> prove a .wtns (GPU) -> verify (GPU, oracle)."""
    from oracle import bn254 as bn
    from oracle import groth16 as og
    from zkfl import native
    b = circuits.build("sgd_verified", 8, 4, 3, 1000)
    rc = read_r1cs(b.r1cs_bytes())
    zk = zkey.groth16_setup(rc, gpu_ctx, zkey.Toxic(tau=21, alpha=22, beta=23, gamma=24, delta=25))
    from zkfl import clients
    inp = clients.Client(1, 8, 4, 3, clients.JsLcg(12345)).training_input(8, 1000, 100000000)[0]
    w = ow.evaluate(b, inp)
    assert rc.check(w)
    key = native.ProvingKey(gpu_ctx, zk)
    proof, pub = key.prove(zkey.wtns_bytes(w), (5).to_bytes(32, "little") + (7).to_bytes(32, "little"))
    key.close()
    assert pub == w[1:1 + rc.n_public]
    vk = groth16.vk_bytes(groth16.export_verification_key(zk, alphabeta=False))
    assert gpu_ctx.verify(vk, groth16.public_bytes(pub), proof)
    z = og.parse_zkey(zk)
    assert proof == og.proof_bytes(og.prove(z, w, r=5, s=7))
    assert og.verify(z, pub, bn.g1_from_bytes_std(proof[:64]), bn.g2_from_bytes_std(proof[64:192]),
                     bn.g1_from_bytes_std(proof[192:]))
