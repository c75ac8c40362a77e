"""C-ABI object lifetimes and a slot-stream configuration on an MI355X (-m gpu).

* zkfl_ctx_destroy may come before zkfl_key_free / zkfl_wprog_free / zkfl_witness_free (the N-API
  finalizers run in an unspecified order): the context is reference-counted by its keys and
  witness programs (csrc/zkfl.hip ctx_retain / ctx_release), so every order is safe.
* ZKFL_SLOT_STREAMS=2 with serialized profiling: the slot owns a second stream but the B2 MSM
  shares B1's sort on the main stream, so k_proof_start must empty the G2 tail too.
"""
import ctypes as C
import os
import subprocess
import sys

import pytest

from oracle import groth16 as og
from oracle import witness as ow

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd")
RS = (0x1234567).to_bytes(32, "little") + (0x7654321).to_bytes(32, "little")


def _poseidon_key(gpu_ctx):
    from zkfl import circuits, zkey
    b = circuits.build("poseidon_hash2")
    zk = zkey.groth16_setup(b, gpu_ctx, zkey.Toxic(tau=31337, alpha=5, beta=6, gamma=7, delta=8))
    return b, zk


@pytest.mark.parametrize("order", ["ctx_first", "children_first", "ctx_middle"])
def test_ctx_destroy_in_any_order(gpu_ctx, order):
    """Raw C ABI: ctx + key + witness program + resident witness; one proof; then the handles are
    released in the given order.  A later context proves the same bytes (the device is intact)."""
    from zkfl import native, wprog, zkey
    b, zk = _poseidon_key(gpu_ctx)
    inp = {"left": 1, "right": 2}
    w = ow.evaluate(b, inp)
    wt = zkey.wtns_bytes(w)
    L = native.lib()
    P = C.c_void_p
    ctx, key, prog, wit = P(), P(), P(), P()
    native.check(L.zkfl_ctx_create(0, C.byref(ctx)))
    native.check(L.zkfl_zkey_load(ctx, zk, len(zk), C.byref(key)))
    img = wprog.compile_program(b)
    native.check(L.zkfl_wprog_load(ctx, img, len(img), C.byref(prog)))
    native.check(L.zkfl_witness_upload(ctx, key, wt, len(wt), C.byref(wit)))
    proof = (C.c_uint8 * 256)()
    native.check(L.zkfl_groth16_prove_resident(ctx, key, wit, RS, proof))
    ref = og.proof_bytes(og.prove(og.parse_zkey(zk), w, r=0x1234567, s=0x7654321))
    assert bytes(proof) == ref
    frees = {"ctx": lambda: L.zkfl_ctx_destroy(ctx), "key": lambda: L.zkfl_key_free(key),
             "prog": lambda: L.zkfl_wprog_free(prog), "wit": lambda: L.zkfl_witness_free(wit)}
    seq = {"ctx_first": ["ctx", "wit", "prog", "key"], "children_first": ["wit", "prog", "key", "ctx"],
           "ctx_middle": ["prog", "ctx", "key", "wit"]}[order]
    for name in seq:
        assert frees[name]() == 0, name
    # the device still serves a new context
    with native.Context(0) as c2:
        k2 = native.ProvingKey(c2, zk)
        assert k2.prove(wt, RS)[0] == ref


def test_slot_streams_2_serialized_profiling_parity(tmp_path):
    """ZKFL_SLOT_STREAMS=2 + serialized profiling (bench.py's stage pass on a two-stream slot): the
    proofs equal the oracle's, including pi_B (the G2 tail emptied by k_proof_start)."""
    script = tmp_path / "s2.py"
    script.write_text(f"""
import sys
sys.path[:0] = [{ROOT!r}, {PKG!r}]
from oracle import groth16 as og, witness as ow
from zkfl import circuits, clients, native, zkey
b = circuits.build("sgd_verified", 8, 4, 3, 1000)
with native.Context(0) as ctx:
    zk = zkey.groth16_setup(b, ctx, zkey.Toxic(tau=31337, alpha=5, beta=6, gamma=7, delta=8))
    z = og.parse_zkey(zk)
    key = native.ProvingKey(ctx, zk)
    key.set_slots(2)
    ctx.set_profiling(True, serialize=True)
    wts, refs = [], []
    for cid in (1, 2, 3):
        inp, _ = clients.Client(cid, 8, 4, 3, clients.JsLcg(12345 + cid)).training_input(8, 1000, 100000000)
        w = ow.evaluate(b, inp)
        wts.append(key.upload(zkey.wtns_bytes(w)))
        refs.append(og.proof_bytes(og.prove(z, w, r=0x1234567 + cid, s=0x7654321 + cid)))
    rs = b"".join((0x1234567 + c).to_bytes(32, "little") + (0x7654321 + c).to_bytes(32, "little") for c in (1, 2, 3))
    for rep in range(2):  # the second pass reuses buckets the first left behind
        got = key.prove_batch(wts, rs)
        assert got == refs, [g == r for g, r in zip(got, refs)]
    for w in wts:
        w.close()
    key.close()
print("ok")
""")
    env = dict(os.environ, ZKFL_SLOT_STREAMS="2")
    p = subprocess.run([sys.executable, "-u", str(script)], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), p.stdout + p.stderr
