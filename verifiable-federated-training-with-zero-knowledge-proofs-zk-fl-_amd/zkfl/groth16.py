"""snarkjs-compatible Groth16 surface backed by libzkfl (HIP).

Mirrors the snarkjs API/CLI the reference harness drives:
  ``groth16.prove(zkey, wtns)``            <- ``snarkjs groth16 prove`` (tests/full_system_simulation.mjs:773-776)
  ``groth16.fullProve(input, circuit, zkey)`` <- snarkjs ``groth16.fullProve`` (witness + prove)
  ``wtns_calculate(circuit, input)``       <- ``generate_witness.cjs`` / ``snarkjs wtns calculate`` (:758-767)
  ``export_verification_key(zkey)``        <- ``snarkjs zkey export verificationkey`` (:732-735)
  ``r1cs_info(circuit)``                   <- ``snarkjs r1cs info`` (tests/test_verified_gradient.mjs:351-356)
  ``verify(vkey, public, proof)``          <- ``snarkjs groth16 verify`` (:865-868), on the GPU
Outputs are snarkjs's JSON shapes: proof.json = {pi_a, pi_b, pi_c, protocol, curve} with
decimal strings, public.json = list of decimal strings (witness[1..nPublic]).
"""

from __future__ import annotations

import hashlib
import os

from . import native, wprog
from .field import Q
from .zkey import read_wtns, zkey_header

_RINV_Q = pow(2 ** 256, Q - 2, Q)


def _read(x) -> bytes:
    if isinstance(x, (bytes, bytearray, memoryview)):
        return bytes(x)
    with open(os.fspath(x), "rb") as f:
        return f.read()


def _le(b: bytes, i: int) -> int:
    return int.from_bytes(b[32 * i:32 * i + 32], "little")


def proof_to_json(proof: bytes) -> dict:
    """256-byte C-ABI proof -> snarkjs proof.json object."""
    v = [str(_le(proof, i)) for i in range(8)]
    return {
        "pi_a": [v[0], v[1], "1"],
        "pi_b": [[v[2], v[3]], [v[4], v[5]], ["1", "0"]],
        "pi_c": [v[6], v[7], "1"],
        "protocol": "groth16",
        "curve": "bn128",
    }


def proof_from_json(p: dict) -> bytes:
    vals = [p["pi_a"][0], p["pi_a"][1], p["pi_b"][0][0], p["pi_b"][0][1], p["pi_b"][1][0], p["pi_b"][1][1],
            p["pi_c"][0], p["pi_c"][1]]
    return b"".join(int(x).to_bytes(32, "little") for x in vals)


def _mont_to_std_q(b: bytes):
    return [int.from_bytes(b[i:i + 32], "little") * _RINV_Q % Q for i in range(0, len(b), 32)]


def export_verification_key(zkey, alphabeta: bool = True, ctx: native.Context | None = None) -> dict:
    """snarkjs ``zkey export verificationkey``.  ``vk_alphabeta_12`` = e(alpha1, beta2) is
    computed with the GPU pairing (``zkfl_pairing``); pass ``alphabeta=False`` to skip it (the
    verifier does not read it: snarkjs verify uses the 4-pair product)."""
    h = zkey_header(_read(zkey))

    def g1(b):
        x, y = _mont_to_std_q(b)
        return [str(x), str(y), "1"]

    def g2(b):
        x0, x1, y0, y1 = _mont_to_std_q(b)
        return [[str(x0), str(x1)], [str(y0), str(y1)], ["1", "0"]]

    vk = {
        "protocol": "groth16", "curve": "bn128", "nPublic": h["nPublic"],
        "vk_alpha_1": g1(h["alpha1"]), "vk_beta_2": g2(h["beta2"]), "vk_gamma_2": g2(h["gamma2"]),
        "vk_delta_2": g2(h["delta2"]),
    }
    if alphabeta:
        c = ctx or _prover().ctx
        gt = c.pairing(_g1_bytes(vk["vk_alpha_1"]), _g2_bytes(vk["vk_beta_2"]))
        v = [str(_le(gt, i)) for i in range(12)]
        vk["vk_alphabeta_12"] = [[v[6 * i + 2 * j:6 * i + 2 * j + 2] for j in range(3)] for i in range(2)]
    vk["IC"] = [g1(p) for p in h["IC"]]
    return vk


def _g1_bytes(p) -> bytes:
    """snarkjs JSON G1 [x, y, z] (z = "1", or "0" for infinity) -> 64 B std LE (infinity = zeros)."""
    if int(p[2]) == 0:
        return bytes(64)
    assert int(p[2]) == 1, "projective JSON points are not supported"
    return int(p[0]).to_bytes(32, "little") + int(p[1]).to_bytes(32, "little")


def _g2_bytes(p) -> bytes:
    if int(p[2][0]) == 0 and int(p[2][1]) == 0:
        return bytes(128)
    assert int(p[2][0]) == 1 and int(p[2][1]) == 0, "projective JSON points are not supported"
    return b"".join(int(x).to_bytes(32, "little") for x in (p[0][0], p[0][1], p[1][0], p[1][1]))


def vk_bytes(vk: dict) -> bytes:
    """vkey.json -> the C-ABI vk image (include/zkfl.h, zkfl_groth16_verify)."""
    return (int(vk["nPublic"]).to_bytes(4, "little") + _g1_bytes(vk["vk_alpha_1"]) + _g2_bytes(vk["vk_beta_2"])
            + _g2_bytes(vk["vk_gamma_2"]) + _g2_bytes(vk["vk_delta_2"]) + b"".join(_g1_bytes(p) for p in vk["IC"]))


def public_bytes(public) -> bytes:
    """public.json (decimal strings) -> npub x 32 B std LE.  Values >= 2^256 cannot be encoded
    and are rejected here; values in [r, 2^256) reach the verifier, which reports them invalid."""
    return b"".join(int(x).to_bytes(32, "little") for x in public)


def wtns_calculate(circuit, inputs: dict) -> bytes:
    """Witness generation on the GPU (circom WASM + generate_witness.cjs replacement) -> .wtns
    bytes; an unsatisfied assert raises ZkflError with code ZKFL_E_CONSTRAINT (-7)."""
    return _prover().wtns_calculate(circuit, inputs)


def r1cs_info(circuit) -> dict:
    return {
        "curve": "bn-128", "wires": circuit.n_wires, "constraints": circuit.n_constraints,
        "privateInputs": circuit.n_prv_in, "publicInputs": circuit.n_pub_in,
        "outputs": circuit.n_pub_out, "labels": circuit.n_wires,
    }


class Prover:
    """Keeps one device context and device-resident proving keys (load once, prove many:
    the reference's artifact caching, SURVEY.md §5 checkpoint/resume)."""

    def __init__(self, device: int = 0):
        self.ctx = native.Context(device)
        self._keys = {}
        self._progs = {}

    def program(self, circuit) -> native.WitnessProgram:
        """The circuit's compiled witness program, loaded once (the .wasm's role)."""
        p = self._progs.get(id(circuit))
        if p is None:
            p = (circuit, native.WitnessProgram(self.ctx, wprog.compile_program(circuit)))
            self._progs[id(circuit)] = p
        return p[1]

    def wtns_calculate(self, circuit, inputs: dict) -> bytes:
        return self.program(circuit).compute([wprog.input_bytes(circuit, inputs)])[0]

    def key(self, zkey) -> native.ProvingKey:
        buf = _read(zkey)
        digest = hashlib.sha256(buf).digest()
        k = self._keys.get(digest)
        if k is None:
            k = native.ProvingKey(self.ctx, buf)
            self._keys[digest] = k
        return k

    def prove(self, zkey, wtns, rs: bytes | None = None):
        """-> (proof.json dict, public.json list)"""
        proof, pub = self.key(zkey).prove(_read(wtns), rs)
        return proof_to_json(proof), [str(x) for x in pub]

    def full_prove(self, inputs: dict, circuit, zkey, rs: bytes | None = None):
        return self.prove(zkey, self.wtns_calculate(circuit, inputs), rs)

    def verify(self, vk: dict, public, proof: dict) -> bool:
        return self.ctx.verify(vk_bytes(vk), public_bytes(public), proof_from_json(proof))

    def verify_batch(self, vk: dict, publics, proofs) -> list:
        """Many proofs against one key in one launch (the server's per-round check)."""
        return self.ctx.verify_batch(vk_bytes(vk), b"".join(public_bytes(p) for p in publics),
                                     b"".join(proof_from_json(p) for p in proofs), int(vk["nPublic"]))

    def close(self):
        for k in self._keys.values():
            k.close()
        self._keys.clear()
        for _, p in self._progs.values():
            p.close()
        self._progs.clear()
        self.ctx.close()


_default = None


def _prover() -> Prover:
    global _default
    if _default is None:
        _default = Prover(int(os.environ.get("LOCAL_RANK", "0")))
    return _default


def prove(zkey, wtns, rs: bytes | None = None):
    return _prover().prove(zkey, wtns, rs)


def fullProve(inputs: dict, circuit, zkey, rs: bytes | None = None):  # noqa: N802 (snarkjs name)
    return _prover().full_prove(inputs, circuit, zkey, rs)


def verify(vk: dict, public, proof: dict) -> bool:
    """snarkjs ``groth16.verify(vKey, publicSignals, proof)`` -> bool (GPU pairing check)."""
    return _prover().verify(vk, public, proof)


__all__ = ["prove", "fullProve", "verify", "Prover", "proof_to_json", "proof_from_json", "export_verification_key",
           "vk_bytes", "public_bytes", "wtns_calculate", "r1cs_info", "read_wtns"]
