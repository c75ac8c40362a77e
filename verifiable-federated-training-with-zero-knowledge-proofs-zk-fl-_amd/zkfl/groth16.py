"""snarkjs-compatible Groth16 surface backed by libzkfl (HIP).

Mirrors the snarkjs API/CLI the reference harness drives:
  ``groth16.prove(zkey, wtns)``            <- ``snarkjs groth16 prove`` (tests/full_system_simulation.mjs:773-776)
  ``groth16.fullProve(input, circuit, zkey)`` <- snarkjs ``groth16.fullProve`` (witness + prove)
  ``wtns_calculate(circuit, input)``       <- ``generate_witness.cjs`` / ``snarkjs wtns calculate`` (:758-767)
  ``export_verification_key(zkey)``        <- ``snarkjs zkey export verificationkey`` (:732-735)
  ``r1cs_info(circuit)``                   <- ``snarkjs r1cs info`` (tests/test_verified_gradient.mjs:351-356)
Outputs are snarkjs's JSON shapes: proof.json = {pi_a, pi_b, pi_c, protocol, curve} with
decimal strings, public.json = list of decimal strings (witness[1..nPublic]).
"""

from __future__ import annotations

import hashlib
import os

from . import native
from .field import Q
from .zkey import read_wtns, wtns_bytes, zkey_header

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


def export_verification_key(zkey) -> dict:
    """snarkjs ``zkey export verificationkey`` (vk_alphabeta_12 omitted: the pairing-based
    verifier recomputes it)."""
    h = zkey_header(_read(zkey))

    def g1(b):
        x, y = _mont_to_std_q(b)
        return [str(x), str(y), "1"]

    def g2(b):
        x0, x1, y0, y1 = _mont_to_std_q(b)
        return [[str(x0), str(x1)], [str(y0), str(y1)], ["1", "0"]]

    return {
        "protocol": "groth16", "curve": "bn128", "nPublic": h["nPublic"],
        "vk_alpha_1": g1(h["alpha1"]), "vk_beta_2": g2(h["beta2"]), "vk_gamma_2": g2(h["gamma2"]),
        "vk_delta_2": g2(h["delta2"]), "IC": [g1(p) for p in h["IC"]],
    }


def wtns_calculate(circuit, inputs: dict) -> bytes:
    """Witness generation (circom WASM replacement); raises ConstraintError on bad inputs."""
    return wtns_bytes(circuit.witness(inputs))


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
        return self.prove(zkey, wtns_calculate(circuit, inputs), rs)

    def close(self):
        for k in self._keys.values():
            k.close()
        self._keys.clear()
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


__all__ = ["prove", "fullProve", "Prover", "proof_to_json", "proof_from_json", "export_verification_key",
           "wtns_calculate", "r1cs_info", "read_wtns"]
