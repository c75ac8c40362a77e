#!/usr/bin/env python3
"""Groth16 verification on the GPU: latency (batch 1) and throughput (batched, one lane per proof).

Circuit: sgd_verified(8,4,3,1000) (6 public signals), dev ceremony, one proof replicated.
Prints one JSON line per batch size.  Not part of the bench.py contract (verification is a
correctness gate in SURVEY.md §8 a9, not the metric).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd"))

from zkfl import circuits, clients, groth16, native, wprog  # noqa: E402
from zkfl import zkey  # noqa: E402


def main():
    sizes = [int(x) for x in (sys.argv[1:] or ["1", "64", "1024", "8192"])]
    b = circuits.build("sgd_verified", 8, 4, 3, 1000)
    inp, _ = clients.Client(1, 8, 4, 3, clients.JsLcg(12345)).training_input(8, 1000, 100000000)
    ctx = native.Context(0)
    zk = zkey.groth16_setup(b, ctx, zkey.Toxic(tau=77, alpha=1, beta=2, gamma=3, delta=4))
    key = native.ProvingKey(ctx, zk)
    wp = native.WitnessProgram(ctx, wprog.compile_program(b))
    proof, pub = key.prove(wp.compute([wprog.input_bytes(b, inp)])[0])
    vk = groth16.vk_bytes(groth16.export_verification_key(zk, alphabeta=False))
    pubb = groth16.public_bytes(pub)
    assert ctx.verify(vk, pubb, proof)  # also prepares and caches the key
    for n in sizes:
        reps = max(1, min(20, 2048 // n))
        t0 = time.perf_counter()
        for _ in range(reps):
            res = ctx.verify_batch(vk, pubb * n, proof * n, len(pub))
        dt = (time.perf_counter() - t0) / reps
        assert all(res)
        print(json.dumps({"batch": n, "ms_per_batch": round(dt * 1e3, 3), "verifications_per_s": round(n / dt, 1),
                          "npub": len(pub)}), flush=True)
    key.close()
    ctx.close()


if __name__ == "__main__":
    main()
