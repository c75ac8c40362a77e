#!/usr/bin/env python3
"""Config-5 stage probe (GPU box): what bounds the c5 leg -- the GPU witness engine, the proofs, or
their pipeline.  Same keys and inputs as bench.py's c5 leg (8 clients x {training, secure
aggregation} per round):
  witness  zkfl_witness_compute_resident of each key's 8 witnesses per round, round after round
  proofs   resident witnesses -> zkfl_groth16_prove_batch, one key at a time (its slots in flight)
  prove2   the two keys' resident witnesses alternately, one batch each per round (host-serialized)
  full     the c5 leg itself (zkfl_groth16_full_prove_multi)
    python3 tools/c5_stage_probe.py [--rounds 16 --slots 8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=16)
    ap.add_argument("--slots", type=int, default=8)
    args = ap.parse_args()
    from zkfl import circuits, clients, native, wprog, zkey
    ctx = native.Context(0)
    circ = {"train": circuits.build("sgd_verified", 8, 4, 3, 1000), "secagg": circuits.build("secure_masked_update", 4, 7)}
    keys, progs, images = {}, {}, {}
    for i, (nm, b) in enumerate(circ.items()):
        zk = zkey.groth16_setup(b, ctx, zkey.Toxic(tau=0xC5 + i, alpha=3, beta=5, gamma=7, delta=11 + i))
        keys[nm] = native.ProvingKey(ctx, zk)
        keys[nm].set_slots(args.slots)
        images[nm] = wprog.compile_program(b)
        progs[nm] = native.WitnessProgram(ctx, images[nm])
    inputs = {"train": [], "secagg": []}
    for r in range(args.rounds):
        for tr, sa, _ in clients.federated_round(8, rnd=r + 1, first_id=1):
            inputs["train"].append(native.parse_inputs(images["train"], json.dumps(tr)))
            inputs["secagg"].append(native.parse_inputs(images["secagg"], json.dumps(sa)))
    n = 16 * args.rounds
    # witness engine alone
    for nm in keys:
        progs[nm].compute_resident(keys[nm], inputs[nm][:8])  # warm-up
    t0 = time.perf_counter()
    res = {nm: [] for nm in keys}
    for r in range(args.rounds):
        for nm in keys:
            res[nm] += progs[nm].compute_resident(keys[nm], inputs[nm][8 * r:8 * r + 8])
    tw = time.perf_counter() - t0
    # proofs alone, one key at a time
    for nm in keys:
        keys[nm].prove_batch(res[nm][:8])
    t0 = time.perf_counter()
    for nm in keys:
        keys[nm].prove_batch(res[nm])
    tp = time.perf_counter() - t0
    # the two keys per round, host-serialized batches of 8
    t0 = time.perf_counter()
    for r in range(args.rounds):
        for nm in keys:
            keys[nm].prove_batch(res[nm][8 * r:8 * r + 8])
    tr2 = time.perf_counter() - t0
    # both keys at once from resident witnesses: one host thread per key (the C calls release the GIL)
    import threading
    t0 = time.perf_counter()
    th = [threading.Thread(target=keys[nm].prove_batch, args=(res[nm],)) for nm in keys]
    for t in th:
        t.start()
    for t in th:
        t.join()
    tboth = time.perf_counter() - t0
    print(f"  proofs of both keys at once from resident witnesses ({args.slots} slots each): {n / tboth:.1f} /s",
          flush=True)
    for nm in keys:
        for w in res[nm]:
            w.close()
        progs[nm].close()
        keys[nm].close()  # its slot streams would hold hardware queues beside the c5 leg's own keys
    s, _ = bench.c5_leg(ctx, 0, 1, args.rounds, args.slots, None, 0)
    print(f"witness {n / tw:.1f} /s | proofs (one key at a time, {args.slots} slots) {n / tp:.1f} /s | "
          f"proofs (per-round batches of 8) {n / tr2:.1f} /s | full c5 {s['value']:.1f} proofs/s", flush=True)


if __name__ == "__main__":
    main()
