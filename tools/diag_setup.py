#!/usr/bin/env python3
"""Timing probe of the ceremony primitives (zkfl_setup_*) on the GPU box: each call on tiny inputs,
printed as it completes, so a slow or stuck primitive is named."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd"))
sys.path.insert(0, ROOT)


def step(name, fn):
    t0 = time.perf_counter()
    print(f"{name} ...", flush=True)
    r = fn()
    print(f"{name}: {time.perf_counter() - t0:.3f} s", flush=True)
    return r


def main():
    from zkfl import native, ptau
    ctx = step("context", lambda: native.Context(0))
    step("g1_gen_mul x1", lambda: ctx.g1_gen_mul((5).to_bytes(32, "little")))
    g1 = ptau.G1_ONE
    g2 = ptau.G2_ONE
    for n in (1, 64, 4096):
        step(f"g1_scale x{n}", lambda: ctx.g1_scale(g1 * n, (7).to_bytes(32, "little") * n))
    for n in (1, 64):
        step(f"g2_scale x{n}", lambda: ctx.g2_scale(g2 * n, (7).to_bytes(32, "little") * n))
    for lg in (0, 3, 10):
        step(f"g1_lagrange 2^{lg}", lambda: ctx.g1_lagrange(g1 * (1 << lg), lg))
    step("g2_lagrange 2^3", lambda: ctx.g2_lagrange(g2 * 8, 3))
    step("g1_lincomb", lambda: ctx.g1_lincomb(g1 * 4, [0, 2, 5], [0, 1, 2, 3, 0], (3).to_bytes(32, "little") * 5))
    step("g2_lincomb", lambda: ctx.g2_lincomb(g2 * 4, [0, 2, 5], [0, 1, 2, 3, 0], (3).to_bytes(32, "little") * 5))
    ctx.close()


if __name__ == "__main__":
    main()
