#!/usr/bin/env python3
"""Throughput probe for knock-out experiments (GPU box): the bench's timed region on M without
any verification, so a deliberately broken library variant (a stage compiled out with
-DZK_KNOCKOUT=mask, tools/build_ab.sh) can be timed.  1 / throughput differences between a
variant and the full build give a stage's marginal cost per proof in the concurrent regime.
Never a benchmark of record: the proofs of a knocked-out build are wrong.

    ZKFL_LIB=build_ab/ko1/libzkfl.so python3 tools/ko_probe.py [--steps 48 --warmup 8 --slots 20]
    --e2e: time the input.json -> proof path (zkfl_groth16_full_prove_json_batch) instead
    --latency N: N proofs one at a time (prove_batch of one -> the low-latency schedule); prints
    the median host wall clock per proof
"""
import argparse
import os
import sys
import time

os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("ZKFL_HW_QUEUES", "28")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd"))


def _thread_cpu():
    """{tid: (name, utime + stime ticks)} of this process's threads."""
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                st = f.read()
        except OSError:
            continue
        name = st[st.index("(") + 1:st.rindex(")")]
        fields = st[st.rindex(")") + 2:].split()
        out[tid] = (name, int(fields[11]) + int(fields[12]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--slots", type=int, default=20)
    ap.add_argument("--e2e", action="store_true")
    ap.add_argument("--latency", type=int, default=0)
    ap.add_argument("--c5-first", action="store_true", help="run bench.py's config-5 leg first (as bench.py does)")
    ap.add_argument("--threads", action="store_true",
                    help="also print each thread's host CPU over the timed batch (/proc/self/task)")
    ap.add_argument("--circuit", default="M", help="bench.py circuit name (M: the metric, M19: the 2^19 leg)")
    args = ap.parse_args()
    from zkfl import circuits, clients, native, wprog, zkey
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    name, (bt, dim, depth, prec) = bench.CIRCUITS[args.circuit]
    b = circuits.build(name, bt, dim, depth, prec)
    objs = [clients.Client(c + 1, bt, dim, depth, clients.JsLcg(12345 + c)).training_input(bt, prec, 100000000)[0]
            for c in range(4)]
    ctx = native.Context(0)
    if args.c5_first:
        bench.c5_leg(ctx, 0, 1, 4, 8, None, 0)
    zk = zkey.groth16_setup(b, ctx, zkey.Toxic(tau=0x5EED, alpha=0xA1, beta=0xB2, gamma=0xC3, delta=0xD4))
    key = native.ProvingKey(ctx, zk)
    key.set_slots(args.slots)
    wp = native.WitnessProgram(ctx, wprog.compile_program(b))
    n = args.steps * args.slots
    if args.latency:
        import statistics
        res = wp.compute_resident(key, [wprog.input_bytes(b, o) for o in objs])
        for i in range(args.warmup):
            key.prove_batch([res[i % 4]])
        ts = []
        for i in range(args.latency):
            t0 = time.perf_counter()
            key.prove_batch([res[i % 4]])
            ts.append((time.perf_counter() - t0) * 1e3)
        print(f"{os.environ.get('ZKFL_LIB', 'in-tree')}: latency min {min(ts):.3f} max {max(ts):.3f}: "
              f"{statistics.median(ts):.3f} ms median")
        return
    if args.e2e:
        import json
        texts = [json.dumps(o) for o in objs]
        key.full_prove_json_batch(wp, [texts[i % 4] for i in range(args.warmup * args.slots)])
        t0 = time.perf_counter()
        key.full_prove_json_batch(wp, [texts[i % 4] for i in range(n)])
    else:
        res = wp.compute_resident(key, [wprog.input_bytes(b, o) for o in objs])
        key.prove_batch([res[i % 4] for i in range(args.warmup * args.slots)])
        ctx.synchronize()
        c0 = _thread_cpu() if args.threads else None
        t0 = time.perf_counter()
        key.prove_batch([res[i % 4] for i in range(n)])
    ctx.synchronize()
    dt = time.perf_counter() - t0
    if args.threads and c0 is not None:
        c1 = _thread_cpu()
        tick = os.sysconf("SC_CLK_TCK")
        use = sorted(((c1[t][1] - c0.get(t, (None, 0))[1], c1[t][0], t) for t in c1), reverse=True)
        for ticks, name, tid in use[:8]:
            print(f"  thread {tid} {name}: {ticks / tick * 1e3 / n:.3f} ms host CPU per proof", flush=True)
    print(f"{os.environ.get('ZKFL_LIB', 'in-tree')}: {n / dt:.2f} proofs/s ({dt / n * 1e3:.3f} ms per proof)")


if __name__ == "__main__":
    main()
