#!/usr/bin/env python3
"""Groth16 proofs/sec on the ZK-FL training-step circuit (~2^18 constraints), 1..N MI355X.

Workload (BASELINE.json metric): TrainingStepVerified(BATCH=128,
DIM=4, DEPTH=7, PRECISION=1000) — the reference's sgd_verified.circom at the Report's N=128
scale — with synthetic client inputs from the reference harness's seeded generator
(tests/full_system_simulation.mjs:273-303, weights = 0, tau^2 = 1e8, round 1).
A step = one full Groth16 proof (ABC, 3x coset NTT, 4 G1 + 1 G2 MSM, assembly) from a
device-resident witness with the proving key resident in HBM; r, s from the OS CSPRNG.
Multi-GPU: one process per GPU, independent proofs per rank (weak scaling, no collective on
the data path); the barrier / max-over-ranks timing uses torch.distributed.

Prints ONE JSON line on rank 0 (see DESIGN.md §Measurement for the roofline definitions).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

# Each in-flight proof slot drives one HIP stream; HIP maps a process's streams onto
# GPU_MAX_HW_QUEUES hardware queues (HIP default 4, which the GPU boxes also export), and streams
# sharing a queue serialize.  Set it before anything initializes HIP.  Measured on MI355X
# (tools/concurrency_probe.hip): kernels on distinct streams run concurrently up to ~20 at 24
# queues, while 32 queues oversubscribe the hardware queue slots; 20 slots x 1 stream at 28 queues
# is the best measured configuration (322.2 / 320.0 against 317.4 for 16 x 24,
# profiles/r01_experiments.md).  ZKFL_HW_QUEUES overrides the value used here.
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("ZKFL_HW_QUEUES", "28")

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd")
sys.path.insert(0, PKG_DIR)

METRIC = "Groth16 proofs/sec (training-step circuit, ~2^18 constraints) at 1/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# algorithmic bytes per accumulated (base, window) entry: sorted bucket key (2 B) + entry index
# (4 B) + the affine base it names (64 B G1, 128 B G2)
BYTES_PER_ENTRY = {"msm_accumulate_g1": 2 + 4 + 64, "msm_accumulate_g2": 2 + 4 + 128}
# Fq multiplications per entry: XYZZ mixed addition madd-2008-s = 8M + 2S over Fq (G1), over Fq2
# (G2: 3 Fq products per Fq2 product, Karatsuba)
FQMUL_PER_ENTRY = {"msm_accumulate_g1": 10, "msm_accumulate_g2": 30}
# the integer-VALU ceiling: Fq Montgomery multiplications/s of the library's fp_mul at full
# occupancy, measured on MI355X by tools/fp_microbench.hip (tools/README.md)
FQMUL_PEAK_GPS = 125.1
# rocprofv3 kernel names of the instrumented kernels (profiles/pmc_traffic.json keys)
KERNEL_SYMBOL = {"msm_accumulate_g1": "k_msm_accumulate<zkfl::FqOps",   # FqOpsLazy (G1 compute type)
                 "msm_accumulate_g2": "k_msm_accumulate<zkfl::Fq2"}     # Fq2PairOps
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "pmc_traffic.json")
PROFILED = ("msm_accumulate_g1", "msm_accumulate_g2", "ntt", "abc", "prove")

CIRCUITS = {
    "M": ("sgd_verified", (128, 4, 7, 1000)),
    "C2": ("sgd_verified", (8, 4, 3, 1000)),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline_leg(zk: bytes, wt: bytes, seconds_budget=20.0):
    """Oracle ("port") on the host cores: the C restatement (oracle/c/groth16_ref.c) proving
    the same zkey/wtns, bounded to ~seconds_budget, reported as proofs/s."""
    sys.path.insert(0, ROOT)
    from oracle import cbaseline
    return cbaseline.time_prove(zk, wt, seconds_budget)


def timed_run(key, warm_w, steps_w, ctx, dist):
    """W untimed proofs, then exactly K timed proofs bracketed by barrier + synchronize on both
    sides; returns (max-over-ranks elapsed seconds, proofs)."""

    def barrier_sync():
        ctx.synchronize()
        if dist is not None:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            dist.barrier()

    if warm_w:
        key.prove_batch(warm_w)
    barrier_sync()
    t_start = time.perf_counter()
    proofs = key.prove_batch(steps_w)          # K proofs, `slots` in flight
    barrier_sync()
    elapsed = time.perf_counter() - t_start
    if dist is not None:
        import torch
        dev = "cuda" if torch.cuda.is_available() and dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, proofs


def roofline_pass(key, ctx, ws, slots, n=6):
    """Per-kernel HIP-event timings with every kernel running alone (one slot, a proof's three
    streams serialized onto one), after the timed region: the roofline's average launch time."""
    key.set_slots(1)
    key.prove_batch(ws[:1])
    ctx.profile_reset()
    ctx.set_profiling(True, serialize=True)
    key.prove_batch([ws[i % len(ws)] for i in range(n)])
    ctx.set_profiling(False)
    prof = {k: ctx.profile(k) for k in PROFILED}
    ctx.profile_reset()
    key.set_slots(slots)
    return prof, n


def _pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed PMC summary (tools/rocpd_summary.py)."""
    try:
        with open(PMC_TRAFFIC) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    for name, v in d.get("kernels", {}).items():
        if KERNEL_SYMBOL[kernel] in name:
            return v["traffic"]
    return None


def report(args, world, elapsed, prof, config, cpu, prof_proofs=1):
    """The one JSON line (rank 0)."""
    ms_per_step = elapsed / args.steps * 1e3
    value = world * args.steps / elapsed
    cand = {k: v for k, v in prof.items() if k in BYTES_PER_ENTRY and v[1] > 0}
    roofline = None
    if cand:
        dom = max(cand, key=lambda k: cand[k][0])
        ms_tot, launches, units, med_ms = prof[dom]
        avg_s = med_ms / 1e3        # median launch: robust to a one-off stalled dispatch
        entries = units / launches
        achieved = entries * BYTES_PER_ENTRY[dom] / avg_s / 1e9 if avg_s > 0 else 0.0
        fq = entries * FQMUL_PER_ENTRY[dom] / avg_s / 1e9 if avg_s > 0 else 0.0
        roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": _pmc_traffic(dom),
                    "algorithmic_bytes": round(entries * BYTES_PER_ENTRY[dom]),
                    "avg_launch_ms": round(avg_s * 1e3, 4), "mean_launch_ms": round(ms_tot / launches, 4),
                    "launches": launches,
                    "entries_per_launch": round(entries),
                    "valu": {"achieved": round(fq, 2), "peak": FQMUL_PEAK_GPS, "unit": "G Fq-mul/s",
                             "frac": round(fq / FQMUL_PEAK_GPS, 4)}}
    stage_ms = {k: round(v[3] * v[1] / max(1, prof_proofs), 3) for k, v in prof.items()}  # median x launches
    return {
        "metric": METRIC, "value": round(value, 4), "unit": "proofs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (reference harness seeded client generator)",
        "config": config, "roofline": roofline, "stage_ms_isolated_per_proof": stage_ms, "cpu_baseline": cpu,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=256)   # ~1 s at 16 proofs in flight
    ap.add_argument("--warmup", type=int, default=32)
    ap.add_argument("--circuit", default="M", choices=sorted(CIRCUITS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--slots", type=int, default=20, help="proofs in flight per GPU (one HIP stream each)")
    ap.add_argument("--clients", type=int, default=4, help="distinct synthetic client witnesses, cycled")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist_mod
        dist = dist_mod
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
        dist.init_process_group(backend=backend)

    from zkfl import circuits, clients, native, wprog, zkey

    name, params = CIRCUITS[args.circuit]
    t0 = time.perf_counter()
    b = circuits.build(name, *params)
    batch, dim, depth, precision = params
    inputs = []
    for c in range(args.clients):
        client = clients.Client(rank * args.clients + c + 1, batch, dim, depth, clients.JsLcg(12345 + c))
        inputs.append(wprog.input_bytes(b, client.training_input(batch, precision, 100000000)[0]))
    log(f"[bench r{rank}] circuit {name}{params}: {b.n_constraints} constraints, {b.n_wires} wires "
        f"({time.perf_counter() - t0:.1f} s)")

    ctx = native.Context(local_rank)
    t0 = time.perf_counter()
    zk = zkey.groth16_setup(b, ctx, zkey.Toxic(tau=0x5EED, alpha=0xA1, beta=0xB2, gamma=0xC3, delta=0xD4))
    log(f"[bench r{rank}] dev setup {len(zk) / 1e6:.0f} MB zkey ({time.perf_counter() - t0:.1f} s)")
    t0 = time.perf_counter()
    key = native.ProvingKey(ctx, zk)
    key.set_slots(args.slots)
    wp = native.WitnessProgram(ctx, wprog.compile_program(b))
    log(f"[bench r{rank}] key + witness program load ({time.perf_counter() - t0:.1f} s), domain {key.domain_size}, "
        f"slots {args.slots}")
    t0 = time.perf_counter()
    res = wp.compute_resident(key, inputs)      # GPU witness generation straight into HBM
    log(f"[bench r{rank}] {len(res)} client witnesses on the GPU ({(time.perf_counter() - t0) * 1e3:.1f} ms)")
    steps_w = [res[i % len(res)] for i in range(args.steps)]
    warm_w = [res[i % len(res)] for i in range(max(args.warmup, args.slots) if args.warmup else 0)]

    elapsed, proofs = timed_run(key, warm_w, steps_w, ctx, dist)
    prof, nprof = roofline_pass(key, ctx, res, args.slots)
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline_leg(zk, wp.compute(inputs[:1])[0])
            except Exception as e:  # noqa: BLE001
                log(f"[bench] cpu baseline failed: {e}")
        config = {"workload": f"groth16 prove, {name}{params} (BATCH,DIM,DEPTH,PRECISION)",
                  "constraints": b.n_constraints, "wires": b.n_wires, "domain": key.domain_size,
                  "global_batch": world, "parallelism": f"replicas{world}", "slots_in_flight": args.slots,
                  "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))}
        print(json.dumps(report(args, world, elapsed, prof, config, cpu, nprof)), flush=True)
    assert len(proofs) == args.steps and all(len(p) == 256 for p in proofs)
    for r_ in res:
        r_.close()
    wp.close()
    key.close()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
