#!/usr/bin/env python3
"""Config-5 probe (GPU box): bench.py's c5 leg alone -- federated rounds of 8 clients x {training,
secure aggregation} through zkfl_groth16_full_prove_multi, every proof verified -- printing one
line tools/ab.sh can alternate:  <lib>: <v> proofs/s (host CPU <c> ms per proof, <k> cores busy)

    ZKFL_GRAPH=1 python3 tools/c5_probe.py [--rounds 16 --slots 8]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (sets GPU_MAX_HW_QUEUES before HIP starts, puts the package on sys.path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=16)
    ap.add_argument("--slots", type=int, default=8)
    ap.add_argument("--weak", type=int, default=0, help="also the weak leg with this many rounds (as bench.py)")
    ap.add_argument("--repeat", type=int, default=1, help="run the leg(s) this many times in one process")
    ap.add_argument("--no-check", action="store_true",
                    help="do not fail on proofs that do not verify (knock-out builds, tools/build_ab.sh)")
    args = ap.parse_args()
    from zkfl import native
    ctx = native.Context(0)
    for it in range(args.repeat):
        s, w = bench.c5_leg(ctx, 0, 1, args.rounds, args.slots, None, args.weak, check=not args.no_check)
        if w is not None or args.repeat > 1:
            for tag, x in (("strong", s), ("weak", w)):
                if x is not None:
                    print(f"  pass {it} {tag}: {x['value']:.2f} proofs/s, host CPU {x['host_cpu_ms_per_proof']} ms "
                          f"per proof, {x['host_cpu_cores_busy']} cores busy", flush=True)
    print(f"{os.environ.get('ZKFL_LIB', 'in-tree')}: {s['value']:.2f} proofs/s (host CPU "
          f"{s['host_cpu_ms_per_proof']} ms per proof, {s['host_cpu_cores_busy']} cores busy)", flush=True)


if __name__ == "__main__":
    main()
