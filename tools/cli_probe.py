"""Attribution probe for the CLI leg (bench.py cli_leg): the harness's `npx snarkjs groth16 prove`
string at C2 / M under controlled conditions, with the shim's and the library's stage marks.

  python tools/cli_probe.py [--runs 5] [--names C2,M] [--hold none|ctx|key] [--child-queues N]

--hold: what this (parent) process holds on the GPU while the CLI children run -- nothing (the
        context for the verifier is made after the runs), a bare context, or the metric key with 20
        proof slots (20 streams over the parent's hardware queues, as bench.py's main leg leaves it
        before key.set_slots(1)).
--child-queues: GPU_MAX_HW_QUEUES of the CLI children (bench.py's process exports 28; a harness
        shell has the box's default, 4).
Prints one JSON line per circuit (the cli_leg record) tagged with the conditions."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (sets GPU_MAX_HW_QUEUES=28 for this process, as the bench does)


class LazyCtx:
    """The verifier's context, made on first use (after the CLI runs of the first circuit)."""

    def __init__(self):
        self.ctx = None

    def verify_batch(self, *a):
        from zkfl import native
        if self.ctx is None:
            self.ctx = native.Context(0)
        return self.ctx.verify_batch(*a)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--names", default="C2")
    ap.add_argument("--hold", default="none", choices=["none", "ctx", "key"])
    ap.add_argument("--child-queues", type=int, default=0)
    args = ap.parse_args()
    from zkfl import native
    held = []
    ctx = LazyCtx()
    if args.hold != "none":
        native.lib()
        ctx = native.Context(0)
        if args.hold == "key":
            from zkfl import circuits, zkey
            name, params = bench.CIRCUITS["M"]
            b = circuits.build(name, *params)
            zk = zkey.groth16_setup(b, ctx, zkey.Toxic(tau=0x5EED, alpha=0xA1, beta=0xB2, gamma=0xC3, delta=0xD4))
            key = native.ProvingKey(ctx, zk)
            key.set_slots(20)
            held.append(key)
    if args.child_queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.child_queues)
    out = bench.cli_leg(ctx, args.runs, tuple(args.names.split(",")))
    out["probe"] = {"hold": args.hold, "child_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                    "parent_queues": os.environ.get("ZKFL_HW_QUEUES", "28")}
    print(json.dumps(out), flush=True)
    for k in held:
        k.close()


if __name__ == "__main__":
    main()
