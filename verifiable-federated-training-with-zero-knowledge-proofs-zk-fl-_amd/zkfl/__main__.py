"""Command line: the circom + snarkjs commands the reference harness runs, on this framework.

    python -m zkfl compile <circuit> [params..] [-o DIR]    circom <c>.circom --r1cs --wasm
        -> DIR/<name>.r1cs, DIR/<name>.zkwp (witness program: the .wasm's role)
        --circom-layout: also DIR/<name>_js/<name>.wasm (the witness-program image under circom's
        name) + DIR/<name>_js/generate_witness.cjs, so the harness's
        `node <name>_js/generate_witness.cjs <name>_js/<name>.wasm in.json out.wtns` runs unchanged
    python -m zkfl info <circuit> [params..]                 snarkjs r1cs info (tests/test_verified_gradient.mjs:351-356)
    python -m zkfl r1cs-info <file.r1cs>                     snarkjs r1cs info on a circom-compiled .r1cs
    python -m zkfl setup-r1cs <file.r1cs> [-o DIR]           snarkjs groth16 setup (+ contribute, export vk) on a
                                                             circom .r1cs (zkfl/r1cs_file.py); prove its circom
                                                             .wtns with `prove`
    python -m zkfl setup <circuit> [params..] [-o DIR]       snarkjs groth16 setup + zkey contribute + zkey export
        -> DIR/<name>_final.zkey, DIR/verification_key.json  verificationkey (tests/full_system_simulation.mjs:713-735)
                                                             DEVELOPMENT ceremony: fresh random toxic waste, discarded
    python -m zkfl export-vk <zkey> <vkey.json>              snarkjs zkey export verificationkey
    python -m zkfl wtns <circuit.zkwp> <input.json> <out.wtns>              generate_witness.cjs (:758-767)
    python -m zkfl prove <zkey> <wtns> <proof.json> <public.json>           snarkjs groth16 prove (:773-776)
    python -m zkfl verify <vkey.json> <public.json> <proof.json>            snarkjs groth16 verify (:865-868)

<circuit> is one of zkfl.circuits.CIRCUITS (poseidon_hash2, sgd_verified, sgd_step_v5,
balance_unified, secure_masked_update) followed by its integer template parameters.  GPU
commands use device $LOCAL_RANK (default 0).  Exit status 0 on success; verify exits 1 on an
invalid proof, like snarkjs.
"""

from __future__ import annotations

import argparse
import json
import os
import secrets
import sys

from . import circuits, groth16, native, r1cs_file, snarkjs_cli, wprog, zkey


def _circuit(args):
    params = tuple(int(x) for x in args.params)
    b = circuits.build(args.circuit, *params)
    name = args.name or "_".join([args.circuit] + [str(p) for p in params])
    return b, name


def _ctx():
    return native.Context(int(os.environ.get("LOCAL_RANK", "0")))


def cmd_compile(args):
    b, name = _circuit(args)
    os.makedirs(args.out, exist_ok=True)
    with open(os.path.join(args.out, name + ".r1cs"), "wb") as f:
        f.write(b.r1cs_bytes())
    with open(os.path.join(args.out, name + ".zkwp"), "wb") as f:
        f.write(wprog.compile_program(b))
    if args.circom_layout:
        js = os.path.join(args.out, name + "_js")
        os.makedirs(js, exist_ok=True)
        with open(os.path.join(js, name + ".wasm"), "wb") as f:
            f.write(wprog.compile_program(b))
        gen = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "node", "generate_witness.cjs")
        with open(os.path.join(js, "generate_witness.cjs"), "w") as f:
            f.write("// written by `python -m zkfl compile --circom-layout`: circom's generate_witness.cjs over libzkfl\n"
                    f"require({json.dumps(gen)}).main(process.argv.slice(2));\n")
    print(f"template instances: {args.circuit}{tuple(args.params)}")
    print(f"non-linear constraints: {b.n_constraints}")
    print(f"wires: {b.n_wires}")
    print(f"written: {name}.r1cs, {name}.zkwp in {args.out}")


def _print_info(info):
    print(f"[INFO]  snarkJS: Curve: {info['curve']}")
    print(f"[INFO]  snarkJS: # of Wires: {info['wires']}")
    print(f"[INFO]  snarkJS: # of Constraints: {info['constraints']}")
    print(f"[INFO]  snarkJS: # of Private Inputs: {info['privateInputs']}")
    print(f"[INFO]  snarkJS: # of Public Inputs: {info['publicInputs']}")
    print(f"[INFO]  snarkJS: # of Labels: {info['labels']}")
    print(f"[INFO]  snarkJS: # of Outputs: {info['outputs']}")


def cmd_info(args):
    b, _ = _circuit(args)
    _print_info(groth16.r1cs_info(b))


def _read_r1cs(path):
    with open(path, "rb") as f:
        return r1cs_file.read_r1cs(f.read())


def cmd_r1cs_info(args):
    rc = _read_r1cs(args.r1cs)
    info = groth16.r1cs_info(rc)
    info["labels"] = rc.n_labels
    _print_info(info)


def _setup(b, name, out):
    os.makedirs(out, exist_ok=True)
    rnd = lambda: secrets.randbelow(zkey.R - 1) + 1  # noqa: E731
    with _ctx() as ctx:
        zk = zkey.groth16_setup(b, ctx, zkey.Toxic(tau=rnd(), alpha=rnd(), beta=rnd(), gamma=rnd(), delta=rnd()))
        vk = groth16.export_verification_key(zk, ctx=ctx)
    with open(os.path.join(out, name + "_final.zkey"), "wb") as f:
        f.write(zk)
    with open(os.path.join(out, "verification_key.json"), "w") as f:
        json.dump(vk, f, indent=1)
    print(f"written: {name}_final.zkey ({len(zk)} bytes), verification_key.json in {out}")


def cmd_setup_r1cs(args):
    name = args.name or os.path.splitext(os.path.basename(args.r1cs))[0]
    _setup(_read_r1cs(args.r1cs), name, args.out)


def cmd_setup(args):
    b, name = _circuit(args)
    _setup(b, name, args.out)


def cmd_export_vk(args):
    with _ctx() as ctx:
        vk = groth16.export_verification_key(open(args.zkey, "rb").read(), ctx=ctx)
    with open(args.vkey, "w") as f:
        json.dump(vk, f, indent=1)


def cmd_wtns(args):
    with _ctx() as ctx:
        wp = native.WitnessProgram(ctx, open(args.program, "rb").read())
        wt = wp.compute_json(open(args.input).read())
        wp.close()
    with open(args.out, "wb") as f:
        f.write(wt)


def cmd_prove(args):
    p = groth16.Prover(int(os.environ.get("LOCAL_RANK", "0")))
    proof, public = p.prove(args.zkey, args.wtns)
    p.close()
    with open(args.proof, "w") as f:
        json.dump(proof, f, indent=1)
    with open(args.public, "w") as f:
        json.dump(public, f, indent=1)


def cmd_verify(args):
    p = groth16.Prover(int(os.environ.get("LOCAL_RANK", "0")))
    ok = p.verify(json.load(open(args.vkey)), json.load(open(args.public)), json.load(open(args.proof)))
    p.close()
    if ok:
        print("[INFO]  snarkJS: OK!")
        return 0
    print("[ERROR] snarkJS: Invalid proof", file=sys.stderr)
    return 1


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    if argv and argv[0] in snarkjs_cli.VERBS:   # snarkjs ceremony strings (zkfl/snarkjs_cli.py)
        return snarkjs_cli.run(argv)
    ap = argparse.ArgumentParser(prog="python -m zkfl", description=__doc__.split("\n")[0])
    sub = ap.add_subparsers(dest="cmd", required=True)

    def circuit_args(sp, out=False):
        sp.add_argument("circuit", choices=sorted(circuits.CIRCUITS))
        sp.add_argument("params", nargs="*")
        sp.add_argument("--name", default=None, help="output base name (default: circuit_params)")
        if out:
            sp.add_argument("-o", "--out", default=".")

    sp = sub.add_parser("compile")
    circuit_args(sp, out=True)
    sp.add_argument("--circom-layout", action="store_true",
                    help="also write <name>_js/<name>.wasm + generate_witness.cjs (circom's output layout)")
    circuit_args(sub.add_parser("info"))
    circuit_args(sub.add_parser("setup"), out=True)
    sp = sub.add_parser("r1cs-info")
    sp.add_argument("r1cs")
    sp = sub.add_parser("setup-r1cs")
    sp.add_argument("r1cs")
    sp.add_argument("--name", default=None, help="output base name (default: the .r1cs file's)")
    sp.add_argument("-o", "--out", default=".")
    sp = sub.add_parser("export-vk")
    sp.add_argument("zkey")
    sp.add_argument("vkey")
    sp = sub.add_parser("wtns")
    sp.add_argument("program")
    sp.add_argument("input")
    sp.add_argument("out")
    sp = sub.add_parser("prove")
    for a in ("zkey", "wtns", "proof", "public"):
        sp.add_argument(a)
    sp = sub.add_parser("verify")
    for a in ("vkey", "public", "proof"):
        sp.add_argument(a)
    args = ap.parse_args(argv)
    fn = {"compile": cmd_compile, "info": cmd_info, "setup": cmd_setup,
          "r1cs-info": cmd_r1cs_info, "setup-r1cs": cmd_setup_r1cs, "export-vk": cmd_export_vk,
          "wtns": cmd_wtns, "prove": cmd_prove, "verify": cmd_verify}[args.cmd]
    try:
        return fn(args) or 0
    except native.ZkflError as e:
        print(f"[ERROR] zkfl: {e}", file=sys.stderr)
        return 1


if __name__ == "__main__":
    sys.exit(main())
