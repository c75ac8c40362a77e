"""The snarkjs ceremony commands, with snarkjs's argument order, options and exit codes.

Served for `python -m zkfl <snarkjs argv>` and, through it, for the Node shim's `npx snarkjs ...`
(node/snarkjs_shim.js hands these verbs to this module), so the reference's strings run unchanged:
  powersoftau new bn128 <power> <out.ptau> [-v]                  tests/test_secureagg.cjs:25-31
  powersoftau contribute <in.ptau> <out.ptau> [-v] [-e=..] [--name=..]                 :32-38
  powersoftau prepare phase2 <in.ptau> <out.ptau>                                       :41-47
  groth16 setup <c.r1cs> <pot.ptau> <c_0000.zkey>     :48-57, tests/full_system_simulation.mjs:714-716
  zkey contribute <in.zkey> <out.zkey> [--name=..] [-e=..]   tests/full_system_simulation.mjs:723-726
  zkey export verificationkey <c.zkey> <vkey.json>    :732-735, tests/test_secureagg.cjs:58-64
and the snarkjs aliases ptn, ptc, pt2, g16s, zkn (= groth16 setup), zkc, zkev.  The group work runs
on the GPU (zkfl/ptau.py, zkfl/zkey.py -> libzkfl zkfl_setup_*).  Exit status 0 on success, 1 with
an `[ERROR] snarkJS: ...` line otherwise (snarkjs's CLI convention).
"""

from __future__ import annotations

import json
import os
import sys

VERBS = ("powersoftau", "ptn", "ptc", "pt2", "groth16", "g16s", "zkey", "zkn", "zkc", "zkev")
ALIASES = {"ptn": ["powersoftau", "new"], "ptc": ["powersoftau", "contribute"],
           "pt2": ["powersoftau", "prepare", "phase2"], "g16s": ["groth16", "setup"], "zkn": ["groth16", "setup"],
           "zkc": ["zkey", "contribute"], "zkev": ["zkey", "export", "verificationkey"]}


def parse(argv):
    """-> (positional words, {entropy, name}); -v / --verbose and unknown flags are ignored."""
    pos, opts = [], {"entropy": None, "name": None}
    it = iter(argv)
    for a in it:
        if not a.startswith("-") or a == "-":
            pos.append(a)
            continue
        key, eq, val = a.partition("=")
        field = {"-e": "entropy", "--entropy": "entropy", "-n": "name", "--name": "name"}.get(key)
        if field is None:
            continue
        if not eq:
            val = next(it, "")
        opts[field] = val.strip('"').strip("'")
    if pos and pos[0] in ALIASES:
        pos = ALIASES[pos[0]] + pos[1:]
    if pos[:2] == ["zkey", "new"]:
        pos = ["groth16", "setup"] + pos[2:]
    return pos, opts


def _info(msg):
    print(f"[INFO]  snarkJS: {msg}")


def _ctx():
    from . import native
    return native.Context(int(os.environ.get("LOCAL_RANK", "0")))


def _read(path):
    with open(path, "rb") as f:
        return f.read()


def _write(path, data):
    with open(path, "wb") as f:
        f.write(data)


def run(argv) -> int:
    from . import groth16, ptau, r1cs_file, zkey
    pos, opts = parse(argv)
    try:
        if pos[:2] == ["powersoftau", "new"] and len(pos) >= 5:
            if pos[2] not in ("bn128", "bn254", "alt_bn128"):
                raise ValueError(f"curve not supported: {pos[2]}")
            power = int(pos[3])
            _write(pos[4], ptau.new(power))
            _info(f"powersoftau new: power {power} -> {pos[4]}")
        elif pos[:2] == ["powersoftau", "contribute"] and len(pos) >= 4:
            src = _read(pos[2])
            e = opts["entropy"] or ""
            tau, alpha, beta = (ptau.derive_secret(e, k) for k in ("tau", "alpha", "beta"))
            with _ctx() as ctx:
                out = ptau.contribute(src, ctx, tau, alpha, beta, name=opts["name"] or "")
            _write(pos[3], out)
            _info(f"Contribution {ptau.Ptau(out).contributions()[0]} written to {pos[3]}")
        elif pos[:3] == ["powersoftau", "prepare", "phase2"] and len(pos) >= 5:
            src = _read(pos[3])
            with _ctx() as ctx:
                out = ptau.prepare_phase2(src, ctx)
            _write(pos[4], out)
            _info(f"prepare phase2: Lagrange sections 12-15 written to {pos[4]}")
        elif pos[:2] == ["groth16", "setup"] and len(pos) >= 5:
            cs = r1cs_file.read_r1cs(_read(pos[2]))
            pt = _read(pos[3])
            with _ctx() as ctx:
                zk = zkey.setup_from_ptau(cs, pt, ctx)
            _write(pos[4], zk)
            _info(f"Circuit hash written; {cs.n_constraints} constraints, domain {zkey.domain_size_for(cs)}")
        elif pos[:2] == ["zkey", "contribute"] and len(pos) >= 4:
            src = _read(pos[2])
            d = ptau.derive_secret(opts["entropy"] or "", "delta")
            with _ctx() as ctx:
                out = zkey.zkey_contribute(src, ctx, d, name=opts["name"] or "")
            _write(pos[3], out)
            _info(f"zkey contribution written to {pos[3]}")
        elif pos[:3] == ["zkey", "export", "verificationkey"] and len(pos) >= 5:
            with _ctx() as ctx:
                vk = groth16.export_verification_key(_read(pos[3]), ctx=ctx)
            with open(pos[4], "w") as f:
                json.dump(vk, f, indent=1)
            _info("EXPORT VERIFICATION KEY FINISHED")
        else:
            print("usage: snarkjs powersoftau new bn128 <power> <out.ptau>\n"
                  "       snarkjs powersoftau contribute <in.ptau> <out.ptau> [-e=entropy] [--name=name]\n"
                  "       snarkjs powersoftau prepare phase2 <in.ptau> <out.ptau>\n"
                  "       snarkjs groth16 setup <circuit.r1cs> <pot.ptau> <circuit_0000.zkey>\n"
                  "       snarkjs zkey contribute <in.zkey> <out.zkey> [--name=name] [-e=entropy]\n"
                  "       snarkjs zkey export verificationkey <circuit.zkey> <vkey.json>", file=sys.stderr)
            return 99
    except (ValueError, OSError) as e:
        print(f"[ERROR] snarkJS: {e}", file=sys.stderr)
        return 1
    except Exception as e:  # noqa: BLE001 (native.ZkflError and friends: non-zero exit like snarkjs)
        print(f"[ERROR] snarkJS: {e}", file=sys.stderr)
        return 1
    return 0
