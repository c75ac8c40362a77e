"""The reference harness's exact command strings, resolved by `npx` to this package — MI355X (-m gpu).

A throwaway Node project depends on the package (`"zkfl-snarkjs": "file:<pkg>"`, installed with
`npm install --offline`: npm links the package's `snarkjs` bin into node_modules/.bin), and a circuit
directory is laid out the way circom + snarkjs leave it (`python -m zkfl compile --circom-layout`,
`python -m zkfl setup`).  Then, with cwd = the circuit directory, the strings of
tests/full_system_simulation.mjs run unchanged:
  node "<c>_js/generate_witness.cjs" "<c>_js/<c>.wasm" "<input>" "<w>.wtns"           (:758-763)
  npx snarkjs groth16 prove <c>_final.zkey <w>.wtns <proof>.json <public>.json        (:773-776)
  npx snarkjs groth16 verify "<vkey>" "<public>" "<proof>"                            (:865-868)
  npx snarkjs zkey export verificationkey <c>_final.zkey <c>_vkey.json                (:732-735)
  npx snarkjs r1cs info <c>.r1cs  (+ the regex of tests/test_verified_gradient.mjs:356)
plus `groth16 fullprove` and the JS API `groth16.fullProve` / `groth16.verify` (north_star).  Every
proof is checked by the CPU oracle's pairing too; the exported vkey equals the Python export.
"""
import json
import os
import re
import shutil
import subprocess
import sys

import pytest

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(shutil.which("node") is None or shutil.which("npm") is None, reason="needs node")]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd")


def _run(cmd, cwd, ok=True):
    env = dict(os.environ, PYTHONPATH=PKG + os.pathsep + os.environ.get("PYTHONPATH", ""))
    p = subprocess.run(cmd, cwd=cwd, shell=True, capture_output=True, text=True, timeout=180, env=env)
    if ok:
        assert p.returncode == 0, f"{cmd}\n{p.stdout}\n{p.stderr}"
    return p


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    from zkfl import clients
    proj = tmp_path_factory.mktemp("harness")
    (proj / "package.json").write_text(json.dumps({"name": "harness", "version": "1.0.0", "private": True,
                                                   "dependencies": {"zkfl-snarkjs": "file:" + PKG}}))
    _run("npm install --offline --no-audit --no-fund", proj)
    assert os.path.exists(proj / "node_modules" / ".bin" / "snarkjs")
    circ = proj / "circuits" / "training"
    circ.mkdir(parents=True)
    name = "sgd_verified"
    py = sys.executable
    _run(f"{py} -m zkfl compile sgd_verified 8 4 3 1000 --name {name} --circom-layout -o .", circ)
    _run(f"{py} -m zkfl setup sgd_verified 8 4 3 1000 --name {name} -o .", circ)
    inp, _ = clients.Client(1, 8, 4, 3, clients.JsLcg(12346)).training_input(8, 1000, 100000000)
    (circ / "client1_training_input.json").write_text(json.dumps(inp))
    return proj, circ, name, inp


def _oracle_verify(zkey_path, public, proof):
    """proof.json + public.json checked by the CPU oracle's pairing (oracle/groth16.py::verify)."""
    from oracle import bn254 as bn
    from oracle import groth16 as og
    from zkfl import groth16
    z = og.parse_zkey(open(zkey_path, "rb").read())
    pb = groth16.proof_from_json(proof)
    return og.verify(z, [int(x) for x in public], bn.g1_from_bytes_std(pb[:64]), bn.g2_from_bytes_std(pb[64:192]),
                     bn.g1_from_bytes_std(pb[192:]))


def test_reference_command_strings(harness):
    proj, circ, name, inp = harness
    circuitDir = str(circ)
    cjsPath = os.path.join(circuitDir, f"{name}_js", "generate_witness.cjs")
    wasmPath = os.path.join(circuitDir, f"{name}_js", f"{name}.wasm")
    inputPath = os.path.join(circuitDir, "client1_training_input.json")
    witnessPath = os.path.join(circuitDir, "client1_training.wtns")
    proofPath = os.path.join(circuitDir, "client1_training_proof.json")
    publicPath = os.path.join(circuitDir, "client1_training_public.json")
    # tests/full_system_simulation.mjs:758-763 and :773-776, verbatim
    _run(f'node "{cjsPath}" "{wasmPath}" "{inputPath}" "{witnessPath}"', circuitDir)
    _run(f"npx snarkjs groth16 prove {name}_final.zkey {witnessPath} {proofPath} {publicPath}", circuitDir)
    proof, public = json.load(open(proofPath)), json.load(open(publicPath))
    assert proof["protocol"] == "groth16" and proof["curve"] == "bn128" and proof["pi_a"][2] == "1"
    assert public == [inp[k] for k in ("client_id", "round", "root_D", "root_G", "root_W", "tauSquared")]
    # :732-735 (the harness's vkey name), then :865-868 verbatim
    _run(f"npx snarkjs zkey export verificationkey {name}_final.zkey {name}_vkey.json", circuitDir)
    vkeyPath = os.path.join(circuitDir, f"{name}_vkey.json")
    assert json.load(open(vkeyPath)) == json.load(open(os.path.join(circuitDir, "verification_key.json")))
    p = _run(f'npx snarkjs groth16 verify "{vkeyPath}" "{publicPath}" "{proofPath}"', circuitDir)
    assert "OK!" in p.stdout
    assert _oracle_verify(os.path.join(circuitDir, f"{name}_final.zkey"), public, proof)
    bad = list(public)
    bad[3] = str(int(bad[3]) + 1)
    badPath = os.path.join(circuitDir, "bad_public.json")
    json.dump(bad, open(badPath, "w"))
    p = _run(f'npx snarkjs groth16 verify "{vkeyPath}" "{badPath}" "{proofPath}"', circuitDir, ok=False)
    assert p.returncode == 1 and "Invalid proof" in p.stderr
    # tests/test_verified_gradient.mjs:351-356: the constraint count through the harness's regex
    p = _run(f"npx snarkjs r1cs info {name}.r1cs", circuitDir)
    m = re.search(r"# of Constraints:\s*(\d+)", p.stdout)
    from zkfl import circuits
    assert m and int(m.group(1)) == circuits.build("sgd_verified", 8, 4, 3, 1000).n_constraints
    # an unsatisfiable input fails like circom ("Assert Failed"): non-zero exit
    wrong = dict(inp)
    wrong["remainder"] = [str(int(wrong["remainder"][0]) + 1)] + wrong["remainder"][1:]
    json.dump(wrong, open(os.path.join(circuitDir, "wrong.json"), "w"))
    p = _run(f'node "{cjsPath}" "{wasmPath}" wrong.json w2.wtns', circuitDir, ok=False)
    assert p.returncode != 0


def test_fullprove_cli_and_js_api(harness):
    proj, circ, name, inp = harness
    circuitDir = str(circ)
    _run(f"npx snarkjs groth16 fullprove client1_training_input.json {name}_js/{name}.wasm {name}_final.zkey "
         "fp_proof.json fp_public.json", circuitDir)
    public = json.load(open(os.path.join(circuitDir, "fp_public.json")))
    proof = json.load(open(os.path.join(circuitDir, "fp_proof.json")))
    assert public[0] == inp["client_id"] and len(public) == 6
    assert _oracle_verify(os.path.join(circuitDir, f"{name}_final.zkey"), public, proof)
    script = proj / "api.js"
    script.write_text(f"""
const snarkjs = require('zkfl-snarkjs');
const fs = require('fs');
(async () => {{
  const dir = {json.dumps(circuitDir)};
  const input = JSON.parse(fs.readFileSync(dir + '/client1_training_input.json', 'utf8'));
  const {{ proof, publicSignals }} = await snarkjs.groth16.fullProve(input, dir + '/{name}_js/{name}.wasm',
                                                                    dir + '/{name}_final.zkey');
  const vKey = await snarkjs.zKey.exportVerificationKey(dir + '/{name}_final.zkey');
  const ok = await snarkjs.groth16.verify(vKey, publicSignals, proof);
  publicSignals[0] = '99';
  const bad = await snarkjs.groth16.verify(vKey, publicSignals, proof);
  console.log(JSON.stringify({{ ok, bad, proof }}));
  process.exit(0);
}})().catch((e) => {{ console.error(e); process.exit(1); }});
""")
    p = _run("node api.js", proj)
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["ok"] is True and r["bad"] is False
    assert _oracle_verify(os.path.join(circuitDir, f"{name}_final.zkey"), public, r["proof"])


def test_addon_gc_any_finalizer_order(harness):
    """A long-lived Node process drops every reference and forces GC before a normal exit: the
    context's external goes first (its finalizer runs before the key's and the program's), which
    is safe because the C ABI keeps the context alive for its children (zkfl_ctx_destroy only drops
    the handle's reference).  Then a second context proves again and the process exits normally
    (no quickExit)."""
    proj, circ, name, inp = harness
    circuitDir = str(circ)
    addon = os.path.join(PKG, "node", "zkfl.node")
    script = proj / "gc.js"
    script.write_text(f"""
const a = require({json.dumps(addon)});
const fs = require('fs');
const dir = {json.dumps(circuitDir)};
const zk = fs.readFileSync(dir + '/{name}_final.zkey');
const wp = fs.readFileSync(dir + '/{name}_js/{name}.wasm');
const input = fs.readFileSync(dir + '/client1_training_input.json', 'utf8');
const tick = () => new Promise((r) => setImmediate(r));
(async () => {{
  let c = a.createContext(0);
  let k = a.loadKey(c, zk);
  let p = a.loadProgram(c, wp);
  const r1 = await a.fullProve(c, k, p, input);
  c = null;                       // the context first
  for (let i = 0; i < 4; i++) {{ global.gc(); await tick(); }}
  k = null; p = null;             // then its children
  for (let i = 0; i < 4; i++) {{ global.gc(); await tick(); }}
  const c2 = a.createContext(0);
  const k2 = a.loadKey(c2, zk);
  const r2 = await a.fullProve(c2, k2, a.loadProgram(c2, wp), input);
  console.log(JSON.stringify({{ n1: r1.proof.length, n2: r2.proof.length, pub: r1.publicSignals.equals(r2.publicSignals) }}));
}})().catch((e) => {{ console.error(e); process.exit(1); }});
""")
    p = _run("node --expose-gc gc.js", proj)
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r == {"n1": 256, "n2": 256, "pub": True}
