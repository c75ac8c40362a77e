"""The reference's ceremony strings and its circomlibjs import, through `npx` -> this package — MI355X.

A throwaway Node project depends on the package as `zkfl-snarkjs` (its `snarkjs` bin) and on
node/circomlibjs as `circomlibjs`, installed with `npm install --offline` (both `file:`), so:
  * tests/test_secureagg.cjs:25-64 (powersoftau new / contribute / prepare phase2, groth16 setup,
    zkey export verificationkey) runs verbatim, then its wtns calculate / prove / verify strings
    (:108-142) on the secure-aggregation circuit (SecureMaskedUpdate(4, 2) compiled here under the
    test's file names: circom is absent);
  * a harness-shaped script restating Client._runZKProof (tests/full_system_simulation.mjs:673-788)
    finds pot17_final.ptau by the :677-695 search, sets the training circuit up with the :713-738
    strings, and proves; the server side verifies with the :865-868 string;
  * `import { buildPoseidon } from 'circomlibjs'` (:25) with the harness's own vectorHash /
    gradientCommitment / buildMerkleTree (:139-223) reproduces data/test_input_v5.json's root_G, its
    leaf hashes, root_D through the 8 paths, and the circomlibjs vectors; the GPU tree extension
    equals the harness's tree.
ZKFL_DETERMINISTIC_SETUP=1 makes the ceremony secrets a function of the -e entropy strings, so the
keys can be compared with the known-tau ceremony.
"""
import json
import os
import shutil
import subprocess
import sys

import pytest

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(shutil.which("node") is None or shutil.which("npm") is None, reason="needs node")]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden", "test_input_v5.json")


def _run(cmd, cwd, ok=True, timeout=240):
    env = dict(os.environ, PYTHONPATH=PKG + os.pathsep + os.environ.get("PYTHONPATH", ""),
               ZKFL_DETERMINISTIC_SETUP="1")
    p = subprocess.run(cmd, cwd=cwd, shell=True, capture_output=True, text=True, timeout=timeout, env=env)
    if ok:
        assert p.returncode == 0, f"{cmd}\n{p.stdout}\n{p.stderr}"
    return p


@pytest.fixture(scope="module")
def proj(tmp_path_factory):
    proj = tmp_path_factory.mktemp("ceremony")
    (proj / "package.json").write_text(json.dumps({
        "name": "harness", "version": "1.0.0", "private": True,
        "dependencies": {"zkfl-snarkjs": "file:" + PKG, "circomlibjs": "file:" + os.path.join(PKG, "node", "circomlibjs")}}))
    _run("npm install --offline --no-audit --no-fund", proj)
    assert os.path.exists(proj / "node_modules" / ".bin" / "snarkjs")
    return proj


def _sections(buf):
    from zkfl import ptau
    s = ptau.read_sections(buf, b"zkey")
    return {t: buf[o:o + n] for t, (o, n) in s.items()}


def test_circomlibjs_fixture_roots(proj):
    script = proj / "roots.mjs"
    script.write_text(r"""
import { buildPoseidon, zkfl } from 'circomlibjs';
import fs from 'fs';

const CONFIG = { CHUNK_SIZE: 16,
  FIELD_PRIME: 21888242871839275222246405745257275088548364400416034343698204186575808495617n };
let poseidon, F;

// tests/full_system_simulation.mjs:139-223, the harness's own helpers
function vectorHash(values) {
  if (values.length <= CONFIG.CHUNK_SIZE) return F.toObject(poseidon(values.map(v => BigInt(v))));
  const chunkHashes = [];
  for (let c = 0; c < Math.ceil(values.length / CONFIG.CHUNK_SIZE); c++) {
    const chunk = values.slice(c * CONFIG.CHUNK_SIZE, Math.min((c + 1) * CONFIG.CHUNK_SIZE, values.length));
    chunkHashes.push(F.toObject(poseidon(chunk.map(v => BigInt(v)))));
  }
  return F.toObject(poseidon(chunkHashes));
}
function gradientCommitment(g, clientId, round) {
  const gradHash = vectorHash(g);
  const metaHash = F.toObject(poseidon([BigInt(clientId), BigInt(round)]));
  return F.toObject(poseidon([BigInt(gradHash), BigInt(metaHash)]));
}
function buildMerkleTree(leafHashes, depth) {
  const zeroHash = F.toObject(poseidon([BigInt(0)]));
  const leaves = [...leafHashes];
  while (leaves.length < 2 ** depth) leaves.push(zeroHash);
  const tree = [leaves];
  let cur = leaves;
  while (cur.length > 1) {
    const next = [];
    for (let i = 0; i < cur.length; i += 2) next.push(F.toObject(poseidon([BigInt(cur[i]), BigInt(cur[i + 1])])));
    tree.push(next);
    cur = next;
  }
  return tree;
}

async function main() {
  poseidon = await buildPoseidon();
  F = poseidon.F;
  const d = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
  const grad = d.gradPos.map((p, i) => BigInt(p) - BigInt(d.gradNeg[i]));
  const gField = grad.map(g => ((g % CONFIG.FIELD_PRIME) + CONFIG.FIELD_PRIME) % CONFIG.FIELD_PRIME);
  const leaves = d.features.map((f, i) => vectorHash([...f, d.labels[i]]));
  // the fixture holds the batch's 8 samples of a larger dataset: root_D through their paths
  // (getMerkleProof's siblings / pathIndices, :225-238), each hashed with the circomlibjs API
  const pathRoots = leaves.map((leaf, i) => {
    let cur = leaf;
    d.siblings[i].forEach((sib, l) => {
      cur = d.pathIndices[i][l] === '0' || d.pathIndices[i][l] === 0
        ? F.toObject(poseidon([cur, BigInt(sib)])) : F.toObject(poseidon([BigInt(sib), cur]));
    });
    return cur.toString();
  });
  // buildMerkleTree (:198-223) over the 8 leaves, depth 3: the harness's loop vs the GPU tree
  const tree = buildMerkleTree(leaves, 3);
  const gpuTree = zkfl.buildMerkleTree(leaves, 3);
  const batch = poseidon.batch([[1, 2], [3, 4]]);
  console.log(JSON.stringify({
    root_G: gradientCommitment(gField, d.client_id, d.round).toString(),
    path_roots: pathRoots,
    tree: tree.map((lv) => lv.map((x) => x.toString())),
    gpu_tree: gpuTree.map((lv) => lv.map((x) => x.toString())),
    p12: F.toString(poseidon([1, 2])), p0: F.toObject(poseidon([0])).toString(),
    p1: F.toObject(poseidon([1n])).toString(), batch0: batch[0].toString(),
    neg: F.toObject(poseidon([-1, '2'])).toString(), negRef: F.toObject(poseidon([CONFIG.FIELD_PRIME - 1n, 2])).toString(),
    leaf0: leaves[0].toString(), sib: d.siblings[1][0],
    vh: zkfl.vectorHash([...d.features[0], d.labels[0]]).toString(),
  }));
}
main().catch((e) => { console.error(e); process.exit(1); });
""")
    p = _run(f"node roots.mjs {GOLDEN}", proj)
    r = json.loads(p.stdout.strip().splitlines()[-1])
    d = json.load(open(GOLDEN))
    assert r["root_G"] == d["root_G"]
    assert r["path_roots"] == [d["root_D"]] * 8
    assert r["tree"] == r["gpu_tree"] and len(r["tree"]) == 4 and len(r["tree"][0]) == 8
    assert r["leaf0"] == r["sib"] == r["vh"]                   # level-0 sibling of leaf 1 = leaf 0
    assert r["p12"] == r["batch0"] == "7853200120776062878684798364095072458815029376092732009249414926327459813530"
    assert r["p0"] == "19014214495641488759237505126948346942972912379615652741039992445865937985820"
    assert r["p1"] == "18586133768512220936620570745912940619677854269274689475585506675881198879027"
    assert r["neg"] == r["negRef"]


def test_secureagg_ceremony_strings(proj):
    """tests/test_secureagg.cjs:25-64 verbatim (buildDir = <proj>/build), then :108-142."""
    from zkfl import circuits, clients, native, ptau, zkey
    buildDir = str(proj / "build")
    os.makedirs(buildDir, exist_ok=True)
    j = os.path.join
    py = sys.executable
    # circom (:14-22) is absent: the secure-aggregation circuit is compiled here under the test's names
    _run(f"{py} -m zkfl compile secure_masked_update 4 2 --name secure_agg_client --circom-layout -o {buildDir}", proj)
    _run(f'npx --yes snarkjs powersoftau new bn128 12 {j(buildDir, "pot12_0000.ptau")} -v', proj)
    _run(f'npx --yes snarkjs powersoftau contribute {j(buildDir, "pot12_0000.ptau")} {j(buildDir, "pot12_0001.ptau")} '
         '-v -e="codex-test"', proj)
    _run(f'npx --yes snarkjs powersoftau prepare phase2 {j(buildDir, "pot12_0001.ptau")} {j(buildDir, "pot12_final.ptau")}',
         proj)
    _run(f'npx --yes snarkjs groth16 setup {j(buildDir, "secure_agg_client.r1cs")} {j(buildDir, "pot12_final.ptau")} '
         f'{j(buildDir, "secure_agg_client_0000.zkey")}', proj)
    _run(f'npx --yes snarkjs zkey export verificationkey {j(buildDir, "secure_agg_client_0000.zkey")} '
         f'{j(buildDir, "vkey.json")}', proj)
    # the key equals the known-tau ceremony for the secrets the entropy string selects (gamma =
    # delta = 1: no zkey contribution in this test); H from the truncated top block (2^12 = 2^power)
    os.environ["ZKFL_DETERMINISTIC_SETUP"] = "1"
    try:
        tau, alpha, beta = (ptau.derive_secret("codex-test", k) for k in ("tau", "alpha", "beta"))
    finally:
        del os.environ["ZKFL_DETERMINISTIC_SETUP"]
    pt = ptau.Ptau(open(j(buildDir, "pot12_final.ptau"), "rb").read())
    assert pt.power == 12 and pt.prepared and pt.contributions()[0] == 1
    b = circuits.build("secure_masked_update", 4, 2)
    zk = open(j(buildDir, "secure_agg_client_0000.zkey"), "rb").read()
    with native.Context(0) as ctx:
        known = zkey.groth16_setup(b, ctx, zkey.Toxic(tau=tau, alpha=alpha, beta=beta, gamma=1, delta=1))
    got, ref = _sections(zk), _sections(known)
    for t in (1, 2, 3, 5, 6, 7, 8, 10):
        assert got[t] == ref[t], t
    # :66-142 with this circuit's input.json (the stale test's own inputs belong to the legacy circuit)
    c = clients.Client(1, 8, 4, 3, clients.JsLcg(12346))
    tr, grad = c.training_input(8, 1000, 100000000)
    inp = clients.secagg_input(1, [2, 3], grad, 1, 100000000, c.root_D, int(tr["root_W"]))
    open(j(buildDir, "input.json"), "w").write(json.dumps(inp))
    _run(f'npx --yes snarkjs wtns calculate {j(buildDir, "secure_agg_client_js", "secure_agg_client.wasm")} '
         f'{j(buildDir, "input.json")} {j(buildDir, "witness.wtns")}', proj)
    _run(f'npx --yes snarkjs groth16 prove {j(buildDir, "secure_agg_client_0000.zkey")} {j(buildDir, "witness.wtns")} '
         f'{j(buildDir, "proof.json")} {j(buildDir, "public.json")}', proj)
    p = _run(f'npx --yes snarkjs groth16 verify {j(buildDir, "vkey.json")} {j(buildDir, "public.json")} '
             f'{j(buildDir, "proof.json")}', proj)
    assert "OK!" in p.stdout
    public = json.load(open(j(buildDir, "public.json")))
    assert public[:2] == ["1", "1"] and len(public) == 13


HARNESS = r"""
// Client._runZKProof (tests/full_system_simulation.mjs:673-788) and the server's verify (:865-868),
// restated with the same paths, search order and command strings.
import { execSync } from 'child_process';
import fs from 'fs';
import path from 'path';

const ROOT = process.argv[2];
const CONFIG = {
  TRAINING_DIR: path.join(ROOT, 'artifacts', 'training'),
  KEYS_DIR: path.join(ROOT, 'artifacts', 'keys'),
  PROJECT_ROOT: ROOT,
};
function runCommand(cmd, cwd) {
  try { execSync(cmd, { cwd, stdio: 'pipe' }); return { success: true }; }
  catch (error) { return { success: false, error: error.message }; }
}
function log(x) { console.log(x); }

async function runZKProof(circuitDir, circuitName, inputPath, outputPrefix) {
  const wasmPath = path.join(circuitDir, `${circuitName}_js`, `${circuitName}.wasm`);
  const zkeyPath = path.join(circuitDir, `${circuitName}_final.zkey`);
  let ptauFile = null;
  const possiblePtau = ['pot17_final.ptau', 'pot14_final.ptau'];
  const possibleDirs = [CONFIG.KEYS_DIR, CONFIG.PROJECT_ROOT, circuitDir];
  for (const dir of possibleDirs) {
    for (const ptau of possiblePtau) {
      if (fs.existsSync(path.join(dir, ptau))) { ptauFile = path.join(dir, ptau); break; }
    }
    if (ptauFile) break;
  }
  if (!ptauFile) { log('No ptau file found!'); return null; }
  log('ptau: ' + ptauFile);
  if (!fs.existsSync(wasmPath) || !fs.existsSync(zkeyPath)) {
    if (!fs.existsSync(zkeyPath)) {
      let result = runCommand(`npx snarkjs groth16 setup ${circuitName}.r1cs "${ptauFile}" ${circuitName}_0000.zkey`, circuitDir);
      if (!result.success) { log('Setup failed ' + result.error); return null; }
      result = runCommand(`npx snarkjs zkey contribute ${circuitName}_0000.zkey ${circuitName}_final.zkey --name="test" -e="entropy"`, circuitDir);
      if (!result.success) { log('Contribution failed ' + result.error); return null; }
      runCommand(`npx snarkjs zkey export verificationkey ${circuitName}_final.zkey ${circuitName}_vkey.json`, circuitDir);
      try { fs.unlinkSync(path.join(circuitDir, `${circuitName}_0000.zkey`)); } catch (e) {}
      log('setup done');
    }
  }
  const cjsPath = path.join(circuitDir, `${circuitName}_js`, 'generate_witness.cjs');
  const witnessPath = path.join(circuitDir, `${outputPrefix}.wtns`);
  let result = runCommand(`node "${cjsPath}" "${wasmPath}" "${inputPath}" "${witnessPath}"`, circuitDir);
  if (!result.success) { log('Witness generation failed ' + result.error); return null; }
  const proofPath = path.join(circuitDir, `${outputPrefix}_proof.json`);
  const publicPath = path.join(circuitDir, `${outputPrefix}_public.json`);
  result = runCommand(`npx snarkjs groth16 prove ${circuitName}_final.zkey ${witnessPath} ${proofPath} ${publicPath}`, circuitDir);
  if (!result.success) { log('Proof generation failed ' + result.error); return null; }
  return { proof: JSON.parse(fs.readFileSync(proofPath, 'utf8')), publicSignals: JSON.parse(fs.readFileSync(publicPath, 'utf8')),
           proofPath, publicPath };
}

async function main() {
  const dir = CONFIG.TRAINING_DIR;
  const res = await runZKProof(dir, 'sgd_verified', path.join(dir, 'client1_training_input.json'), 'client1_training');
  if (!res) process.exit(2);
  const vkeyPath = path.join(dir, 'sgd_verified_vkey.json');
  const v = runCommand(`npx snarkjs groth16 verify "${vkeyPath}" "${res.publicPath}" "${res.proofPath}"`, dir);
  console.log(JSON.stringify({ verified: v.success, publicSignals: res.publicSignals }));
}
main().catch((e) => { console.error(e); process.exit(1); });
"""


def test_harness_runzkproof_flow(proj):
    """pot17_final.ptau made by the ceremony strings in artifacts/keys, a fresh circuit directory
    holding only what circom writes (.r1cs, _js/), and the harness's flow from there."""
    from zkfl import clients
    keys = proj / "artifacts" / "keys"
    train = proj / "artifacts" / "training"
    keys.mkdir(parents=True)
    train.mkdir(parents=True)
    py = sys.executable
    _run("npx snarkjs powersoftau new bn128 17 pot17_0000.ptau -v", keys)
    _run('npx snarkjs powersoftau contribute pot17_0000.ptau pot17_0001.ptau --name="First" -v -e="harness"', keys)
    _run("npx snarkjs powersoftau prepare phase2 pot17_0001.ptau pot17_final.ptau -v", keys, timeout=600)
    _run(f"{py} -m zkfl compile sgd_verified 8 4 3 1000 --name sgd_verified --circom-layout -o .", train)
    inp, _ = clients.Client(1, 8, 4, 3, clients.JsLcg(12346)).training_input(8, 1000, 100000000)
    (train / "client1_training_input.json").write_text(json.dumps(inp))
    (proj / "harness.mjs").write_text(HARNESS)
    p = _run(f"node harness.mjs {proj}", proj, timeout=600)
    lines = p.stdout.strip().splitlines()
    assert any(ln.startswith("ptau: ") and ln.endswith(os.path.join("keys", "pot17_final.ptau")) for ln in lines), p.stdout
    assert "setup done" in lines
    r = json.loads(lines[-1])
    assert r["verified"] is True
    assert r["publicSignals"] == [inp[k] for k in ("client_id", "round", "root_D", "root_G", "root_W", "tauSquared")]
    assert not (train / "sgd_verified_0000.zkey").exists() and (train / "sgd_verified_final.zkey").exists()
