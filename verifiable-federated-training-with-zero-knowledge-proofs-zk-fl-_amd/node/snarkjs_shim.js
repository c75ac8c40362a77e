#!/usr/bin/env node
// snarkjs-compatible CLI/API over the N-API addon (zkfl.node -> libzkfl.so -> HIP).
//
// Installed as the `snarkjs` bin of package.json, so the reference harness's command strings resolve
// to it unchanged (`npx snarkjs ...` with cwd = the circuit directory):
//   snarkjs groth16 prove <circuit_final.zkey> <witness.wtns> <proof.json> <public.json>
//       (tests/full_system_simulation.mjs:773-776)
//   snarkjs groth16 verify <verification_key.json> <public.json> <proof.json>
//       (:865-868; exit 0 + "OK!" when valid, exit 1 + "Invalid proof" otherwise)
//   snarkjs groth16 fullprove <input.json> <circuit.wasm> <circuit_final.zkey> <proof.json> <public.json>
//   snarkjs wtns calculate <circuit.wasm> <input.json> <witness.wtns>   (tests/test_secureagg.cjs:108-118)
//   snarkjs zkey export verificationkey <circuit_final.zkey> <vkey.json>  (:732-735)
//   snarkjs r1cs info <circuit.r1cs>                                    (tests/test_verified_gradient.mjs:351-356)
// "circuit.wasm" is the witness-program image `python -m zkfl compile --circom-layout` writes under
// the .wasm name (magic "zkwp"); a real circom .wasm is accepted when `<circuit>.zkwp` sits beside it.
//
// API (snarkjs shape, Promise-based):
//   const { groth16, wtns, zKey, r1cs } = require('zkfl-snarkjs');
//   const { proof, publicSignals } = await groth16.fullProve(input, 'c_js/c.wasm', 'c_final.zkey');
//   const { proof, publicSignals } = await groth16.prove('c_final.zkey', 'w.wtns');
//   const ok = await groth16.verify(vKey, publicSignals, proof);
//   const wtnsBuffer = await wtns.calculate(input, 'c_js/c.wasm');
//   const vKey = await zKey.exportVerificationKey('c_final.zkey');
//   const info = await r1cs.info('c.r1cs');
'use strict';
// ZKFL_CLI_TIMING=<file>: one JSON line per invocation with the stages of the CLI (ms since this
// node process started): bench.py's cli_prove leg breaks `npx snarkjs groth16 prove` down with it.
const T_ENTRY = process.uptime() * 1000;
const TIMING = process.env.ZKFL_CLI_TIMING || null;
const marks = [['entry', T_ENTRY]];
function mark(name) { if (TIMING) marks.push([name, process.uptime() * 1000]); }
const fs = require('fs');
const path = require('path');

const addon = require(path.join(__dirname, 'zkfl.node'));
mark('addon');
if (TIMING) {
  process.on('exit', () => {
    mark('exit');
    fs.appendFileSync(TIMING, JSON.stringify({ argv: process.argv.slice(2), marks }) + '\n');
  });
}

const Q = BigInt('21888242871839275222246405745257275088696311157297823662689037894645226208583');
let ctx = null;
const keys = new Map();
const progs = new Map();

function context() {
  if (ctx === null) ctx = addon.createContext(parseInt(process.env.LOCAL_RANK || '0', 10));
  return ctx;
}

function leToBig(buf, off) {
  let v = BigInt(0);
  for (let i = 31; i >= 0; i--) v = (v << BigInt(8)) | BigInt(buf[off + i]);
  return v;
}

function leToDec(buf, off) { return leToBig(buf, off).toString(); }

function proofToJson(p) {
  const v = [];
  for (let i = 0; i < 8; i++) v.push(leToDec(p, 32 * i));
  return {
    pi_a: [v[0], v[1], '1'],
    pi_b: [[v[2], v[3]], [v[4], v[5]], ['1', '0']],
    pi_c: [v[6], v[7], '1'],
    protocol: 'groth16',
    curve: 'bn128',
  };
}

function publicToJson(buf) {
  const pub = [];
  for (let i = 0; i < buf.length / 32; i++) pub.push(leToDec(buf, 32 * i));
  return pub;
}

function read(x) { return Buffer.isBuffer(x) ? x : fs.readFileSync(x); }

function key(zkey) {
  const id = Buffer.isBuffer(zkey) ? zkey : path.resolve(zkey);
  let k = keys.get(id);
  if (!k) {
    // the context comes up on a thread of its own (addon.createContext) while this thread maps and
    // parses the key file (zkfl_zkey_file_open); the load then waits for it
    const c = context();
    mark('context');
    if (Buffer.isBuffer(zkey)) {
      k = addon.loadKey(c, zkey);
    } else {
      const f = addon.openKeyFile(id);
      mark('zkey_read');
      addon.contextReady(c);
      mark('context_wait');
      k = addon.loadKeyFile(c, f);
    }
    mark('key_load');
    keys.set(id, k);
  }
  return k;
}

// The circuit's witness program: the image itself, or a compiled .zkwp beside a circom .wasm.
function programImage(wasm) {
  if (Buffer.isBuffer(wasm)) return wasm;
  const buf = fs.readFileSync(wasm);
  if (buf.length >= 4 && buf.toString('latin1', 0, 4) === 'zkwp') return buf;
  const stem = path.basename(wasm).replace(/\.wasm$/, '');
  for (const d of [path.dirname(wasm), path.dirname(path.dirname(wasm))]) {
    const cand = path.join(d, stem + '.zkwp');
    if (fs.existsSync(cand)) return fs.readFileSync(cand);
  }
  throw new Error(`${wasm}: a circom WASM witness calculator; compile the circuit with ` +
                  '`python -m zkfl compile --circom-layout` (or place <circuit>.zkwp beside it)');
}

function program(wasm) {
  const id = Buffer.isBuffer(wasm) ? wasm : path.resolve(wasm);
  let p = progs.get(id);
  if (!p) {
    p = addon.loadProgram(context(), programImage(wasm));
    progs.set(id, p);
  }
  return p;
}

function inputText(input) {
  if (typeof input === 'string') return input;
  return JSON.stringify(input, (k, v) => (typeof v === 'bigint' ? v.toString() : v));
}

async function prove(zkey, wtnsFile) {
  const k = key(zkey);
  const wtns = read(wtnsFile);
  mark('wtns_read');
  const r = await addon.prove(context(), k, wtns);
  mark('prove');
  return { proof: proofToJson(r.proof), publicSignals: publicToJson(r.publicSignals) };
}

// snarkjs groth16.fullProve(input, wasmFile, zkeyFileName): the witness is computed on the GPU
// straight into HBM and proven there (zkfl_groth16_full_prove_json); nothing but the proof and
// the public signals comes back.
async function fullProve(input, wasmFile, zkeyFileName) {
  const r = await addon.fullProve(context(), key(zkeyFileName), program(wasmFile), inputText(input));
  return { proof: proofToJson(r.proof), publicSignals: publicToJson(r.publicSignals) };
}

function decToLe(x) {
  let v = BigInt(x);
  const b = Buffer.alloc(32);
  for (let i = 0; i < 32; i++) { b[i] = Number(v & BigInt(255)); v >>= BigInt(8); }
  if (v !== BigInt(0)) throw new Error('value does not fit in 256 bits: ' + x);
  return b;
}

function g1Buf(p) {
  if (BigInt(p[2]) === BigInt(0)) return Buffer.alloc(64);
  return Buffer.concat([decToLe(p[0]), decToLe(p[1])]);
}

function g2Buf(p) {
  if (BigInt(p[2][0]) === BigInt(0) && BigInt(p[2][1]) === BigInt(0)) return Buffer.alloc(128);
  return Buffer.concat([decToLe(p[0][0]), decToLe(p[0][1]), decToLe(p[1][0]), decToLe(p[1][1])]);
}

// vkey.json -> the C-ABI vk image (include/zkfl.h, zkfl_groth16_verify)
function vkBuffer(vk) {
  const n = Buffer.alloc(4);
  n.writeUInt32LE(vk.nPublic, 0);
  return Buffer.concat([n, g1Buf(vk.vk_alpha_1), g2Buf(vk.vk_beta_2), g2Buf(vk.vk_gamma_2), g2Buf(vk.vk_delta_2),
    ...vk.IC.map(g1Buf)]);
}

async function verify(vk, publicSignals, proof) {
  const pr = Buffer.concat([g1Buf(proof.pi_a), g2Buf(proof.pi_b), g1Buf(proof.pi_c)]);
  const pub = Buffer.concat(publicSignals.map(decToLe).concat([Buffer.alloc(0)]));
  return addon.verify(context(), vkBuffer(vk), pub, pr);
}

async function wtnsCalculate(input, wasm) {
  return addon.witness(context(), program(wasm), inputText(input));
}

// --- iden3 binfile readers for the setup-side commands (SURVEY.md Appendix A) ---
function sections(buf, magic) {
  if (buf.length < 12 || buf.toString('latin1', 0, 4) !== magic) throw new Error(`not a ${magic} file`);
  const n = buf.readUInt32LE(8);
  const out = {};
  let off = 12;
  for (let i = 0; i < n; i++) {
    if (off + 12 > buf.length) throw new Error('truncated section header');
    const type = buf.readUInt32LE(off);
    const size = Number(buf.readBigUInt64LE(off + 4));
    off += 12;
    if (size > buf.length - off) throw new Error('truncated section');
    if (!(type in out)) out[type] = buf.subarray(off, off + size);
    off += size;
  }
  return out;
}

function modpow(b, e, m) {
  let r = BigInt(1);
  b %= m;
  while (e > BigInt(0)) {
    if (e & BigInt(1)) r = (r * b) % m;
    b = (b * b) % m;
    e >>= BigInt(1);
  }
  return r;
}

// snarkjs `zkey export verificationkey`: zkey section 2 points are Montgomery form over q.
async function exportVerificationKey(zkeyFile) {
  const s = sections(read(zkeyFile), 'zkey');
  const h = s[2];
  if (!h || h.length < 84 + 64 * 3 + 128 * 3 || !s[3]) throw new Error('zkey: header');
  const rinv = modpow(BigInt(2) ** BigInt(256) % Q, Q - BigInt(2), Q);
  const fq = (b, o) => ((leToBig(b, o) * rinv) % Q);
  const g1 = (b, o) => {
    const x = fq(b, o), y = fq(b, o + 32);
    return x === BigInt(0) && y === BigInt(0) ? ['0', '1', '0'] : [x.toString(), y.toString(), '1'];
  };
  const g2 = (b, o) => [[fq(b, o).toString(), fq(b, o + 32).toString()],
    [fq(b, o + 64).toString(), fq(b, o + 96).toString()], ['1', '0']];
  const nPublic = h.readUInt32LE(76);
  const p = 84;  // alpha1 64 | beta1 64 | beta2 128 | gamma2 128 | delta1 64 | delta2 128
  const vk = {
    protocol: 'groth16', curve: 'bn128', nPublic,
    vk_alpha_1: g1(h, p), vk_beta_2: g2(h, p + 128), vk_gamma_2: g2(h, p + 256), vk_delta_2: g2(h, p + 448),
  };
  const gt = addon.pairing(context(), g1Buf(vk.vk_alpha_1), g2Buf(vk.vk_beta_2));   // e(alpha1, beta2) on the GPU
  const v = [];
  for (let i = 0; i < 12; i++) v.push(leToDec(gt, 32 * i));
  vk.vk_alphabeta_12 = [0, 1].map((i) => [0, 1, 2].map((j) => v.slice(6 * i + 2 * j, 6 * i + 2 * j + 2)));
  vk.IC = [];
  for (let i = 0; i <= nPublic; i++) vk.IC.push(g1(s[3], 64 * i));
  return vk;
}

// snarkjs `r1cs info`: header section 1 of the .r1cs (iden3 r1cs v1)
async function r1csInfo(r1csFile) {
  const h = sections(read(r1csFile), 'r1cs')[1];
  if (!h || h.length < 4) throw new Error('r1cs: header');
  const n8 = h.readUInt32LE(0);
  const o = 4 + n8;
  return {
    curve: 'bn-128', nVars: h.readUInt32LE(o), nOutputs: h.readUInt32LE(o + 4), nPubInputs: h.readUInt32LE(o + 8),
    nPrvInputs: h.readUInt32LE(o + 12), nLabels: Number(h.readBigUInt64LE(o + 16)), nConstraints: h.readUInt32LE(o + 24),
  };
}

module.exports = {
  groth16: { prove, fullProve, verify },
  wtns: { calculate: wtnsCalculate },
  zKey: { exportVerificationKey },
  r1cs: { info: r1csInfo },
  addon, proofToJson, vkBuffer,
};

// A CLI command's end: its outputs are written (synchronously) by now, so after the 'exit'
// listeners (the timing record) the process leaves with _exit -- the device memory of its key and
// context goes back with the process, without the HIP runtime's teardown (tens of ms for a large
// key).  ZKFL_CLI_FULL_EXIT=1: a normal process.exit.
function quit(code) {
  if (addon.quickExit && !process.env.ZKFL_CLI_FULL_EXIT) {
    process.emit('exit', code);
    addon.quickExit(code);
  }
  process.exit(code);
}

function done(p) {
  p.then((code) => quit(code || 0)).catch((e) => { console.error('[ERROR] snarkJS: ' + e.message); quit(1); });
}

// The one-time ceremony commands (powersoftau new|contribute|prepare phase2, groth16 setup,
// zkey new|contribute and their aliases; tests/test_secureagg.cjs:25-57,
// tests/full_system_simulation.mjs:713-730) are served by the package's Python host, which drives
// the same libzkfl (zkfl_setup_*: scalar multiplications, group FFTs and sparse combinations on the
// GPU): `python3 -m zkfl <the same argv>` as a child process, its exit status passed through.
const CEREMONY = new Set(['powersoftau', 'ptn', 'ptc', 'pt2', 'g16s', 'zkn', 'zkc']);

function isCeremony(argv) {
  const a = argv.filter((x) => !x.startsWith('-'));
  return CEREMONY.has(a[0]) || (a[0] === 'groth16' && a[1] === 'setup') ||
    (a[0] === 'zkey' && (a[1] === 'new' || a[1] === 'contribute'));
}

function runCeremony(argv) {
  const { spawnSync } = require('child_process');
  const pkg = path.join(__dirname, '..');
  const env = Object.assign({}, process.env, {
    PYTHONPATH: pkg + (process.env.PYTHONPATH ? path.delimiter + process.env.PYTHONPATH : ''),
  });
  const r = spawnSync(process.env.ZKFL_PYTHON || 'python3', ['-m', 'zkfl'].concat(argv), { stdio: 'inherit', env });
  if (r.error) {
    console.error('[ERROR] snarkJS: cannot start the zkfl ceremony host: ' + r.error.message);
    return 1;
  }
  return r.status === null ? 1 : r.status;
}

if (require.main === module && isCeremony(process.argv.slice(2))) {
  process.exit(runCeremony(process.argv.slice(2)));
} else if (require.main === module) {
  const a = process.argv.slice(2).filter((x) => !x.startsWith('-'));
  const [cmd, sub] = a;
  const w = (f, o) => fs.writeFileSync(f, JSON.stringify(o, null, 1));
  if (cmd === 'groth16' && sub === 'prove' && a.length >= 6) {
    done(prove(a[2], a[3]).then(({ proof, publicSignals }) => {
      w(a[4], proof);
      w(a[5], publicSignals);
      mark('json_write');
    }));
  } else if (cmd === 'groth16' && sub === 'fullprove' && a.length >= 7) {
    done(fullProve(fs.readFileSync(a[2], 'utf8'), a[3], a[4]).then(({ proof, publicSignals }) => {
      w(a[5], proof);
      w(a[6], publicSignals);
    }));
  } else if (cmd === 'groth16' && sub === 'verify' && a.length >= 5) {
    const rd = (f) => JSON.parse(fs.readFileSync(f, 'utf8'));
    done(verify(rd(a[2]), rd(a[3]), rd(a[4])).then((ok) => {
      if (ok) { console.log('[INFO]  snarkJS: OK!'); return 0; }
      console.error('[ERROR] snarkJS: Invalid proof');
      return 1;
    }));
  } else if (cmd === 'wtns' && sub === 'calculate' && a.length >= 5) {
    done(wtnsCalculate(fs.readFileSync(a[3], 'utf8'), a[2]).then((buf) => fs.writeFileSync(a[4], buf)));
  } else if (cmd === 'zkey' && sub === 'export' && a[2] === 'verificationkey' && a.length >= 5) {
    done(exportVerificationKey(a[3]).then((vk) => w(a[4], vk)));
  } else if (cmd === 'r1cs' && sub === 'info' && a.length >= 3) {
    done(r1csInfo(a[2]).then((i) => {
      console.log(`[INFO]  snarkJS: Curve: ${i.curve}`);
      console.log(`[INFO]  snarkJS: # of Wires: ${i.nVars}`);
      console.log(`[INFO]  snarkJS: # of Constraints: ${i.nConstraints}`);
      console.log(`[INFO]  snarkJS: # of Private Inputs: ${i.nPrvInputs}`);
      console.log(`[INFO]  snarkJS: # of Public Inputs: ${i.nPubInputs}`);
      console.log(`[INFO]  snarkJS: # of Labels: ${i.nLabels}`);
      console.log(`[INFO]  snarkJS: # of Outputs: ${i.nOutputs}`);
    }));
  } else if (cmd === 'version' || process.argv.includes('--version')) {
    console.log('zkfl-snarkjs (libzkfl ABI ' + addon.version() + ')');
  } else {
    console.error('usage: snarkjs groth16 prove <zkey> <wtns> <proof.json> <public.json>\n' +
                  '       snarkjs groth16 fullprove <input.json> <circuit.wasm> <zkey> <proof.json> <public.json>\n' +
                  '       snarkjs groth16 verify <vkey.json> <public.json> <proof.json>\n' +
                  '       snarkjs wtns calculate <circuit.wasm> <input.json> <out.wtns>\n' +
                  '       snarkjs zkey export verificationkey <zkey> <vkey.json>\n' +
                  '       snarkjs r1cs info <circuit.r1cs>\n' +
                  '       snarkjs powersoftau new bn128 <power> <out.ptau>\n' +
                  '       snarkjs powersoftau contribute <in.ptau> <out.ptau> [-e=entropy] [--name=name]\n' +
                  '       snarkjs powersoftau prepare phase2 <in.ptau> <out.ptau>\n' +
                  '       snarkjs groth16 setup <circuit.r1cs> <pot.ptau> <circuit_0000.zkey>\n' +
                  '       snarkjs zkey contribute <in.zkey> <out.zkey> [--name=name] [-e=entropy]');
    process.exit(99);
  }
}
