#!/usr/bin/env node
// snarkjs-compatible CLI/API shim over the N-API addon (zkfl.node -> libzkfl.so -> HIP).
//
// CLI (same argument order and files as the reference's execSync strings,
// tests/full_system_simulation.mjs:773-776):
//   node snarkjs_shim.js groth16 prove <circuit_final.zkey> <witness.wtns> <proof.json> <public.json>
//   node snarkjs_shim.js groth16 verify <verification_key.json> <public.json> <proof.json>
//   node snarkjs_shim.js wtns calculate <circuit.zkwp> <input.json> <witness.wtns>
//     (snarkjs wtns calculate / generate_witness.cjs, :758-767; the .zkwp witness program image
//      from `python -m zkfl compile` plays the role of the circuit's .wasm)
//     (:865-868; exit 0 + "OK!" when valid, exit 1 + "Invalid proof" otherwise)
// API (snarkjs shape):
//   const { groth16 } = require('./snarkjs_shim.js');
//   const { proof, publicSignals } = await groth16.prove(zkeyFileOrBuffer, wtnsFileOrBuffer);
//   const ok = await groth16.verify(vKeyObject, publicSignals, proof);
//   const wtnsBuffer = await wtns.calculate(inputObject, zkwpFileOrBuffer);
'use strict';
const fs = require('fs');
const path = require('path');

const addon = require(path.join(__dirname, 'zkfl.node'));

let ctx = null;
const keys = new Map();

function leToDec(buf, off) {
  let v = BigInt(0);
  for (let i = 31; i >= 0; i--) v = (v << BigInt(8)) | BigInt(buf[off + i]);
  return v.toString();
}

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

function read(x) { return Buffer.isBuffer(x) ? x : fs.readFileSync(x); }

async function prove(zkey, wtns) {
  if (ctx === null) ctx = addon.createContext(parseInt(process.env.LOCAL_RANK || '0', 10));
  const id = Buffer.isBuffer(zkey) ? zkey : path.resolve(zkey);
  let key = keys.get(id);
  if (!key) {
    key = addon.loadKey(ctx, read(zkey));
    keys.set(id, key);
  }
  const r = await addon.prove(ctx, key, read(wtns));
  const pub = [];
  for (let i = 0; i < r.publicSignals.length / 32; i++) pub.push(leToDec(r.publicSignals, 32 * i));
  return { proof: proofToJson(r.proof), publicSignals: pub };
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
  if (ctx === null) ctx = addon.createContext(parseInt(process.env.LOCAL_RANK || '0', 10));
  const pr = Buffer.concat([g1Buf(proof.pi_a), g2Buf(proof.pi_b), g1Buf(proof.pi_c)]);
  const pub = Buffer.concat(publicSignals.map(decToLe).concat([Buffer.alloc(0)]));
  return addon.verify(ctx, vkBuffer(vk), pub, pr);
}

const progs = new Map();

async function wtnsCalculate(input, zkwp) {
  if (ctx === null) ctx = addon.createContext(parseInt(process.env.LOCAL_RANK || '0', 10));
  const id = Buffer.isBuffer(zkwp) ? zkwp : path.resolve(zkwp);
  let prog = progs.get(id);
  if (!prog) {
    prog = addon.loadProgram(ctx, read(zkwp));
    progs.set(id, prog);
  }
  const text = typeof input === 'string' ? input : JSON.stringify(input, (k, v) => (typeof v === 'bigint' ? v.toString() : v));
  return addon.witness(ctx, prog, text);
}

module.exports = { groth16: { prove, verify }, wtns: { calculate: wtnsCalculate }, addon, proofToJson, vkBuffer };

if (require.main === module) {
  const [cmd, sub, zkeyF, wtnsF, proofF, publicF] = process.argv.slice(2);
  if (cmd === 'groth16' && sub === 'prove' && publicF) {
    prove(zkeyF, wtnsF).then(({ proof, publicSignals }) => {
      fs.writeFileSync(proofF, JSON.stringify(proof, null, 1));
      fs.writeFileSync(publicF, JSON.stringify(publicSignals, null, 1));
      process.exit(0);
    }).catch((e) => { console.error(e.message); process.exit(1); });
  } else if (cmd === 'groth16' && sub === 'verify' && proofF) {
    // argument order: verify <vkey.json> <public.json> <proof.json>
    const [vkF, pubF, prF] = [zkeyF, wtnsF, proofF];
    const rd = (f) => JSON.parse(fs.readFileSync(f, 'utf8'));
    verify(rd(vkF), rd(pubF), rd(prF)).then((ok) => {
      if (ok) { console.log('[INFO]  snarkJS: OK!'); process.exit(0); }
      console.error('[ERROR] snarkJS: Invalid proof');
      process.exit(1);
    }).catch((e) => { console.error(e.message); process.exit(1); });
  } else if (cmd === 'wtns' && sub === 'calculate' && proofF) {
    // argument order: wtns calculate <circuit.zkwp> <input.json> <out.wtns>
    const [progF, inputF, outF] = [zkeyF, wtnsF, proofF];
    wtnsCalculate(fs.readFileSync(inputF, 'utf8'), progF).then((w) => {
      fs.writeFileSync(outF, w);
      process.exit(0);
    }).catch((e) => { console.error(e.message); process.exit(1); });
  } else if (cmd === 'version') {
    console.log('zkfl ' + addon.version());
  } else {
    console.error('usage: snarkjs_shim.js groth16 prove <zkey> <wtns> <proof.json> <public.json>\n' +
                  '       snarkjs_shim.js groth16 verify <vkey.json> <public.json> <proof.json>\n' +
                  '       snarkjs_shim.js wtns calculate <circuit.zkwp> <input.json> <out.wtns>');
    process.exit(99);
  }
}
