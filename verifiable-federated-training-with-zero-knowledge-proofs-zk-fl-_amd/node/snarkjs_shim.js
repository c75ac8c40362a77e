#!/usr/bin/env node
// snarkjs-compatible CLI/API shim over the N-API addon (zkfl.node -> libzkfl.so -> HIP).
//
// CLI (same argument order and files as the reference's execSync strings,
// tests/full_system_simulation.mjs:773-776):
//   node snarkjs_shim.js groth16 prove <circuit_final.zkey> <witness.wtns> <proof.json> <public.json>
// API (snarkjs shape):
//   const { groth16 } = require('./snarkjs_shim.js');
//   const { proof, publicSignals } = await groth16.prove(zkeyFileOrBuffer, wtnsFileOrBuffer);
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

module.exports = { groth16: { prove }, addon, proofToJson };

if (require.main === module) {
  const [cmd, sub, zkeyF, wtnsF, proofF, publicF] = process.argv.slice(2);
  if (cmd === 'groth16' && sub === 'prove' && publicF) {
    prove(zkeyF, wtnsF).then(({ proof, publicSignals }) => {
      fs.writeFileSync(proofF, JSON.stringify(proof, null, 1));
      fs.writeFileSync(publicF, JSON.stringify(publicSignals, null, 1));
      process.exit(0);
    }).catch((e) => { console.error(e.message); process.exit(1); });
  } else if (cmd === 'version') {
    console.log('zkfl ' + addon.version());
  } else {
    console.error('usage: snarkjs_shim.js groth16 prove <zkey> <wtns> <proof.json> <public.json>');
    process.exit(99);
  }
}
