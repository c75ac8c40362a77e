#!/usr/bin/env node
// circom's `<circuit>_js/generate_witness.cjs <circuit>.wasm <input.json> <output.wtns>` over libzkfl:
// the witness is computed by the GPU witness engine (zkfl_witness_compute_json) instead of the
// circuit's WASM.  The reference harness runs exactly this command line
// (tests/full_system_simulation.mjs:758-763).  `python -m zkfl compile --circom-layout` writes
// `<circuit>_js/<circuit>.wasm` as the witness-program image (magic "zkwp") and a
// generate_witness.cjs that loads this file, so the harness's command runs unchanged.  A real
// circom .wasm is accepted when a compiled `<circuit>.zkwp` sits next to it (or one directory up).
'use strict';
const { wtns } = require('./snarkjs_shim.js');
const fs = require('fs');

function main(args) {
  const [wasmF, inputF, outF] = args;
  if (!outF) {
    console.error('Usage: node generate_witness.cjs <file.wasm> <input.json> <output.wtns>');
    process.exit(1);
  }
  wtns.calculate(fs.readFileSync(inputF, 'utf8'), wasmF).then((w) => {
    fs.writeFileSync(outF, w);
    process.exit(0);
  }).catch((e) => { console.error(e.message); process.exit(1); });
}

module.exports = { main };

if (require.main === module) main(process.argv.slice(2));
