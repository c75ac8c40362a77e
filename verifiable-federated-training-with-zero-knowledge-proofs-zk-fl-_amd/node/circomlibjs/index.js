// circomlibjs-shaped Poseidon on the GPU (zkfl.node -> libzkfl zkfl_poseidon_batch).
//
// The reference harness imports `buildPoseidon` from circomlibjs [ext]
// (tests/full_system_simulation.mjs:25, :134-137; tests/test_secureagg.cjs:67-69) and computes every
// off-circuit commitment with it: vectorHash (:139-155), gradientCommitment (:159-164),
// weightCommitment (:168-170), keyMaterialCommitment (:174-177), derivePairwiseMask (:181-196),
// buildMerkleTree / getMerkleProof (:198-238).  This package answers that import: installed as
// `circomlibjs` (a `file:` dependency on this directory), `await buildPoseidon()` returns a
// callable with circomlibjs's contract
//     poseidon(inputs[, initState = 0, nOut = 1]) -> field element    (1..16 inputs)
//     poseidon.F: e, toObject, toString, fromObject, eq, isZero, add, sub, mul, neg, square, inv,
//                 div, zero, one, p, n8
// where an element is a 32-byte Uint8Array in Montgomery form (little-endian x * 2^256 mod r), as
// in ffjavascript's WasmField1, and inputs may be BigInt, number, decimal / 0x string or elements
// (reduced mod r, negatives included).  The hash is circomlib's Poseidon (t = n + 1, R_F = 8),
// bit-identical on the GPU (csrc/poseidon.h; pinned by data/test_input_v5.json in the tests).
// Extensions beyond circomlibjs, for batched server-side work on the same device:
//     poseidon.batch(rows) -> [BigInt]             one GPU launch for many equal-arity hashes
//     zkfl.vectorHash(values) / zkfl.vectorHashBatch(vectors) -> BigInt / [BigInt]
//     zkfl.buildMerkleTree(leafHashes, depth) -> levels of BigInt (the harness's `tree`)
'use strict';
const path = require('path');

const addon = require(path.join(__dirname, '..', 'zkfl.node'));

const P = BigInt('21888242871839275222246405745257275088548364400416034343698204186575808495617');
const R256 = (BigInt(1) << BigInt(256)) % P;

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
const RINV = modpow(R256, P - BigInt(2), P);

let ctx = null;
function context() {
  if (ctx === null) ctx = addon.createContext(parseInt(process.env.LOCAL_RANK || '0', 10));
  return ctx;
}

function mod(x) {
  const v = x % P;
  return v < BigInt(0) ? v + P : v;
}

function leWrite(buf, off, v) {
  for (let i = 0; i < 32; i++) {
    buf[off + i] = Number(v & BigInt(255));
    v >>= BigInt(8);
  }
}

function leRead(buf, off) {
  let v = BigInt(0);
  for (let i = 31; i >= 0; i--) v = (v << BigInt(8)) | BigInt(buf[off + i]);
  return v;
}

function isElement(x) { return x instanceof Uint8Array && x.length === 32; }

// any accepted input -> standard-form BigInt in [0, r)
function toStd(x) {
  if (isElement(x)) return mod(leRead(x, 0) * RINV);
  if (typeof x === 'bigint') return mod(x);
  if (typeof x === 'number') {
    if (!Number.isInteger(x)) throw new Error('field element from a non-integer number: ' + x);
    return mod(BigInt(x));
  }
  if (typeof x === 'string') {
    const s = x.trim();
    return mod(s.startsWith('-') ? -BigInt(s.slice(1)) : BigInt(s));
  }
  throw new Error('unsupported field element type: ' + typeof x);
}

function fromStd(v) {
  const out = new Uint8Array(32);
  leWrite(out, 0, mod(v * R256));
  return out;
}

const F = {
  p: P,
  n8: 32,
  e: (x) => (isElement(x) ? x : fromStd(toStd(x))),
  fromObject: (x) => fromStd(toStd(x)),
  toObject: (a) => toStd(a),
  toString: (a, radix) => toStd(a).toString(radix || 10),
  eq: (a, b) => toStd(a) === toStd(b),
  isZero: (a) => toStd(a) === BigInt(0),
  add: (a, b) => fromStd(toStd(a) + toStd(b)),
  sub: (a, b) => fromStd(toStd(a) - toStd(b)),
  mul: (a, b) => fromStd(toStd(a) * toStd(b)),
  neg: (a) => fromStd(-toStd(a)),
  square: (a) => fromStd(toStd(a) * toStd(a)),
  inv: (a) => fromStd(modpow(toStd(a), P - BigInt(2), P)),
  div: (a, b) => fromStd(toStd(a) * modpow(toStd(b), P - BigInt(2), P)),
};
F.zero = fromStd(BigInt(0));
F.one = fromStd(BigInt(1));

function packRows(rows, width) {
  const buf = Buffer.alloc(32 * width * rows.length);
  rows.forEach((row, i) => {
    if (!Array.isArray(row) || row.length !== width) throw new Error('poseidon: rows must have equal length');
    row.forEach((x, j) => leWrite(buf, 32 * (i * width + j), toStd(x)));
  });
  return buf;
}

function unpack(buf) {
  const out = [];
  for (let i = 0; i < buf.length / 32; i++) out.push(leRead(buf, 32 * i));
  return out;
}

function poseidon(inputs, initState, nOut) {
  if (!Array.isArray(inputs) || inputs.length < 1 || inputs.length > 16) {
    throw new Error('poseidon: between 1 and 16 inputs');
  }
  if (initState !== undefined && initState !== null && toStd(initState) !== BigInt(0)) {
    throw new Error('poseidon: only initState = 0 (circomlib Poseidon) is supported');
  }
  if (nOut !== undefined && nOut !== 1) throw new Error('poseidon: only nOut = 1 is supported');
  const out = addon.poseidon(context(), inputs.length, 1, packRows([inputs], inputs.length));
  return fromStd(leRead(out, 0));
}
poseidon.F = F;
poseidon.batch = (rows) => {
  if (!rows.length) return [];
  const w = rows[0].length;
  if (w < 1 || w > 16) throw new Error('poseidon.batch: between 1 and 16 inputs per row');
  return unpack(addon.poseidon(context(), w, rows.length, packRows(rows, w)));
};

async function buildPoseidon() { return poseidon; }

const zkfl = {
  vectorHash: (values) => unpack(addon.vectorHash(context(), values.length, 1, packRows([values], values.length)))[0],
  vectorHashBatch: (vectors) => {
    if (!vectors.length) return [];
    const n = vectors[0].length;
    return unpack(addon.vectorHash(context(), n, vectors.length, packRows(vectors, n)));
  },
  buildMerkleTree: (leafHashes, depth) => {
    const flat = unpack(addon.merkleBuild(context(), packRows(leafHashes.map((x) => [x]), 1), depth));
    const tree = [];
    let pos = 0;
    for (let l = 0; l <= depth; l++) {
      const w = 1 << (depth - l);
      tree.push(flat.slice(pos, pos + w));
      pos += w;
    }
    return tree;
  },
};

module.exports = {
  buildPoseidon,
  buildPoseidonReference: buildPoseidon,
  buildPoseidonOpt: buildPoseidon,
  buildPoseidonWasm: buildPoseidon,
  zkfl,
};
