// ES-module entry of the circomlibjs face (`import { buildPoseidon } from 'circomlibjs'`,
// tests/full_system_simulation.mjs:25); the implementation is index.js.
import cjs from './index.js';

export const { buildPoseidon, buildPoseidonReference, buildPoseidonOpt, buildPoseidonWasm, zkfl } = cjs;
export default cjs;
