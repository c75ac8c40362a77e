// Host interface of the GPU Poseidon / vector-hash / Merkle-tree engine (csrc/merkle.hip), used by
// the C ABI in csrc/zkfl.hip.  Replaces the reference's server/data-side circomlibjs hashing
// (tests/full_system_simulation.mjs:139-238: vectorHash, gradient/weight/key commitments,
// buildMerkleTree, getMerkleProof; computeDatasetCommitment :309-335).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "field.h"

namespace zkfl {

constexpr uint32_t POS_MAX_ARITY = 16;  // circomlib Poseidon(n): t = n + 1 <= 17
constexpr uint32_t VHASH_CHUNK = 16;    // CONFIG.CHUNK_SIZE / vector_hash.circom:59

// circomlib parameter generation restated on the host (Grain LFSR, zkfl/field.py): width t in
// 2..17 -> raw standard-form round constants (count (8 + R_P(t)) * t) and the Cauchy points
// x[t] | y[t] whose MDS is M[i][j] = 1 / (x_i + y_j).  32 B little-endian each.
uint32_t pos_rp(uint32_t t);
void pos_params_raw(uint32_t t, uint8_t* consts_out, uint8_t* xy_out);

struct PosTables;  // device-resident Montgomery constants for every width (built once per context)
int pos_tables_create(PosTables** out, hipStream_t st, std::string& err);
void pos_tables_free(PosTables* p);

// out[i] = in[i] in Montgomery form (device, n elements)
hipError_t fr_to_mont_batch(const Fr* in, size_t n, Fr* out, hipStream_t st);

// out[i] = Poseidon(in[i*arity .. i*arity+arity)) for n rows; std form in and out (device).
hipError_t poseidon_batch(const PosTables* P, uint32_t arity, size_t n, const Fr* in, Fr* out, hipStream_t st);

// out[i] = vectorHash(in[i*len .. i*len+len)) (len <= 256: chunks of 16, then Poseidon of the
// chunk hashes).  in std; out Montgomery when out_mont (tree leaves), else std.  scratch: n *
// ceil(len/16) Fr when len > 16.
hipError_t vector_hash_batch(const PosTables* P, uint32_t len, size_t n, const Fr* in, Fr* out, bool out_mont,
                             Fr* scratch, hipStream_t st);

// buildMerkleTree over n Montgomery-form leaves (device) padded to 2^depth with Poseidon([0]):
// tree_std receives the full padded levels in standard form, level 0 (2^depth) first, root last
// ((2^(depth+1) - 1) Fr).  work: merkle_work_size(n, depth) Fr of scratch.
size_t merkle_work_size(size_t n, uint32_t depth);
hipError_t merkle_build(const PosTables* P, const Fr* leaves_mont, size_t n, uint32_t depth, Fr* tree_std, Fr* work,
                        hipStream_t st);

}  // namespace zkfl
