// Host interface of the GPU Groth16 verifier / pairing (csrc/verify.hip), used by the C ABI in
// csrc/zkfl.hip.  Replaces `snarkjs groth16 verify` [ext] (tests/full_system_simulation.mjs:865-868).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace zkfl {

struct VkDev;  // prepared verification key (device tables + lines), opaque

// vk image: nPublic u32 | alpha1 (64) | beta2 (128) | gamma2 (128) | delta2 (128) | IC[(nPub+1) x 64],
// standard-form little-endian affine coordinates (the proof's encoding).  Returns a ZKFL_* code.
int vk_prepare(const uint8_t* vk, size_t len, hipStream_t st, VkDev** out, std::string& err);
void vk_free(VkDev* vk);
bool vk_same(const VkDev* vk, const uint8_t* bytes, size_t len);
uint32_t vk_npub(const VkDev* vk);

// results[i] = 1 valid / 0 invalid for n proofs (256 B each) with npub public signals each (32 B).
int verify_batch(const VkDev* vk, size_t n, const uint8_t* pubs, const uint8_t* proofs, int32_t* results,
                 hipStream_t st, std::string& err);

// e(P_i, Q_i) (final_exp != 0) or the bare Miller loop value, 384 B std-form Fq12 each
// (ffjavascript toObject order).  Points that are off-curve / out of G2 -> ZKFL_E_ARG.
int pairing_batch(size_t n, const uint8_t* g1, const uint8_t* g2, int final_exp, uint8_t* out, hipStream_t st,
                  std::string& err);

}  // namespace zkfl
