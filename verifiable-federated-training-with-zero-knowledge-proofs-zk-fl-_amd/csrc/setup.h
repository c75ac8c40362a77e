// Setup-side group primitives for gfx950: the bulk work of the snarkjs ceremony commands
// [ext] that the reference runs once per circuit (tests/test_secureagg.cjs:25-57,
// tests/full_system_simulation.mjs:713-730):
//   powersoftau contribute     tauG1[i] *= tau^i, alphaTauG1[i] *= alpha tau^i, ...  -> setup_scale
//   powersoftau prepare phase2 Lagrange bases = inverse FFT over the group              -> setup_lagrange
//   groth16 setup              A_i = sum_j a_ij L_j(tau) G1, ... (sparse combinations)   -> setup_lincomb
//   zkey contribute            delta *= d, C_i and H_j *= 1/d                           -> setup_scale
// Points are affine Montgomery (the LEM bytes of ptau / zkey sections, infinity = all zero),
// scalars 32-byte little-endian standard form.  All three are one lane per point operation
// over XYZZ coordinates (curve.h); they are one-time setup work, not on the proving path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace zkfl {

// out[i] = k_i * P_i, n points.
hipError_t setup_scale(bool g2, hipStream_t st, const uint8_t* points, const uint8_t* scalars, size_t n,
                       uint8_t* out);

// out[j] = (1/N) sum_i w^{-ij} P_i, N = 2^logn, w = Fr.w[logn] (ffjavascript roots, nqr = 5).
// For P_i = tau^i G this is L_j(tau) G, the snarkjs `prepare phase2` Lagrange evaluation.
hipError_t setup_lagrange(bool g2, hipStream_t st, const uint8_t* points, int logn, uint8_t* out);

// out[r] = sum_{t in [rowptr[r], rowptr[r+1])} coefs[t] * bases[idx[t]], n_out rows (empty row ->
// infinity).  The caller validated idx[t] < n_bases and the row pointers (host side).
hipError_t setup_lincomb(bool g2, hipStream_t st, const uint8_t* bases, size_t n_bases, size_t n_out,
                         const uint64_t* rowptr, const uint32_t* idx, const uint8_t* coefs, uint8_t* out);

}  // namespace zkfl
