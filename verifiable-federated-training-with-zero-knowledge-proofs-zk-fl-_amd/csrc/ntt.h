// Radix-2 NTT over Fr for the Groth16 H polynomial on gfx950.
//
// Replaces ffjavascript `Fr.ifft` / `Fr.batchApplyKey` / `Fr.fft` as used by snarkjs
// groth16_prove:  a_coef = ifft(a); a_odd[i] = a_coef[i] * inc^i with
// inc = w[power+1] (shift when power == 28); a_odd_T = fft(a_odd).  Values are Fr in
// Montgomery form; results are field-identical to ffjavascript's (natural order in / out).
//
// Layout: the inverse transform is a decimation-in-frequency pass (natural in, bit-reversed
// out), the coset scale (incl. 1/n) is applied in bit-reversed order, and the forward
// transform is decimation-in-time (bit-reversed in, natural out), so no explicit bit
// reversal pass exists.  Stages whose butterfly span is < 2^NTT_LDS_LOG run fused inside
// LDS (one 1024-element tile = 32 KiB per workgroup); the remaining large-span stages are
// one coalesced global pass each (HBM-bound: 2 x 32 B read + write per butterfly).
#pragma once
#include "common.h"
#include "field.h"

namespace zkfl {

struct NttPlan {
  int logn = 0;
  size_t n = 0;
  Fr* tw_fwd = nullptr;   // [n/2] forward root powers
  Fr* tw_inv = nullptr;   // [n/2] inverse root powers
  Fr* coset = nullptr;    // [n] inc^{bitrev(p)} / n
};

hipError_t ntt_plan_alloc(NttPlan& pl, int logn, hipStream_t st);
void ntt_plan_free(NttPlan& pl);
// In place: nvec vectors (stride vstride) of evaluations on the domain -> evaluations on
// the odd coset (snarkjs ifft + batchApplyKey + fft).
hipError_t ntt_coset_shift(const NttPlan& pl, Fr* d, int nvec, size_t vstride, hipStream_t st);

}  // namespace zkfl
