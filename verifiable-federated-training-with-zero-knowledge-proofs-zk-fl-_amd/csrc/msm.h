// Pippenger multi-scalar multiplication on gfx950 for G1 (Fq) and G2 (Fq2).
//
// Replaces ffjavascript `G1.multiExpAffine` / `G2.multiExpAffine` as called by snarkjs
// groth16_prove for the A, B1, B2, C and H queries (reference
// call site tests/full_system_simulation.mjs:773-776).  Result semantics are identical:
// sum_i s_i * P_i with scalars in standard form and affine bases in Montgomery form,
// (0,0) bases and zero scalars contributing nothing.
//
// MI355X design:
//  * Bases are fixed per proving key, so at key-load time every base P_i is expanded into
//    W = 16 window copies 2^(16 j) P_i (affine, Montgomery), laid out [i][j] (64 B / 128 B
//    each).  One MSM is then a single bucket set: every (i, j) with a non-zero signed 16-bit
//    digit d_ij lands in bucket |d_ij|-1 (2^15 buckets), no per-window bucket reduction and
//    no window combination.  288 GB of HBM makes the 16x base expansion (~2 GB for the
//    2^18-constraint training circuit) free.
//  * Signed digits in [-2^15, 2^15]; the sign is applied by negating y on the fly.
//  * (bucket, entry) pairs are radix-sorted (rocPRIM, 16 key bits), bucket ranges found by
//    adjacent-key compare.  The sorted entries are cut into fixed chunks of L entries, one lane
//    each, independent of bucket boundaries: every lane does exactly L additions (no idle lanes
//    behind a short bucket tail, no task->bucket search), emits a partial sum at each bucket
//    change (first segment -> head[chunk], last -> tail[chunk], a bucket wholly inside the chunk
//    -> its final sum), and k_msm_bucket_sum stitches each bucket from its chunks' partials.
//  * Accumulation uses XYZZ + affine mixed additions (10 Fq mul for G1).
//  * Bucket reduction sum_b (b+1) S_b uses grouped running sums (groups of RG buckets),
//    recursively on the group sums, then a Horner combination.
#pragma once
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "msm_api.h"

namespace zkfl {

// Accumulation kernel configuration per curve (measured on MI355X): G1 fits its
// working set in 128 VGPRs -> 4 waves/SIMD with the pipelined gather; G2's Fq2 working set needs
// > 256 registers, so it runs at 1 wave/SIMD (2 waves cost 130-280 spills in every schedule tried).
#ifndef MSM_G1_WAVES
#define MSM_G1_WAVES 4
#endif
#ifndef MSM_G1_PF
#define MSM_G1_PF true
#endif
#ifndef MSM_G2_WAVES
#define MSM_G2_WAVES 1
#endif
#ifndef MSM_G2_PF
#define MSM_G2_PF true
#endif

// ---------------------------------------------------------------------------
// Key-load-time window expansion: out[i*W + j] = 2^(16 j) * in[i]  (affine)
// ---------------------------------------------------------------------------
template <class F>
__global__ void __launch_bounds__(64) k_msm_expand(const Affine<F>* __restrict__ in, size_t n, Affine<F>* __restrict__ out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  using T = typename F::T;
  Affine<F> p = in[i];
  if (aff_is_inf(p)) {
    for (int j = 0; j < MSM_W; j++) out[i * MSM_W + j] = p;
    return;
  }
  // Keep the 16 window copies in XYZZ in the output slots' scratch (global), with a
  // Montgomery batch inversion of their ZZZ over the 16 copies.
  XYZZ<F> acc = xyzz_from_affine<F>(p);
  T pref[MSM_W];
  XYZZ<F> pts[MSM_W];
  for (int j = 0; j < MSM_W; j++) {
    pts[j] = acc;
    pref[j] = (j == 0) ? acc.ZZZ : F::mul(pref[j - 1], acc.ZZZ);
    if (j + 1 < MSM_W)
      for (int k = 0; k < MSM_C; k++) acc = xyzz_dbl<F>(acc);
  }
  T inv = F::inv(pref[MSM_W - 1]);
  for (int j = MSM_W - 1; j >= 0; j--) {
    T iZZZ = (j == 0) ? inv : F::mul(inv, pref[j - 1]);
    if (j > 0) inv = F::mul(inv, pts[j].ZZZ);
    T iZ = F::mul(pts[j].ZZ, iZZZ);
    Affine<F> a;
    a.x = F::mul(pts[j].X, F::sqr(iZ));
    a.y = F::mul(pts[j].Y, iZZZ);
    out[i * MSM_W + j] = a;
  }
}

// ---------------------------------------------------------------------------
// Per-MSM kernels
// ---------------------------------------------------------------------------
// Signed-digit decomposition; entry (i, j) -> key = bucket, val = (i*W+j) | sign<<31.
static __global__ void k_msm_digits(const uint32_t* __restrict__ scalars, const uint32_t* __restrict__ extra,
                                    const uint32_t* __restrict__ sidx, uint32_t extra_start, size_t n,
                                    uint16_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t si = sidx ? sidx[i] : (uint32_t)i;
  const uint32_t* src = si < extra_start ? scalars + (size_t)si * 8 : extra + (size_t)(si - extra_start) * 8;
  const uint4* sp = reinterpret_cast<const uint4*>(src);
  uint4 a = sp[0], b = sp[1];
  uint32_t s[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint32_t carry = 0;
#pragma unroll
  for (int j = 0; j < MSM_W; j++) {
    uint32_t raw = (s[j >> 1] >> ((j & 1) * 16)) & 0xFFFFu;
    int32_t d = (int32_t)(raw + carry);
    if (d > MSM_NB) {
      d -= (1 << MSM_C);
      carry = 1;
    } else {
      carry = 0;
    }
    size_t e = i * MSM_W + j;
    if (d == 0) {
      keys[e] = MSM_KEY_NONE;
      vals[e] = 0;
    } else {
      uint32_t mag = (uint32_t)(d < 0 ? -d : d);
      keys[e] = (uint16_t)(mag - 1);
      vals[e] = (uint32_t)e | (d < 0 ? 0x80000000u : 0u);
    }
  }
}

static __global__ void k_msm_bounds(const uint16_t* __restrict__ keys, size_t m,
                             uint32_t* __restrict__ bstart, uint32_t* __restrict__ bend,
                             uint32_t* __restrict__ nnz) {
  size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= m) return;
  uint16_t k = keys[p];
  if (k == MSM_KEY_NONE) return;
  if (p == 0 || keys[p - 1] != k) bstart[k] = (uint32_t)p;
  const bool last = (p == m - 1 || keys[p + 1] != k);
  if (last) bend[k] = (uint32_t)(p + 1);
  if (p == m - 1 || keys[p + 1] == MSM_KEY_NONE) *nnz = (uint32_t)(p + 1);  // non-zero digits
}

// Lane c adds the sorted entries [c*L, min(c*L+L, nnz)).  Software-pipelined: the key/index of
// entry p+1 and its base are in flight while entry p is added.
// MINW: minimum waves per SIMD the register allocator must allow; PF: software-pipeline the
// next entry's key/index/base loads behind the current addition (costs one affine point of
// registers).  Chosen per curve in msm_run.
template <class F, int MINW, bool PF>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MINW))) k_msm_accumulate(
                                                        const uint16_t* __restrict__ keys,
                                                        const uint32_t* __restrict__ vals,
                                                        const Affine<F>* __restrict__ bases,
                                                        const uint32_t* __restrict__ nnz_ptr,
                                                        XYZZ<F>* __restrict__ head,
                                                        XYZZ<F>* __restrict__ tail,
                                                        XYZZ<F>* __restrict__ buckets) {
  const size_t c = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nnz = *nnz_ptr;
  const size_t p0 = c * MSM_L;
  if (p0 >= nnz) return;
  const uint32_t p1 = (uint32_t)(p0 + MSM_L < nnz ? p0 + MSM_L : nnz);
  XYZZ<F> acc = xyzz_inf<F>();
  uint32_t cur = keys[p0];
  bool first = true;
  if (PF) {
    uint32_t v0 = vals[p0], k1 = 0, v1 = 0;
    if (p0 + 1 < p1) {
      k1 = keys[p0 + 1];
      v1 = vals[p0 + 1];
    }
    Affine<F> a = bases[v0 & 0x7FFFFFFFu];
    for (uint32_t p = (uint32_t)p0; p < p1; p++) {
      Affine<F> an;
      uint32_t k2 = 0, v2 = 0;
      if (p + 1 < p1) an = bases[v1 & 0x7FFFFFFFu];
      if (p + 2 < p1) {
        k2 = keys[p + 2];
        v2 = vals[p + 2];
      }
      acc = xyzz_madd<F>(acc, (v0 & 0x80000000u) ? aff_neg<F>(a) : a);
      if (p + 1 < p1 && k1 != cur) {  // bucket boundary inside the chunk
        if (first) head[c] = acc;
        else buckets[cur] = acc;     // starts and ends inside this chunk: complete
        first = false;
        acc = xyzz_inf<F>();
        cur = k1;
      }
      v0 = v1;
      v1 = v2;
      k1 = k2;
      a = an;
    }
  } else {
    for (uint32_t p = (uint32_t)p0; p < p1; p++) {
      const uint32_t k = keys[p], v = vals[p];
      if (k != cur) {
        if (first) head[c] = acc;
        else buckets[cur] = acc;
        first = false;
        acc = xyzz_inf<F>();
        cur = k;
      }
      Affine<F> a = bases[v & 0x7FFFFFFFu];
      acc = xyzz_madd<F>(acc, (v & 0x80000000u) ? aff_neg<F>(a) : a);
    }
  }
  if (first) head[c] = acc;
  else tail[c] = acc;
}

// Bucket b = its entries [s, e): stitched from the partials of chunks c0 = s/L .. c1 = (e-1)/L.
template <class F>
__global__ void __launch_bounds__(64) k_msm_bucket_sum(const uint32_t* __restrict__ bstart,
                                                        const uint32_t* __restrict__ bend,
                                                        const uint32_t* __restrict__ nnz_ptr,
                                                        const XYZZ<F>* __restrict__ head,
                                                        const XYZZ<F>* __restrict__ tail,
                                                        XYZZ<F>* __restrict__ buckets) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= MSM_NB) return;
  const uint32_t s = bstart[b], e = bend[b];
  if (s == e) {
    buckets[b] = xyzz_inf<F>();
    return;
  }
  const uint32_t c0 = s / MSM_L, c1 = (e - 1) / MSM_L;
  const bool starts_chunk = (s == c0 * MSM_L);
  if (c0 == c1) {
    const uint32_t nnz = *nnz_ptr;
    const uint32_t cend = (c0 + 1) * MSM_L < nnz ? (c0 + 1) * MSM_L : nnz;
    if (starts_chunk) buckets[b] = head[c0];
    else if (e == cend) buckets[b] = tail[c0];
    return;  // otherwise wholly inside the chunk: written by k_msm_accumulate
  }
  XYZZ<F> acc = starts_chunk ? head[c0] : tail[c0];
  for (uint32_t c = c0 + 1; c <= c1; c++) acc = xyzz_add<F>(acc, head[c]);
  buckets[b] = acc;
}

// One level of the grouped running-sum bucket reduction over in[0..K):
//   acc[g] = sum_{k in group} (k - g*RG + 1) * in[k],   run[g] = sum_{k in group} in[k]
// acc[g] is pre-scaled by RG^level (level doublings) so all levels sum together.
template <class F>
__global__ void __launch_bounds__(64) k_msm_reduce_level(const XYZZ<F>* __restrict__ in, int K, int shift_dbls,
                                   XYZZ<F>* __restrict__ acc_out, XYZZ<F>* __restrict__ run_out) {
  int g = blockIdx.x * blockDim.x + threadIdx.x;
  int G = (K + MSM_RG - 1) / MSM_RG;
  if (g >= G) return;
  int lo = g * MSM_RG;
  int hi = lo + MSM_RG;
  if (hi > K) hi = K;
  XYZZ<F> run = xyzz_inf<F>();
  XYZZ<F> acc = xyzz_inf<F>();
  for (int k = hi - 1; k >= lo; k--) {
    run = xyzz_add<F>(run, in[k]);
    acc = xyzz_add<F>(acc, run);
  }
  for (int d = 0; d < shift_dbls; d++) acc = xyzz_dbl<F>(acc);
  acc_out[g] = acc;
  run_out[g] = run;
}

// out[i] = sum of in[i*8 .. i*8+8)
template <class F>
__global__ void __launch_bounds__(64) k_msm_sum8(const XYZZ<F>* __restrict__ in, int n, XYZZ<F>* __restrict__ out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  int lo = i * 8;
  if (lo >= n) return;
  int hi = lo + 8;
  if (hi > n) hi = n;
  XYZZ<F> acc = in[lo];
  for (int k = lo + 1; k < hi; k++) acc = xyzz_add<F>(acc, in[k]);
  out[i] = acc;
}

// ---------------------------------------------------------------------------
// Host-side plan
// ---------------------------------------------------------------------------
template <class F>
hipError_t msm_bases_alloc(MsmBases<F>& b, size_t n) {
  b.n = n;
  ZK_CHECK(hipMalloc(&b.bases_w, (n ? n : 1) * MSM_W * sizeof(Affine<F>)));
  return hipSuccess;
}

template <class F>
void msm_bases_free(MsmBases<F>& b) {
  if (b.bases_w) (void)hipFree(b.bases_w);
  if (b.sidx) (void)hipFree(b.sidx);
  b = MsmBases<F>();
}

// Expand b.n affine bases (device pointer) into the window table; h_sidx (host, b.n entries)
// is the scalar index map or nullptr for identity.
template <class F>
hipError_t msm_bases_set(MsmBases<F>& b, const Affine<F>* d_bases, const uint32_t* h_sidx, uint32_t extra_start,
                         hipStream_t st) {
  // identity maps never address the extra slots (H has domainSize > nVars entries on small circuits)
  b.extra_start = h_sidx ? extra_start : 0xFFFFFFFFu;
  if (h_sidx && b.n) {
    ZK_CHECK(hipMalloc(&b.sidx, b.n * sizeof(uint32_t)));
    ZK_CHECK(hipMemcpyAsync(b.sidx, h_sidx, b.n * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  }
  if (b.n) hipLaunchKernelGGL(k_msm_expand<F>, dim3(zk_grid(b.n, 64)), dim3(64), 0, st, d_bases, b.n, b.bases_w);
  return hipGetLastError();
}

template <class F>
hipError_t msm_scratch_alloc(MsmScratch<F>& s, size_t cap, hipStream_t st) {
  s.cap = cap;
  const size_t m = cap * MSM_W;
  ZK_CHECK(hipMalloc(&s.keys_in, m * sizeof(uint16_t)));
  ZK_CHECK(hipMalloc(&s.keys_out, m * sizeof(uint16_t)));
  ZK_CHECK(hipMalloc(&s.vals_in, m * sizeof(uint32_t)));
  ZK_CHECK(hipMalloc(&s.vals_out, m * sizeof(uint32_t)));
  ZK_CHECK(rocprim::radix_sort_pairs(nullptr, s.sort_tmp_bytes, s.keys_in, s.keys_out, s.vals_in, s.vals_out, m, 0,
                                     16, st));
  ZK_CHECK(hipMalloc(&s.sort_tmp, s.sort_tmp_bytes));
  ZK_CHECK(hipMalloc(&s.bstart, MSM_NB * sizeof(uint32_t)));
  ZK_CHECK(hipMalloc(&s.bend, MSM_NB * sizeof(uint32_t)));
  s.max_chunks = (m + MSM_L - 1) / MSM_L;
  ZK_CHECK(hipMalloc(&s.head, s.max_chunks * sizeof(XYZZ<F>)));
  ZK_CHECK(hipMalloc(&s.tail, s.max_chunks * sizeof(XYZZ<F>)));
  ZK_CHECK(hipMalloc(&s.buckets, MSM_NB * sizeof(XYZZ<F>)));
  ZK_CHECK(hipMalloc(&s.red_acc, MSM_NB * sizeof(XYZZ<F>)));
  ZK_CHECK(hipMalloc(&s.red_run, MSM_NB * sizeof(XYZZ<F>)));
  ZK_CHECK(hipMalloc(&s.red_tmp, MSM_NB * sizeof(XYZZ<F>)));
  ZK_CHECK(hipMalloc(&s.nnz, sizeof(uint32_t)));
  return hipSuccess;
}

template <class F>
void msm_scratch_free(MsmScratch<F>& s) {
  void* ptrs[] = {s.keys_in, s.keys_out, s.vals_in, s.vals_out, s.sort_tmp, s.bstart, s.bend,
                  s.head, s.tail, s.buckets, s.red_acc, s.red_run, s.red_tmp, s.nnz};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  s = MsmScratch<F>();
}

// One MSM: n = b.n standard-form scalars (8 x u32, device) -> *d_out (device XYZZ).
template <class F>
__global__ void k_msm_set_inf(XYZZ<F>* out) {
  *out = xyzz_inf<F>();
}

template <class F>
hipError_t msm_run(const MsmBases<F>& b, MsmScratch<F>& pl, const uint32_t* d_scalars, const uint32_t* d_extra,
                   XYZZ<F>* d_out, hipStream_t st, Profiler* prof = nullptr, const char* tag = nullptr) {
  if (b.n > pl.cap) return hipErrorInvalidValue;
  if (b.n == 0) {
    hipLaunchKernelGGL(k_msm_set_inf<F>, dim3(1), dim3(1), 0, st, d_out);
    return hipGetLastError();
  }
  const size_t m = b.n * MSM_W;
  const size_t chunks = (m + MSM_L - 1) / MSM_L;
  size_t need = 0;
  ZK_CHECK(rocprim::radix_sort_pairs(nullptr, need, pl.keys_in, pl.keys_out, pl.vals_in, pl.vals_out, m, 0, 16, st));
  if (need > pl.sort_tmp_bytes || chunks > pl.max_chunks) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_msm_digits, dim3(zk_grid(b.n, 256)), dim3(256), 0, st, d_scalars, d_extra, b.sidx,
                     b.extra_start, b.n, pl.keys_in, pl.vals_in);
  ZK_CHECK(rocprim::radix_sort_pairs(pl.sort_tmp, need, pl.keys_in, pl.keys_out, pl.vals_in, pl.vals_out, m, 0, 16,
                                     st));
  ZK_CHECK(hipMemsetAsync(pl.bstart, 0, MSM_NB * sizeof(uint32_t), st));
  ZK_CHECK(hipMemsetAsync(pl.bend, 0, MSM_NB * sizeof(uint32_t), st));
  ZK_CHECK(hipMemsetAsync(pl.nnz, 0, sizeof(uint32_t), st));
  hipLaunchKernelGGL(k_msm_bounds, dim3(zk_grid(m, 256)), dim3(256), 0, st, pl.keys_out, m, pl.bstart, pl.bend,
                     pl.nnz);
  const int pidx = prof ? prof->begin(tag, st) : -1;
  constexpr bool G1 = sizeof(typename F::T) == 32;
  hipLaunchKernelGGL((k_msm_accumulate<F, G1 ? MSM_G1_WAVES : MSM_G2_WAVES, G1 ? MSM_G1_PF : MSM_G2_PF>),
                     dim3(zk_grid(chunks, 64)), dim3(64), 0, st, pl.keys_out, pl.vals_out,
                     b.bases_w, pl.nnz, pl.head, pl.tail, pl.buckets);
  if (prof) prof->end(pidx, st, 0.0, pl.nnz);
  hipLaunchKernelGGL(k_msm_bucket_sum<F>, dim3(zk_grid(MSM_NB, 64)), dim3(64), 0, st, pl.bstart, pl.bend, pl.nnz,
                     pl.head, pl.tail, pl.buckets);
  // grouped running-sum reduction
  const XYZZ<F>* in = pl.buckets;
  int K = MSM_NB;
  int level = 0;
  int nacc = 0;
  XYZZ<F>* run_bufs[2] = {pl.red_run, pl.red_tmp};
  while (K > 0) {
    int G = (K + MSM_RG - 1) / MSM_RG;
    int shift = 3 * level;  // RG = 8 = 2^3
    XYZZ<F>* run_out = run_bufs[level & 1];
    hipLaunchKernelGGL(k_msm_reduce_level<F>, dim3(zk_grid(G, 64)), dim3(64), 0, st, in, K, shift,
                       pl.red_acc + nacc, run_out);
    nacc += G;
    in = run_out + 1;
    K = G - 1;
    level++;
  }
  // sum all acc entries
  XYZZ<F>* src = pl.red_acc;
  XYZZ<F>* dst = pl.red_tmp;
  int cnt = nacc;
  while (cnt > 1) {
    int nout = (cnt + 7) / 8;
    hipLaunchKernelGGL(k_msm_sum8<F>, dim3(zk_grid(nout, 64)), dim3(64), 0, st, src, cnt, dst);
    XYZZ<F>* t = src;
    src = dst;
    dst = (t == pl.red_acc) ? pl.red_run : t;
    cnt = nout;
  }
  ZK_CHECK(hipMemcpyAsync(d_out, src, sizeof(XYZZ<F>), hipMemcpyDeviceToDevice, st));
  return hipGetLastError();
}

// Non-template entry points (one translation unit per curve: msm_g1.hip / msm_g2.hip).
#define ZKFL_MSM_DEFINE(SUF, F)                                                                          \
  hipError_t msm_bases_alloc_##SUF(MsmBases<F>& b, size_t n) { return msm_bases_alloc(b, n); }           \
  hipError_t msm_bases_set_##SUF(MsmBases<F>& b, const Affine<F>* src, const uint32_t* h_sidx,          \
                                 uint32_t extra_start, hipStream_t st) {                                 \
    return msm_bases_set(b, src, h_sidx, extra_start, st);                                               \
  }                                                                                                      \
  void msm_bases_free_##SUF(MsmBases<F>& b) { msm_bases_free(b); }                                       \
  hipError_t msm_scratch_alloc_##SUF(MsmScratch<F>& s, size_t cap, hipStream_t st) {                     \
    return msm_scratch_alloc(s, cap, st);                                                                \
  }                                                                                                      \
  void msm_scratch_free_##SUF(MsmScratch<F>& s) { msm_scratch_free(s); }                                 \
  hipError_t msm_run_##SUF(const MsmBases<F>& b, MsmScratch<F>& s, const uint32_t* sc, const uint32_t* ex, \
                           XYZZ<F>* out, hipStream_t st, Profiler* prof, const char* tag) {              \
    return msm_run(b, s, sc, ex, out, st, prof, tag);                                                    \
  }

}  // namespace zkfl
