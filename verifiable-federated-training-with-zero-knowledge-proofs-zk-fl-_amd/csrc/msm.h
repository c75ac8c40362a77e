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
//    W window copies 2^(c j) P_i (affine, Montgomery; c bits per key, msm_pick_c: 16 x 16 or
//    19 x 14 for small keys, W = ceil(255 / c)), laid out [i][j] (64 B / 128 B each).  One MSM is then a single bucket set:
//    every (i, j) with a non-zero signed c-bit digit d_ij lands in bucket |d_ij|-1 (2^(c-1)
//    buckets), no per-window bucket reduction and no window combination.  288 GB of HBM makes
//    the Wx base expansion (~2 GB for the 2^18-constraint training circuit) free.
//  * Signed digits in [-(2^(c-1) - 1), 2^(c-1)]; the sign is applied on the fly (f29_madd_signed).
//  * (bucket, entry) pairs are bucket-sorted (two counting passes over the (c-1)-bit bucket
//    number, k_msm_bin_*; zero digits dropped).  The sorted entries are cut
//    into fixed chunks of L entries, one lane each, independent of bucket boundaries: every lane
//    does exactly L additions.  A bucket run that starts and ends inside its chunk is final and
//    written to its bucket; a run cut by a chunk edge becomes an "item" (<= 2 per chunk).
//  * Stitching levels apply the same run logic to the items, SG per lane, until one lane holds
//    what is left: a bucket spread over many chunks is summed by a shallow tree instead of one
//    lane walking its chunks (that serial walk, not the arithmetic, used to set the MSM's latency).
//  * Accumulation uses XYZZ + affine mixed additions (10 Fq mul for G1).
//  * Bucket reduction sum_b (b+1) S_b: 8 buckets folded serially per lane, then 64-lane blocks
//    (LDS suffix scan + trees); two levels for the 2^(c-1) buckets, the second writing the MSM result.
#pragma once
#include <algorithm>
#include <cstring>

#include "field29.h"
#include "msm_api.h"
#include "wtrace.h"

namespace zkfl {

// Kernel occupancy per curve (measured on MI355X).  G1: the accumulation fits 128
// VGPRs (4 waves/SIMD); its stitching/reduction kernels run at 2-3.  G2 runs on lane pairs
// (Fq2PairOps): the accumulation 168 VGPRs (3 waves/SIMD), the tails 179-241 (2 waves/SIMD), no
// spills; one lane per G2 point needed > 256 registers, so a single wave owned the whole SIMD
// for the kernel's duration (measured 186 -> 208 proofs/s moving G2 to lane pairs).
// G1 in 29-bit limbs (field29.h) needs ~140 VGPRs in the accumulation: 3 waves/SIMD without
// spills measured 352.8 proofs/s against 342.9 at 4 waves with 17 spilled VGPRs (32-bit limbs,
// 4 waves: 331.3).
#ifndef MSM_G1_WAVES
#define MSM_G1_WAVES 3
#endif
// G2 in 29-bit limbs: 168 VGPRs + 14 spilled at 3 waves/SIMD, 180 without spills at 2 -- equal
// throughput (399.5 vs 400.9 proofs/s, profiles/r02_s5_ab_limb29_g2.log); 2 keeps scratch out.
#ifndef MSM_G2_WAVES
#define MSM_G2_WAVES 2
#endif
// 1: the next entry's base is loaded while the current one is added (one affine point of
// registers); 0: loaded after it, latency hidden by the other waves only.  Without it G1 at 4
// waves/SIMD spills 3 VGPRs instead of 19 (1.71 -> 1.65 ms per proof) and G2 fits 3 waves/SIMD
// without spills (1.00 -> 0.955 ms per proof); measured.
#ifndef MSM_G1_PREFETCH
#define MSM_G1_PREFETCH 0
#endif
#ifndef MSM_G2_PREFETCH
#define MSM_G2_PREFETCH 0
#endif
// 1: the next entry's base is fetched straight into LDS (global_load_lds_dwordx4, 4 x 16 B per
// lane, double-buffered, 8 KB per wave) while the current one is added, so the gather latency is
// hidden without holding the point in VGPRs (which spilled / cost occupancy: MSM_G*_PREFETCH).
#ifndef MSM_LDS_PF
#define MSM_LDS_PF 1
#endif
#ifndef MSM_G2_TAIL_WAVES
#define MSM_G2_TAIL_WAVES 2
#endif
#ifndef MSM_G1_TAIL_WAVES
#define MSM_G1_TAIL_WAVES 2
#endif
#ifndef MSM_G1_STITCH_WAVES
#define MSM_G1_STITCH_WAVES MSM_G1_TAIL_WAVES
#endif

// Compute type -> storage: how the point kernels read and write the stored points.  G1 and plain
// Fq2 hold a point per lane; Fq2PairOps holds it across a lane pair (component h of every
// coordinate in lane 2k+h), reading and writing Affine/XYZZ<Fq2Ops> memory.
// PIECES: 16-B LDS-DMA pieces of one lane's share of a base record.
template <class F>
struct MsmIO {
  using S = F;
  static constexpr int LANES = 1;
  static constexpr int PIECES = 4;
  static ZK_DEV Affine<F> ld_aff(const Affine<S>* p, size_t i) { return p[i]; }
  // the 16-B piece q < 4 of this lane's share of base i, and a share rebuilt from its pieces
  // (G1: the whole 64-B point; the LDS-DMA prefetch of k_msm_accumulate)
  static ZK_DEV const uint4* piece(const Affine<S>* p, size_t i, int q) {
    return reinterpret_cast<const uint4*>(p + i) + q;
  }
  static ZK_DEV Affine<F> from_pieces(const uint32_t (&w)[4 * PIECES]) {
    Affine<F> a;
    memcpy(&a, w, sizeof(a));
    return a;
  }
  static ZK_DEV XYZZ<F> ld(const XYZZ<S>* p, size_t i) { return p[i]; }
  static ZK_DEV void st(XYZZ<S>* p, size_t i, const XYZZ<F>& v) { p[i] = v; }
};
template <>
struct MsmIO<Fq2PairOps> {
  using S = Fq2Ops;
  static constexpr int LANES = 2;
  static constexpr int PIECES = 4;
  static ZK_DEV Affine<Fq2PairOps> ld_aff(const Affine<S>* p, size_t i) {
    const Fq* q = reinterpret_cast<const Fq*>(p + i);
    const uint32_t h = pair_half();
    return {q[h], q[2 + h]};
  }
  // lane 2k+h holds x.c_h, y.c_h: pieces 0, 1 = x.c_h, 2, 3 = y.c_h
  static ZK_DEV const uint4* piece(const Affine<S>* p, size_t i, int q) {
    return reinterpret_cast<const uint4*>(p + i) + 2 * pair_half() + (q & 1) + (q >> 1) * 4;
  }
  static ZK_DEV Affine<Fq2PairOps> from_pieces(const uint32_t (&w)[4 * PIECES]) {
    Affine<Fq2PairOps> a;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      a.x.v[k] = w[k];
      a.y.v[k] = w[8 + k];
    }
    return a;
  }
  static ZK_DEV XYZZ<Fq2PairOps> ld(const XYZZ<S>* p, size_t i) {
    const Fq* q = reinterpret_cast<const Fq*>(p + i);
    const uint32_t h = pair_half();
    return {q[h], q[2 + h], q[4 + h], q[6 + h]};
  }
  static ZK_DEV void st(XYZZ<S>* p, size_t i, const XYZZ<Fq2PairOps>& v) {
    Fq* q = reinterpret_cast<Fq*>(p + i);
    const uint32_t h = pair_half();
    q[h] = v.X;
    q[2 + h] = v.Y;
    q[4 + h] = v.ZZ;
    q[6 + h] = v.ZZZ;
  }
};
// G1 compute types with another arithmetic over the same storage (one lane per point).
template <class F>
struct MsmIOSameLayout {
  using S = FqOps;
  static constexpr int LANES = 1;
  static constexpr int PIECES = 4;
  static ZK_DEV Affine<F> ld_aff(const Affine<S>* p, size_t i) { return reinterpret_cast<const Affine<F>*>(p)[i]; }
  static ZK_DEV const uint4* piece(const Affine<S>* p, size_t i, int q) {
    return reinterpret_cast<const uint4*>(p + i) + q;
  }
  static ZK_DEV Affine<F> from_pieces(const uint32_t (&w)[4 * PIECES]) {
    Affine<F> a;
    memcpy(&a, w, sizeof(a));
    return a;
  }
  static ZK_DEV XYZZ<F> ld(const XYZZ<S>* p, size_t i) { return reinterpret_cast<const XYZZ<F>*>(p)[i]; }
  static ZK_DEV void st(XYZZ<S>* p, size_t i, const XYZZ<F>& v) { reinterpret_cast<XYZZ<F>*>(p)[i] = v; }
};
template <>
struct MsmIO<FqOpsCompact> : MsmIOSameLayout<FqOpsCompact> {};
template <>
struct MsmIO<FqOpsLazy> : MsmIOSameLayout<FqOpsLazy> {};
// G1 in 29-bit limbs (field29.h): the same 8 x 32-bit storage, converted on every load / store
// (stored values < 2^256, in the 2^261 Montgomery domain)
// (pre-packed 128-B records of nine 29-bit limbs per coordinate were measured neutral in round 5,
// 430.4 vs 430.1 proofs/s for twice the window table, and removed: DESIGN.md §13)
template <>
struct MsmIO<FqOps29> {
  using S = FqOps;
  static constexpr int LANES = 1;
  static constexpr int PIECES = 4;
  static ZK_DEV Affine<FqOps29> ld_aff(const Affine<S>* p, size_t i) {
    const Affine<S> a = p[i];
    return {f29_pack(a.x.v), f29_pack(a.y.v)};
  }
  static ZK_DEV const uint4* piece(const Affine<S>* p, size_t i, int q) {
    return reinterpret_cast<const uint4*>(p + i) + q;
  }
  // the record's words as read from LDS (word by word: a memcpy through HIP's uint4 was lowered to
  // byte permutes, ~45 VALU instructions per entry)
  static ZK_DEV Affine<FqOps29> from_pieces(const uint32_t (&w)[4 * PIECES]) {
    Affine<FqOps29> a;
    uint32_t x[8], y[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      x[k] = w[k];
      y[k] = w[8 + k];
    }
    a.x = f29_pack(x);
    a.y = f29_pack(y);
    return a;
  }
  static ZK_DEV XYZZ<FqOps29> ld(const XYZZ<S>* p, size_t i) {
    const XYZZ<S> a = p[i];
    return {f29_pack(a.X.v), f29_pack(a.Y.v), f29_pack(a.ZZ.v), f29_pack(a.ZZZ.v)};
  }
  static ZK_DEV void st(XYZZ<S>* p, size_t i, const XYZZ<FqOps29>& v) {
    XYZZ<S> a;
    f29_unpack(a.X.v, f29_below256(v.X));
    f29_unpack(a.Y.v, f29_below256(v.Y));
    f29_unpack(a.ZZ.v, v.ZZ);
    f29_unpack(a.ZZZ.v, v.ZZZ);
    p[i] = a;
  }
};
// Compute type the MSM kernels use for a stored curve (G1: redundant [0, 2p) arithmetic with
// the compact multiply; MSM_G1_NO_LAZY: canonical values, compact multiply).
template <class F>
struct MsmCompute {
  using type = F;
};
template <>
struct MsmIO<Fq2Pair29> {
  using S = Fq2Ops;
  static constexpr int LANES = 2;
  static constexpr int PIECES = 4;
  static ZK_DEV Affine<Fq2Pair29> ld_aff(const Affine<S>* p, size_t i) {
    const Fq* q = reinterpret_cast<const Fq*>(p + i);
    const uint32_t h = pair_half();
    return {f29_pack(q[h].v), f29_pack(q[2 + h].v)};
  }
  static ZK_DEV const uint4* piece(const Affine<S>* p, size_t i, int q) {
    return reinterpret_cast<const uint4*>(p + i) + 2 * pair_half() + (q & 1) + (q >> 1) * 4;
  }
  static ZK_DEV Affine<Fq2Pair29> from_pieces(const uint32_t (&w)[4 * PIECES]) {
    uint32_t x[8], y[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      x[k] = w[k];
      y[k] = w[8 + k];
    }
    return {f29_pack(x), f29_pack(y)};
  }
  static ZK_DEV XYZZ<Fq2Pair29> ld(const XYZZ<S>* p, size_t i) {
    const Fq* q = reinterpret_cast<const Fq*>(p + i);
    const uint32_t h = pair_half();
    return {f29_pack(q[h].v), f29_pack(q[2 + h].v), f29_pack(q[4 + h].v), f29_pack(q[6 + h].v)};
  }
  static ZK_DEV void st(XYZZ<S>* p, size_t i, const XYZZ<Fq2Pair29>& v) {
    Fq* q = reinterpret_cast<Fq*>(p + i);
    const uint32_t h = pair_half();
    f29_unpack(q[h].v, f29_below256(v.X));
    f29_unpack(q[2 + h].v, f29_below256(v.Y));
    f29_unpack(q[4 + h].v, v.ZZ);
    f29_unpack(q[6 + h].v, v.ZZZ);
  }
};
// MSM_G1_F29 (default): 29-bit limbs (field29.h); 0: 32-bit limbs in [0, 2p) (FqOpsLazy).
#ifndef MSM_G1_F29
#define MSM_G1_F29 1
#endif
template <>
struct MsmCompute<FqOps> {
#if MSM_G1_F29
  using type = FqOps29;
#elif !defined(MSM_G1_NO_LAZY)
  using type = FqOpsLazy;
#else
  using type = FqOpsCompact;
#endif
};

// Base coordinates (n Fq values) into the 29-bit compute types' Montgomery domain:
// x 2^261 = fp_mul(x 2^256, 2^261 mod p)
static __global__ void __launch_bounds__(256) k_msm_to_m29(Fq* __restrict__ a, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fq c;
#pragma unroll
  for (int k = 0; k < 8; k++) c.v[k] = P29::C261[k];
  a[i] = fp_mul(a[i], c);
}
// MSM_G2_F29 (default): lane pairs in 29-bit limbs (Fq2Pair29); 0: 32-bit limbs (Fq2PairOps).
#ifndef MSM_G2_F29
#define MSM_G2_F29 1
#endif
template <>
struct MsmCompute<Fq2Ops> {
#if MSM_G2_F29
  using type = Fq2Pair29;
#else
  using type = Fq2PairOps;
#endif
};

// ---------------------------------------------------------------------------
// Key-load-time window expansion: out[i*W + j] = 2^(c j) * in[i]  (affine)
// ---------------------------------------------------------------------------
template <class F, int C>
__global__ void __launch_bounds__(64) k_msm_expand(const Affine<F>* __restrict__ in, size_t n, Affine<F>* __restrict__ out) {
  constexpr int W = msm_w_of(C);
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  using T = typename F::T;
  Affine<F> p = in[i];
  if (aff_is_inf(p)) {
    for (int j = 0; j < W; j++) out[i * W + j] = p;
    return;
  }
  // Keep the W window copies in XYZZ in the output slots' scratch (global), with a
  // Montgomery batch inversion of their ZZZ over the 16 copies.
  XYZZ<F> acc = xyzz_from_affine<F>(p);
  T pref[W];
  XYZZ<F> pts[W];
  for (int j = 0; j < W; j++) {
    pts[j] = acc;
    pref[j] = (j == 0) ? acc.ZZZ : F::mul(pref[j - 1], acc.ZZZ);
    if (j + 1 < W)
      for (int k = 0; k < C; k++) acc = xyzz_dbl<F>(acc);
  }
  T inv = F::inv(pref[W - 1]);
  for (int j = W - 1; j >= 0; j--) {
    T iZZZ = (j == 0) ? inv : F::mul(inv, pref[j - 1]);
    if (j > 0) inv = F::mul(inv, pts[j].ZZZ);
    T iZ = F::mul(pts[j].ZZ, iZZZ);
    Affine<F> a;
    a.x = F::mul(pts[j].X, F::sqr(iZ));
    a.y = F::mul(pts[j].Y, iZZZ);
    out[i * W + j] = a;
  }
}

// ---------------------------------------------------------------------------
// Per-MSM kernels
// ---------------------------------------------------------------------------
// Window j of a 256-bit scalar (8 x 32-bit words): bits [c j, c j + c) (j is unrolled, so the
// word index and shifts are constants).
template <int C>
ZK_DEV uint32_t msm_window(const uint32_t (&s)[8], int j) {
  const int b = C * j, w = b >> 5, sh = b & 31;
  uint32_t x = s[w] >> sh;
  if (sh + C > 32 && w + 1 < 8) x |= s[w + 1] << (32 - sh);
  return x & ((1u << C) - 1u);
}

// ---------------------------------------------------------------------------
// Bucket sort of the digits (rocPRIM's onesweep radix sort until round 2: DESIGN.md §5).
// Keys are (c-1)-bit bucket numbers, so two counting passes put every non-zero digit in bucket
// order with no look-back and no memsets:
//   count   per block of bases: digits -> LDS histogram of the high key bits -> cnt[bin][block]
//   scan    one workgroup: cnt (bin-major) -> exclusive offsets, bin starts, nnz
//   scatter per block: digits again (the scalars are 2 B per entry, the pairs 6) -> each pair
//           to its high bin at an LDS-atomic cursor
//   bins    one workgroup per high bin: LDS histogram of the low bits, then each pair to its
//           bucket at an LDS-atomic cursor
// Zero digits are dropped (the accumulation reads only the first nnz pairs).  The order inside
// a bucket is arbitrary: a bucket's sum does not depend on it, and the proof is affine.
// ---------------------------------------------------------------------------
constexpr int MSM_SORT_T = 256;           // threads per block in count / scatter
constexpr int MSM_SORT_HB = 1 << MSM_SORT_HIGH_BITS; // high bins (every window width)
// key bits sorted inside a high bin at window width C, and its low counters
template <int C>
constexpr int msm_sort_lb() {
  return C - 1 - MSM_SORT_HIGH_BITS;
}
template <int C>
constexpr int msm_sort_nl() {
  return 1 << msm_sort_lb<C>();
}
constexpr int MSM_SORT_MAXBLK = 32768 / MSM_SORT_HB; // count/scatter blocks (the scan holds cnt in LDS)
static_assert(MSM_SORT_HB <= MSM_SORT_T, "bucket sort split");
constexpr int MSM_SORT_BT = 1024;         // threads of the scan workgroup
constexpr int MSM_SORT_BINT = MSM_SORT_BIN_THREADS;  // threads per high-bin workgroup
static_assert(MSM_SORT_HB * MSM_SORT_MAXBLK == 32 * MSM_SORT_BT, "scan: 32 counters per thread");

// Signed digits of base i: fn(key, val) for every non-zero digit d of its scalar (window j),
// key = |d| - 1 (the bucket), val = (i W + j) | sign << 31
template <int C, class Fn>
ZK_DEV void msm_for_digits(const uint32_t* __restrict__ scalars, const uint32_t* __restrict__ extra,
                           const uint32_t* __restrict__ sidx, uint32_t extra_start, size_t i, Fn&& fn) {
  constexpr int W = msm_w_of(C), NB = msm_nb_of(C);
  const uint32_t si = sidx ? sidx[i] : (uint32_t)i;
  const uint32_t* src = si < extra_start ? scalars + (size_t)si * 8 : extra + (size_t)(si - extra_start) * 8;
  const uint4* sp = reinterpret_cast<const uint4*>(src);
  const uint4 a = sp[0], b = sp[1];
  const uint32_t s[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint32_t carry = 0;
#pragma unroll
  for (int j = 0; j < W; j++) {
    const uint32_t raw = msm_window<C>(s, j);
    int32_t d = (int32_t)(raw + carry);
    carry = d > NB ? 1u : 0u;
    if (carry) d -= (1 << C);
    if (d != 0) {
      const uint32_t mag = (uint32_t)(d < 0 ? -d : d);
      fn(mag - 1, (uint32_t)(i * W + j) | (d < 0 ? 0x80000000u : 0u));
    }
  }
}

// One sort of a launch (blockIdx.y): its scalars and base map, its blocking (per_blk bases per
// count / scatter block, nblk blocks) and its scratch.  Every sort launch takes a table of up to
// MSM_TAIL_MAX of them, so independent MSMs of a proof sort in the same four launches.
struct MsmSortJob {
  const uint32_t* scalars;
  const uint32_t* extra;
  const uint32_t* sidx;
  uint32_t extra_start;
  uint32_t n, per_blk, nblk;
  uint32_t* cnt;        // [HB][nblk] counts, then exclusive offsets
  uint32_t* bin_start;  // [HB + 1]
  uint32_t* nnz;
  uint16_t* keys_in;
  uint32_t* vals_in;
  uint16_t* keys_out;
  uint32_t* vals_out;
};
struct MsmSortArgs {
  MsmSortJob j[MSM_TAIL_MAX];
};

template <int C>
__global__ void __launch_bounds__(MSM_SORT_T) k_msm_bin_count(const MsmSortArgs A) {
  ZK_WT(WT_SORT_COUNT);
  ZK_LIGHT();
  constexpr int LB = msm_sort_lb<C>();
  const MsmSortJob& J = A.j[blockIdx.y];
  if (blockIdx.x >= J.nblk) return;
  __shared__ uint32_t h[MSM_SORT_HB];
  if (threadIdx.x < MSM_SORT_HB) h[threadIdx.x] = 0;
  __syncthreads();
  const size_t i0 = (size_t)blockIdx.x * J.per_blk, i1 = i0 + J.per_blk < J.n ? i0 + J.per_blk : J.n;
  for (size_t i = i0 + threadIdx.x; i < i1; i += MSM_SORT_T)
    msm_for_digits<C>(J.scalars, J.extra, J.sidx, J.extra_start, i,
                      [&](uint32_t key, uint32_t) { atomicAdd(&h[key >> LB], 1u); });
  __syncthreads();
  if (threadIdx.x < MSM_SORT_HB) J.cnt[(size_t)threadIdx.x * J.nblk + blockIdx.x] = h[threadIdx.x];
}

// cnt[HB * nblk] (bin-major) -> exclusive offsets in place; bin_start[HB + 1]; *nnz.
// The scan keeps all 32 K counters in LDS (~139 KB): gfx950's 160 KB per workgroup.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "the bucket sort's scan needs gfx950's 160 KB of LDS"
#endif
static __global__ void __launch_bounds__(MSM_SORT_BT) k_msm_bin_scan(const MsmSortArgs A) {
  ZK_WT(WT_SORT_SCAN);
  ZK_LIGHT();
  const MsmSortJob& J = A.j[blockIdx.y];
  uint32_t* __restrict__ cnt = J.cnt;
  uint32_t* __restrict__ bin_start = J.bin_start;
  const uint32_t nblk = J.nblk;
  __shared__ uint32_t c[MSM_SORT_HB * MSM_SORT_MAXBLK + MSM_SORT_BT];  // +1 word per 32: no bank conflicts
  __shared__ uint32_t part[MSM_SORT_BT];
  const uint32_t total = MSM_SORT_HB * nblk, t = threadIdx.x;
  for (uint32_t k = t; k < total; k += MSM_SORT_BT) c[k + (k >> 5)] = cnt[k];
  __syncthreads();
  uint32_t s = 0;
  for (uint32_t q = 0; q < 32; q++) {
    const uint32_t k = t * 32 + q;
    if (k < total) s += c[k + (k >> 5)];
  }
  part[t] = s;
  __syncthreads();
  for (uint32_t off = 1; off < MSM_SORT_BT; off <<= 1) {
    const uint32_t v = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - s;
  for (uint32_t q = 0; q < 32; q++) {
    const uint32_t k = t * 32 + q;
    if (k < total) {
      const uint32_t v = c[k + (k >> 5)];
      c[k + (k >> 5)] = run;
      run += v;
    }
  }
  __syncthreads();
  for (uint32_t k = t; k < total; k += MSM_SORT_BT) {
    const uint32_t v = c[k + (k >> 5)];
    cnt[k] = v;
    if (k % nblk == 0) bin_start[k / nblk] = v;
  }
  if (t == MSM_SORT_BT - 1) {
    bin_start[MSM_SORT_HB] = part[t];
    *J.nnz = part[t];
  }
}

template <int C>
__global__ void __launch_bounds__(MSM_SORT_T) k_msm_bin_scatter(const MsmSortArgs A) {
  ZK_WT(WT_SORT_SCATTER);
  ZK_LIGHT();
  constexpr int LB = msm_sort_lb<C>();
  const MsmSortJob& J = A.j[blockIdx.y];
  if (blockIdx.x >= J.nblk) return;
  __shared__ uint32_t cur[MSM_SORT_HB];
  if (threadIdx.x < MSM_SORT_HB) cur[threadIdx.x] = J.cnt[(size_t)threadIdx.x * J.nblk + blockIdx.x];
  __syncthreads();
  uint16_t* __restrict__ keys = J.keys_in;
  uint32_t* __restrict__ vals = J.vals_in;
  const size_t i0 = (size_t)blockIdx.x * J.per_blk, i1 = i0 + J.per_blk < J.n ? i0 + J.per_blk : J.n;
  for (size_t i = i0 + threadIdx.x; i < i1; i += MSM_SORT_T)
    msm_for_digits<C>(J.scalars, J.extra, J.sidx, J.extra_start, i, [&](uint32_t key, uint32_t val) {
      const uint32_t p = atomicAdd(&cur[key >> LB], 1u);
      keys[p] = (uint16_t)key;
      vals[p] = val;
    });
}

// One workgroup per high bin: [bin_start[b], bin_start[b+1]) of (tk, tv) -> buckets in (ko, vo).
// BINT threads per workgroup (MSM_SORT_BINT).  A 256-thread variant for small MSMs measured
// neutral on config 5 (1906.7 vs 1894.0 proofs/s, 3 alternations, profiles/r04_ab_c5_small_keys.log).
template <int BINT, int NL>
__global__ void __launch_bounds__(BINT) k_msm_bin_sort(const MsmSortArgs A) {
  static_assert(BINT >= NL && BINT <= 1024 && NL >= 64, "bins: one thread per low counter");
  ZK_WT(WT_SORT_BINS);
  ZK_LIGHT();
  const MsmSortJob& J = A.j[blockIdx.y];
  const uint32_t* __restrict__ bin_start = J.bin_start;
  const uint16_t* __restrict__ tk = J.keys_in;
  const uint32_t* __restrict__ tv = J.vals_in;
  uint16_t* __restrict__ ko = J.keys_out;
  uint32_t* __restrict__ vo = J.vals_out;
  __shared__ uint32_t c[NL];
  const uint32_t b0 = bin_start[blockIdx.x], b1 = bin_start[blockIdx.x + 1], t = threadIdx.x;
  if (b0 == b1) return;
  if (t < NL) c[t] = 0;
  __syncthreads();
#if MSM_SORT_STAGE
  // a bin that fits is read from memory once: its pairs wait in LDS for the placing loop
  __shared__ uint16_t sk[MSM_SORT_STAGE];
  __shared__ uint32_t sv[MSM_SORT_STAGE];
  const bool staged = b1 - b0 <= MSM_SORT_STAGE;
  for (uint32_t p = b0 + t; p < b1; p += BINT) {
    const uint16_t key = tk[p];
    if (staged) {
      sk[p - b0] = key;
      sv[p - b0] = tv[p];
    }
    atomicAdd(&c[key & (NL - 1)], 1u);
  }
#else
  for (uint32_t p = b0 + t; p < b1; p += BINT) atomicAdd(&c[tk[p] & (NL - 1)], 1u);
#endif
  __syncthreads();
  // exclusive scan of the low counters by the first waves (wave scan + wave totals)
  uint32_t v = 0, x = 0;
  if (t < NL) {
    v = c[t];
    x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if ((t & 63) >= (uint32_t)o) x += y;
    }
  }
  __shared__ uint32_t wt[NL / 64];
  if (t < NL && (t & 63) == 63) wt[t >> 6] = x;
  __syncthreads();
  if (t < NL) {
    uint32_t base = b0;
    for (uint32_t w = 0; w < (t >> 6); w++) base += wt[w];
    c[t] = base + x - v;
  }
  __syncthreads();
  for (uint32_t p = b0 + t; p < b1; p += BINT) {
#if MSM_SORT_STAGE
    const uint16_t key = staged ? sk[p - b0] : tk[p];
    const uint32_t val = staged ? sv[p - b0] : tv[p];
#else
    const uint16_t key = tk[p];
    const uint32_t val = tv[p];
#endif
    const uint32_t q = atomicAdd(&c[key & (NL - 1)], 1u);
    ko[q] = key;
    vo[q] = val;
  }
}

// Where a bucket run found by one lane goes (shared by the accumulation and stitching levels).
// A run [a, b] of bucket k inside a lane's range [q0, q1) is open on the left if it starts the
// range and the previous range ends in the same bucket, open on the right likewise.  A closed
// run is the whole bucket: written to buckets[k].  An open run becomes an item of the next
// stitching level: the left-open run in slot 0, a (only) right-open run in slot 1.  Unused
// slots are dummies carrying the range's first / last bucket, so item keys stay sorted.
template <class F, class S = typename MsmIO<F>::S>
ZK_DEV void msm_emit_run(uint32_t k, const XYZZ<F>& acc, bool real, bool open_left, bool open_right,
                         XYZZ<S>* __restrict__ buckets, uint32_t* __restrict__ okey, XYZZ<S>* __restrict__ oval,
                         bool& slot0, bool& slot1) {
  using IO = MsmIO<F>;
  if (!open_left && !open_right) {
    if (real) IO::st(buckets, k, acc);
  } else if (open_left) {
    okey[0] = real ? k : (k | MSM_ITEM_DUMMY);
    if (real) IO::st(oval, 0, acc);
    slot0 = true;
  } else {
    okey[1] = real ? k : (k | MSM_ITEM_DUMMY);
    if (real) IO::st(oval, 1, acc);
    slot1 = true;
  }
}

// Marks stitching level `level` live when any lane of the wave emitted a real open run.
ZK_DEV void msm_mark_live(uint32_t* __restrict__ live, int level, bool open) {
  const uint64_t b = __ballot(open);
  if (b && (threadIdx.x & 63) == (uint32_t)(__ffsll((unsigned long long)b) - 1)) live[level] = 1u;
}

// Level 0: lane c adds the sorted entries [c*L, min(c*L+L, nnz)) (fixed-size chunks, independent
// of bucket boundaries, so every lane does the same work; L = msm_chunk_len(nnz, target)).
// Software-pipelined: the key/index of entry p+1 and its base are in flight while entry p is
// added.  MINW: minimum waves per SIMD the register allocator must allow (chosen per curve,
// DESIGN.md §5).
// Chunk c of one MSM (the body of k_msm_accumulate and k_msm_accumulate_multi; 64-thread blocks).
template <class F, class S = typename MsmIO<F>::S>
ZK_DEV void msm_acc_chunk(const uint16_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                          const Affine<S>* __restrict__ bases, const uint32_t* __restrict__ nnz_ptr,
                          uint32_t* __restrict__ item_key, XYZZ<S>* __restrict__ item_val,
                          XYZZ<S>* __restrict__ buckets, uint32_t target, uint32_t* __restrict__ live, size_t c) {
  using IO = MsmIO<F>;
  constexpr bool PF = sizeof(typename S::T) == 32 ? MSM_G1_PREFETCH : MSM_G2_PREFETCH;
  const uint32_t nnz = *nnz_ptr;
  const uint32_t L = msm_chunk_len<S>(nnz, target);
  const size_t p0 = c * L;
  if (p0 >= nnz) return;
  const uint32_t p1 = (uint32_t)(p0 + L < nnz ? p0 + L : nnz);
  // the neighbouring chunks' keys and the item slots are only read at a run's end (registers are
  // the G1 kernel's limit at 4 waves/SIMD)
  bool slot0 = false, slot1 = false, first_run = true, open = false;
  XYZZ<F> acc = xyzz_inf<F>();
  uint32_t cur = keys[p0];
  uint32_t v0 = vals[p0], k1 = 0, v1 = 0;
  if (p0 + 1 < p1) {
    k1 = keys[p0 + 1];
    v1 = vals[p0 + 1];
  }
#if MSM_LDS_PF
  // lane l's piece q of buffer b lands at pf[b][q][l] (an LDS-DMA writes base + lane x 16 B).  A
  // native 4 x u32 vector type: with HIP's uint4 struct the reads below were lowered to 32
  // ds_read_u16 plus ~100 byte-reassembly instructions per entry (gfx950, ROCm 7.2)
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  constexpr int NP = IO::PIECES;
  __shared__ v4u pf[2][NP][64];
  const uint32_t ln = threadIdx.x;
  auto fetch = [&](uint32_t idx, int b) {
#pragma unroll
    for (int q = 0; q < NP; q++)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)IO::piece(bases, idx, q),
                                       (__attribute__((address_space(3))) void*)&pf[b][q][0], 16, 0, 0);
  };
  fetch(v0 & 0x7FFFFFFFu, 0);
  uint32_t it = 0;
#else
  Affine<F> a = IO::ld_aff(bases, v0 & 0x7FFFFFFFu);
#endif
  for (uint32_t p = (uint32_t)p0; p < p1; p++) {
#if MSM_LDS_PF
    const int b = it++ & 1;
    // the LDS-DMA of this buffer must have landed: with the native vector type the compiler no
    // longer connects these reads to the global_load_lds writes and dropped the vmcnt wait on the
    // first iteration (wrong first base, found by the GPU proof tests) -- so wait explicitly
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t u[4 * NP];
#pragma unroll
    for (int q = 0; q < NP; q++) {  // ds_read_b128
      const v4u x = pf[b][q][ln];
      u[4 * q] = x.x;
      u[4 * q + 1] = x.y;
      u[4 * q + 2] = x.z;
      u[4 * q + 3] = x.w;
    }
    const Affine<F> a = IO::from_pieces(u);
    if (p + 1 < p1) fetch(v1 & 0x7FFFFFFFu, b ^ 1);
#else
    Affine<F> an;
    if (PF && p + 1 < p1) an = IO::ld_aff(bases, v1 & 0x7FFFFFFFu);
#endif
    uint32_t k2 = 0, v2 = 0;
    if (p + 2 < p1) {
      k2 = keys[p + 2];
      v2 = vals[p + 2];
    }
    acc = xyzz_madd_signed<F>(acc, a, (v0 & 0x80000000u) != 0);
    const bool last = p + 1 == p1;
    if (last || k1 != cur) {
      const bool open_left = first_run && p0 > 0 && keys[p0 - 1] == cur;
      const bool open_right = last && p1 < nnz && keys[p1] == cur;
      msm_emit_run<F>(cur, acc, true, open_left, open_right, buckets, item_key + 2 * c, item_val + 2 * c, slot0,
                      slot1);
      open = open || open_left || open_right;
      acc = xyzz_inf<F>();
      cur = k1;
      first_run = false;
    }
    v0 = v1;
    v1 = v2;
    k1 = k2;
#if !MSM_LDS_PF
    if (PF) a = an;
    else if (p + 1 < p1) a = IO::ld_aff(bases, v0 & 0x7FFFFFFFu);
#endif
  }
  if (!slot0) item_key[2 * c] = (uint32_t)keys[p0] | MSM_ITEM_DUMMY;
  if (!slot1) item_key[2 * c + 1] = (uint32_t)keys[p1 - 1] | MSM_ITEM_DUMMY;
  msm_mark_live(live, 0, open);
}

template <class F, int MINW, class S = typename MsmIO<F>::S>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MINW))) k_msm_accumulate(
    const uint16_t* __restrict__ keys, const uint32_t* __restrict__ vals, const Affine<S>* __restrict__ bases,
    const uint32_t* __restrict__ nnz_ptr, uint32_t* __restrict__ item_key, XYZZ<S>* __restrict__ item_val,
    XYZZ<S>* __restrict__ buckets, uint32_t target, uint32_t* __restrict__ live) {
  ZK_WT(WT_ACC | (MsmIO<F>::LANES == 2 ? WT_G2 : 0u));
  msm_acc_chunk<F>(keys, vals, bases, nnz_ptr, item_key, item_val, buckets, target, live,
                   ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / MsmIO<F>::LANES);
}

// The accumulations of up to MSM_TAIL_MAX independent MSMs of one curve in one launch (blockIdx.y
// = MSM): a small key's A, B1 and C + H, so the proof's chain waits for one launch, not three.
template <class S>
struct MsmAccArgs {
  const uint16_t* keys[MSM_TAIL_MAX];
  const uint32_t* vals[MSM_TAIL_MAX];
  const Affine<S>* bases[MSM_TAIL_MAX];
  const uint32_t* nnz[MSM_TAIL_MAX];
  uint32_t* item_key[MSM_TAIL_MAX];
  XYZZ<S>* item_val[MSM_TAIL_MAX];
  XYZZ<S>* buckets[MSM_TAIL_MAX];
  uint32_t target[MSM_TAIL_MAX];
  uint32_t* live[MSM_TAIL_MAX];
};
template <class F, int MINW, class S = typename MsmIO<F>::S>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MINW))) k_msm_accumulate_multi(
    const MsmAccArgs<S> A) {
  ZK_WT(WT_ACC | (MsmIO<F>::LANES == 2 ? WT_G2 : 0u) | WT_JOINT);
  const int y = blockIdx.y;
  msm_acc_chunk<F>(A.keys[y], A.vals[y], A.bases[y], A.nnz[y], A.item_key[y], A.item_val[y], A.buckets[y],
                   A.target[y], A.live[y], ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / MsmIO<F>::LANES);
}

}  // namespace zkfl
namespace zkfl {

// Item count of stitching level `level` (>= 1), derived on the device from nnz.
template <class S>
ZK_DEV uint32_t msm_items_at(uint32_t nnz, int level, uint32_t target) {
  const uint32_t L = msm_chunk_len<S>(nnz, target);
  uint32_t n = 2 * ((nnz + L - 1) / L);
  for (int l = 1; l < level; l++) n = 2 * ((n + MSM_SG - 1) / MSM_SG);
  return n;
}

// Stitching level: the same run logic over the previous level's items (SG per lane), so a
// bucket spread over many chunks is summed by a tree of depth log_{SG/2}, not by one lane.
// Kernel argument of the batched tail launches: up to MSM_TAIL_MAX MSMs, one per blockIdx.y.
template <class S>
struct MsmTailArgs {
  uint32_t* key[MSM_TAIL_MAX][2];
  XYZZ<S>* val[MSM_TAIL_MAX][2];
  XYZZ<S>* buckets[MSM_TAIL_MAX];
  XYZZ<S>* red_a[MSM_TAIL_MAX];
  XYZZ<S>* red_s[MSM_TAIL_MAX];
  const uint32_t* nnz[MSM_TAIL_MAX];
  XYZZ<S>* out[MSM_TAIL_MAX];
  uint32_t* live[MSM_TAIL_MAX];
  uint32_t target[MSM_TAIL_MAX];
  int c;  // window bits of every MSM in the batch
};

// Zero the buckets (ZZ = 0: infinity) and the nnz counter of every tail in the batch: one launch
// for all MSMs of a proof instead of two memsets each.
template <class S>
__global__ void __launch_bounds__(256) k_msm_tail_reset(const MsmTailArgs<S> ta) {
  ZK_WT(WT_TAIL_RESET | (sizeof(typename S::T) == 32 ? 0u : WT_G2));
  ZK_LIGHT();
  const int y = blockIdx.y;
  uint4* b = reinterpret_cast<uint4*>(ta.buckets[y]);
  const size_t nv = (size_t)msm_nb_of(ta.c) * sizeof(XYZZ<S>) / sizeof(uint4);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (size_t)gridDim.x * blockDim.x)
    b[i] = make_uint4(0, 0, 0, 0);
  if (blockIdx.x == 0 && threadIdx.x == 0) *const_cast<uint32_t*>(ta.nnz[y]) = 0;
  if (blockIdx.x == 0 && threadIdx.x < MSM_LIVE_LEVELS) ta.live[y][threadIdx.x] = 0;
}

// One stitching level for lane g of MSM y (N = the level's item count).
template <class F, class S = typename MsmIO<F>::S>
ZK_DEV void msm_stitch_lane(const MsmTailArgs<S>& ta, int y, int level, int src, uint32_t g, uint32_t N) {
  using IO = MsmIO<F>;
  const uint32_t* __restrict__ in_key = ta.key[y][src];
  const XYZZ<S>* __restrict__ in_val = ta.val[y][src];
  uint32_t* __restrict__ out_key = ta.key[y][src ^ 1];
  XYZZ<S>* __restrict__ out_val = ta.val[y][src ^ 1];
  XYZZ<S>* __restrict__ buckets = ta.buckets[y];
  const uint32_t q0 = g * MSM_SG;
  const uint32_t q1 = q0 + MSM_SG < N ? q0 + MSM_SG : N;
  constexpr uint32_t KM = ~MSM_ITEM_DUMMY;
  const uint32_t kprev = q0 > 0 ? (in_key[q0 - 1] & KM) : 0xFFFFFFFFu;
  const uint32_t knext = q1 < N ? (in_key[q1] & KM) : 0xFFFFFFFFu;
  uint32_t* okey = out_key + 2 * g;
  XYZZ<S>* oval = out_val + 2 * g;
  bool slot0 = false, slot1 = false, real = false, open = false;
  XYZZ<F> acc = xyzz_inf<F>();
  uint32_t kq = in_key[q0];
  uint32_t cur = kq & KM, run_start = q0;
  for (uint32_t q = q0; q < q1; q++) {
    const uint32_t kn = q + 1 < q1 ? in_key[q + 1] : 0xFFFFFFFFu;
    if (!(kq & MSM_ITEM_DUMMY)) {
      acc = xyzz_add<F>(acc, IO::ld(in_val, q));
      real = true;
    }
    const bool last = q + 1 == q1;
    if (last || (kn & KM) != cur) {
      const bool ol = run_start == q0 && kprev == cur, orr = last && knext == cur;
      msm_emit_run<F>(cur, acc, real, ol, orr, buckets, okey, oval, slot0, slot1);
      open = open || (real && (ol || orr));
      acc = xyzz_inf<F>();
      real = false;
      cur = kn & KM;
      run_start = q + 1;
    }
    kq = kn;
  }
  if (!slot0) okey[0] = (in_key[q0] & KM) | MSM_ITEM_DUMMY;
  if (!slot1) okey[1] = (in_key[q1 - 1] & KM) | MSM_ITEM_DUMMY;
  if (level < MSM_LIVE_LEVELS && open) ta.live[y][level] = 1u;
}

template <class F, int MINW, class S = typename MsmIO<F>::S>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MINW))) k_msm_stitch(
    const MsmTailArgs<S> ta, int level, int src) {
  ZK_WT(WT_STITCH | (MsmIO<F>::LANES == 2 ? WT_G2 : 0u));
  ZK_LIGHT();
  const int y = blockIdx.y;
  // the level before emitted no real open run: every bucket is final already
  if (ta.live[y][level - 1] == 0u) return;
  const uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) / MsmIO<F>::LANES;
  const uint32_t N = msm_items_at<S>(*ta.nnz[y], level, ta.target[y]);
  if (g * MSM_SG >= N) return;
  msm_stitch_lane<F>(ta, y, level, src, g, N);
}

// The last stitching levels of MSM y in one workgroup (blockIdx.y = MSM): from `level` on, every
// level has at most MSM_STITCH_LAST lanes, so the workgroup runs them back to back with a barrier
// between levels (the items pass through global memory inside one CU) until one lane holds every
// item -- one launch instead of ~4 dependent ones per tail batch.
constexpr int MSM_STITCH_LAST = 128;
// MSM y's last stitching levels on this workgroup (k_msm_stitch_last, k_msm_stitch_last_joint)
template <class F, class S>
ZK_DEV void msm_stitch_last_block(const MsmTailArgs<S>& ta, int y, int level, int src) {
  const uint32_t g = threadIdx.x / MsmIO<F>::LANES;
  const uint32_t nnz = *ta.nnz[y];
  for (; level < MSM_LIVE_LEVELS; level++, src ^= 1) {
    const uint32_t N = msm_items_at<S>(nnz, level, ta.target[y]);
    if (ta.live[y][level - 1] != 0u && g * MSM_SG < N) msm_stitch_lane<F>(ta, y, level, src, g, N);
    __threadfence_block();
    __syncthreads();
    if (N <= (uint32_t)MSM_SG) break;
  }
}
template <class F, int MINW, class S = typename MsmIO<F>::S>
__global__ void __launch_bounds__(MSM_STITCH_LAST * MsmIO<F>::LANES) k_msm_stitch_last(const MsmTailArgs<S> ta,
                                                                                       int level, int src) {
  ZK_WT(WT_STITCH | (MsmIO<F>::LANES == 2 ? WT_G2 : 0u));
  ZK_LIGHT();
  msm_stitch_last_block<F>(ta, blockIdx.y, level, src);
}

// Weighted bucket reduction sum_b (b+1) S_b.  An item i stands for a group of g = 2^log2g
// consecutive buckets: s_i = its bucket sum, a_i = sum (b - first + 1) S_b; items combine as
//   a' = sum_k a_k + g * sum_k k s_k,   s' = sum_k s_k,   sum_k k s_k = sum_{k>=1} R_k
// with the suffix sums R_k = sum_{j>=k} s_j.  Each logical lane first folds Q consecutive items
// serially (running sum, 2 additions per bucket), then a 64-lane block combines the lanes with an
// LDS suffix scan and two trees (depth ~18).  Level 0 reads the buckets as both a and s (g = 1,
// Q = 8: 64 blocks); level 1 (Q = 1) combines the 64 block results into the MSM result.  Serial
// folding first keeps the waves few: the reduction's cost is its waves' register-time.
// Q0: buckets folded serially per lane at level 0 (per curve: the reduction's waves hold their
// registers for the whole serial fold, but fewer, longer lanes do less scan/tree work per bucket)
#ifndef MSM_G1_WSUM_Q
#define MSM_G1_WSUM_Q 16
#endif
#ifndef MSM_G2_WSUM_Q
#define MSM_G2_WSUM_Q 16
#endif
template <class S>
constexpr int msm_wsum_q0() {
  return sizeof(typename S::T) == 32 ? MSM_G1_WSUM_Q : MSM_G2_WSUM_Q;
}
// Q0 of the latency schedule's reduction (one proof alone, msm_tails(..., fast = true)): 128
// level-0 blocks (4 buckets per lane at c = 16, 1 at c = 14), a 128-lane level 1 -- about 45
// dependent point operations on the chain instead of ~70, for ~1.8x the reduction's (small) work
template <int C>
constexpr int msm_wsum_q_fast() {
  return msm_nb_of(C) / (MSM_RB * 128);
}
// lanes of a reduction block: level 0 one wave (MSM_RB), level 1 one lane per level-0 block
template <bool L0, int Q0, int C>
constexpr int msm_wsum_rb() {
  return L0 || msm_nb_of(C) / (MSM_RB * Q0) <= MSM_RB ? MSM_RB : msm_nb_of(C) / (MSM_RB * Q0);
}
template <int Q0, int C>
constexpr bool msm_wsum_fits() {
  return Q0 >= 1 && msm_nb_of(C) % (MSM_RB * Q0) == 0 && msm_wsum_rb<false, Q0, C>() <= 2 * MSM_RB;
}
// One reduction block: MSM yb's reduction block bx at this level, this thread's logical lane t
// (< RB), the block's LDS arrays sh / shy (RB points each); store = false runs the block (its
// barriers) without writing a result (the idle half of a joint G1 block, k_msm_wsum_joint).
template <class F, bool L0, int Q0, int C, class S = typename MsmIO<F>::S>
ZK_DEV void msm_wsum_block(const MsmTailArgs<S>& ta, int yb, int bx, int t, XYZZ<S>* sh, XYZZ<S>* shy, bool store) {
  static_assert(msm_wsum_fits<Q0, C>(), "two reduction levels cover the buckets; red_a / red_s hold 2 x the level-1 block");
  constexpr int NB = msm_nb_of(C);
  // One kernel per level (template L0): level 0 keeps only the running sums R, W live through its
  // fold, level 1 has no fold at all, so neither carries the other's registers.
  const XYZZ<S>* __restrict__ in_a = L0 ? ta.buckets[yb] : ta.red_a[yb];
  const XYZZ<S>* __restrict__ in_s = L0 ? ta.buckets[yb] : ta.red_s[yb];
  constexpr int B0 = NB / (MSM_RB * Q0);  // level-0 blocks = level-1 items
  constexpr int RB = msm_wsum_rb<L0, Q0, C>();
  constexpr int N = L0 ? NB : B0, Q = L0 ? Q0 : 1;
  constexpr int log2g = L0 ? 0 : __builtin_ctz((unsigned)(Q0 * MSM_RB));
  XYZZ<S>* __restrict__ out_a = L0 ? ta.red_a[yb] : ta.out[yb];
  XYZZ<S>* __restrict__ out_s = L0 ? ta.red_s[yb] : ta.red_s[yb] + RB;
  using IO = MsmIO<F>;
  const int i0 = (bx * RB + t) * Q;  // this lane's items [i0, i0 + Q)
  XYZZ<F> R = xyzz_inf<F>(), y = xyzz_inf<F>();
  if constexpr (L0) {  // serial fold over Q buckets (a = s: the buckets themselves, g = 1)
    XYZZ<F> W = xyzz_inf<F>();
#pragma unroll 1
    for (int k = Q - 1; k >= 0; k--) {
      if (i0 + k < N) R = xyzz_add<F>(R, IO::ld(in_s, i0 + k));
      if (k >= 1) W = xyzz_add<F>(W, R);
    }
    y = xyzz_add<F>(R, W);  // this lane's item: a group of Q buckets
  } else if (i0 < N) {  // one block result per lane
    R = IO::ld(in_s, i0);
    y = IO::ld(in_a, i0);
  }
#pragma unroll 1
  for (int d = 1; d < RB; d <<= 1) {  // suffix scan of s
    IO::st(sh, t, R);
    __syncthreads();
    if (t + d < RB) R = xyzz_add<F>(R, IO::ld(sh, t + d));
    __syncthreads();
  }
  // The tree sums of R_{t>=1} (x) and of a (y) side by side: at step d, lanes [0, d) add x
  // pairs and lanes [RB/2, RB/2 + d) add y pairs, so both trees cost one tree's latency.
  IO::st(sh, t, t >= 1 ? R : xyzz_inf<F>());
  IO::st(shy, t, y);
  __syncthreads();
  constexpr int H = RB / 2;
  const bool ty = t >= H;
  const int tt = ty ? t - H : t;
  XYZZ<S>* tree = ty ? shy : sh;
#pragma unroll 1
  for (int d = H; d >= 1; d >>= 1) {
    XYZZ<F> v;
    if (tt < d) v = xyzz_add<F>(IO::ld(tree, tt), IO::ld(tree, tt + d));
    __syncthreads();
    if (tt < d) IO::st(tree, tt, v);
    __syncthreads();
  }
  XYZZ<F> x;
  if (t == 0 && store) {
    x = IO::ld(sh, 0);
    y = IO::ld(shy, 0);
    constexpr int lq = __builtin_ctz((unsigned)Q);
    for (int k = 0; k < log2g + lq; k++) x = xyzz_dbl<F>(x);
    const XYZZ<F> a = xyzz_add<F>(y, x);
    // canonical (and, for FqOps29, back in the 2^256 domain) only when it leaves the MSM
    IO::st(out_a, bx, L0 ? a : xyzz_canon<F>(a));
    IO::st(out_s, bx, R);
  }
}

template <class F, int MINW, bool L0, int Q0, int C, class S = typename MsmIO<F>::S>
__global__ void __launch_bounds__((msm_wsum_rb<L0, Q0, C>() * MsmIO<F>::LANES)) __attribute__((amdgpu_waves_per_eu(MINW)))
k_msm_wsum(const MsmTailArgs<S> ta) {
  ZK_WT((L0 ? WT_WSUM0 : WT_WSUM1) | (MsmIO<F>::LANES == 2 ? WT_G2 : 0u));
  ZK_LIGHT();
  constexpr int RB = msm_wsum_rb<L0, Q0, C>();
  __shared__ XYZZ<S> sh[RB], shy[RB];
  msm_wsum_block<F, L0, Q0, C>(ta, blockIdx.y, blockIdx.x, threadIdx.x / MsmIO<F>::LANES, sh, shy, true);
}

// ---------------------------------------------------------------------------
// Joint tails: the G1 tails of a proof and its G2 tail as ONE launch sequence (blockIdx.y: the n1
// G1 MSMs, then the G2 ones), so the latency-bound stitching levels and reduction blocks of both
// curves run side by side instead of one chain after the other.  A joint block is 128 threads:
// 128 G1 lanes, or 64 G2 lane pairs (the stitching); two G1 reduction blocks or one G2 block (the
// reduction).  The kernels hold both curves' code, so they take the larger register budget of the
// two (2 waves/SIMD, as both tails' kernels already run).
// ---------------------------------------------------------------------------
template <class S1, class S2>
struct MsmJointArgs {
  MsmTailArgs<S1> a;  // G1 tails (blockIdx.y < n1)
  MsmTailArgs<S2> b;  // G2 tails (blockIdx.y - n1)
  int n1;
};
constexpr int MSM_JOINT_T = 128;

template <class F1, class F2, int MINW, class S1 = typename MsmIO<F1>::S, class S2 = typename MsmIO<F2>::S>
__global__ void __launch_bounds__(MSM_JOINT_T) __attribute__((amdgpu_waves_per_eu(MINW)))
k_msm_stitch_joint(const MsmJointArgs<S1, S2> ja, int level, int src) {
  ZK_WT(WT_STITCH | WT_JOINT);
  ZK_LIGHT();
  const int y = blockIdx.y;
  if (y < ja.n1) {
    if (ja.a.live[y][level - 1] == 0u) return;
    const uint32_t g = (blockIdx.x * MSM_JOINT_T + threadIdx.x) / MsmIO<F1>::LANES;
    const uint32_t N = msm_items_at<S1>(*ja.a.nnz[y], level, ja.a.target[y]);
    if (g * MSM_SG < N) msm_stitch_lane<F1>(ja.a, y, level, src, g, N);
  } else {
    const int z = y - ja.n1;
    if (ja.b.live[z][level - 1] == 0u) return;
    const uint32_t g = (blockIdx.x * MSM_JOINT_T + threadIdx.x) / MsmIO<F2>::LANES;
    const uint32_t N = msm_items_at<S2>(*ja.b.nnz[z], level, ja.b.target[z]);
    if (g * MSM_SG < N) msm_stitch_lane<F2>(ja.b, z, level, src, g, N);
  }
}

template <class F1, class F2, int MINW, class S1 = typename MsmIO<F1>::S, class S2 = typename MsmIO<F2>::S>
__global__ void __launch_bounds__(2 * MSM_STITCH_LAST) k_msm_stitch_last_joint(const MsmJointArgs<S1, S2> ja, int level,
                                                                                int src) {
  static_assert(MsmIO<F1>::LANES == 1 && MsmIO<F2>::LANES == 2, "joint tails: G1 lanes, G2 lane pairs");
  ZK_WT(WT_STITCH | WT_JOINT);
  ZK_LIGHT();
  const int y = blockIdx.y;
  if (y < ja.n1)
    msm_stitch_last_block<F1>(ja.a, y, level, src);  // threads >= MSM_STITCH_LAST have no lane
  else
    msm_stitch_last_block<F2>(ja.b, y - ja.n1, level, src);
}

// One reduction level of every tail: a G1 joint block runs two G1 reduction blocks (its two 64-
// or 128-lane halves), a G2 joint block one G2 block on lane pairs
template <class F1, class F2, int MINW, bool L0, int Q0, int C, class S1 = typename MsmIO<F1>::S,
          class S2 = typename MsmIO<F2>::S>
__global__ void __launch_bounds__((2 * msm_wsum_rb<L0, Q0, C>())) __attribute__((amdgpu_waves_per_eu(MINW)))
k_msm_wsum_joint(const MsmJointArgs<S1, S2> ja) {
  ZK_WT((L0 ? WT_WSUM0 : WT_WSUM1) | WT_JOINT);
  ZK_LIGHT();
  constexpr int RB = msm_wsum_rb<L0, Q0, C>();
  constexpr int NBLK = L0 ? msm_nb_of(C) / (MSM_RB * Q0) : 1;  // reduction blocks per MSM at this level
  constexpr size_t B1 = 2 * 2 * RB * sizeof(XYZZ<S1>), B2 = 2 * RB * sizeof(XYZZ<S2>);
  __shared__ __attribute__((aligned(16))) unsigned char lds[B1 > B2 ? B1 : B2];
  const int y = blockIdx.y;
  if (y < ja.n1) {
    if (2 * (int)blockIdx.x >= NBLK) return;  // the G1 blocks fit the first half of the grid
    const int half = threadIdx.x / RB, bx = 2 * blockIdx.x + half;
    XYZZ<S1>* sh = reinterpret_cast<XYZZ<S1>*>(lds) + half * 2 * RB;
    msm_wsum_block<F1, L0, Q0, C>(ja.a, y, bx, threadIdx.x % RB, sh, sh + RB, bx < NBLK);
  } else {
    XYZZ<S2>* sh = reinterpret_cast<XYZZ<S2>*>(lds);
    msm_wsum_block<F2, L0, Q0, C>(ja.b, y - ja.n1, blockIdx.x, threadIdx.x / MsmIO<F2>::LANES, sh, sh + RB, true);
  }
}

// ---------------------------------------------------------------------------
// Host-side plan
// ---------------------------------------------------------------------------
// fn(std::integral_constant<int, C>) for the window width c of a base set (MSM_C or MSM_C_SMALL:
// the widths whose kernels are instantiated)
template <class Fn>
hipError_t msm_with_c(int c, Fn&& fn) {
  if (c == MSM_C) return fn(std::integral_constant<int, MSM_C>());
  if constexpr (MSM_C_SMALL != MSM_C)
    if (c == MSM_C_SMALL) return fn(std::integral_constant<int, MSM_C_SMALL>());
  return hipErrorInvalidValue;
}

template <class F>
hipError_t msm_bases_alloc(MsmBases<F>& b, size_t n, int c) {
  if (c != MSM_C && c != MSM_C_SMALL) return hipErrorInvalidValue;
  b.n = n;
  b.c = c;
  ZK_CHECK(hipMalloc(&b.bases_w, (n ? n : 1) * msm_w_of(c) * sizeof(Affine<F>)));
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
  using FC = typename MsmCompute<F>::type;
  const size_t m = b.n * msm_w_of(b.c);
  if (b.n)
    ZK_CHECK(msm_with_c(b.c, [&](auto cc) {
      hipLaunchKernelGGL((k_msm_expand<F, decltype(cc)::value>), dim3(zk_grid(b.n, 64)), dim3(64), 0, st, d_bases,
                         b.n, b.bases_w);
      return hipSuccess;
    }));
  if constexpr (std::is_same<FC, FqOps29>::value || std::is_same<FC, Fq2Pair29>::value) {
    const size_t nfq = m * (sizeof(Affine<F>) / sizeof(Fq));
    if (nfq)
      hipLaunchKernelGGL(k_msm_to_m29, dim3(zk_grid(nfq, 256)), dim3(256), 0, st, reinterpret_cast<Fq*>(b.bases_w), nfq);
  }
  return hipGetLastError();
}

template <class F>
hipError_t msm_scratch_alloc(MsmScratch<F>& s, size_t cap, int c, hipStream_t st) {
  s.cap = cap;
  s.c = c;
  const size_t m = cap * msm_w_of(c);
  ZK_CHECK(hipMalloc(&s.keys_in, m * sizeof(uint16_t)));
  ZK_CHECK(hipMalloc(&s.keys_out, m * sizeof(uint16_t)));
  ZK_CHECK(hipMalloc(&s.vals_in, m * sizeof(uint32_t)));
  ZK_CHECK(hipMalloc(&s.vals_out, m * sizeof(uint32_t)));
  s.sort_tmp_bytes = (MSM_SORT_HB * MSM_SORT_MAXBLK + MSM_SORT_HB + 1) * sizeof(uint32_t);
  ZK_CHECK(hipMalloc(&s.sort_tmp, s.sort_tmp_bytes));
  (void)st;
  return hipSuccess;
}

template <class F>
void msm_scratch_free(MsmScratch<F>& s) {
  void* ptrs[] = {s.keys_in, s.keys_out, s.vals_in, s.vals_out, s.sort_tmp};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  s = MsmScratch<F>();
}

// Accumulation lanes (chunks) the device holds at once for this curve's k_msm_accumulate: the
// occupancy of its 64-thread blocks x the CUs x chunks per block (0 when unknown: fixed L).
template <class F>
uint32_t msm_resident_chunks() {
#if !MSM_ADAPTIVE_L
  return 0;
#else
  // tests: ZKFL_MSM_TARGET=<chunks> forces a small target, so small MSMs run long chunks too
  if (const char* e = getenv("ZKFL_MSM_TARGET")) return (uint32_t)strtoul(e, nullptr, 10);
  using FC = typename MsmCompute<F>::type;
  constexpr int AW = sizeof(typename F::T) == 32 ? MSM_G1_WAVES : MSM_G2_WAVES;
  int dev = 0, ncu = 0, nb = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_msm_accumulate<FC, AW>, 64, 0) != hipSuccess) return 0;
  if (ncu <= 0 || nb <= 0) return 0;
  const uint32_t t = (uint32_t)ncu * (uint32_t)nb * (64u / MsmIO<FC>::LANES);
  // A/B knob: ZKFL_MSM_TARGET_SCALE=<x> resizes the target (x < 1: longer chunks, fewer items)
  if (const char* e = getenv("ZKFL_MSM_TARGET_SCALE")) return std::max<uint32_t>(64, (uint32_t)(t * atof(e)));
  return t;
#endif
}

// Minimum entries per accumulation lane for an MSM of `cap` bases.  Small MSMs (<= 2^16 bases:
// config 5's keys) are latency-bound chains, so they take short chunks: a shorter serial walk
// per lane for a few more stitching items (config 5 1970 vs 1893 proofs/s at 8 vs 16, same box,
// DESIGN.md §12).  ZKFL_MSM_L0 / ZKFL_MSM_L0_SMALL override (A/B knobs).
template <class F>
uint32_t msm_tail_l0(size_t cap) {
  const bool small = cap <= ((size_t)1 << 16);
  const char* e = getenv(small ? "ZKFL_MSM_L0_SMALL" : "ZKFL_MSM_L0");
  const uint32_t l = e ? (uint32_t)atoi(e) : (small ? MSM_SMALL_L : (uint32_t)MsmChunk<F>::L);
  return l < 1 ? 1u : l > 255 ? 255u : l;
}

template <class F>
hipError_t msm_tail_alloc(MsmTail<F>& t, size_t cap, int c) {
  if (c != MSM_C && c != MSM_C_SMALL) return hipErrorInvalidValue;
  t.c = c;
  const size_t m = cap * msm_w_of(c);
  t.target = std::min<uint32_t>(msm_resident_chunks<F>(), 0xFFFFFFu);
  t.l0 = msm_tail_l0<F>(cap);
  t.max_chunks = (m + t.l0 - 1) / t.l0;
  if (t.target) t.max_chunks = std::min<size_t>(t.max_chunks, t.target);  // msm_chunk_len bounds the lanes
  t.item_cap[0] = 2 * t.max_chunks;
  t.item_cap[1] = 2 * ((t.item_cap[0] + MSM_SG - 1) / MSM_SG);
  for (int k = 0; k < 2; k++) {
    ZK_CHECK(hipMalloc(&t.item_key[k], (t.item_cap[k] ? t.item_cap[k] : 2) * sizeof(uint32_t)));
    ZK_CHECK(hipMalloc(&t.item_val[k], (t.item_cap[k] ? t.item_cap[k] : 2) * sizeof(XYZZ<F>)));
  }
  ZK_CHECK(hipMalloc(&t.buckets, msm_nb_of(c) * sizeof(XYZZ<F>)));
  // <= 2 level-1 blocks (fast: 128 lanes)
  ZK_CHECK(hipMalloc(&t.red_a, MSM_TAIL_RED * sizeof(XYZZ<F>)));
  ZK_CHECK(hipMalloc(&t.red_s, MSM_TAIL_RED * sizeof(XYZZ<F>)));
  ZK_CHECK(hipMalloc(&t.nnz, sizeof(uint32_t)));
  ZK_CHECK(hipMalloc(&t.live, MSM_LIVE_LEVELS * sizeof(uint32_t)));
  return hipSuccess;
}

template <class F>
void msm_tail_free(MsmTail<F>& t) {
  void* ptrs[] = {t.item_key[0], t.item_key[1], t.item_val[0], t.item_val[1], t.buckets, t.red_a, t.red_s, t.nnz,
                  t.live};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  t = MsmTail<F>();
}

// (one window width per batch: msm_tails_* reject a batch that mixes them)
template <class F>
MsmTailArgs<F> msm_tail_args(MsmTail<F>* const* t, XYZZ<F>* const* outs, int n) {
  MsmTailArgs<F> ta = {};
  ta.c = n > 0 ? t[0]->c : MSM_C;
  for (int i = 0; i < n; i++) {
    for (int k = 0; k < 2; k++) {
      ta.key[i][k] = t[i]->item_key[k];
      ta.val[i][k] = t[i]->item_val[k];
    }
    ta.buckets[i] = t[i]->buckets;
    ta.red_a[i] = t[i]->red_a;
    ta.red_s[i] = t[i]->red_s;
    ta.nnz[i] = t[i]->nnz;
    ta.out[i] = outs ? outs[i] : nullptr;
    ta.live[i] = t[i]->live;
    ta.target[i] = msm_target_arg(*t[i]);
  }
  return ta;
}

// Empty buckets and zero nnz for n tails (before their accumulations).
template <class F>
bool msm_tails_one_c(MsmTail<F>* const* t, int n) {
  for (int i = 1; i < n; i++)
    if (t[i]->c != t[0]->c) return false;
  return true;
}

template <class F>
hipError_t msm_tails_reset(MsmTail<F>* const* t, int n, hipStream_t st) {
  if (n < 1 || n > MSM_TAIL_MAX || !msm_tails_one_c(t, n)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_msm_tail_reset<F>, dim3(128, n), dim3(256), 0, st, msm_tail_args<F>(t, nullptr, n));
  return hipGetLastError();
}

// digits (+ nnz) -> sort by bucket into pl.keys_out / pl.vals_out (the first *nnz pairs; the sort
// writes *nnz), for n <= MSM_TAIL_MAX independent MSMs of one window width at once (blockIdx.y =
// MSM): the same four launches whatever n, each MSM with its own scratch.
template <class F>
hipError_t msm_sort_multi(const MsmBases<F>* const* b, MsmScratch<F>* const* pl, uint32_t* const* nnz,
                          const uint32_t* const* sc, const uint32_t* const* ex, int n, hipStream_t st) {
  if (n < 1 || n > MSM_TAIL_MAX) return hipErrorInvalidValue;
  MsmSortArgs A = {};
  uint32_t gx = 0;
  int ny = 0;
  bool sorted = true;
  const int c = b[0]->c;
  for (int i = 0; i < n; i++) {
    const size_t m = b[i]->n;
    if (m > pl[i]->cap || b[i]->c != c || pl[i]->c != c) return hipErrorInvalidValue;
    if (m == 0) {  // nothing to sort: nnz = 0 (the tail reset left it so)
      continue;
    }
    // count / scan / scatter / bins (see k_msm_bin_count); keys_in/vals_in hold the high-bin order
    const size_t per_blk = (m + MSM_SORT_MAXBLK - 1) / MSM_SORT_MAXBLK < MSM_SORT_T
                               ? (size_t)MSM_SORT_T
                               : ((m + MSM_SORT_MAXBLK - 1) / MSM_SORT_MAXBLK + MSM_SORT_T - 1) / MSM_SORT_T * MSM_SORT_T;
    const uint32_t nblk = (uint32_t)((m + per_blk - 1) / per_blk);
    if (nblk > MSM_SORT_MAXBLK) return hipErrorInvalidValue;
    MsmSortJob& J = A.j[ny++];
    J = {sc[i], ex[i], b[i]->sidx, b[i]->extra_start, (uint32_t)m, (uint32_t)per_blk, nblk,
         static_cast<uint32_t*>(pl[i]->sort_tmp), static_cast<uint32_t*>(pl[i]->sort_tmp) + MSM_SORT_HB * MSM_SORT_MAXBLK,
         nnz[i], pl[i]->keys_in, pl[i]->vals_in, pl[i]->keys_out, pl[i]->vals_out};
    gx = std::max(gx, nblk);
    sorted = sorted && pl[i]->ko_sorted;
    pl[i]->ko_sorted = 1;
  }
  if (ny == 0) return hipSuccess;
  return msm_with_c(c, [&](auto cc) {
    constexpr int C = decltype(cc)::value;
    constexpr int NL = msm_sort_nl<C>();
    static_assert(NL >= 64 && NL <= 1024 && MSM_SORT_BINT >= NL, "bins: one thread per low counter");
    hipLaunchKernelGGL((k_msm_bin_count<C>), dim3(gx, ny), dim3(MSM_SORT_T), 0, st, A);
    hipLaunchKernelGGL(k_msm_bin_scan, dim3(1, ny), dim3(MSM_SORT_BT), 0, st, A);
    if (!(ZK_KNOCKOUT & 2) || !sorted) {  // knock-out: an MSM's own scratch keeps its first sort
      hipLaunchKernelGGL((k_msm_bin_scatter<C>), dim3(gx, ny), dim3(MSM_SORT_T), 0, st, A);
      hipLaunchKernelGGL((k_msm_bin_sort<MSM_SORT_BINT, NL>), dim3(MSM_SORT_HB, ny), dim3(MSM_SORT_BINT), 0, st, A);
    }
    return hipGetLastError();
  });
}

template <class F>
hipError_t msm_sort(const MsmBases<F>& b, MsmScratch<F>& pl, uint32_t* nnz, const uint32_t* d_scalars,
                    const uint32_t* d_extra, hipStream_t st) {
  const MsmBases<F>* bp = &b;
  MsmScratch<F>* pp = &pl;
  return msm_sort_multi(&bp, &pp, &nnz, &d_scalars, &d_extra, 1, st);
}

// Accumulation (level 0: fixed chunks, closed runs straight into the buckets, open runs as items)
// over sorted (bucket, entry) pairs and t.nnz.  The pairs may come from another MSM with the same
// scalars and base index map (B1's sort serves B2: msm_sort once, accumulate on both curves).
template <class F>
hipError_t msm_accumulate_sorted(const MsmBases<F>& b, const uint16_t* keys, const uint32_t* vals, MsmTail<F>& t,
                                 hipStream_t st, Profiler* prof = nullptr, const char* tag = nullptr) {
  if (b.n == 0) return hipSuccess;
  if (b.c != t.c) return hipErrorInvalidValue;
  const size_t m = b.n * msm_w_of(b.c);
  size_t chunks = (m + t.l0 - 1) / t.l0;
  if (t.target) chunks = std::min<size_t>(chunks, t.target);  // lanes of msm_chunk_len(nnz, target)
  if (chunks > t.max_chunks) return hipErrorInvalidValue;
  const int pidx = prof ? prof->begin(tag, st) : -1;
  using FC = typename MsmCompute<F>::type;
  constexpr int LN = MsmIO<FC>::LANES;
  constexpr int AW = sizeof(typename F::T) == 32 ? MSM_G1_WAVES : MSM_G2_WAVES;
  // measurement knob: ZKFL_ACC_PAD_LDS=<bytes> reserves unused LDS per accumulation block, which
  // lowers the number of resident waves without changing the chunking (PMC traffic attribution)
  static const size_t pad_lds = getenv("ZKFL_ACC_PAD_LDS") ? strtoul(getenv("ZKFL_ACC_PAD_LDS"), nullptr, 10) : 0;
  if (!((ZK_KNOCKOUT & 64) && LN == 1))
    hipLaunchKernelGGL((k_msm_accumulate<FC, AW>), dim3(zk_grid(chunks * LN, 64)), dim3(64), pad_lds, st, keys, vals,
                       b.bases_w, t.nnz, t.item_key[0], t.item_val[0], t.buckets, msm_target_arg(t), t.live);
  if (prof) prof->end(pidx, st, 0.0, t.nnz);
  return hipGetLastError();
}

// The accumulations of n <= MSM_TAIL_MAX MSMs of one curve over their sorted pairs (keys[i],
// vals[i]) in ONE launch (k_msm_accumulate_multi); each tail must have been reset.
template <class F>
hipError_t msm_accumulate_sorted_multi(const MsmBases<F>* const* b, const uint16_t* const* keys,
                                       const uint32_t* const* vals, MsmTail<F>* const* t, int n, hipStream_t st) {
  if (n < 1 || n > MSM_TAIL_MAX) return hipErrorInvalidValue;
  using FC = typename MsmCompute<F>::type;
  constexpr int LN = MsmIO<FC>::LANES;
  constexpr int AW = sizeof(typename F::T) == 32 ? MSM_G1_WAVES : MSM_G2_WAVES;
  MsmAccArgs<F> A = {};
  size_t gx = 0;
  int ny = 0;
  for (int i = 0; i < n; i++) {
    if (b[i]->n == 0) continue;
    if (b[i]->c != t[i]->c) return hipErrorInvalidValue;
    const size_t m = b[i]->n * msm_w_of(b[i]->c);
    size_t chunks = (m + t[i]->l0 - 1) / t[i]->l0;
    if (t[i]->target) chunks = std::min<size_t>(chunks, t[i]->target);
    if (chunks > t[i]->max_chunks) return hipErrorInvalidValue;
    gx = std::max<size_t>(gx, zk_grid(chunks * LN, 64));
    A.keys[ny] = keys[i];
    A.vals[ny] = vals[i];
    A.bases[ny] = b[i]->bases_w;
    A.nnz[ny] = t[i]->nnz;
    A.item_key[ny] = t[i]->item_key[0];
    A.item_val[ny] = t[i]->item_val[0];
    A.buckets[ny] = t[i]->buckets;
    A.target[ny] = msm_target_arg(*t[i]);
    A.live[ny] = t[i]->live;
    ny++;
  }
  if (ny && !((ZK_KNOCKOUT & 64) && LN == 1))
    hipLaunchKernelGGL((k_msm_accumulate_multi<FC, AW>), dim3((uint32_t)gx, ny), dim3(64), 0, st, A);
  return hipGetLastError();
}

// digits (+ nnz) -> radix sort by bucket -> accumulate.  The tail must have been reset
// (msm_tails_reset).  An MSM with no bases leaves nnz = 0 and empty buckets: its tail yields
// infinity.
template <class F>
hipError_t msm_accumulate(const MsmBases<F>& b, MsmScratch<F>& pl, MsmTail<F>& t, const uint32_t* d_scalars,
                          const uint32_t* d_extra, hipStream_t st, Profiler* prof = nullptr,
                          const char* tag = nullptr) {
  ZK_CHECK(msm_sort(b, pl, t.nnz, d_scalars, d_extra, st));
  return msm_accumulate_sorted(b, pl.keys_out, pl.vals_out, t, st, prof, tag);
}

// Tails of n accumulated MSMs in one batch: stitching levels until one lane holds every
// remaining item (item counts here are host-side upper bounds; the kernels use each nnz), then
// the two weighted-reduction levels, the last writing outs[i].  fast: the latency schedule's
// reduction (MSM_WSUM_Q_FAST: shorter dependent chain, more waves).
template <class F>
hipError_t msm_stitch(MsmTail<F>* const* t, int n, hipStream_t st) {
  if (n < 1 || n > MSM_TAIL_MAX || !msm_tails_one_c(t, n)) return hipErrorInvalidValue;
  using FC = typename MsmCompute<F>::type;
  constexpr int LN = MsmIO<FC>::LANES;
  constexpr int SW = sizeof(typename F::T) == 32 ? MSM_G1_STITCH_WAVES : MSM_G2_TAIL_WAVES;
  const MsmTailArgs<F> ta = msm_tail_args<F>(t, nullptr, n);
  size_t N = 0;
  for (int i = 0; i < n; i++) N = std::max(N, t[i]->item_cap[0]);
  N = std::max<size_t>(N, 2);
  int cur = 0;
  static const bool last_kernel = !getenv("ZKFL_STITCH_LAST") || atoi(getenv("ZKFL_STITCH_LAST")) != 0;
  for (int level = 1; !(ZK_KNOCKOUT & 8); level++) {
    if (level >= MSM_LIVE_LEVELS) return hipErrorInvalidValue;  // liveness flags per level
    const size_t lanes = (N + MSM_SG - 1) / MSM_SG;
    if (last_kernel && lanes <= (size_t)MSM_STITCH_LAST) {  // the remaining levels in one workgroup
      hipLaunchKernelGGL((k_msm_stitch_last<FC, SW>), dim3(1, n), dim3(MSM_STITCH_LAST * LN), 0, st, ta, level, cur);
      break;
    }
    hipLaunchKernelGGL((k_msm_stitch<FC, SW>), dim3(zk_grid(lanes * LN, 64), n), dim3(64), 0, st, ta, level, cur);
    if (N <= (size_t)MSM_SG) break;
    N = 2 * lanes;
    cur ^= 1;
  }
  return hipGetLastError();
}

// The two weighted-reduction levels of n bucket sets (ta: buckets, red_a, red_s, out of each)
template <class F>
hipError_t msm_wsum(const MsmTailArgs<F>& ta, int n, hipStream_t st, bool fast) {
  if (n < 1 || n > MSM_TAIL_MAX) return hipErrorInvalidValue;
  if (ZK_KNOCKOUT & 16) return hipGetLastError();
  using FC = typename MsmCompute<F>::type;
  constexpr int LN = MsmIO<FC>::LANES;
  constexpr int TW = sizeof(typename F::T) == 32 ? MSM_G1_TAIL_WAVES : MSM_G2_TAIL_WAVES;
  return msm_with_c(ta.c, [&](auto cc) {
    constexpr int C = decltype(cc)::value, NB = msm_nb_of(C);
    constexpr int Q0 = msm_wsum_q0<F>(), QF = msm_wsum_q_fast<C>();
    if (fast) {
      hipLaunchKernelGGL((k_msm_wsum<FC, TW, true, QF, C>), dim3(NB / (MSM_RB * QF), n), dim3(MSM_RB * LN), 0, st, ta);
      hipLaunchKernelGGL((k_msm_wsum<FC, TW, false, QF, C>), dim3(1, n), dim3(msm_wsum_rb<false, QF, C>() * LN), 0, st,
                         ta);
    } else {
      hipLaunchKernelGGL((k_msm_wsum<FC, TW, true, Q0, C>), dim3(NB / (MSM_RB * Q0), n), dim3(MSM_RB * LN), 0, st, ta);
      hipLaunchKernelGGL((k_msm_wsum<FC, TW, false, Q0, C>), dim3(1, n), dim3(msm_wsum_rb<false, Q0, C>() * LN), 0, st,
                         ta);
    }
    return hipGetLastError();
  });
}

template <class F>
hipError_t msm_tails(MsmTail<F>* const* t, XYZZ<F>* const* outs, int n, hipStream_t st, bool fast = false) {
  ZK_CHECK(msm_stitch(t, n, st));
  return msm_wsum(msm_tail_args<F>(t, outs, n), n, st, fast);
}

// The G1 tails t1[0..n1) and G2 tails t2[0..n2) of one proof as one launch sequence (the joint
// kernels above): stitching levels until every tail is down to one workgroup, the last levels of
// all of them in one launch, then the two reduction levels -> o1[i], o2[i].  Same results as
// msm_tails on each curve; one window width for all.
template <class S1, class S2>
hipError_t msm_tails_joint(MsmTail<S1>* const* t1, XYZZ<S1>* const* o1, int n1, MsmTail<S2>* const* t2,
                           XYZZ<S2>* const* o2, int n2, hipStream_t st, bool fast) {
  if (n1 < 1 || n1 > MSM_TAIL_MAX || n2 < 1 || n2 > MSM_TAIL_MAX || !msm_tails_one_c(t1, n1) ||
      !msm_tails_one_c(t2, n2) || t1[0]->c != t2[0]->c)
    return hipErrorInvalidValue;
  using F1 = typename MsmCompute<S1>::type;
  using F2 = typename MsmCompute<S2>::type;
  static_assert(msm_wsum_q0<S1>() == msm_wsum_q0<S2>(), "joint reduction: one fold per curve");
  constexpr int W = MSM_G1_TAIL_WAVES < MSM_G2_TAIL_WAVES ? MSM_G1_TAIL_WAVES : MSM_G2_TAIL_WAVES;
  constexpr int L1 = MsmIO<F1>::LANES, L2 = MsmIO<F2>::LANES;
  static_assert(L1 == 1 && L2 == 2, "joint tails: G1 lanes, G2 lane pairs");
  MsmJointArgs<S1, S2> ja;
  ja.a = msm_tail_args<S1>(t1, o1, n1);
  ja.b = msm_tail_args<S2>(t2, o2, n2);
  ja.n1 = n1;
  const int ny = n1 + n2;
  size_t N1 = 2, N2 = 2;  // host-side upper bounds of the items per level (the kernels use each nnz)
  for (int i = 0; i < n1; i++) N1 = std::max(N1, t1[i]->item_cap[0]);
  for (int i = 0; i < n2; i++) N2 = std::max(N2, t2[i]->item_cap[0]);
  int cur = 0;
  for (int level = 1; !(ZK_KNOCKOUT & 8); level++) {
    if (level >= MSM_LIVE_LEVELS) return hipErrorInvalidValue;
    const size_t lanes1 = (N1 + MSM_SG - 1) / MSM_SG, lanes2 = (N2 + MSM_SG - 1) / MSM_SG;
    if (lanes1 <= (size_t)MSM_STITCH_LAST && lanes2 <= (size_t)MSM_STITCH_LAST) {
      hipLaunchKernelGGL((k_msm_stitch_last_joint<F1, F2, W>), dim3(1, ny), dim3(2 * MSM_STITCH_LAST), 0, st, ja,
                         level, cur);
      break;
    }
    const size_t bx = std::max(zk_grid(lanes1 * L1, MSM_JOINT_T), zk_grid(lanes2 * L2, MSM_JOINT_T));
    hipLaunchKernelGGL((k_msm_stitch_joint<F1, F2, W>), dim3((uint32_t)bx, ny), dim3(MSM_JOINT_T), 0, st, ja, level, cur);
    if (N1 > (size_t)MSM_SG) N1 = 2 * lanes1;
    if (N2 > (size_t)MSM_SG) N2 = 2 * lanes2;
    cur ^= 1;
  }
  if (ZK_KNOCKOUT & 16) return hipGetLastError();
  return msm_with_c(t1[0]->c, [&](auto cc) {
    constexpr int C = decltype(cc)::value, NB = msm_nb_of(C);
    constexpr int Q0 = msm_wsum_q0<S1>(), QF = msm_wsum_q_fast<C>();
    if (fast) {
      hipLaunchKernelGGL((k_msm_wsum_joint<F1, F2, W, true, QF, C>), dim3(NB / (MSM_RB * QF), ny),
                         dim3(2 * msm_wsum_rb<true, QF, C>()), 0, st, ja);
      hipLaunchKernelGGL((k_msm_wsum_joint<F1, F2, W, false, QF, C>), dim3(1, ny), dim3(2 * msm_wsum_rb<false, QF, C>()),
                         0, st, ja);
    } else {
      hipLaunchKernelGGL((k_msm_wsum_joint<F1, F2, W, true, Q0, C>), dim3(NB / (MSM_RB * Q0), ny),
                         dim3(2 * msm_wsum_rb<true, Q0, C>()), 0, st, ja);
      hipLaunchKernelGGL((k_msm_wsum_joint<F1, F2, W, false, Q0, C>), dim3(1, ny), dim3(2 * msm_wsum_rb<false, Q0, C>()),
                         0, st, ja);
    }
    return hipGetLastError();
  });
}

template <class F>
hipError_t msm_run(const MsmBases<F>& b, MsmScratch<F>& pl, MsmTail<F>& t, const uint32_t* d_scalars,
                   const uint32_t* d_extra, XYZZ<F>* d_out, hipStream_t st, Profiler* prof = nullptr,
                   const char* tag = nullptr) {
  MsmTail<F>* tp = &t;
  ZK_CHECK(msm_tails_reset(&tp, 1, st));
  ZK_CHECK(msm_accumulate(b, pl, t, d_scalars, d_extra, st, prof, tag));
  return msm_tails(&tp, &d_out, 1, st);
}

// Non-template entry points (one translation unit per curve: msm_g1.hip / msm_g2.hip).
#define ZKFL_MSM_DEFINE(SUF, F)                                                                          \
  hipError_t zk_wtrace_bind_##SUF(const WtBuf& b) { return zk_wtrace_bind_tu(b); }                      \
  hipError_t msm_bases_alloc_##SUF(MsmBases<F>& b, size_t n, int c) { return msm_bases_alloc(b, n, c); } \
  hipError_t msm_bases_set_##SUF(MsmBases<F>& b, const Affine<F>* src, const uint32_t* h_sidx,          \
                                 uint32_t extra_start, hipStream_t st) {                                 \
    return msm_bases_set(b, src, h_sidx, extra_start, st);                                               \
  }                                                                                                      \
  void msm_bases_free_##SUF(MsmBases<F>& b) { msm_bases_free(b); }                                       \
  hipError_t msm_scratch_alloc_##SUF(MsmScratch<F>& s, size_t cap, int c, hipStream_t st) {              \
    return msm_scratch_alloc(s, cap, c, st);                                                             \
  }                                                                                                      \
  void msm_scratch_free_##SUF(MsmScratch<F>& s) { msm_scratch_free(s); }                                 \
  hipError_t msm_tail_alloc_##SUF(MsmTail<F>& t, size_t cap, int c) { return msm_tail_alloc(t, cap, c); } \
  void msm_tail_free_##SUF(MsmTail<F>& t) { msm_tail_free(t); }                                          \
  hipError_t msm_accumulate_##SUF(const MsmBases<F>& b, MsmScratch<F>& s, MsmTail<F>& t, const uint32_t* sc, \
                                  const uint32_t* ex, hipStream_t st, Profiler* prof, const char* tag) { \
    return msm_accumulate(b, s, t, sc, ex, st, prof, tag);                                               \
  }                                                                                                      \
  hipError_t msm_sort_##SUF(const MsmBases<F>& b, MsmScratch<F>& s, uint32_t* nnz, const uint32_t* sc,      \
                            const uint32_t* ex, hipStream_t st) {                                        \
    return msm_sort(b, s, nnz, sc, ex, st);                                                              \
  }                                                                                                      \
  hipError_t msm_accumulate_sorted_##SUF(const MsmBases<F>& b, const uint16_t* keys, const uint32_t* vals,  \
                                         MsmTail<F>& t, hipStream_t st, Profiler* prof, const char* tag) { \
    return msm_accumulate_sorted(b, keys, vals, t, st, prof, tag);                                       \
  }                                                                                                      \
  hipError_t msm_sort_multi_##SUF(const MsmBases<F>* const* b, MsmScratch<F>* const* s, uint32_t* const* nnz, \
                                  const uint32_t* const* sc, const uint32_t* const* ex, int n, hipStream_t st) { \
    return msm_sort_multi(b, s, nnz, sc, ex, n, st);                                                     \
  }                                                                                                      \
  hipError_t msm_accumulate_sorted_multi_##SUF(const MsmBases<F>* const* b, const uint16_t* const* keys,      \
                                               const uint32_t* const* vals, MsmTail<F>* const* t, int n,  \
                                               hipStream_t st) {                                          \
    return msm_accumulate_sorted_multi(b, keys, vals, t, n, st);                                         \
  }                                                                                                      \
  hipError_t msm_tails_##SUF(MsmTail<F>* const* t, XYZZ<F>* const* outs, int n, hipStream_t st, bool fast) { \
    return msm_tails(t, outs, n, st, fast);                                                              \
  }                                                                                                      \
  hipError_t msm_tails_reset_##SUF(MsmTail<F>* const* t, int n, hipStream_t st) {                        \
    return msm_tails_reset(t, n, st);                                                                    \
  }                                                                                                      \
  hipError_t msm_run_##SUF(const MsmBases<F>& b, MsmScratch<F>& s, MsmTail<F>& t, const uint32_t* sc,     \
                           const uint32_t* ex, XYZZ<F>* out, hipStream_t st, Profiler* prof, const char* tag) { \
    return msm_run(b, s, t, sc, ex, out, st, prof, tag);                                                 \
  }

}  // namespace zkfl
