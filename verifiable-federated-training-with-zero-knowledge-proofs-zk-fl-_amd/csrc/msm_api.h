// MSM plan object and non-template entry points (see msm.h for the algorithm).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "common.h"
#include "curve.h"
#include "prof.h"

namespace zkfl {

// Window width c of the signed-digit decomposition.  Scalars are < r < 2^254; with signed digits
// d in [-(2^(c-1) - 1), 2^(c-1)] the top window absorbs the last carry when c W >= 255, so
// W = ceil(255 / c): 19 windows at c = 14, 16 at c = 16, 15 at c = 17.  Every base is expanded into
// its W window copies at key load, so an MSM accumulates one entry per non-zero digit into ONE set
// of 2^(c-1) buckets: a wider window cuts the entries of a full-width scalar and multiplies the
// buckets the (latency-bound) reduction folds.  Bucket keys are |d| - 1 < 2^(c-1),
// a u16 for c <= 17.
// The width is chosen per MSM base set (per proving key: msm_pick_c): MSM_C for large keys, where
// the accumulation dominates, MSM_C_SMALL for keys of at most MSM_SMALL_C_BASES bases, whose
// proofs are chains of latency-bound reduction launches (config 5: 2,335 vs 2,152 proofs/s at 14
// vs 16 bits, the metric key 388 vs 427 -- profiles/r05_ab_window_bits.log).  17 bits (15 windows,
// 2^16 buckets) was measured and rejected in round 5 (config 5 -11%, M within noise:
// profiles/r05_ab_c17_c5_latency.log, r05_ab_c17_large_keys.log) and is no longer accepted.
#ifndef MSM_WINDOW_BITS
#define MSM_WINDOW_BITS 16
#endif
#ifndef MSM_WINDOW_BITS_SMALL
#define MSM_WINDOW_BITS_SMALL 14
#endif
#ifndef MSM_SMALL_C_BASES
#define MSM_SMALL_C_BASES (1 << 16)
#endif
constexpr int MSM_C = MSM_WINDOW_BITS;     // window bits of large keys
constexpr int MSM_C_SMALL = MSM_WINDOW_BITS_SMALL;
__host__ __device__ constexpr int msm_w_of(int c) { return (255 + c - 1) / c; }  // windows: 254-bit scalars + the last carry
__host__ __device__ constexpr int msm_nb_of(int c) { return 1 << (c - 1); }     // buckets (signed digits)
constexpr int MSM_W = msm_w_of(MSM_C);
constexpr int MSM_NB = msm_nb_of(MSM_C);
constexpr int MSM_W_MAX = msm_w_of(MSM_C < MSM_C_SMALL ? MSM_C : MSM_C_SMALL);
static_assert(MSM_C >= 14 && MSM_C <= 16 && MSM_C_SMALL >= 14 && MSM_C_SMALL <= 16,
              "window width: the widths the GPU parity suite runs (>= 64 low counters per high bin of the bucket sort)");
// Knock-out builds for marginal-cost measurements (tools/ko_probe.py; proofs are WRONG, timing
// only): 1 assembly, 2 digit sort, 4 NTT, 8 stitching, 16 bucket reduction, 32 the G2 MSM,
// 64 the G1 accumulation kernel.  0 in every real build; a non-zero value only compiles together
// with ZK_KNOCKOUT_AB_ONLY (tools/build_ab.sh sets both), so a wrong-proof library cannot be built
// by a stray define.
#ifndef ZK_KNOCKOUT
#define ZK_KNOCKOUT 0
#endif
#if ZK_KNOCKOUT != 0 && !defined(ZK_KNOCKOUT_AB_ONLY)
#error "ZK_KNOCKOUT builds compute wrong proofs: timing A/B only (define ZK_KNOCKOUT_AB_ONLY to acknowledge)"
#endif
// high key bits of the bucket sort (its high bins, every window width): the low c - 1 - HIGH_BITS
// bits are sorted inside one high bin (6 at c = 14, 8 at c = 16, 9 at c = 17)
#ifndef MSM_SORT_HIGH_BITS
#define MSM_SORT_HIGH_BITS 7
#endif
// pairs of one high bin staged in LDS by the bucket sort's bins pass (0: the bin is read twice)
#ifndef MSM_SORT_STAGE
#define MSM_SORT_STAGE 0
#endif
// threads per high-bin workgroup of the bucket sort's bins pass
#ifndef MSM_SORT_BIN_THREADS
#define MSM_SORT_BIN_THREADS 1024
#endif
#ifndef MSM_G1_L
#define MSM_G1_L 16
#endif
#ifndef MSM_STITCH_SG
#define MSM_STITCH_SG 8
#endif
constexpr int MSM_L = MSM_G1_L;            // sorted entries per accumulation lane (fixed-size chunks)
constexpr int MSM_SG = MSM_STITCH_SG;      // partial sums per lane in each stitching level
constexpr int MSM_RB = 64;                 // items per block (one wave) in the weighted bucket reduction
constexpr uint32_t MSM_ITEM_DUMMY = 0x80000000u;  // stitch item flag: padding (its value is infinity)
#ifndef MSM_G2_L
#define MSM_G2_L 16
#endif
// minimum chunk length of small MSMs (<= 2^16 bases), both curves (msm_tail_l0)
#ifndef MSM_SMALL_L
#define MSM_SMALL_L 8
#endif
// Chunk length per curve (storage field type S)
template <class S>
struct MsmChunk {
  static constexpr int L = MSM_L;
};
template <>
struct MsmChunk<Fq2Ops> {
  static constexpr int L = MSM_G2_L;
};
// 1 (default): the chunk length grows with the MSM so that one accumulation launch is ONE full
// round of resident lanes (msm_chunk_len); 0: every MSM uses MsmChunk<S>::L (A/B builds).
#ifndef MSM_ADAPTIVE_L
#define MSM_ADAPTIVE_L 1
#endif
// Entries per accumulation lane for an MSM with nnz sorted non-zero digits: the minimum L0, or the
// fewest that keep the lanes within `target` = the lanes the device holds at once for the
// accumulation kernel (0: always the minimum).  The kernel argument carries both: bits 0-23 the
// lanes, bits 24-31 the tail's minimum L0 (0: MsmChunk<S>::L) -- msm_target_arg.  A longer chunk leaves fewer chunk
// edges inside a bucket, and every such edge costs one full point addition in the stitching;
// the launch stays one full round of lanes, so the accumulation's own duration does not change.
// The accumulation and the stitching levels derive the same value from nnz on the device.
template <class S>
__host__ __device__ inline uint32_t msm_chunk_len(uint32_t nnz, uint32_t target) {
  const uint32_t L0 = (target >> 24) ? (target >> 24) : (uint32_t)MsmChunk<S>::L;
  target &= 0xFFFFFFu;
  if (target == 0) return L0;
  const uint32_t l = (uint32_t)(((uint64_t)nnz + target - 1) / target);
  return l > L0 ? l : L0;
}
constexpr int MSM_LIVE_LEVELS = 32;  // stitching levels with a liveness flag (level 0 = accumulation)


// Read-only, per proving key: every base expanded into its W window copies.
// Bases are compacted at key load (infinity points dropped); sidx[i] maps compacted base i to
// its scalar: sidx < extra_start -> scalars_main[sidx], else scalars_extra[sidx - extra_start]
// (the proof's 1 / r / s / -rs blinding slots).  sidx == nullptr means identity.
template <class F>
struct MsmBases {
  size_t n = 0;                  // number of (compacted) bases incl. augmentation slots
  int c = MSM_C;                 // window bits (msm_pick_c)
  Affine<F>* bases_w = nullptr;  // [n][W] expanded affine bases (device)
  uint32_t* sidx = nullptr;      // [n] scalar index map (device) or nullptr
  uint32_t extra_start = 0xFFFFFFFFu;
};

// Mutable, per in-flight proof (one stream at a time): digit/sort scratch shared by the MSMs a
// slot runs one after another.
template <class F>
struct MsmScratch {
  size_t cap = 0;                // max number of bases served
  int c = MSM_C;                 // window bits of the base sets served
  uint16_t* keys_in = nullptr;
  uint16_t* keys_out = nullptr;
  uint32_t* vals_in = nullptr;
  uint32_t* vals_out = nullptr;
  void* sort_tmp = nullptr;
  size_t sort_tmp_bytes = 0;
  int ko_sorted = 0;             // sort knock-out builds only: this scratch holds a sort already
};

// Per MSM of a proof: what the accumulation leaves for the tail (stitching + reduction), so the
// tails of several MSMs can run as one batch (one launch per level for all of them).
template <class F>
struct MsmTail {
  size_t max_chunks = 0;        // ceil(cap * W / L)
  int c = MSM_C;                // window bits of the MSMs it serves
  // stitching items (ping-pong): 2 per chunk / per stitching lane, sorted by bucket
  uint32_t* item_key[2] = {nullptr, nullptr};   // bucket | MSM_ITEM_DUMMY
  XYZZ<F>* item_val[2] = {nullptr, nullptr};
  size_t item_cap[2] = {0, 0};
  XYZZ<F>* buckets = nullptr;   // [NB]
  XYZZ<F>* red_a = nullptr;     // weighted-reduction block outputs
  XYZZ<F>* red_s = nullptr;
  uint32_t* nnz = nullptr;      // number of non-zero digits of the last run (device)
  // live[l] != 0: level l (0 = the accumulation) emitted a real open run, so level l + 1 has
  // something to stitch; a level whose predecessor emitted none returns at once (device)
  uint32_t* live = nullptr;
  uint32_t target = 0;          // accumulation lanes resident at once (msm_chunk_len; 0: fixed L)
  uint32_t l0 = 0;              // minimum entries per accumulation lane (msm_tail_l0)
};

// msm_chunk_len's argument: resident lanes (bits 0-23) | minimum chunk length (bits 24-31)
template <class F>
inline uint32_t msm_target_arg(const MsmTail<F>& t) {
  return (t.l0 << 24) | (t.target & 0xFFFFFFu);
}

// Window bits for a base set of n bases; ZKFL_MSM_C=<MSM_C | MSM_C_SMALL> forces one (tests, A/B)
inline int msm_pick_c(size_t n) {
  if (const char* e = getenv("ZKFL_MSM_C")) {
    const int c = atoi(e);
    if (c == MSM_C || c == MSM_C_SMALL) return c;
  }
  return n <= (size_t)MSM_SMALL_C_BASES ? MSM_C_SMALL : MSM_C;
}

constexpr int MSM_TAIL_MAX = 4;  // MSM tails per batched launch (the 4 G1 MSMs of a proof)
constexpr int MSM_TAIL_RED = 4 * MSM_RB;  // reduction block outputs per bucket set (<= 2 level-1 blocks of 128 lanes)

#define ZKFL_MSM_DECLARE(SUF, F)                                                                    \
  hipError_t msm_bases_alloc_##SUF(MsmBases<F>& b, size_t n, int c);                                \
  hipError_t msm_bases_set_##SUF(MsmBases<F>& b, const Affine<F>* src, const uint32_t* h_sidx,      \
                                 uint32_t extra_start, hipStream_t st);                              \
  void msm_bases_free_##SUF(MsmBases<F>& b);                                                        \
  hipError_t msm_scratch_alloc_##SUF(MsmScratch<F>& s, size_t cap, int c, hipStream_t st);          \
  void msm_scratch_free_##SUF(MsmScratch<F>& s);                                                    \
  hipError_t msm_tail_alloc_##SUF(MsmTail<F>& t, size_t cap, int c);                                \
  void msm_tail_free_##SUF(MsmTail<F>& t);                                                          \
  /* digits -> sort -> accumulation into t (the MSM is finished by msm_tails) */                    \
  hipError_t msm_accumulate_##SUF(const MsmBases<F>& b, MsmScratch<F>& s, MsmTail<F>& t,            \
                                  const uint32_t* scalars, const uint32_t* extra, hipStream_t st,    \
                                  Profiler* prof, const char* tag);                                  \
  /* empty buckets + zero nnz of n <= MSM_TAIL_MAX tails (before their accumulations) */              \
  hipError_t msm_tails_reset_##SUF(MsmTail<F>* const* t, int n, hipStream_t st);                     \
  hipError_t msm_sort_##SUF(const MsmBases<F>& b, MsmScratch<F>& s, uint32_t* nnz, const uint32_t* sc,  \
                            const uint32_t* ex, hipStream_t st);                                        \
  hipError_t msm_accumulate_sorted_##SUF(const MsmBases<F>& b, const uint16_t* keys, const uint32_t* vals, \
                                         MsmTail<F>& t, hipStream_t st, Profiler* prof, const char* tag);  \
  /* stitching + bucket reduction of n <= MSM_TAIL_MAX accumulated MSMs -> outs[i] (device) */      \
  hipError_t msm_tails_##SUF(MsmTail<F>* const* t, XYZZ<F>* const* outs, int n, hipStream_t st,     \
                             bool fast = false);                                                      \
  hipError_t msm_run_##SUF(const MsmBases<F>& b, MsmScratch<F>& s, MsmTail<F>& t, const uint32_t* scalars, \
                           const uint32_t* extra, XYZZ<F>* out, hipStream_t st, Profiler* prof, const char* tag); \
  /* n <= MSM_TAIL_MAX independent MSMs of one window width: their sorts in the same four launches, */   \
  /* their accumulations in one launch (blockIdx.y = MSM) */                                             \
  hipError_t msm_sort_multi_##SUF(const MsmBases<F>* const* b, MsmScratch<F>* const* s, uint32_t* const* nnz, \
                                  const uint32_t* const* sc, const uint32_t* const* ex, int n, hipStream_t st); \
  hipError_t msm_accumulate_sorted_multi_##SUF(const MsmBases<F>* const* b, const uint16_t* const* keys,      \
                                               const uint32_t* const* vals, MsmTail<F>* const* t, int n,  \
                                               hipStream_t st);

ZKFL_MSM_DECLARE(g1, FqOps)
ZKFL_MSM_DECLARE(g2, Fq2Ops)

// The G1 tails and the G2 tail of one proof as ONE launch sequence (msm_joint.hip): stitching and
// reduction of both curves side by side, blockIdx.y over all n1 + n2 MSMs
hipError_t msm_tails_joint(MsmTail<FqOps>* const* t1, XYZZ<FqOps>* const* o1, int n1, MsmTail<Fq2Ops>* const* t2,
                           XYZZ<Fq2Ops>* const* o2, int n2, hipStream_t st, bool fast);

}  // namespace zkfl
