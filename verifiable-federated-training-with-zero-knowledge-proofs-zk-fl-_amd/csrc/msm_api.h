// MSM plan object and non-template entry points (see msm.h for the algorithm).
#pragma once
#include <hip/hip_runtime.h>

#include "common.h"
#include "curve.h"
#include "prof.h"

namespace zkfl {

constexpr int MSM_C = 16;                  // window bits
constexpr int MSM_W = 16;                  // windows covering 256 bits (scalars < r < 2^254)
constexpr int MSM_NB = 1 << (MSM_C - 1);   // buckets (signed digits)
constexpr int MSM_L = 32;                  // entries per accumulation task
constexpr int MSM_RG = 8;                  // running-sum group size in the bucket reduction
constexpr uint16_t MSM_KEY_NONE = 0xFFFFu; // zero digit: sorted past every bucket


template <class F>
struct MsmPlan {
  size_t n = 0;                  // number of bases (including augmentation slots)
  Affine<F>* bases_w = nullptr;  // [n][W] expanded affine bases (device)
  // scratch
  uint16_t* keys_in = nullptr;
  uint16_t* keys_out = nullptr;
  uint32_t* vals_in = nullptr;
  uint32_t* vals_out = nullptr;
  void* sort_tmp = nullptr;
  size_t sort_tmp_bytes = 0;
  void* scan_tmp = nullptr;
  size_t scan_tmp_bytes = 0;
  uint32_t* bstart = nullptr;  // [NB]
  uint32_t* bend = nullptr;    // [NB]
  uint32_t* tcount = nullptr;  // [NB]
  uint32_t* toff = nullptr;    // [NB + 1]
  size_t max_tasks = 0;
  XYZZ<F>* partials = nullptr;  // [max_tasks]
  XYZZ<F>* buckets = nullptr;   // [NB]
  XYZZ<F>* red_acc = nullptr;   // reduction scratch (all levels), [NB]
  XYZZ<F>* red_run = nullptr;   // [NB]
  XYZZ<F>* red_tmp = nullptr;   // [NB]
  uint32_t* nnz = nullptr;      // number of non-zero digits of the last run (device)
};

hipError_t msm_alloc_g1(MsmPlan<FqOps>& pl, size_t n, hipStream_t st);
void msm_free_g1(MsmPlan<FqOps>& pl);
hipError_t msm_set_bases_g1(MsmPlan<FqOps>& pl, const Affine<FqOps>* b, hipStream_t st);
hipError_t msm_run_g1(MsmPlan<FqOps>& pl, const uint32_t* s, XYZZ<FqOps>* out, hipStream_t st, Profiler* prof,
                      const char* tag);
hipError_t msm_alloc_g2(MsmPlan<Fq2Ops>& pl, size_t n, hipStream_t st);
void msm_free_g2(MsmPlan<Fq2Ops>& pl);
hipError_t msm_set_bases_g2(MsmPlan<Fq2Ops>& pl, const Affine<Fq2Ops>* b, hipStream_t st);
hipError_t msm_run_g2(MsmPlan<Fq2Ops>& pl, const uint32_t* s, XYZZ<Fq2Ops>* out, hipStream_t st, Profiler* prof,
                      const char* tag);

}  // namespace zkfl
