// Wave-level timeline of the prover's kernels (build flag ZK_WTRACE=1; 0, the default, compiles
// it out).  Every instrumented kernel's waves append one record {kind, HW_ID, start, end, start
// cycle, end cycle}: the start when the wave begins, the end when its last lane leaves (64-bit
// atomicMax), from s_memrealtime (100 MHz) and s_memtime (shader clock) -- so each wave also gives
// the clock it ran at.  rocprofv3's kernel trace cost the 20-slot bench a third of its
// throughput (275 vs 420 proofs/s); these records cost one atomic and one store per wave, so the
// timeline they give is the unperturbed one: which kernels share the GPU, how many waves each
// keeps resident, how long a wave of each takes under load.  Records go to a device buffer that
// each translation unit binds (zk_wtrace_bind_*), driven by zkfl_debug_wtrace (tools/wtrace.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef ZK_WTRACE
#define ZK_WTRACE 0
#endif

namespace zkfl {

struct WtRec {
  uint32_t kind, hwid;
  unsigned long long t0, t1;  // s_memrealtime (100 MHz)
  unsigned long long c0, c1;  // s_memtime (shader clock cycles): (c1 - c0) / (t1 - t0) = the clock
};
struct WtBuf {
  WtRec* rec = nullptr;
  uint32_t* cnt = nullptr;
  uint32_t cap = 0;
};

// kinds (tools/wtrace.py names them); G2 variants of the MSM kernels add WT_G2, the joint tails WT_JOINT
enum : uint32_t {
  WT_ACC = 1, WT_STITCH, WT_WSUM0, WT_WSUM1, WT_SORT_COUNT, WT_SORT_SCAN, WT_SORT_SCATTER, WT_SORT_BINS,
  WT_TAIL_RESET, WT_NTT_COLS_INV, WT_NTT_LDS, WT_NTT_COLS_FWD, WT_ABC, WT_ABC_ROWS, WT_JOIN, WT_ASSEMBLE,
  WT_SET_EXTRA, WT_WITNESS, WT_G2 = 32, WT_JOINT = 64  // joint G1 + G2 tail kernels
};

#if ZK_WTRACE
static __device__ WtBuf zk_wt;  // one per translation unit, bound by its zk_wtrace_bind_*

struct WtScope {
  WtRec* r = nullptr;
  __device__ explicit WtScope(uint32_t kind) {
    const uint64_t act = __ballot(1);
    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)act) - 1;
    const bool lead = (threadIdx.x & 63) == leader;
    uint32_t idx = 0xFFFFFFFFu;
    if (lead && zk_wt.rec) idx = atomicAdd(zk_wt.cnt, 1u);
    idx = __shfl(idx, (int)leader);
    if (idx < zk_wt.cap) {
      r = zk_wt.rec + idx;
      if (lead) {
        const unsigned long long t = wall_clock64();
        r->kind = kind;
        r->hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID: wave, SIMD, CU, SH, SE
        const unsigned long long c = clock64();
        r->t0 = t;
        r->t1 = t;
        r->c0 = c;
        r->c1 = c;
      }
    }
  }
  __device__ ~WtScope() {
    if (r) {
      atomicMax(&r->t1, (unsigned long long)wall_clock64());
      atomicMax(&r->c1, (unsigned long long)clock64());
    }
  }
};
#define ZK_WT(kind) ::zkfl::WtScope zk_wt_scope_(kind)
static inline hipError_t zk_wtrace_bind_tu(const WtBuf& b) {
  return hipMemcpyToSymbol(HIP_SYMBOL(zk_wt), &b, sizeof(b));
}
#else
#define ZK_WT(kind) ((void)0)
static inline hipError_t zk_wtrace_bind_tu(const WtBuf&) { return hipErrorNotSupported; }
#endif

// binders of the other translation units (msm_g1.hip, msm_g2.hip, ntt.hip, witness.hip)
hipError_t zk_wtrace_bind_g1(const WtBuf& b);
hipError_t zk_wtrace_bind_g2(const WtBuf& b);
hipError_t zk_wtrace_bind_ntt(const WtBuf& b);
hipError_t zk_wtrace_bind_wit(const WtBuf& b);
hipError_t zk_wtrace_bind_joint(const WtBuf& b);

}  // namespace zkfl
