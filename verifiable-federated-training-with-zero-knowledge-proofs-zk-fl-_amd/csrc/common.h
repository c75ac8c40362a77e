// Small shared helpers for the HIP translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace zkfl {

#define ZK_CHECK(x)                                                             \
  do {                                                                          \
    hipError_t _e = (x);                                                        \
    if (_e != hipSuccess) return _e;                                            \
  } while (0)

// Issue priority (s_setprio, 0..3) of the latency-bound kernels of a proof (sort, NTT, ABC,
// stitching, bucket reduction, assembly).  Under the 20-slot load their waves share SIMDs with
// VALU-saturating accumulation waves and, at equal priority, ran 2-10x slower than alone
// (tools/wtrace.py: sort_bins 205 vs 68 us, NTT columns 97 vs 44 us), holding their registers all
// that time.  Raised, their few instructions issue first and their registers come back sooner;
// the accumulations lose only the issue slots that work needs anyway.  0: no priority (A/B).
#ifndef ZK_LIGHT_PRIO
#define ZK_LIGHT_PRIO 3
#endif
#if defined(__HIP_DEVICE_COMPILE__)
#define ZK_LIGHT()                                                     \
  do {                                                                 \
    if (ZK_LIGHT_PRIO > 0) __builtin_amdgcn_s_setprio(ZK_LIGHT_PRIO);  \
  } while (0)
#else
#define ZK_LIGHT() ((void)0)
#endif

static inline unsigned zk_grid(size_t n, unsigned block) {
  return (unsigned)((n + block - 1) / block);
}

}  // namespace zkfl
