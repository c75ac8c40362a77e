// The joint G1 + G2 tails (msm.h k_msm_*_joint): both curves' tail kernels in one translation unit.
#include "msm.h"

namespace zkfl {
hipError_t zk_wtrace_bind_joint(const WtBuf& b) { return zk_wtrace_bind_tu(b); }
hipError_t msm_tails_joint(MsmTail<FqOps>* const* t1, XYZZ<FqOps>* const* o1, int n1, MsmTail<Fq2Ops>* const* t2,
                           XYZZ<Fq2Ops>* const* o2, int n2, hipStream_t st, bool fast) {
  return msm_tails_joint<FqOps, Fq2Ops>(t1, o1, n1, t2, o2, n2, st, fast);
}
}  // namespace zkfl
