// G1 instantiation of the MSM engine (separate TU: parallel build, smaller register-allocation units).
#include "msm.h"

namespace zkfl {
ZKFL_MSM_DEFINE(g1, FqOps)
}  // namespace zkfl
