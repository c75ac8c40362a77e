// G2 (Fq2) instantiation of the MSM engine.
#include "msm.h"

namespace zkfl {
ZKFL_MSM_DEFINE(g2, Fq2Ops)
}  // namespace zkfl
