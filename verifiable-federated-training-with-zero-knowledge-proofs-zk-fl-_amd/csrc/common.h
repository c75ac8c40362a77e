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

static inline unsigned zk_grid(size_t n, unsigned block) {
  return (unsigned)((n + block - 1) / block);
}

}  // namespace zkfl
