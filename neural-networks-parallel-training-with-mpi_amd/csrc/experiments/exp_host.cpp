// Host-side experiment entry points (NNMPI_BUILD_EXPERIMENTS=1 builds only; the production
// library reaches them through weak references in kernels/kernels.h, null there).
#include <hip/hip_ext.h>

#include "kernels/kernels.h"

namespace nnmpi {

// A stream restricted to a set of CUs (bit i of word i / 32 = CU i): the CU-partitioned
// concurrency A/B of round 4 (scripts/r4_cu_split_ab.py).
hipError_t exp_cu_mask_stream(const uint32_t* mask, int words, hipStream_t* out) {
  return hipExtStreamCreateWithCUMask(out, (uint32_t)words, mask);
}

}  // namespace nnmpi
