// sort.hip -- rocPRIM pair sort for the kNN initialisation's Morton order (knn.hip).  The
// rasterizer's depth sort is dsort.hip.  Kept in its own translation unit: rocPRIM's templates
// dominate compile time.
#include <cstring>
#include <rocprim/rocprim.hpp>
#include "gsr_launch.h"

namespace gsr {

namespace {
// rocPRIM routes radix sorts of up to 2^20 items through block-sort + 10 merge passes; for the
// P ~ 1M depth keys that is ~150 us/frame on MI355X vs a few onesweep passes.  Cap the merge path.
#ifndef GSR_DEPTH_RADIX_BITS
#define GSR_DEPTH_RADIX_BITS 0
#endif
#if GSR_DEPTH_RADIX_BITS
using OnesweepCfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 12>, rocprim::kernel_config<256, 12>,
                                        GSR_DEPTH_RADIX_BITS>,
    8192>;
#else
using OnesweepCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                               rocprim::default_config, 8192>;
#endif

}  // namespace

size_t sort_pairs_temp_bytes(size_t n, int end_bit) {
    size_t bytes = 0;
    rocprim::radix_sort_pairs<OnesweepCfg>(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                           (const uint32_t *)nullptr, (uint32_t *)nullptr, n > 0 ? n : 1, 0, end_bit);
    return bytes;
}

hipError_t sort_pairs(void *tmp, size_t tmp_bytes, const uint32_t *kin, uint32_t *kout, const uint32_t *vin,
                      uint32_t *vout, size_t n, int end_bit, hipStream_t s) {
    if (n == 0) return hipSuccess;
    return rocprim::radix_sort_pairs<OnesweepCfg>(tmp, tmp_bytes, kin, kout, vin, vout, n, 0, end_bit, s);
}

}  // namespace gsr
